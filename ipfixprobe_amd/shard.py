"""Multi-GPU sharding of the path.

The reference scales by running one independent pipeline -- input thread + private
NHTFlowCache -- per NIC queue, with symmetric RSS keeping both directions of a biflow on the
same queue (ipfixprobe.cpp:381-464, dpdkDevice.cpp:230-262); caches never exchange state.
Here: one process and one engine per GPU, and a direction-free flow hash
`lo = min(XXH64(key), XXH64(key_inv))` picks the rank, so both directions of a biflow land on
the same GPU.  It stands for the NIC's symmetric RSS hash and is not the table key (that is
XXH64 of the canonical-order key, ipxg_table.hpp; cache.cpp:84-92 keys on the forward and the
inverse hash): ownership only needs some function both directions share.  The only exchange is
the gather of the per-GPU export buffers to rank 0: `gather_records` (an all-gather of the
record counts, then point-to-point transfers) or, for the IPFIX message streams formatted on
each GPU every step, `StreamGather` (the exact stream bytes, point to point, sized by headers
gathered one step earlier, so no rank waits on the host for the others' sizes and the exchange
runs on a side stream behind the next step's kernels).  RCCL over xGMI on GPUs; gloo on CPU
tensors in the tests.
"""
import numpy as np

RECORD_BYTES = 128  # sizeof(ipxg_flow_record)


def owner(lo, world):
    """Rank owning canonical hash `lo` (numpy uint64 array or int): its low 32 bits split into
    `world` equal ranges.  (Not the high bits: lo is the minimum of two hashes, so its high
    bits are skewed towards zero -- rank 0 of 8 would own 23 % of the flows; the low bits of
    the minimum are uniform.)"""
    if isinstance(lo, np.ndarray):
        lo = lo.astype(np.uint64)
        return (((lo & np.uint64(0xFFFFFFFF)) * np.uint64(world)) >> np.uint64(32)).astype(np.int64)
    return ((int(lo) & 0xFFFFFFFF) * world) >> 32


def canonical(hash_fwd, hash_inv):
    """The table key of a packet from its two key hashes (the parser's hash_fwd/hash_inv)."""
    return np.minimum(np.asarray(hash_fwd, dtype=np.uint64), np.asarray(hash_inv, dtype=np.uint64))


def gather_records(buf, n, rank, world, device):
    """Gather every rank's first `n` export records (`buf`: a uint8 tensor on `device` holding
    at least n * 128 bytes) into rank 0.  Returns the concatenation (uint8 tensor, rank order)
    on rank 0 and None elsewhere.  Collective: every rank must call it."""
    import torch
    import torch.distributed as dist
    cnt = torch.tensor([n], dtype=torch.int64, device=device)
    counts = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    mine = buf[: n * RECORD_BYTES]
    if rank == 0:
        out = torch.empty(sum(counts) * RECORD_BYTES, dtype=torch.uint8, device=device)
        out[: n * RECORD_BYTES].copy_(mine)
        off = n * RECORD_BYTES
        reqs = []
        for r in range(1, world):
            if counts[r]:
                reqs.append(dist.irecv(out[off: off + counts[r] * RECORD_BYTES], src=r))
            off += counts[r] * RECORD_BYTES
        for q in reqs:
            q.wait()
        return out
    if n:
        dist.send(mine.contiguous(), dst=0)
    return None


class StreamGather:
    """Exact-size gather of every rank's per-step byte stream (its IPFIX messages) to rank 0 --
    the path's only exchange.  Step k: each rank copies its stream into a buffer of
    its own (the producer may then reuse its buffer) and gathers a 16-byte header (stream bytes,
    records) to rank 0; the streams themselves move one step later, point to point, exactly the
    bytes each rank produced, sized by the headers rank 0 gathered the step before -- by then
    long complete, so rank 0's host reads them from pinned memory without waiting on the
    exchange, and nothing is padded to a worst case.  A stream of any size fits (the buffers
    grow), so no rank can fail alone inside a collective.

    Every rank calls push() the same number of times and then flush() (collective).  On GPUs the
    caller runs it inside `with torch.cuda.stream(side)`; `copied` (a torch.cuda.Event, optional)
    is recorded once the stream has been copied.  On CPU tensors (gloo) every call is
    synchronous.  Rank 0 keeps what it received of the last step (`last`: [(rank, uint8 tensor,
    records)]) and the totals (`received_bytes`, `received_records`, `header_bytes`)."""

    HEADER = 16  # two little-endian int64: stream bytes, records

    def __init__(self, rank, world, device, keep_last=True):
        import torch
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.bufs = [torch.zeros(256, dtype=torch.uint8, device=self.device) for _ in range(2)]
        self.hdr = [torch.zeros(2, dtype=torch.int64, device=self.device) for _ in range(2)]
        self.hdrs = [[torch.zeros(2, dtype=torch.int64, device=self.device) for _ in range(world)]
                     for _ in range(2)] if rank == 0 else None
        self.hdr_host = [torch.zeros((world, 2), dtype=torch.int64, pin_memory=self.cuda) for _ in range(2)] \
            if rank == 0 else None
        self.hdr_ev = [None, None]
        self.prev = None  # (buffer index, own bytes, own records)
        self.k = 0
        self.keep_last = keep_last
        self.last = []
        self.sent_bytes = self.sent_records = 0  # this rank's streams
        self.received_bytes = self.received_records = self.header_bytes = 0  # rank 0

    def push(self, src, nbytes, records, copied=None, counts=None, copy=True):
        """Step k's stream: `src` (uint8 tensor) holding `nbytes` bytes of `records` records.
        `counts` (optional): a 2-element int64 tensor on the device holding the same {nbytes,
        records}, written by the producer in stream order (Engine.device_ipfix_counts) -- the
        header is then a device copy, no host value in it.  copy=False: `src` is sent as it is,
        one push later -- the producer keeps it valid until then (the engine's two alternating
        message buffers) and may overwrite it once `copied` has fired, which is recorded after
        that send."""
        import torch
        import torch.distributed as dist
        self._move_prev()
        i = self.k % 2
        if not copy:
            self.bufs[i] = src
        else:
            if self.bufs[i].numel() < nbytes:
                self.bufs[i] = torch.zeros(max(nbytes, 2 * self.bufs[i].numel()), dtype=torch.uint8, device=self.device)
            if nbytes:
                self.bufs[i][:nbytes].copy_(src[:nbytes])
        if counts is not None:
            self.hdr[i].copy_(counts)  # the producer's own device counts
        else:
            self.hdr[i][0].fill_(int(nbytes))
            self.hdr[i][1].fill_(int(records))
        if copied is not None:
            copied.record()  # (copy: the producer's buffer is free from here; else: the previous one is)
        if self.world > 1:
            dist.gather(self.hdr[i], self.hdrs[i] if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.hdr_host[i].copy_(torch.stack(self.hdrs[i]) if self.world > 1 else self.hdr[i].view(1, 2),
                                   non_blocking=self.cuda)
            if self.cuda:
                self.hdr_ev[i] = torch.cuda.Event()
                self.hdr_ev[i].record()
            self.header_bytes += self.HEADER * self.world
        self.prev = (i, int(nbytes), int(records))
        self.sent_bytes += int(nbytes)
        self.sent_records += int(records)
        self.k += 1

    def flush(self):
        self._move_prev()

    def _move_prev(self):
        import torch
        import torch.distributed as dist
        if self.prev is None:
            return
        i, nb, nr = self.prev
        self.prev = None
        ops = []
        if self.rank == 0:
            if self.hdr_ev[i] is not None:
                self.hdr_ev[i].synchronize()  # the step-before's header gather: long complete
            sizes = self.hdr_host[i].tolist()
            got = [(0, self.bufs[i][:nb], nr)]
            for r in range(1, self.world):
                n, rec = int(sizes[r][0]), int(sizes[r][1])
                t = torch.empty(n, dtype=torch.uint8, device=self.device)
                if n:
                    ops.append(dist.P2POp(dist.irecv, t, r))
                got.append((r, t, rec))
                self.received_bytes += n
                self.received_records += rec
            self.received_bytes += nb  # rank 0's own stream: local, not moved
            self.received_records += nr
            if self.keep_last:
                self.last = got
        elif nb:
            ops.append(dist.P2POp(dist.isend, self.bufs[i][:nb], 0))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
