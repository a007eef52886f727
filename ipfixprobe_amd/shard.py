"""Multi-GPU sharding of the path.

The reference scales by running one independent pipeline -- input thread + private
NHTFlowCache -- per NIC queue, with symmetric RSS keeping both directions of a biflow on the
same queue (ipfixprobe.cpp:381-464, dpdkDevice.cpp:230-262); caches never exchange state.
Here: one process and one engine per GPU, and the canonical flow hash
`lo = min(XXH64(key), XXH64(key_inv))` (the table key, cache.cpp:84-92 / ipxg_table.hpp)
picks the rank, so both directions of a biflow land on the same GPU.  The only exchange is
the gather of the per-GPU export buffers to rank 0: `gather_records` (an all-gather of the
record counts, then point-to-point transfers) or, for IPFIX message streams formatted on each
GPU, `gather_slots` (one fixed-size slot per rank -- the stream's length in its header -- so no
rank waits on the host for the others' sizes and the gather can run on a side stream, behind
the next step's kernels).  RCCL over xGMI on GPUs; gloo on CPU tensors in the tests.
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


SLOT_HEADER = 16  # little-endian u64 stream bytes, u64 records


def ipfix_stream_bound(records):
    """Bytes of an IPFIX message stream of `records` basic records, templates included (at
    least 13 records per message of 1458 bytes: 16 + 4 + 13 * 105; two more messages for the
    template message and a flush that splits the two templates' sets)."""
    return 196 + records * 105 + (records // 13 + 3) * 20


def pack_slot(slot, stream, nbytes, records):
    """Header + the first nbytes of `stream` (uint8 tensor) into `slot` (uint8 tensor of the
    agreed slot size, same device), with stream-ordered copies (no host synchronisation)."""
    if SLOT_HEADER + nbytes > slot.numel():
        raise ValueError("IPFIX stream of %d bytes exceeds the slot (%d)" % (nbytes, slot.numel()))
    hdr = slot[:SLOT_HEADER].view(torch_int64())  # two scalar fills on the device
    hdr[0] = nbytes
    hdr[1] = records
    if nbytes:
        slot[SLOT_HEADER:SLOT_HEADER + nbytes].copy_(stream[:nbytes])


def torch_int64():
    import torch
    return torch.int64


def gather_slots(slot, rank, world):
    """Every rank's slot into rank 0 (dist.gather on the current stream): a list of world
    tensors on rank 0, None elsewhere.  Collective: every rank must call it."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [slot]
    out = [torch.empty_like(slot) for _ in range(world)] if rank == 0 else None
    dist.gather(slot, out, dst=0)
    return out


def unpack_slots(slots):
    """[(stream bytes as a numpy uint8 array, records)] from gathered slots (host copies)."""
    res = []
    for s in slots:
        a = s.cpu().numpy()
        nb, nr = (int(v) for v in a[:SLOT_HEADER].view(np.int64))
        res.append((a[SLOT_HEADER:SLOT_HEADER + nb], nr))
    return res
