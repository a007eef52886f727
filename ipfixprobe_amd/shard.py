"""Multi-GPU sharding of the path.

The reference scales by running one independent pipeline -- input thread + private
NHTFlowCache -- per NIC queue, with symmetric RSS keeping both directions of a biflow on the
same queue (ipfixprobe.cpp:381-464, dpdkDevice.cpp:230-262); caches never exchange state.
Here: one process and one engine per GPU, and the canonical flow hash
`lo = min(XXH64(key), XXH64(key_inv))` (the table key, cache.cpp:84-92 / ipxg_table.hpp)
picks the rank, so both directions of a biflow land on the same GPU.  The only exchange is
the gather of the per-GPU export buffers to rank 0 (`gather_records`): an all-gather of the
record counts, then point-to-point transfers (RCCL over xGMI on GPUs; gloo on CPU tensors
in the tests).
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
