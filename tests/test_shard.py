"""Multi-GPU sharding (ipfixprobe_amd/shard.py): flows partitioned by the
canonical hash never share state, so the union of per-rank results equals one run over the
whole capture; the export gather runs over torch.distributed (gloo on CPU here, RCCL on the
GPUs in bench.py)."""
import os
import socket
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))

import flowcmp  # noqa: E402
import oracle_py  # noqa: E402
import synth  # noqa: E402
from ipfixprobe_amd import shard  # noqa: E402
from pcaputil import FLOW_DTYPE  # noqa: E402


def _capture(seed=21):
    return synth.flow_stream(seed=seed, n_flows=120, n_pkts=2500, frag=False, v6_share=0.3,
                             vlan_share=0.2).batch()


def _owners(arena, desc, world):
    pk, _ = oracle_py.parse_batch(arena, desc, 1)
    return shard.owner(shard.canonical(pk["hash_fwd"], pk["hash_inv"]), world)


def test_owner_covers_ranks_and_is_symmetric():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 2**64, 20000, dtype=np.uint64)  # two independent key hashes
    b = rng.integers(0, 2**64, 20000, dtype=np.uint64)
    for world in (1, 2, 4, 8):
        o = shard.owner(shard.canonical(a, b), world)
        assert o.min() >= 0 and o.max() < world
        assert np.array_equal(o, shard.owner(shard.canonical(b, a), world))  # both directions
        if world > 1:
            share = np.bincount(o, minlength=world) / len(o)
            assert share.min() > 0.85 / world and share.max() < 1.15 / world  # balanced
    assert shard.owner(0xFFFFFFFF, 8) == 7 and shard.owner(0xFFFFFFFF00000000, 8) == 0


def test_shard_union_equals_whole_capture_oracle():
    """The sharding rule itself: per-shard caches over the shards' packets give exactly the
    records of one cache over everything (so ranks never need to exchange flow state)."""
    arena, desc = _capture()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    own = _owners(arena, desc, 4)
    parts = []
    for r in range(4):
        got, _ = oracle_py.run_capture(arena, np.ascontiguousarray(desc[own == r]), 1, cache_exp=20)
        parts.append(got)
    d = flowcmp.diff(np.concatenate(parts), want)
    assert not d, d


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena, desc = _capture()
        own = _owners(arena, desc, world)
        got, _ = oracle_py.run_capture(arena, np.ascontiguousarray(desc[own == rank]), 1, cache_exp=20)
        buf = torch.from_numpy(np.ascontiguousarray(got).view(np.uint8).copy())
        out = shard.gather_records(buf, len(got), rank, world, torch.device("cpu"))
        if rank == 0:
            recs = out.numpy().view(FLOW_DTYPE)
            want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
            d = flowcmp.diff(recs, want)
            assert not d, d
        else:
            assert out is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shards_gather_to_rank0(world):
    """world_size > 1 on CPU: each rank handles its shard, gather_records brings every
    record to rank 0, which matches one run over the whole capture."""
    import torch.multiprocessing as mp
    mp.spawn(_gloo_worker, args=(world, _free_port()), nprocs=world, join=True)


@pytest.mark.gpu
def test_engine_shards_union_equals_whole_capture():
    """One engine per shard (as one per GPU): the union of their exports is the oracle's
    result over the whole capture."""
    from ipfixprobe_amd import run_capture
    arena, desc = _capture(seed=22)
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    own = _owners(arena, desc, 2)
    parts = [run_capture(arena, np.ascontiguousarray(desc[own == r]))[0] for r in range(2)]
    d = flowcmp.diff(np.concatenate(parts), want)
    assert not d, d


@pytest.mark.gpu
def test_rccl_gather_single_rank_aliases_device_exports():
    """bench.py's N > 1 step on one rank: the export buffer aliased zero-copy as a torch tensor
    (__cuda_array_interface__) and gathered over RCCL (world size 1) equals ipxg_poll_exports."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    import bench
    from ipfixprobe_amd import Engine
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        arena, desc = _capture(seed=24)
        with Engine() as e:
            e.submit(arena, desc)
            e.finish()
            ptr, n = e.device_exports()
            buf = torch.as_tensor(bench._DevArray(ptr, max(n, 1) * 128), device=dev)
            out = shard.gather_records(buf, n, 0, 1, dev)
            got = out.cpu().numpy().view(FLOW_DTYPE)
            want = e.poll()
        assert n == len(want) > 0
        assert got.tobytes() == want.tobytes()
    finally:
        dist.destroy_process_group()
