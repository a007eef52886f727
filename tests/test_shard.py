"""Multi-GPU sharding (ipfixprobe_amd/shard.py): flows partitioned by the
canonical hash never share state, so the union of per-rank results equals one run over the
whole capture; the export gather runs over torch.distributed (gloo on CPU here, RCCL on the
GPUs in bench.py)."""
import json
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


def _gloo_ipfix_worker(rank, world, port, q):
    """bench.py's N > 1 export step on CPU: each rank's flows exported as IPFIX streams (the
    oracle's exporter, observation domain = rank) over two steps, moved to rank 0 by
    StreamGather, which decodes every stream."""
    import torch
    import torch.distributed as dist
    import ipfixdec
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena, desc = _capture(seed=31)
        own = _owners(arena, desc, world)
        got, _ = oracle_py.run_capture(arena, np.ascontiguousarray(desc[own == rank]), 1, cache_exp=20)
        x = oracle_py.ipfix_exporter(odid=rank, export_time=5)
        half = len(got) // 2
        g = shard.StreamGather(rank, world, "cpu")
        streams = []
        for part in (got[:half], got[half:]):  # two steps: the second without the template message
            stream, _ = oracle_py.ipfix_export(x, part)
            g.push(torch.from_numpy(stream.copy()), len(stream), len(part))
            streams.append(len(stream))
            if rank == 0 and len(streams) == 2:
                first = [(r, t.numpy().copy(), nr) for r, t, nr in g.last]
        g.flush()
        if rank == 0:
            recs, wire = [], 0
            for (r, b0, n0), (r1, b1, n1) in zip(first, g.last):
                assert r == r1
                msgs, tm, rr0, _, _ = ipfixdec.decode(b0)
                msgs1, _, rr1, _, _ = ipfixdec.decode(b1, tm)
                assert all(m["odid"] == r for m in msgs + msgs1) and len(rr0) == n0 and len(rr1) == n1
                recs += [rr0, rr1]
                wire += len(b0) + len(b1)
            want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
            allr = np.concatenate(recs)
            assert ipfixdec.basic_view(allr) == ipfixdec.basic_view(want)
            q.put((wire, g.received_bytes, g.received_records))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_gloo_ipfix_streams_gather_to_rank0(world):
    """world_size 4 / 8 on CPU: the exact N > 1 export step of bench.py (IPFIX stream per rank
    and step -> StreamGather to rank 0); the union of the decoded records is the whole capture's,
    and rank 0 received exactly the streams' bytes (DESIGN.md 6's volume: no padding)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_gloo_ipfix_worker, args=(world, _free_port(), q), nprocs=world, join=True)
    wire, moved, nrec = q.get(timeout=10)
    assert nrec > 100 and moved == wire


@pytest.mark.gpu
def test_bench_export_gather_single_rank():
    """bench.py's N > 1 export step (ExportGather: device IPFIX stream -> StreamGather on a side
    stream) at world size 1 over RCCL: the streams rank 0 holds decode to the engine's flows."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    import bench
    import ipfixdec
    from ipfixprobe_amd import Engine
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(_free_port()))
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        arena, desc = _capture(seed=25)
        want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
        with Engine() as e:
            g = bench.ExportGather(e, 0, 1, dev)
            got = []
            for _ in range(2):  # two steps: the second stream has no template message
                e.submit(arena, desc)
                e.finish()
                g.step()
                torch.cuda.synchronize()
                got.append([(r, t.cpu().numpy().copy(), nr) for r, t, nr in g.g.last])
            g.flush()
            torch.cuda.synchronize()
            got.append([(r, t.cpu().numpy().copy(), nr) for r, t, nr in g.g.last])
            assert g.device_ms() > 0
        # got[1] holds step 0's stream (moved during step 1's push), got[2] step 1's (the flush)
        (_, b0, n0), = got[1]
        (_, b1, n1), = got[2]
        _, t0, _, _, _ = ipfixdec.decode(b0)
        msgs, _, recs, _, _ = ipfixdec.decode(b1, t0)
        assert n1 == len(want) == len(recs) and all(s[0] != 2 for m in msgs for s in m["sets"])
        w = want.copy()
        w["end_reason"] = 0  # the oracle's sweep and the engine close open flows with different reasons
        recs["end_reason"] = 0
        assert ipfixdec.basic_view(recs) == ipfixdec.basic_view(w)
        assert g.g.received_bytes == len(b0) + len(b1)
        # the headers were device copies of the engine's own counts (ipxg_device_ipfix_counts)
        assert sorted(tuple(int(v) for v in h[0]) for h in g.g.hdr_host) == sorted([(len(b0), n0), (len(b1), n1)])
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_bench_gather_flag_single_gpu():
    """bench.py --gather: the N > 1 exchange at world size 1, no launcher --
    every exported flow's IPFIX record reaches rank 0's stream, the stream bytes rank 0 holds
    equal the bytes produced, and the line reports the side stream's per-step cost."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gather", "--steps", "20", "--warmup", "2",
                        "--no-cpu-baseline", "--no-e2e"], capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    g = line["gather"]
    assert line["n_gpus"] == 1 and g is not None
    assert g["device_ms_per_step"] > 0
    # (receives lag the pushes by one step: equal up to one step's difference in stream size)
    assert g["rank0_stream_bytes_per_step"] > 0
    assert abs(g["rank0_receives_bytes_per_step"] - g["rank0_stream_bytes_per_step"]) <= 0.01 * g["rank0_stream_bytes_per_step"]
    # 100k flows exported per udp64 step, 81 bytes each (IPv4 basic record) plus message headers
    assert 81 * line["flows_exported_per_step"] < g["rank0_stream_bytes_per_step"] < 90 * line["flows_exported_per_step"]
