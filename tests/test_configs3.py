"""configs[3] (BASELINE.json): IMIX, 1G packets over 10M flows, flow-key-hash sharded across 8
GPUs.  What one GPU of that job does is `bench.py --workload imix10m --shard R/8`: the 10M-flow
IMIX mix (Zipf 1.1), restricted to the flows whose canonical hash rank R owns (shard.owner, the
NIC-RSS analogue of the reference's one-pipeline-per-queue model, ipfixprobe.cpp:381-464,
dpdkDevice.cpp:230-262), 125M packets per step in 13 batches of 9,615,385 (a batch's arena stays
inside the descriptors' 32-bit offsets).

CPU: the shard split of the 10M flows (canonical hashes by the oracle's XXH64).
GPU: oracle parity on 2M packets of shard 0's mix (four batches, flows carried across them), and
the bench's full shard step -- 125M packets in 13 batches -- conserved exactly."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))

import bench  # noqa: E402
import flowcmp  # noqa: E402
import oracle_py  # noqa: E402
import pcaputil  # noqa: E402
import synthgen  # noqa: E402

FLOWS, WORLD, PKTS, NB = 10_000_000, 8, 9_615_385, 13
_MIX = {}


def _mix():
    if "m" not in _MIX:
        _MIX["m"] = synthgen.Mix("imix", FLOWS, seed=1234, zipf=1.1)  # bench's make_workload, imix10m
    return _MIX["m"]


def _owners(hasher):
    key = "own_cpu" if hasher is oracle_py.xxh64_batch else "own_gpu"
    if key not in _MIX:
        _MIX[key] = bench.flow_owners(_mix(), WORLD, hasher=hasher)
    return _MIX[key]


def test_shards_split_the_flows_evenly():
    """Every one of the 8 shards owns 12.5 +- 0.5 % of the 10M flows.  Packets: the bench gives
    every rank the same count -- its own Zipf(1.1) stream over its flows in popularity order
    (Mix.restrict), every GPU at the same load as an RSS queue of its own would be -- while one
    shared 1G-packet stream split by flow hash would not be balanced: the most popular flow alone
    carries 11.6 % of its packets, and the most loaded shard 22.4 % (1.79x the mean).  Those
    shares are pinned here from the mix's Zipf weights."""
    mix = _mix()
    own = _owners(oracle_py.xxh64_batch)
    share = np.bincount(own, minlength=WORLD) / len(own)
    assert np.all(np.abs(share - 1.0 / WORLD) < 0.005), share
    w = np.arange(1, FLOWS + 1, dtype=np.float64) ** -1.1
    w /= w.sum()
    assert abs(w[0] - 0.1164) < 0.001
    pk = np.bincount(own[mix.rank_flow.astype(np.int64)], weights=w, minlength=WORLD)
    assert abs(pk.sum() - 1.0) < 1e-9
    assert abs(pk.max() - 0.2236) < 0.001 and int(np.argmax(pk)) == int(own[mix.rank_flow[0]]), pk
    # the restricted mix of shard 0: its flows, in the full mix's popularity order
    import copy
    keep = np.nonzero(own == 0)[0]
    sub = copy.copy(mix)  # (restrict() replaces the arrays, the full mix stays as it is)
    sub.restrict(keep)
    assert len(sub.flows) == len(keep)
    pos = np.empty(FLOWS, dtype=np.int64)
    pos[mix.rank_flow] = np.arange(FLOWS)
    order = pos[keep]
    assert np.array_equal(sub.flows["mac_id"], mix.flows["mac_id"][keep[np.argsort(order, kind="stable")]])


def _shard_gen(rank=0):
    """bench.make_workload's generator for imix10m --shard rank/8."""
    import copy
    import torch
    mix = copy.copy(_mix())
    mix.restrict(np.nonzero(_owners(None) == rank)[0])
    return synthgen.Generator(mix, torch.device("cuda", 0), seed=1234 + 7919 * rank)


@pytest.mark.gpu
def test_shard_mix_parity_against_oracle():
    """2M packets of shard 0's mix (1.25M flows, Zipf 1.1 over them), submitted as four device
    batches with flows carried across them: every record equals the oracle's."""
    import torch
    from ipfixprobe_amd import Engine
    gen = _shard_gen(0)
    assert abs(len(gen.mix.flows) - FLOWS / WORLD) < 0.005 * FLOWS
    n, nb = 500_000, 4
    batches = [gen.batch(k * n, n) for k in range(nb)]
    torch.cuda.synchronize()
    with Engine(bench.engine_params(len(gen.mix.flows))) as e:
        for fr, de in batches:
            e.submit(fr, de, device=True)
        e.finish()
        got = e.poll()
        gst = e.stats()
    c = oracle_py.OracleCache(cache_exp=22)
    for fr, de in batches:
        c.run(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1)
    c.finish()
    want = c.take()
    wst = c.stats()
    c.close()
    assert wst["end_no_res"] == 0
    d = flowcmp.diff(got, want)
    assert not d, d
    assert gst["parsed_packets"] == n * nb


@pytest.mark.gpu
def test_shard_full_step_conservation():
    """The bench's imix10m --shard 0/8 step: 125M packets in 13 batches of 9,615,385 (arenas near
    the 32-bit descriptor-offset limit) into one table of the shard's 1.25M flows, then finish.
    Every packet is accounted to exactly one record, the record count equals the flows the
    generator drew (its host restatement), and no record is split."""
    import torch
    from ipfixprobe_amd import Engine
    gen = _shard_gen(0)
    F = len(gen.mix.flows)
    drawn = np.zeros(F, dtype=bool)
    with Engine(bench.engine_params(F)) as e:
        for k in range(NB):
            fr, de = gen.batch(k * PKTS, PKTS)
            assert fr.numel() > 3_000_000_000  # (the arena of a 9.6M IMIX batch: ~3.5 GB)
            e.submit(fr, de, device=True)
            del fr, de
            f, _, _, _, _ = synthgen.host_plan(gen, k * PKTS, PKTS)
            drawn[f] = True
        e.finish()
        recs = e.poll()
        st = e.stats()
        torch.cuda.synchronize()
    assert st["parsed_packets"] == PKTS * NB
    assert int(recs["src_packets"].sum() + recs["dst_packets"].sum()) == PKTS * NB
    assert len(recs) == int(drawn.sum())
    assert st["end_forced"] == len(recs)
    assert len(np.unique(recs["flow_hash"])) == len(recs)
