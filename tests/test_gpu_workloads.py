"""The BASELINE.json workloads beyond configs[1] through the HIP path: the device generator
(tools/synth) against its host restatement, the engine against the oracle on the configs[2]
IMIX/Zipf mix and the configs[4] QUIC/encapsulation mix at oracle-checkable sizes (several
batches, flows carried across them), and size-independent properties at the bench's full sizes.
"""
import os
import sys

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
import synthgen  # noqa: E402

MIXES = {"imix": dict(zipf=1.1), "quic": dict(zipf=None)}


def _gen(name, flows, seed=1234):
    import torch
    mix = synthgen.Mix(name, flows, seed=seed, **MIXES[name])
    return synthgen.Generator(mix, torch.device("cuda", 0), seed=seed)


@pytest.mark.parametrize("name", sorted(MIXES))
def test_generator_matches_host_restatement(name):
    gen = _gen(name, 50_000)
    arena, desc = gen.batch(123_457, 4000)
    a = arena.cpu().numpy()
    d = desc.cpu().numpy().view(pcaputil.DESC_DTYPE)
    ha, hd = synthgen.host_batch(gen, 123_457, 4000)
    assert np.array_equal(d, hd)
    for i in range(len(d)):
        o, c = int(d["offset"][i]), int(d["caplen"][i])
        assert np.array_equal(a[o:o + c], ha[o:o + c]), i


def _run_batches(params, batches, finish=True):
    from ipfixprobe_amd import Engine
    with Engine(params) as e:
        for fr, de in batches:
            e.submit(fr, de, device=True)
        if finish:
            e.finish()
        recs = e.poll()
        st = e.stats()
    return recs, st


@pytest.mark.parametrize("walk", ["", ";walk=wide", ";walk=narrow"])
@pytest.mark.parametrize("name", sorted(MIXES))
def test_workload_parity(name, walk):
    """2M packets of the mix over 1M flows, submitted as four device batches with flows carried
    across them, against the oracle run over the same packets in one pass; with the engine's
    choice of header walk per batch and with each walk pinned."""
    import torch
    gen = _gen(name, 1_000_000)
    n, nb = 500_000, 4
    batches = [gen.batch(k * n, n) for k in range(nb)]
    torch.cuda.synchronize()
    got, gst = _run_batches("s=21" + walk, batches)
    if walk != ";walk=narrow":
        assert gst["walked_packets"] > 0
    want, wst = [], None
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
    for k in ("seen_packets", "parsed_packets", "ipv4_packets", "ipv6_packets", "tcp_packets", "udp_packets",
              "vlan_packets", "mpls_packets", "pppoe_packets"):
        assert gst[k] == wst[k], k
    assert gst["parsed_packets"] == n * nb


def test_imix_batch_parity_against_oracle_single_batch():
    """One 1M-packet IMIX batch (the Zipf elephant flows concentrate ~12 % of the packets on one
    flow: the binned ingest's skew handling) bit-exact against the oracle."""
    import torch
    gen = _gen("imix", 1_000_000, seed=99)
    fr, de = gen.batch(0, 1_000_000)
    torch.cuda.synchronize()
    got, gst = _run_batches("s=21", [(fr, de)])
    want, wst = oracle_py.run_capture(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1, cache_exp=22)
    d = flowcmp.diff(got, want)
    assert not d, d


@pytest.mark.parametrize("name,n,nb", [("imix", 10_000_000, 10), ("quic", 5_000_000, 4)])
def test_workload_full_size_conservation(name, n, nb):
    """The bench's full step (imix: 100M packets, 1M flows; quic: 20M, 1M): every packet is
    accounted to exactly one record, the record count equals the distinct flows the generator
    drew (host restatement of its plan), and no record is split (no timeouts, no FIN/RST)."""
    import torch
    gen = _gen(name, 1_000_000)
    from ipfixprobe_amd import Engine
    drawn = np.zeros(1_000_000, dtype=bool)
    with Engine("s=21") as e:
        for k in range(nb):
            fr, de = gen.batch(k * n, n)
            e.submit(fr, de, device=True)
            del fr, de
            f, _, _, _, _ = synthgen.host_plan(gen, k * n, n)
            drawn[f] = True
        e.finish()
        recs = e.poll()
        st = e.stats()
        torch.cuda.synchronize()
    assert st["parsed_packets"] == n * nb
    assert int(recs["src_packets"].sum() + recs["dst_packets"].sum()) == n * nb
    assert len(recs) == int(drawn.sum())
    assert st["end_forced"] == len(recs)
    assert len(np.unique(recs["flow_hash"])) == len(recs)
