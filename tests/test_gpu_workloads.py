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
import synth

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


def _run_batches(params, batches, finish=True, offset16=False, asynchronous=False):
    from ipfixprobe_amd import Engine
    with Engine(params) as e:
        for fr, de in batches:
            e.submit(fr, de, device=True, offset16=offset16, asynchronous=asynchronous)
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


@pytest.mark.parametrize("group", ["1", "3", "8"])
@pytest.mark.parametrize("name", sorted(MIXES))
def test_slow_lists_grouped(name, group, monkeypatch):
    """k_bin_slow workgroups taking several k_bin workgroups' slow lists (BinView::slow_group; the
    engine picks it from the previous batch's slow count, IPXG_SLOW_GROUP pins it): 1 (one list
    each), 3 (the last group short of lists) and 8, on three batches of each mix (every batch in
    units as well as bytes would double the time; bytes here) against the oracle, with the
    packet statistics."""
    import torch
    monkeypatch.setenv("IPXG_SLOW_GROUP", group)
    gen = _gen(name, 200_000, seed=321)
    n, nb = 400_000, 3
    batches = [gen.batch(k * n, n) for k in range(nb)]
    torch.cuda.synchronize()
    got, gst = _run_batches("s=20", batches)
    c = oracle_py.OracleCache(cache_exp=21)
    for fr, de in batches:
        c.run(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1)
    c.finish()
    want = c.take()
    wst = c.stats()
    c.close()
    d = flowcmp.diff(got, want)
    assert not d, d
    for k in ("seen_packets", "parsed_packets", "ipv6_packets", "mpls_packets", "pppoe_packets"):
        assert gst[k] == wst[k], k


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


@pytest.mark.parametrize("name,n,nb,units", [("imix", 10_000_000, 10, False), ("quic", 5_000_000, 4, False),
                                              ("imix", 14_285_715, 7, True), ("quic", 10_000_000, 2, True)])
def test_workload_full_size_conservation(name, n, nb, units):
    """The bench's full step (imix: 100M packets, 1M flows; quic: 20M, 1M), in the batches byte
    offsets allow and in the larger ones of 16-byte unit offsets (the bench's default, arenas past
    4 GiB): every packet is accounted to exactly one record, the record count equals the distinct
    flows the generator drew (host restatement of its plan), and no record is split (no timeouts,
    no FIN/RST)."""
    import torch
    gen = _gen(name, 1_000_000)
    from ipfixprobe_amd import Engine
    drawn = np.zeros(1_000_000, dtype=bool)
    with Engine("s=21") as e:
        for k in range(nb):
            fr, de = gen.batch(k * n, n, offset16=units)
            if units and name == "quic":
                assert fr.numel() > 1 << 32  # (the arena of a 10M configs[4] batch: ~8 GB)
            e.submit(fr, de, device=True, offset16=units)
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


@pytest.mark.parametrize("params", ["s=20", "s=20;walk=narrow", "strict=true;s=17"])
@pytest.mark.parametrize("name", sorted(MIXES))
def test_offset16_batches_match_byte_offsets(name, params):
    """IPXG_BATCH_OFFSET16 (ABI 8): the generator's batches with their offsets in 16-byte units
    (the same arena) -- records and counters equal the byte-offset run's (binned ingest with
    either walk, and the reference's own table: strict), and the oracle's."""
    import torch
    gen = _gen(name, 200_000)
    n, nb = 300_000, 3
    byte = [gen.batch(k * n, n) for k in range(nb)]
    unit = [gen.batch(k * n, n, offset16=True) for k in range(nb)]
    torch.cuda.synchronize()
    for (a1, d1), (a2, d2) in zip(byte, unit):
        assert torch.equal(a1, a2)
        o1 = d1.view(torch.int32).view(-1, 4)
        o2 = d2.view(torch.int32).view(-1, 4)
        assert torch.equal(o1[:, 0], o2[:, 0] * 16) and torch.equal(o1[:, 1:], o2[:, 1:])
    got_b, st_b = _run_batches(params, byte)
    got_u, st_u = _run_batches(params, unit, offset16=True, asynchronous=True)
    d = flowcmp.diff(got_u, got_b)
    assert not d, d
    for k in ("seen_packets", "parsed_packets", "ipv4_packets", "ipv6_packets", "vlan_packets", "mpls_packets"):
        assert st_u[k] == st_b[k], k
    if "strict" not in params:
        c = oracle_py.OracleCache(cache_exp=22)
        for fr, de in byte:
            c.run(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1)
        c.finish()
        want = c.take()
        c.close()
        d = flowcmp.diff(got_u, want)
        assert not d, d


@pytest.mark.parametrize("layout", ["lanes", "blocks"])
def test_arena_past_4gib(layout):
    """Frames past 4 GiB (IPXG_BATCH_OFFSET16): the configs[4] mix's frames copied 4.5 GiB up a
    larger arena for every other packet ('lanes': a wave's frames lie 4.5 GiB apart) or every
    other 4096-packet block ('blocks': whole waves read past 4 GiB) -- records and counters
    against the oracle over the same packets."""
    import torch
    gen = _gen("quic", 100_000)
    n = 200_000
    fr, de = gen.batch(0, n)
    high = 9 << 29  # 4.5 GiB
    big = torch.zeros(high + fr.numel(), dtype=torch.uint8, device=fr.device)
    big[:fr.numel()] = fr
    big[high:] = fr
    d = de.view(torch.int32).view(n, 4).clone()
    idx = torch.arange(n, device=fr.device)
    up = (idx % 2 == 1) if layout == "lanes" else ((idx // 4096) % 2 == 1)
    off = d[:, 0].to(torch.int64)
    d[:, 0] = (torch.where(up, off + high, off) // 16).to(torch.int32)
    desc = d.view(torch.uint8).reshape(-1)
    torch.cuda.synchronize()
    got, st = _run_batches("s=19", [(big, desc)], offset16=True)
    want, wst = oracle_py.run_capture(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1, cache_exp=20)
    del big
    dd = flowcmp.diff(got, want)
    assert not dd, dd
    for k in ("seen_packets", "parsed_packets", "ipv4_packets", "ipv6_packets", "vlan_packets", "mpls_packets"):
        assert st[k] == wst[k], k


@pytest.mark.parametrize("walk", [";walk=narrow", ";walk=wide"])
def test_offset16_frames_past_the_arena_read_as_zeros(walk):
    """with IPXG_BATCH_OFFSET16 the ingest reads heads through 64-bit addresses, which no
    buffer range clamps.  Every other descriptor here points past arena_len (into memory the caller
    still owns, so an unguarded read would parse those frames as flows instead of faulting): k_bin and
    k_bin_slow must read them as zeros -- keyless packets, as the byte-offset path's buffer loads give
    them -- and the records are the oracle's over the packets inside the arena."""
    import torch
    rng = np.random.default_rng(97)
    n = 8192
    sip = (10 << 24) + rng.integers(0, 200, n)
    dip = (192 << 24) + (168 << 16) + rng.integers(0, 50, n)
    arena, desc = synth.udp_frames(sip, dip, rng.integers(1024, 1200, n), rng.integers(1, 30, n))
    inside = np.arange(n) % 2 == 0
    # the inside packets' frames first, the outside ones after arena_len
    order = np.concatenate([np.nonzero(inside)[0], np.nonzero(~inside)[0]])
    frames = arena.reshape(n, 64)[order].reshape(-1)
    pos = np.empty(n, dtype=np.int64)
    pos[order] = np.arange(n)
    d = desc.copy()
    d["offset"] = (pos * 64) // 16
    big = torch.from_numpy(np.ascontiguousarray(frames)).cuda()
    arena_t = big[:int(inside.sum()) * 64]  # arena_len ends before the outside frames
    dt = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8).reshape(-1)).cuda()
    torch.cuda.synchronize()
    got, st = _run_batches("s=18" + walk, [(arena_t, dt)], offset16=True)
    di = desc[inside].copy()
    want, wst = oracle_py.run_capture(arena, di, 1, cache_exp=20)
    dd = flowcmp.diff(got, want)
    assert not dd, dd
    assert st["seen_packets"] == n
