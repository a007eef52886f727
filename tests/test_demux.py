"""Host symmetric demux (ipxg_demux / ipxg_demux_split, SURVEY 8(e) input distribution): the
per-GPU rings of the end-to-end multi-GPU path.  A biflow's packets in both directions and every
fragment of a datagram go to one shard, so per-shard caches over the split batches give exactly
the records of one cache over the whole capture (checked with the oracle on the CPU, and with one
engine per shard on the GPU)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))

import flowcmp  # noqa: E402
import oracle_py  # noqa: E402
import pcaputil  # noqa: E402
import synth  # noqa: E402
from ipfixprobe_amd import engine  # noqa: E402

REF = os.path.join(os.path.dirname(__file__), "golden", "reference")


def _streams():
    yield "vlan_v6", 1, synth.flow_stream(seed=41, n_flows=150, n_pkts=3000, frag=False, v6_share=0.3,
                                          vlan_share=0.3).batch()
    yield "fragments", 1, synth.flow_stream(seed=42, n_flows=80, n_pkts=2500, frag=True).batch()
    for name in ("mixed", "vlan", "mqtt"):
        dl, pk = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
        yield name, dl, pcaputil.to_batch(pk)


@pytest.mark.parametrize("n_shards", [2, 3, 8])
def test_demux_union_equals_whole_capture_oracle(n_shards):
    for name, dl, (arena, desc) in _streams():
        want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=20)
        batches, shard_of = engine.demux(arena, desc, n_shards, dl)
        assert sum(len(d) for _, d in batches) == len(desc)
        parts = [oracle_py.run_capture(a, d, dl, cache_exp=20)[0] for a, d in batches if len(d)]
        d = flowcmp.diff(np.concatenate(parts), want)
        assert not d, (name, n_shards, d)


def test_demux_split_keeps_frames_and_order():
    arena, desc = synth.flow_stream(seed=43, n_flows=60, n_pkts=1200, frag=True, v6_share=0.5).batch()
    batches, shard_of = engine.demux(arena, desc, 4)
    for k, (a, d) in enumerate(batches):
        src = np.nonzero(shard_of == k)[0]
        assert len(src) == len(d)
        assert np.array_equal(d["ts_sec"], desc["ts_sec"][src]) and np.array_equal(d["ts_usec"], desc["ts_usec"][src])
        assert np.array_equal(d["caplen"], desc["caplen"][src]) and np.all(d["offset"] % 16 == 0)
        for j, i in enumerate(src[:200]):
            o, c = int(desc["offset"][i]), int(desc["caplen"][i])
            assert bytes(a[d["offset"][j]:d["offset"][j] + c]) == bytes(arena[o:o + c])


def test_demux_with_16_byte_unit_offsets():
    """IPXG_BATCH_OFFSET16 (ABI 8): the same frames at the same places, their offsets counted in
    16-byte units -- the same shards, and each shard's batch again in units."""
    arena, desc = synth.flow_stream(seed=45, n_flows=60, n_pkts=1200, frag=True, v6_share=0.5).batch()
    one, _ = engine.demux(arena, desc, 1)  # (frames at 16-byte aligned offsets)
    aligned, adesc = one[0]
    udesc = adesc.copy()
    udesc["offset"] //= 16
    bb, sb = engine.demux(aligned, adesc, 4)
    bu, su = engine.demux(aligned, udesc, 4, offset16=True)
    assert np.array_equal(sb, su)
    for (a1, d1), (a2, d2) in zip(bb, bu):
        assert np.array_equal(a1, a2)
        assert np.array_equal(d1["offset"], d2["offset"] * 16)
        assert np.array_equal(d1["caplen"], d2["caplen"])


def test_demux_is_symmetric_and_balanced():
    """Every packet of a biflow (both directions: one canonical hash) lands on one shard; many
    flows spread evenly over the shards."""
    s = synth.flow_stream(seed=44, n_flows=4000, n_pkts=8000, frag=False, v6_share=0.2)
    arena, desc = s.batch()
    _, fwd = engine.demux(arena, desc, 8)
    share = np.bincount(fwd, minlength=8) / len(fwd)
    assert share.min() > 0.08 and share.max() < 0.17
    pk, _ = oracle_py.parse_batch(arena, desc, 1)
    # the two directions of each biflow: same canonical hash -> same shard
    canon = np.minimum(pk["hash_fwd"], pk["hash_inv"])
    keyed = pk["ip_version"] > 0
    for c in np.unique(canon[keyed])[:500]:
        assert len(np.unique(fwd[keyed & (canon == c)])) == 1


def test_demux_rejects_bad_input():
    arena, desc = synth.flow_stream(seed=45, n_flows=5, n_pkts=50, frag=False).batch()
    with pytest.raises(engine.IpxgError):
        engine.demux(arena, desc, 0)
    bad = desc.copy()
    bad["offset"][3] = len(arena)  # frame past the arena
    with pytest.raises(engine.IpxgError):
        engine.demux(arena, bad, 2)


@pytest.mark.gpu
def test_demux_engines_union_equals_whole_capture():
    """One engine per demuxed shard (as one per GPU, each with its own table) on the GPU: the
    union of their exports is the oracle's result over the whole capture."""
    from ipfixprobe_amd import run_capture
    for name, dl, (arena, desc) in _streams():
        want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=20)
        batches, _ = engine.demux(arena, desc, 3, dl)
        parts = [run_capture(a, d, datalink=dl)[0] for a, d in batches if len(d)]
        d = flowcmp.diff(np.concatenate(parts), want)
        assert not d, (name, d)
