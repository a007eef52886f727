"""Process plugins on the configs[2] / configs[4] mixes (BASELINE.json: "with TLS/HTTP/DNS
process plugins enabled", "QUIC process plugin"): the native stand-ins of
ipfixprobe_amd/host/ipxg_stdplugins.c (include/ipxg_stdplugins.h) registered through the
bridge (ipxg_add_plugin), the engine against the oracle running the same hooks for every
packet.

The stand-ins are pinned by the reference's own goldens through the oracle (CPU): dns and http
(every record equal), tls (the flows the plugin claims = tests/functional/outputs/tls, which keeps
only flows with a TLS extension) and quic."""
import os
import sys
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil
import plugins_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "tests", "golden", "reference")
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def _std(name):
    from ipfixprobe_amd.engine import StdPlugin
    return StdPlugin(name)


def _capture(name):
    dl, pk = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    return dl, arena, desc


@pytest.mark.parametrize("name,pcap", [("dns", "dns"), ("http", "http"), ("tls", "tls"),
                                       ("quic", "quic_initial-sample")])
def test_stand_in_reproduces_reference_golden(name, pcap):
    dl, arena, desc = _capture(pcap)
    pl = _std(name)
    recs, _ = oracle_py.run_capture(arena, desc, dl, plugins=[pl.struct])
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name)))
    if name == "tls":  # the tls test's output keeps the flows with a TLS extension
        recs = recs[recs["ext"] != 0]
    assert Counter(pcaputil.format_records(recs)) == gold
    assert pl.calls()["post_create"] > 0


def test_stand_ins_agree_with_python_stand_ins():
    """dns / http: the C stand-ins and tests/plugins_py.py (each restating dns.cpp / http.cpp)
    end the same flows on the same captures and synthetic HTTP/DNS stream."""
    import test_plugins
    for name, py in (("dns", plugins_py.DnsFlush), ("http", plugins_py.HttpReinsert)):
        for dl, arena, desc in (_capture(name), (1,) + tuple(test_plugins._http_stream())):
            pa, pb = _std(name), py()  # (kept alive while the oracle calls their hooks)
            a, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[pa.struct])
            b, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[pb.struct])
            assert not flowcmp.diff(a, b)


def _mix(name, flows, seed=1234):
    import synthgen
    return synthgen.Mix(name, flows, seed=seed, zipf=1.1 if name == "imix" else None)


def test_mix_plugin_shares():
    """The generator's connections: opening flows (first messages: TLS ClientHello, HTTP request
    line, QUIC long headers) are a small share of the packets, DNS flows rank last (short)."""
    import synthgen

    class G:
        pass
    for name, lo, hi in (("imix", 0.005, 0.03), ("quic", 0.03, 0.12)):
        g = G()
        g.mix, g.seed, g.t0_ns, g.dt_ns = _mix(name, 100_000), 5, 1_700_000_000 * 10**9, 100
        g.q16 = [int(round(x * 65536)) for x in (0.55, 0.005, 0.045)]
        f, _, _, lng, _ = synthgen.host_plan(g, 0, 200_000)
        op = g.mix.flows["opening"][f] != 0
        assert lo < op.mean() < hi, (name, op.mean())
        if name == "quic":
            assert np.array_equal(lng, op & (g.mix.layouts["size_mode"][g.mix.flows["layout"][f]] == 1))


PLUGINS = {"imix": ("dns", "http", "tls"), "quic": ("quic", "dns")}
_CALLS = {}  # hook calls of the single-threaded walk, per mix


@pytest.mark.gpu
@pytest.mark.parametrize("threads,asynchronous", [(1, False), (4, False), (16, False), (16, True)])
@pytest.mark.parametrize("name", sorted(PLUGINS))
def test_plugins_on_workload_match_oracle(name, threads, asynchronous):
    """2M packets of the mix over 1M flows in four device batches with the configs' plugins
    registered: every record (plugin flushes, REINSERTs and the plugins' ext bits included)
    equals the oracle's, which calls the same hooks on every packet; the hooks saw only a small
    share of the packets on the engine (the bridge kept the rest on the device).  The host walk
    on 1, 4 and 16 threads (plugin copies per thread): the same records, and the hook calls of
    all copies sum to the same counts.  asynchronous: device batches submitted back to back with
    IPXG_BATCH_ASYNC, so each batch's k_bin / k_bin_slow run during the previous batch's host walk
    (the early front, its spills deferred): the same records and hook calls."""
    import torch
    import synthgen
    from ipfixprobe_amd import Engine
    gen = synthgen.Generator(_mix(name, 1_000_000), torch.device("cuda", 0), seed=1234)
    n, nb = 500_000, 4
    batches = [gen.batch(k * n, n) for k in range(nb)]
    torch.cuda.synchronize()
    pls = [_std(p) for p in PLUGINS[name]]
    with Engine("s=21") as e:
        e.set_walk_threads(threads)
        for p in pls:
            e.add_plugin(p.struct)
        for fr, de in batches:
            e.submit(fr, de, device=True, asynchronous=asynchronous)
        e.finish()
        got = e.poll()
        st = e.stats()
        overlapped = e.timing()["plugin_overlapped"]
    assert (overlapped >= nb - 2) if asynchronous else overlapped == 0, overlapped
    calls = [p.calls() for p in pls]  # copies folded back into the originals at engine destroy
    if threads == 1:
        _CALLS[name] = calls
    elif name in _CALLS:
        assert calls == _CALLS[name]
    ref = [_std(p) for p in PLUGINS[name]]
    c = oracle_py.OracleCache(cache_exp=22)
    for p in ref:
        c.add_plugin(p.struct)
    for fr, de in batches:
        c.run(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1)
    c.finish()
    want = c.take()
    c.close()
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert (got["ext"] != 0).sum() > 100
    seen = pls[0].calls()["pre_create"]
    assert 0 < seen < 0.25 * n * nb, seen  # the host walk saw the plugin flows' packets only
    assert st["complex_flows"] > 0


class FollowProbe(plugins_py.PyPlugin):
    """QUIC-shaped rule (UDP, long-header bit) with follow_packets = 6: claims a flow on a
    long-header packet and records every later hook call on a claimed flow within its first 6
    packets -- the calls the reference makes (every packet) and the bridge must reproduce."""
    proto_mask = 2

    def __init__(self):
        super().__init__()
        s = self.struct
        s.n_prefixes = 1
        s.prefix_len[0] = 1
        s.prefix[0][0] = 0x80
        s.masked = 1
        s.prefix_mask[0][0] = 0x80
        s.follow_packets = 6
        self.seen = Counter()

    def _note(self, rec, data):
        if data[:1] and data[0] & 0x80:
            rec["ext"] = 1
        elif rec["ext"] and int(rec["src_packets"]) + int(rec["dst_packets"]) < 6:
            self.seen[(int(rec["flow_hash"]), int(rec["src_packets"]) + int(rec["dst_packets"]))] += 1
        return 0

    def post_create(self, rec, p, data):
        return self._note(rec, data)

    def post_update(self, rec, p, data):
        return self._note(rec, data)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [7, 40])
def test_follow_packets_keeps_claimed_flows_on_host(batch):
    """A flow claimed in one batch keeps reaching the plugin's hooks in the next batches (short
    headers, outside the rule) until it holds follow_packets packets; every such call the oracle
    makes, the bridge makes."""
    import synth
    from ipfixprobe_amd import run_capture
    cli, srv = synth.ip4(10), synth.ip4(200)
    frames = []
    for rnd in range(10):
        for f in range(8):
            first = b"\xc0" + b"\x00" * 20 if rnd == 0 and f % 2 == 0 else b"\x40" + b"\x01" * 20
            ip = synth.ipv4(cli, srv, 17, synth.udp(30000 + f, 443, first))
            frames.append(synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) + ip))
    arena, desc = synth.to_batch([(f, len(f), len(f)) for f in frames])
    eng, orc = FollowProbe(), FollowProbe()
    got, _ = run_capture(arena, desc, params="s=16", batch=batch, plugins=[eng.struct])
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=16, plugins=[orc.struct])
    assert not flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert eng.seen == orc.seen and len(orc.seen) == 4 * 4  # packets 2..5 of the 4 claimed flows


@pytest.mark.gpu
def test_expired_followed_flow_leaves_the_host_walk():
    """ipxg_expire exports a followed flow's record with its extension: the slot must stop being
    followed (k_expire cleared only SLOT_LIVE, so the dead slot kept SLOT_FOLLOW, survived
    every rehash and sent the key's next packets to the host walk).  Packets of the same keys after
    the expiry, outside the plugin's rule, stay on the device."""
    import synth
    from ipfixprobe_amd import Engine
    cli, srv = synth.ip4(10), synth.ip4(200)
    nfl = 3000

    def batch(payload, t0):
        fr = [synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) +
                        synth.ipv4(cli, srv, 17, synth.udp(1024 + f, 443, payload))) for f in range(nfl)]
        return synth.to_batch([(f, len(f), len(f)) for f in fr], t0=t0)

    probe = FollowProbe()
    with Engine("s=16") as e:
        e.add_plugin(probe.struct)
        arena, desc = batch(b"\xc0" + b"\x00" * 20, 1000)  # claimed: one long-header packet each
        e.submit(arena, desc)
        t1 = e.timing()["plugin_packets"]
        assert t1 == nfl
        e.expire(1000 + 60)  # every record idle past the inactive timeout (30 s)
        assert e.stats()["flows_in_cache"] == 0
        assert len(e.poll()) == nfl
        arena, desc = batch(b"\x40" + b"\x01" * 20, 1100)  # the same keys, short headers (no rule)
        e.submit(arena, desc)
        assert e.timing()["plugin_packets"] == t1, "an expired flow's slot still sent packets to the host walk"
        e.expire(1100 + 60)
        assert len(e.poll()) == nfl and e.stats()["flows_in_cache"] == 0
