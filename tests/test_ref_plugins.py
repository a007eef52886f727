"""The reference's own process plugins through the bridge: dns.cpp, http.cpp,
tls.cpp and quic.cpp from /root/reference, compiled unmodified by oracle/Makefile (ref_plugins)
into oracle/_ref/libref_plugins.so behind the product's adapter
(ipfixprobe_amd/host/plugin_adapter.hpp: ipxg_plugin hooks -> ipxp::ProcessPlugin virtuals, the
record's ext handle -> an ipxp::Flow holding the RecordExt chain), built against the unmodified
reference headers processPlugin.hpp / packet.hpp / flowifc.hpp.

CPU: the oracle with each real plugin reproduces the reference's golden output of its plugin
test (tests/functional/outputs/<plugin>, basic columns: every record for dns / http / quic, the
flows with a TLS extension for tls).  GPU: the engine's bridge with the real plugins gives the
oracle's records and, record by record, the same extension contents (RecordExt::get_text) --
on the golden captures and on the configs[2] / configs[4] mixes.

The library exists only where the reference tree was present at build time (it travels to the
GPU box in oracle/_ref); the tests skip without it."""
import ctypes
import os
import sys
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "tests", "golden", "reference")
LIB = os.path.join(ROOT, "oracle", "_ref", "libref_plugins.so")
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="oracle/_ref/libref_plugins.so not built")
_L = None


def lib():
    global _L
    if _L is None:
        from ipfixprobe_amd.engine import Plugin
        _L = ctypes.CDLL(LIB)
        _L.ref_plugin_create.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(Plugin)]
        _L.ref_plugin_destroy.argtypes = [ctypes.POINTER(Plugin)]
        _L.ref_ext_text.argtypes = [ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
        _L.ref_ext_free.argtypes = [ctypes.c_uint64]
        _L.ref_ext_count.argtypes = [ctypes.c_uint64]
    return _L


class RefPlugin:
    """A fresh instance of the reference plugin `name` behind the adapter (.struct: its ipxg_plugin)."""

    def __init__(self, name):
        from ipfixprobe_amd.engine import Plugin
        self.struct = Plugin()
        rc = lib().ref_plugin_create(name.encode(), b"", ctypes.byref(self.struct))
        assert rc == 0, (name, rc)

    def __del__(self):
        try:
            lib().ref_plugin_destroy(ctypes.byref(self.struct))
        except Exception:
            pass


def take_exts(recs):
    """Each record's extension texts and extension count (then its Flow is released, as the
    consumer would)."""
    out, cnt = [], []
    buf = ctypes.create_string_buffer(1 << 16)
    for e in recs["ext"]:
        e = int(e)
        if not e:
            out.append("")
            cnt.append(0)
            continue
        n = lib().ref_ext_text(e, buf, len(buf))
        assert n < len(buf)
        out.append(buf.value.decode(errors="replace"))
        cnt.append(lib().ref_ext_count(e))
        lib().ref_ext_free(e)
    return out, np.array(cnt, dtype=np.int64)


def take_texts(recs):
    return take_exts(recs)[0]


def golden_lines(recs, counts):
    """The functional test's lines of these records (basic columns): the reference's UniRec output
    sends one record per extension a flow carries and none for a flow without one
    (unirec.cpp:361-397; tests/functional/scripts/run_test.sh runs `-o unirec` with `-p <plugin>`
    only)."""
    return Counter(pcaputil.format_records(np.repeat(recs, counts)))


def keyed(recs, texts):
    return Counter((flowcmp.rec_key(r), t) for r, t in zip(recs, texts))


GOLDEN = [("dns", "dns"), ("http", "http"), ("tls", "tls"), ("quic", "quic_initial-sample")]
# round 5: the reference's other process plugins behind the same adapter -- rules
# for ntp (port), sip and wg (payload prefixes; wg follows its flows), every packet of every flow
# (ipxg_plugin.all_packets) for the rest -- on their own functional-test captures
# (tests/functional/CMakeLists.txt: plugin -> pcap), compared as that test compares (golden_lines).
MORE = [("ntp", "ntp"), ("sip", "sip"), ("rtsp", "rtsp"), ("wg", "wg"), ("mqtt", "mqtt"), ("pstats", "mixed"),
        ("phists", "mixed"), ("bstats", "bstats"), ("smtp", "smtp"), ("ssdp", "ssdp"), ("dnssd", "dnssd"),
        ("idpcontent", "idpcontent"), ("basicplus", "http"), ("ovpn", "ovpn"), ("ssadetector", "ovpn"),
        ("vlan", "vlan"), ("netbios", "netbios"), ("passivedns", "dns"), ("nettisa", "mixed")]


def _capture(pcap):
    dl, pk = pcaputil.read_capture(os.path.join(REF, pcap + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    return dl, arena, desc


@pytest.mark.parametrize("name,pcap", GOLDEN + MORE)
def test_oracle_with_reference_plugin_reproduces_golden(name, pcap):
    dl, arena, desc = _capture(pcap)
    pl = RefPlugin(name)
    recs, _ = oracle_py.run_capture(arena, desc, dl, plugins=[pl.struct])
    texts, counts = take_exts(recs)
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name)))
    assert golden_lines(recs, counts) == gold
    assert counts.any()


@pytest.mark.parametrize("name,pcap", GOLDEN)
def test_stand_in_decides_like_reference_plugin(name, pcap):
    """The native stand-in (include/ipxg_stdplugins.h) ends and claims the same flows as the real
    plugin on its golden capture."""
    from ipfixprobe_amd.engine import StdPlugin
    dl, arena, desc = _capture(pcap)
    rp, sp = RefPlugin(name), StdPlugin(name)
    a, _ = oracle_py.run_capture(arena, desc, dl, plugins=[rp.struct])
    b, _ = oracle_py.run_capture(arena, desc, dl, plugins=[sp.struct])
    claimed = np.array([t != "" for t in take_texts(a)], dtype=bool)
    assert not flowcmp.diff(a, b)
    assert not flowcmp.diff(a[claimed], b[b["ext"] != 0])


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 5, 7])
@pytest.mark.parametrize("name,pcap", GOLDEN + MORE)
def test_bridge_with_reference_plugin_matches_oracle(name, pcap, batch):
    """The engine's bridge with the reference plugin: records and extension texts equal the
    oracle's, and the basic columns the reference's golden -- in one batch and in batches of 5 / 7
    packets (flows and FLOW_FLUSH(_WITH_REINSERT) boundaries across batches)."""
    from ipfixprobe_amd import run_capture
    dl, arena, desc = _capture(pcap)
    ep, op = RefPlugin(name), RefPlugin(name)
    got, _ = run_capture(arena, desc, datalink=dl, params="s=16", batch=batch, plugins=[ep.struct])
    want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[op.struct])
    (tg, cg), (tw, cw) = take_exts(got), take_exts(want)
    assert keyed(got, zip(tg, cg)) == keyed(want, zip(tw, cw))
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name)))
    assert golden_lines(got, cg) == gold


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 8])
@pytest.mark.parametrize("mix,names", [("imix", ("dns", "http", "tls")), ("quic", ("quic", "dns"))])
def test_bridge_with_reference_plugins_on_workload(mix, names, threads):
    """600k packets of the configs[2] / configs[4] mix (three device batches, flows carried across
    them) with the configs' real plugins: records and extension contents equal the oracle's --
    with the host walk on one thread and split over 8 (each with its own ProcessPlugin::copy())."""
    import torch
    import synthgen
    from ipfixprobe_amd import Engine
    m = synthgen.Mix(mix, 200_000, seed=77, zipf=1.1 if mix == "imix" else None)
    gen = synthgen.Generator(m, torch.device("cuda", 0), seed=77)
    n, nb = 200_000, 3
    batches = [gen.batch(k * n, n) for k in range(nb)]
    torch.cuda.synchronize()
    eps = [RefPlugin(x) for x in names]
    with Engine("s=19") as e:
        e.set_walk_threads(threads)
        for p in eps:
            e.add_plugin(p.struct)
        for fr, de in batches:
            e.submit(fr, de, device=True)
        e.finish()
        got = e.poll()
    ops = [RefPlugin(x) for x in names]
    c = oracle_py.OracleCache(cache_exp=20)
    for p in ops:
        c.add_plugin(p.struct)
    for fr, de in batches:
        c.run(fr.cpu().numpy(), de.cpu().numpy().view(pcaputil.DESC_DTYPE), 1)
    c.finish()
    want = c.take()
    c.close()
    tg, tw = take_texts(got), take_texts(want)
    assert sum(1 for t in tw if t) > 50
    assert keyed(got, tg) == keyed(want, tw)


def _quic_flows_with_short_headers(n_short=20):
    """The golden QUIC capture's packets, each followed by n_short packets of its flow whose UDP
    payload starts as a 1-RTT short header (0x43): the real plugin detects QUIC on the Initial and
    follows the flow (follow_packets), and reads one payload byte of each short-header packet."""
    dl, pk = pcaputil.read_capture(os.path.join(REF, "quic_initial-sample.pcap"))
    out = []
    for (sec, usec, cl, wl, b) in pk:
        out.append((sec, usec, cl, wl, b))
        et = (b[12] << 8) | b[13]
        if et == 0x0800 and b[23] == 17:
            po = 14 + (b[14] & 15) * 4 + 8
        elif et == 0x86DD and b[20] == 17:
            po = 14 + 40 + 8
        else:
            continue
        for k in range(n_short):
            t = usec + 1000 * (k + 1)
            bb = bytearray(b)
            bb[po] = 0x43
            out.append((sec + t // 1_000_000, t % 1_000_000, cl, wl, bytes(bb)))
    return dl, out


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 7])
def test_walk_byte_budget_with_reference_quic(monkeypatch, batch):
    """ipxg_plugin.follow_bytes (ABI 7): the real QUIC plugin reads one payload byte of a packet
    outside its rule (a short header), so with the budget a followed flow's short-header packets
    cross to the host as headers + 1 byte.  Records and extension texts equal the whole-frame
    walk's (IPXG_WALK_FULL=1) and the oracle's; far fewer bytes cross."""
    from ipfixprobe_amd import Engine
    dl, pk = _quic_flows_with_short_headers()
    arena, desc = pcaputil.to_batch(pk)
    out = {}
    for full in ("0", "1"):
        monkeypatch.setenv("IPXG_WALK_FULL", full)
        ep = RefPlugin("quic")
        with Engine("s=16", datalink=dl) as e:
            e.add_plugin(ep.struct)
            e.submit_all(arena, desc, batch)
            e.finish()
            got = e.poll()
            tm = e.timing()
        out[full] = (got, take_texts(got), tm)
    op = RefPlugin("quic")
    want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[op.struct])
    tw = take_texts(want)
    (g0, t0, tm0), (g1, t1, tm1) = out["0"], out["1"]
    assert any(tw)
    assert keyed(g0, t0) == keyed(want, tw)
    assert keyed(g1, t1) == keyed(want, tw)
    assert tm0["plugin_packets"] == tm1["plugin_packets"] >= len(pk)
    assert tm0["plugin_d2h_bytes"] < 0.5 * tm1["plugin_d2h_bytes"]


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 16])
def test_plugin_error_fails_the_call_cleanly(threads):
    """A process plugin that throws PluginError on its 50th hook call: the
    adapter turns it into IPXG_PLUGIN_ERROR, the walk thread stops, and ipxg_submit fails with
    IPXG_EPLUGIN and the plugin's message -- on 1 and on 16 walk threads (every thread's copy
    throws) -- as the reference's input worker reports a PluginError (workers.cpp:107-112).  The
    engine then refuses work (IPXG_ESTATE) until ipxg_reset, runs again after it, and destroys."""
    import synth
    from ipfixprobe_amd import Engine
    from ipfixprobe_amd.engine import IpxgError, Plugin
    lib().ref_failing_plugin_create.argtypes = [ctypes.c_int, ctypes.POINTER(Plugin)]
    nfl, per = 12000, 4
    frames = []
    for i in range(nfl * per):
        f = i % nfl
        ip = synth.ipv4(synth.ip4(0x0A000000 + f), synth.ip4(0xC0A80001), 17, synth.udp(1024 + f % 60000, 53, b"\x00" * 12))
        frames.append(synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) + ip))
    arena, desc = synth.to_batch([(fr, len(fr), len(fr)) for fr in frames])
    pl = Plugin()
    assert lib().ref_failing_plugin_create(50, ctypes.byref(pl)) == 0
    e = Engine("s=17")
    try:
        e.set_walk_threads(threads)
        e.add_plugin(pl)
        with pytest.raises(IpxgError) as ex:
            e.submit(arena, desc)
        assert ex.value.rc == -8, str(ex.value)  # IPXG_EPLUGIN
        assert "PluginError: failing plugin: hook call 50" in str(ex.value)
        with pytest.raises(IpxgError) as ex2:
            e.submit(arena, desc)
        assert ex2.value.rc == -7  # IPXG_ESTATE until reset
        e.reset()
        e.submit(arena, desc)  # (every instance is past its 50th call: no failure now)
        e.finish()
        got = e.poll()
        assert len(got) == nfl and int(got["src_packets"].sum() + got["dst_packets"].sum()) == nfl * per
    finally:
        e.close()  # destroyable after the failure
        lib().ref_plugin_destroy(ctypes.byref(pl))


# ---- round 6: flowhash, icmp and mpls, which have no functional test of their own ----
# flowhash (flow_hash.cpp:54-65) exports Flow::flow_hash as FLOW_ID: through it the reference's own code
# reads every record's flow_hash.  icmp (icmp.cpp:34-48) keeps the type/code of an
# ICMP flow's first packet, mpls (mpls.cpp:45-55) the top MPLS label word the parser left in
# Packet::mplsTop (parser.cpp:614).  All three act in post_create only; behind the bridge they take
# every packet of every flow (rule_for: all_packets).
EXTRA = ("flowhash", "icmp", "mpls")
CAPTURES = sorted(os.path.splitext(f)[0] for f in os.listdir(REF) if f.endswith(".pcap"))


def _flow_ids_match(recs, texts):
    """flowhash's text (RecordExtFLOW_HASH::get_text: flow_id="<hex>") is the record's flow_hash."""
    return all(t == 'flow_id="%x"' % int(r["flow_hash"]) for r, t in zip(recs, texts))


def test_extra_reference_plugins_build():
    for name in EXTRA:
        RefPlugin(name)


@pytest.mark.parametrize("pcap", CAPTURES)
def test_oracle_with_flowhash_icmp_mpls(pcap):
    """The oracle with each plugin on every reference capture: flowhash gives every record exactly one
    extension whose FLOW_ID is the record's flow_hash; icmp's extensions sit on ICMP / ICMPv6 flows only."""
    dl, arena, desc = _capture(pcap)
    for name in EXTRA:
        pl = RefPlugin(name)
        recs, _ = oracle_py.run_capture(arena, desc, dl, plugins=[pl.struct])
        texts, counts = take_exts(recs)
        if name == "flowhash":
            assert (counts == 1).all()  # (arp.pcap: no flow at all)
            assert _flow_ids_match(recs, texts)
        elif name == "icmp":
            assert all(int(r["ip_proto"]) in (1, 58) for r, t in zip(recs, texts) if t)
        else:
            assert all(t.startswith("mpls_label_1=") for t in texts if t)


@pytest.mark.gpu
@pytest.mark.parametrize("pcap", CAPTURES)
def test_bridge_with_flowhash_icmp_mpls_matches_oracle(pcap):
    """The engine's bridge with flowhash, icmp and mpls on every reference capture, in one batch and in
    batches of 7 packets: records and extension texts equal the oracle's, and flowhash's FLOW_ID equals
    the engine's own record's flow_hash."""
    from ipfixprobe_amd import run_capture
    dl, arena, desc = _capture(pcap)
    for name in EXTRA:
        for batch in (None, 7):
            ep, op = RefPlugin(name), RefPlugin(name)
            got, _ = run_capture(arena, desc, datalink=dl, params="s=16", batch=batch, plugins=[ep.struct])
            want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[op.struct])
            (tg, cg), (tw, cw) = take_exts(got), take_exts(want)
            assert keyed(got, zip(tg, cg)) == keyed(want, zip(tw, cw)), (name, batch)
            if name == "flowhash":
                assert (cg == 1).all() and _flow_ids_match(got, tg)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 4096])
def test_bridge_with_flowhash_icmp_mpls_on_fuzz_corpus(batch):
    """The three together on the fuzz corpus (MPLS stacks, EoMPLS, ICMP / ICMPv6, every other
    encapsulation, truncated at every length), where the mpls and icmp plugins find their shapes:
    records and extension texts equal the oracle's."""
    import synth
    from ipfixprobe_amd import run_capture
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=73))
    eps, ops = [RefPlugin(x) for x in EXTRA], [RefPlugin(x) for x in EXTRA]
    got, _ = run_capture(arena, desc, params="s=18", batch=batch, plugins=[p.struct for p in eps])
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, plugins=[p.struct for p in ops])
    (tg, cg), (tw, cw) = take_exts(got), take_exts(want)
    assert keyed(got, zip(tg, cg)) == keyed(want, zip(tw, cw))
    assert sum("mpls_label_1=" in t for t in tw) > 20 and sum("type=" in t for t in tw) > 20
