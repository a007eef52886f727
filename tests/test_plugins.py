"""Process-plugin bridge: hooks at put_pkt_recursive's call sites
(processPlugin.hpp:59-108, cache.cpp:290-491), FLOW_FLUSH and FLOW_FLUSH_WITH_REINSERT.

Pinned by the reference's own goldens: with the DNS stand-in (tests/plugins_py.py, restating
dns.cpp's flush decision) the basic columns of tests/functional/outputs/dns -- which the
plain cache does not reproduce, every DNS message being flushed into a record of its own --
and with the HTTP stand-in those of outputs/http.  The oracle (the same hooks at the same call
sites) is checked against those goldens on the CPU; the engine's bridge (device pre-classifier,
host walk of the plugin flows) against the goldens and the oracle on the GPU, including
synthetic flows whose HTTP requests trigger FLOW_FLUSH_WITH_REINSERT and DNS flows spread over
several batches."""
import ctypes
import os
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil
import plugins_py
import synth
from test_oracle_synth import PKT_BUCKETS

FLOW_EXT_OFFSET = pcaputil.FLOW_DTYPE.fields["ext"][1]  # ipxg_flow_record.ext

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference")


def _capture(name):
    dl, pk = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    return dl, arena, desc


def _gold(name):
    return Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name)))


def test_plain_cache_does_not_reproduce_dns_golden():
    dl, arena, desc = _capture("dns")
    recs, _ = oracle_py.run_capture(arena, desc, dl)
    assert Counter(pcaputil.format_records(recs)) != _gold("dns")


GOLDEN_PLUGINS = [("dns", plugins_py.DnsFlush), ("http", plugins_py.HttpReinsert), ("ntp", plugins_py.NtpFlush),
                  ("sip", plugins_py.SipReinsert)]


def _check_golden(name, recs):
    mine = Counter(pcaputil.format_records(recs))
    gold = _gold(name)
    if name == "sip":  # the sip test's output keeps only the flows with a SIP extension
        assert not (gold - mine)
        assert Counter(pcaputil.format_records(recs[recs["ext"] != 0])) == gold
    else:
        assert mine == gold


@pytest.mark.parametrize("name,plugin", GOLDEN_PLUGINS)
def test_oracle_with_plugin_reproduces_reference_golden(name, plugin):
    dl, arena, desc = _capture(name)
    pl = plugin()
    recs, st = oracle_py.run_capture(arena, desc, dl, plugins=[pl.struct])
    _check_golden(name, recs)
    assert pl.calls["pre_create"] >= st["parsed_packets"] - st["keyless_packets"]


def test_dns_stand_in_decisions():
    q = bytes.fromhex("abcd01000001000000000000") + b"\x07example\x03com\x00" + b"\x00\x01\x00\x01"
    assert plugins_py.dns_valid(q, False)
    assert not plugins_py.dns_valid(q[:11], False)                        # < 12 bytes
    assert plugins_py.dns_valid(q[:-2], False)                            # overflow: returns success
    assert not plugins_py.dns_valid(q[:12] + b"\x40" + b"a" * 64 + b"\x00" + q[-4:], False)  # label > 63
    assert plugins_py.dns_valid(len(q).to_bytes(2, "big") + q, True)
    assert not plugins_py.dns_valid((len(q) + 1).to_bytes(2, "big") + q, True)  # TCP length mismatch


def _http_stream():
    """TCP flows on port 80, three with two requests and two responses each (REINSERT), three
    plain; DNS flows (queries and responses flushed one by one, a non-DNS datagram on port 53
    staying in its flow); other UDP.  The flows are interleaved round-robin, each keeping its
    own packet order."""
    cli, srv = synth.ip4(10), synth.ip4(200)
    get = b"GET /a HTTP/1.1\r\nHost: x\r\n\r\n"
    resp = b"HTTP/1.1 200 OK\r\nContent-Length: 0\r\n\r\n"
    e = lambda ip: synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) + ip)  # noqa: E731
    flows = []
    for f in range(6):
        sp = 40000 + f
        seq = [(0x02, b"", 0), (0x12, b"", 1), (0x10, b"", 0), (0x18, get, 0), (0x18, resp, 1), (0x10, b"", 0)]
        if f % 2 == 0:
            seq += [(0x18, get, 0), (0x18, resp, 1), (0x18, get, 0), (0x10, b"", 1)]
        seq += [(0x11, b"", 0), (0x11, b"", 1)]
        fl = []
        for flags, pay, rev in seq:
            a, b_, s1, s2 = (srv, cli, 80, sp) if rev else (cli, srv, sp, 80)
            fl.append(e(synth.ipv4(a, b_, 6, synth.tcp(s1, s2, flags, payload=pay))))
        flows.append(fl)
    q = bytes.fromhex("abcd01000001000000000000") + b"\x07example\x03com\x00" + b"\x00\x01\x00\x01"
    r = bytes.fromhex("abcd81800001000100000000") + b"\x07example\x03com\x00" + b"\x00\x01\x00\x01" + \
        b"\xc0\x0c\x00\x01\x00\x01\x00\x00\x00\x3c\x00\x04\x01\x02\x03\x04"
    for k in range(7):
        sp = 50000 + k
        fl = []
        for _ in range(6):
            fl.append(e(synth.ipv4(cli, srv, 17, synth.udp(sp, 53, q))))
            fl.append(e(synth.ipv4(srv, cli, 17, synth.udp(53, sp, r))))
            fl.append(e(synth.ipv4(cli, srv, 17, synth.udp(sp, 53, b"\x00\x01"))))  # not DNS
        flows.append(fl)
    for k in range(3):
        flows.append([e(synth.ipv4(cli, srv, 17, synth.udp(7000 + k, 9000, b"x" * 20))) for _ in range(12)])
    frames = []
    for rnd in range(max(len(fl) for fl in flows)):
        for fl in flows:
            if rnd < len(fl):
                frames.append(fl[rnd])
    return synth.to_batch([(f, len(f), len(f)) for f in frames])


def test_oracle_reinsert_splits_http_flows():
    arena, desc = _http_stream()
    plain, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=16)
    pl = plugins_py.HttpReinsert()
    got, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=16, plugins=[pl.struct])
    assert len(got) > len(plain)  # REINSERT exported the flows holding a request already
    # from pre_update the packet goes into the reinserted record only: no packet counted twice
    assert int(got["src_packets"].sum() + got["dst_packets"].sum()) == int(plain["src_packets"].sum() +
                                                                            plain["dst_packets"].sum())
    assert pl.calls["pre_export"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name,plugin", GOLDEN_PLUGINS)
@pytest.mark.parametrize("batch", [None, 7])
def test_bridge_reproduces_reference_golden(name, plugin, batch):
    from ipfixprobe_amd import run_capture
    dl, arena, desc = _capture(name)
    pl = plugin()
    got, st = run_capture(arena, desc, datalink=dl, params="s=16", batch=batch, plugins=[pl.struct])
    _check_golden(name, got)
    ref_pl = plugin()
    want, _ = oracle_py.run_capture(arena, desc, dl, cache_exp=16, plugins=[ref_pl.struct])
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 50, 333])
def test_bridge_reinsert_and_flush_match_oracle(batch):
    from ipfixprobe_amd import run_capture
    arena, desc = _http_stream()
    pls = [plugins_py.HttpReinsert(), plugins_py.DnsFlush()]
    got, st = run_capture(arena, desc, params="s=16", batch=batch, plugins=[p.struct for p in pls])
    ref = [plugins_py.HttpReinsert(), plugins_py.DnsFlush()]
    want, wst = oracle_py.run_capture(arena, desc, 1, cache_exp=16, plugins=[p.struct for p in ref])
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert st["complex_flows"] > 0
    # FlowRecordStats / end reasons count export_flow only (a REINSERT push is not counted)
    for k in PKT_BUCKETS + ["total_exported"]:
        assert st[k] == wst[k], k
    assert st["total_exported"] < len(got)
    # the hooks saw the plugin flows' packets only (other flows stayed on the device)
    assert 0 < pls[0].calls["pre_create"] < len(desc)


@pytest.mark.gpu
def test_bridge_leaves_other_flows_on_device():
    """A stream without any plugin packet: no hook is called, records equal the plain run."""
    from ipfixprobe_amd import run_capture
    arena, desc = synth.flow_stream(seed=61, n_flows=100, n_pkts=3000, frag=False).batch()
    pl = plugins_py.HttpReinsert()
    pl.struct.n_prefixes = 0
    pl.struct.n_ports = 1
    pl.struct.ports[0] = 1  # no packet of the stream uses port 1
    got, _ = run_capture(arena, desc, params="s=16", plugins=[pl.struct])
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=16)
    d = flowcmp.diff(got, want)
    assert not d, d
    assert sum(pl.calls.values()) == 0


class PrefixMarker(plugins_py.PyPlugin):
    """Claims a flow (ext bit) on a packet whose payload starts with its rule's prefixes: 7x under
    the mask F0 (the fuzz corpus' TCP 'x...' and UDP 'y...' payloads), or 'yy' -- exactly the
    packets the pre-classifier must route to the host walk.  Any packet the device misses leaves
    the engine's ext different from the oracle's."""
    proto_mask = 3
    prefixes = (b"\x70", b"yy")

    def __init__(self):
        super().__init__()
        s = self.struct
        s.masked = 1
        s.prefix_mask[0][0] = 0xF0
        self.seen = 0

    def _mark(self, rec, p, data):
        if int(p["ip_proto"]) not in (6, 17) or int(p["frag_off"]):  # outside the rule: no-op
            return 0
        if (data[:1] and (data[0] & 0xF0) == 0x70) or data[:2] == b"yy":
            self.seen += 1
            rec["ext"] = int(rec["ext"]) | 1
        return 0

    def post_create(self, rec, p, data):
        return self._mark(rec, p, data)

    def post_update(self, rec, p, data):
        return self._mark(rec, p, data)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 4096])
def test_classifier_payload_offsets_on_fuzz_corpus(batch):
    """The pre-classifier parses the register-walk shapes (VLAN/QinQ, MPLS, PPPoE, IPv4-in-GRE,
    IPv6 with extension headers, TCP timestamps) from registers and computes their payload offset
    and length itself (parse_medium<PAY>, parser.cpp:780-797): on the fuzz corpus -- every such
    shape, truncated at every length -- the flows it routes to the hooks must be exactly those
    with a rule packet, i.e. the engine's records (ext included) equal the oracle's, whose hooks
    see every packet."""
    from ipfixprobe_amd import run_capture
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=71))
    eng, orc = PrefixMarker(), PrefixMarker()
    got, _ = run_capture(arena, desc, params="s=18", batch=batch, plugins=[eng.struct])
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, plugins=[orc.struct])
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert (want["ext"] != 0).sum() > 100
    assert eng.seen == orc.seen


@pytest.mark.gpu
def test_early_front_defers_spills(monkeypatch):
    """Asynchronous device batches with a plugin registered: each batch's k_bin / k_bin_slow run
    during the previous batch's host walk (the early front), while the walk still owns the table --
    so what overflows a segment is deferred (Params::defer_spill) instead of accumulated into a
    slot, and applied after k_reduce without growing the table.  An elephant flow with the segments
    forced small (IPXG_TILE_AGG=0, IPXG_PART_BITS=8, from the second batch on) overflows them in
    every overlapped batch; the records, the NTP plugin's flushes included, equal the oracle's."""
    import torch
    import test_gpu_semantics
    from ipfixprobe_amd import Engine
    rng = np.random.default_rng(24)
    n, F, nb = 200_000, 5000, 4
    fop = np.where(rng.random(n) < 0.5, 0, rng.integers(1, F, n))
    arena, desc = test_gpu_semantics._udp_batch(rng, fop, F)
    ref = plugins_py.NtpFlush()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, plugins=[ref.struct])
    monkeypatch.setenv("IPXG_TILE_AGG", "0")
    monkeypatch.setenv("IPXG_PART_BITS", "8")
    a = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    ds = [torch.from_numpy(np.ascontiguousarray(desc[k * n // nb:(k + 1) * n // nb]).view(np.uint8).reshape(-1)).cuda()
          for k in range(nb)]
    torch.cuda.synchronize()
    pl = plugins_py.NtpFlush()
    with Engine("s=16") as e:
        e.add_plugin(pl.struct)
        for d in ds:
            e.submit(a, d, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
        tm = e.timing()
    assert tm["plugin_overlapped"] >= nb - 2, tm
    assert st["spilled_packets"] > 0 and st["table_rehashes"] == 0, st
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert (want["ext"] != 0).sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("asynchronous", [False, True])
def test_offset16_fuzz_corpus_with_plugin(asynchronous):
    """IPXG_BATCH_OFFSET16 (ABI 8): the fuzz corpus (every register-walk shape, fragments,
    truncations) at 16-byte aligned offsets, its descriptors counting 16-byte units, in 4096-packet
    device batches with a prefix-rule plugin registered -- records and ext bits equal the oracle's
    over the same packets."""
    import torch
    from ipfixprobe_amd import Engine
    from ipfixprobe_amd import engine as ipe
    arena0, desc0 = synth.to_batch(synth.fuzz_corpus(20000, seed=72))
    one, _ = ipe.demux(arena0, desc0, 1)
    arena, desc = one[0]
    orc = PrefixMarker()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, plugins=[orc.struct])
    udesc = desc.copy()
    udesc["offset"] //= 16
    a = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    step = 4096
    ds = [torch.from_numpy(np.ascontiguousarray(udesc[s:s + step]).view(np.uint8).reshape(-1)).cuda()
          for s in range(0, len(udesc), step)]
    torch.cuda.synchronize()
    eng = PrefixMarker()
    with Engine("s=18") as e:
        e.add_plugin(eng.struct)
        for d in ds:
            e.submit(a, d, device=True, asynchronous=asynchronous, offset16=True)
        e.finish()
        got = e.poll()
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert (want["ext"] != 0).sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("prof", [0, 2])
def test_early_front_on_fuzz_corpus(prof):
    """The fuzz corpus (every register-walk shape, fragments, truncations) in 4096-packet device
    batches submitted back to back with IPXG_BATCH_ASYNC: each batch's k_bin / k_bin_slow run during
    the previous batch's host walk, fragments included (k_bin_slow lists them into the batch's own
    fragment list while the walked batch's replay is done); records and ext bits equal the
    oracle's.  prof: with sampled stage timing (ipxg_profile, every 2nd batch) as bench.py runs it --
    a batch's unrecorded events once left "invalid resource handle" in HIP's last-error slot,
    which failed the next launch check of a plugin batch."""
    import torch
    from ipfixprobe_amd import Engine
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=71))
    orc = PrefixMarker()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, plugins=[orc.struct])
    a = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    step = 4096
    ds = [torch.from_numpy(np.ascontiguousarray(desc[s:s + step]).view(np.uint8).reshape(-1)).cuda()
          for s in range(0, len(desc), step)]
    torch.cuda.synchronize()
    eng = PrefixMarker()
    with Engine("s=18") as e:
        e.add_plugin(eng.struct)
        if prof:
            e.profile(True, prof)
        for d in ds:
            e.submit(a, d, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
        tm = e.timing()
    assert tm["plugin_overlapped"] >= 1, tm
    assert st["fragmented_packets"] > 0, st
    d = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + ["ext"])
    assert not d, d
    assert eng.seen == orc.seen


@pytest.mark.gpu
def test_pre_export_failure_in_poll_fails_the_call():
    """the plugins' pre_export on the records the device exported (ipxg_poll_exports) can
    fail only through the instance's error() (pre_export returns nothing): the poll hands the records
    over, then fails with IPXG_EPLUGIN and the plugin's message, and the engine refuses work until
    ipxg_reset.  A port-53 plugin claims every flow in post_create (a non-zero ext); k_finish exports
    them on the device; the first pre_export fails."""
    from ipfixprobe_amd import Engine
    from ipfixprobe_amd.engine import ERROR_FN, IpxgError

    class FailOnExport(plugins_py.PyPlugin):
        proto_mask = 2
        ports = (53,)

        def __init__(self):
            super().__init__()
            self.msg = ctypes.create_string_buffer(b"pre_export failed on purpose")
            self.failed = False
            self._err = ERROR_FN(self._error)
            self.struct.error = self._err

        def _post_create(self, ctx, flow, view):
            self.calls["post_create"] += 1
            ctypes.c_uint64.from_address(flow + FLOW_EXT_OFFSET).value = 0x5EED  # the flow's state
            return 0

        def _pre_export(self, ctx, flow):
            self.calls["pre_export"] += 1
            self.failed = True

        def _error(self, ctx):
            if not self.failed:
                return None
            self.failed = False
            return ctypes.addressof(self.msg)

    n = 2000
    sip = (10 << 24) + np.arange(n) % 100
    arena, desc = synth.udp_frames(sip, np.full(n, (192 << 24) + 1), np.full(n, 5000), np.full(n, 53))
    pl = FailOnExport()
    with Engine("s=16") as e:
        e.add_plugin(pl.struct)
        e.submit(arena, desc)
        e.finish()
        with pytest.raises(IpxgError) as ex:
            e.poll()
        assert ex.value.rc == -8 and "pre_export failed on purpose" in str(ex.value), str(ex.value)
        with pytest.raises(IpxgError) as ex2:
            e.submit(arena, desc)
        assert ex2.value.rc == -7
        e.reset()
    assert pl.calls["pre_export"] >= 1
