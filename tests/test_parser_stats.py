"""Parser side statistics: TopPorts' TCP/UDP port frequencies
(parser.cpp:484-485, 563-564; topPorts.cpp) and VlanStats with the packet-size histogram
(parser.cpp:798; parser-stats.hpp:42-160).

CPU: the oracle's restatement against an independent per-packet Python restatement over the
reference's own captures and the fuzz corpus (the reference's functional tests do not print these
counters, so they are pinned through the parser fields the goldens do pin: parity of the
counters themselves is unpinned against the reference binary), and the get_top_ports ordering.
GPU: the engine (ps=true) against the oracle on the same packets, bit-exact."""
import os

import numpy as np
import pytest

import oracle_py
import pcaputil
import synth

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "golden", "reference")

BUCKETS = [(0, 64), (65, 127), (128, 255), (256, 511), (512, 1023), (1024, 1517), (1518, 2047), (2048, 4095),
           (4096, 8191), (8192, 65535)]


def top_ports(tcp, udp, n):
    """TopPorts::get_top_ports (topPorts.cpp:35-77) literally: a buffer of n entries, every TCP
    port then every UDP port inserted at lower_bound(frequency >= count)."""
    buf = [(0, 0, 0)] * n  # (port, frequency, protocol)
    inserted = 0
    for proto, arr in ((6, tcp), (17, udp)):
        for port in range(65536):
            f = int(arr[port])
            pos = next((i for i, e in enumerate(buf) if not e[1] >= f), None) if n else None
            if pos is not None:
                buf = buf[:pos] + [(port, f, proto)] + buf[pos:-1]
                inserted += 1
    return buf[:min(n, inserted)]


def _python_stats(arena, desc, dl):
    """Per packet from oracle_parse: ports of valid TCP/UDP packets with frag_off == 0, VlanStats
    of valid packets (sizes = caplen)."""
    pk, _ = oracle_py.parse_batch(arena, desc, dl)
    tcp = np.zeros(65536, dtype=np.uint64)
    udp = np.zeros(65536, dtype=np.uint64)
    vl = np.zeros(4096, dtype=pcaputil.VLAN_STATS_DTYPE)
    for i in range(len(pk)):
        p = pk[i]
        if not p["valid"]:
            continue
        if p["frag_off"] == 0 and p["ip_proto"] in (6, 17):
            arr = tcp if p["ip_proto"] == 6 else udp
            arr[p["src_port"]] += 1
            arr[p["dst_port"]] += 1
        v = vl[p["vlan_id"] & 0xFFF]
        ln = int(desc["caplen"][i])
        if p["ip_version"] == 4:
            v["ipv4_packets"] += 1
            v["ipv4_bytes"] += ln
        elif p["ip_version"] == 6:
            v["ipv6_packets"] += 1
            v["ipv6_bytes"] += ln
        if p["ip_proto"] == 6:
            v["tcp_packets"] += 1
        elif p["ip_proto"] == 17:
            v["udp_packets"] += 1
        v["total_packets"] += 1
        v["total_bytes"] += ln
        b = next(k for k, (lo, hi) in enumerate(BUCKETS) if lo <= ln <= hi)
        v["hist_packets"][b] += 1
        v["hist_bytes"][b] += ln
        vl[p["vlan_id"] & 0xFFF] = v
    return tcp, udp, vl


def _oracle_stats(arena, desc, dl, **kw):
    c = oracle_py.OracleCache(**kw)
    c.run(arena, desc, dl)
    out = c.parser_stats()
    st = c.stats()
    c.close()
    return out, st


@pytest.mark.parametrize("name", ["mixed", "vlan", "http", "dns", "mqtt", "tls"])
def test_oracle_parser_stats_reference_captures(name):
    dl, pkts = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
    arena, desc = pcaputil.to_batch(pkts)
    (tcp, udp, vl), st = _oracle_stats(arena, desc, dl, cache_exp=20)
    ptcp, pudp, pvl = _python_stats(arena, desc, dl)
    assert np.array_equal(udp, pudp) and np.array_equal(vl, pvl)
    assert np.all(tcp >= ptcp)  # + TCP segments dropped after their ports were read
    assert int(vl["total_packets"].sum()) == st["parsed_packets"]
    assert int(vl["ipv4_packets"].sum()) + int(vl["ipv6_packets"].sum()) > 0


def test_oracle_parser_stats_fuzz_corpus():
    corpus = synth.fuzz_corpus(20000, seed=41)
    arena, desc = synth.to_batch(corpus)
    (tcp, udp, vl), st = _oracle_stats(arena, desc, 1, cache_exp=20)
    ptcp, pudp, pvl = _python_stats(arena, desc, 1)
    assert np.array_equal(udp, pudp) and np.array_equal(vl, pvl)
    extra = tcp.astype(np.int64) - ptcp.astype(np.int64)
    assert extra.min() >= 0 and extra.sum() > 0 and extra.sum() % 2 == 0  # dropped TCP: 2 ports each


def test_top_ports_ordering():
    tcp = np.zeros(65536, dtype=np.uint64)
    udp = np.zeros(65536, dtype=np.uint64)
    tcp[[80, 443, 22]] = [5, 9, 5]
    udp[[53, 443, 7]] = [9, 1, 5]
    got = top_ports(tcp, udp, 4)
    assert got == [(443, 9, 6), (53, 9, 17), (22, 5, 6), (80, 5, 6)]  # ties: TCP first, then port order
    assert top_ports(tcp, udp, 10)[-1] == (443, 1, 17) and len(top_ports(tcp, udp, 10)) == 6


def _engine_stats(arena, desc, params, batch=None):
    from ipfixprobe_amd import Engine
    with Engine(params) as e:
        n = len(desc)
        step = batch or n
        for k in range(0, n, step):
            e.submit(arena, np.ascontiguousarray(desc[k:k + step]))
        e.finish()
        tcp, udp, vl = e.parser_stats()
        tp = e.top_ports(12)
    return tcp, udp, vl, tp


def _check(arena, desc, params, okw, batch=None):
    (tcp, udp, vl), _ = _oracle_stats(arena, desc, 1, **okw)
    gt, gu, gv, tp = _engine_stats(arena, desc, params, batch)
    assert np.array_equal(gt, tcp), np.nonzero(gt != tcp)[0][:10]
    assert np.array_equal(gu, udp), np.nonzero(gu != udp)[0][:10]
    assert np.array_equal(gv, vl)
    want = top_ports(tcp, udp, 12)
    assert [(int(r["port"]), int(r["frequency"]), int(r["protocol"])) for r in tp] == want


@pytest.mark.gpu
@pytest.mark.parametrize("walk", ["narrow", "wide"])
def test_gpu_parser_stats_fuzz_corpus(walk):
    corpus = synth.fuzz_corpus(20000, seed=41)
    arena, desc = synth.to_batch(corpus)
    _check(arena, desc, "ps=true;s=20;walk=" + walk, dict(cache_exp=20))


@pytest.mark.gpu
@pytest.mark.parametrize("frag", [True, False])
@pytest.mark.parametrize("batch", [None, 333])
def test_gpu_parser_stats_streams(frag, batch):
    """Fragments (the cache filling ports of non-first fragments, or not), VLAN and IPv6 flows,
    several batches."""
    arena, desc = synth.flow_stream(seed=51, n_flows=150, n_pkts=5000, v6_share=0.4, vlan_share=0.4,
                                    frag=True).batch()
    params = "ps=true;s=20" + ("" if frag else ";fe=false")
    _check(arena, desc, params, dict(cache_exp=20, frag_enable=frag), batch)


@pytest.mark.gpu
def test_gpu_parser_stats_reference_captures():
    for name in ("mixed", "vlan", "http", "tls"):
        dl, pkts = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
        assert dl == 1
        arena, desc = pcaputil.to_batch(pkts)
        _check(arena, desc, "ps=true;s=20", dict(cache_exp=20))


@pytest.mark.gpu
def test_gpu_parser_stats_off_by_default():
    from ipfixprobe_amd import Engine, IpxgError
    with Engine() as e:
        with pytest.raises(IpxgError):
            e.parser_stats()
