"""IPFIX export formatting: the data records of the reference IPFIX
plugin's basic templates.  The oracle (oracle/ipxg_oracle.c oracle_ipfix_basic, a table-
driven restatement of IPFIX_FILL_FIELD / fill_basic_flow, ipfix.cpp:77-96 and :1470-1516) is
pinned here against an independent struct-level packing of BASIC_TMPLT_V4/V6
(ipfix-elements.hpp:328-366); the device formatter is checked against the oracle on real
flow exports."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))

import oracle_py  # noqa: E402
import synth  # noqa: E402
from pcaputil import FLOW_DTYPE  # noqa: E402

EPOCH_DIFF = 2208988800  # ipfix-elements.hpp:50


def _ntp(sec, usec):  # MK_NTP_TS, ipfix-elements.hpp:59-60 (uint64_t arithmetic: wraps)
    return (((sec + EPOCH_DIFF) << 32) | (((usec << 32) // 1000000) & 0xFFFFFFFF)) & (2**64 - 1)


def _pack(r, dir_bit_field):
    """BASIC_TMPLT_V4 / _V6 element by element: end reason, bytes, bytes rev, packets,
    packets rev, flow start, flow end (NTP), L3 proto, L4 proto, TCP flags, TCP flags rev,
    ports, input interface, addresses (network order as stored), src MAC, dst MAC."""
    v4 = int(r["ip_version"]) == 4
    na = 4 if v4 else 16
    return (struct.pack(">BQQQQQQBBBBHHI", int(r["end_reason"]), int(r["src_bytes"]), int(r["dst_bytes"]),
                        int(r["src_packets"]), int(r["dst_packets"]),
                        _ntp(int(r["time_first_sec"]), int(r["time_first_usec"])),
                        _ntp(int(r["time_last_sec"]), int(r["time_last_usec"])),
                        int(r["ip_version"]), int(r["ip_proto"]), int(r["src_tcp_flags"]),
                        int(r["dst_tcp_flags"]), int(r["src_port"]), int(r["dst_port"]), dir_bit_field)
            + bytes(r["src_ip"][:na]) + bytes(r["dst_ip"][:na]) + bytes(r["src_mac"]) + bytes(r["dst_mac"]))


def _random_records(n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, dtype=FLOW_DTYPE)
    for f in ("flow_hash", "src_bytes", "dst_bytes"):
        r[f] = rng.integers(0, 2**63, n, dtype=np.uint64)
    for f in ("time_first_sec", "time_last_sec", "src_packets", "dst_packets"):
        r[f] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for f in ("time_first_usec", "time_last_usec"):
        r[f] = rng.integers(0, 1_000_000, n)
    r["ip_version"] = rng.choice([4, 6], n)
    for f in ("ip_proto", "src_tcp_flags", "dst_tcp_flags", "end_reason"):
        r[f] = rng.integers(0, 256, n)
    for f in ("src_port", "dst_port", "vlan_id"):
        r[f] = rng.integers(0, 65536, n)
    for f, w in (("src_ip", 16), ("dst_ip", 16), ("src_mac", 6), ("dst_mac", 6)):
        r[f] = rng.integers(0, 256, (n, w))
    return r


def test_ipfix_lengths_are_the_templates():
    r = np.zeros(2, dtype=FLOW_DTYPE)
    r["ip_version"] = [4, 6]
    assert len(_pack(r[0], 0)) == 81 and len(_pack(r[1], 0)) == 105


@pytest.mark.parametrize("dir_bit_field", [0, 0x01020304])
def test_oracle_ipfix_matches_struct_packing(dir_bit_field):
    recs = _random_records(500, seed=dir_bit_field & 0xFF)
    got, off = oracle_py.ipfix_basic(recs, dir_bit_field)
    want = b"".join(_pack(r, dir_bit_field) for r in recs)
    assert bytes(got) == want
    lens = np.diff(off.astype(np.int64))
    assert np.array_equal(lens, np.where(recs["ip_version"] == 4, 81, 105))


def test_oracle_ipfix_ntp_edges():
    r = np.zeros(3, dtype=FLOW_DTYPE)
    r["ip_version"] = 4
    r["time_first_usec"] = [0, 999_999, 500_000]
    r["time_first_sec"] = [0, 0xFFFFFFFF, 1_700_000_000]
    got, off = oracle_py.ipfix_basic(r)
    for k in range(3):
        rec = bytes(got[int(off[k]): int(off[k + 1])])
        ntp = struct.unpack(">Q", rec[33:41])[0]
        assert ntp == _ntp(int(r["time_first_sec"][k]), int(r["time_first_usec"][k]))


@pytest.mark.gpu
@pytest.mark.parametrize("dir_bit_field", [0, 7])
def test_device_ipfix_matches_oracle(dir_bit_field):
    from ipfixprobe_amd import Engine
    recs = _random_records(3000, seed=11 + dir_bit_field)
    want, woff = oracle_py.ipfix_basic(recs, dir_bit_field)
    with Engine() as e:
        got, off = e.ipfix_basic(recs, dir_bit_field)
    assert np.array_equal(off, woff)
    assert bytes(got) == bytes(want)


@pytest.mark.gpu
def test_poll_ipfix_of_real_exports():
    """Exports of a capture formatted from the device export buffer: equal to the oracle's
    formatting of the engine's own records, consumed in whole-record prefixes."""
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(seed=23, n_flows=150, n_pkts=3000, frag=False, v6_share=0.4).batch()
    with Engine() as e:
        e.submit(arena, desc)
        e.finish()
        recs = e.poll()
        e.reset()
        e.submit(arena, desc)
        e.finish()
        parts, n_total = [], 0
        cap = 81 * 7 + 50  # a few records per call: prefix semantics
        while e.pending():
            b, n = e.poll_ipfix(3, cap)
            assert n > 0 and len(b) <= cap
            parts.append(bytes(b))
            n_total += n
    assert n_total == len(recs)
    want, _ = oracle_py.ipfix_basic(recs, 3)
    # export order may differ between the two runs: compare the records as multisets
    assert sorted(_split(b"".join(parts))) == sorted(_split(bytes(want)))


def _split(stream):
    """IPFIX basic records back to back -> list of records (length from L3_PROTO at +49)."""
    out, k = [], 0
    while k < len(stream):
        n = 81 if stream[k + 49] == 4 else 105
        out.append(stream[k: k + n])
        k += n
    assert k == len(stream)
    return out


# ---- IPFIX messages: templates + MTU-bounded data messages (ipfix.cpp:385-398, 537-795) ------
import json  # noqa: E402

import ipfixdec  # noqa: E402

GOLDEN_TMPL = os.path.join(os.path.dirname(__file__), "golden", "ipfix_basic_templates.json")


def _v4_first(recs):
    return np.concatenate([recs[recs["ip_version"] != 6], recs[recs["ip_version"] == 6]])


def test_oracle_templates_match_reference_header():
    """The template message's records equal BASIC_TMPLT_V4/V6 as the reference header expands
    them (tests/golden/gen_ipfix_template.py compiles ipfix-elements.hpp), ids 258 / 259."""
    with open(GOLDEN_TMPL) as f:
        gold = json.load(f)
    recs = _random_records(2, seed=3)
    recs["ip_version"] = [4, 6]
    b, nm = oracle_py.ipfix_export(oracle_py.ipfix_exporter(), recs)
    msgs, tmpl, _, _, _ = ipfixdec.decode(b)
    assert msgs[0]["sets"][0][0] == 2 and len(msgs[0]["sets"]) == 1
    assert [list(t) for t in tmpl[258]] == gold["BASIC_TMPLT_V4"]
    assert [list(t) for t in tmpl[259]] == gold["BASIC_TMPLT_V6"]


def test_oracle_ntp_matches_reference_macro():
    with open(GOLDEN_TMPL) as f:
        gold = json.load(f)
    r = np.zeros(len(gold["MK_NTP_TS"]), dtype=FLOW_DTYPE)
    r["ip_version"] = 4
    r["time_first_sec"] = [g[0] for g in gold["MK_NTP_TS"]]
    r["time_first_usec"] = [g[1] for g in gold["MK_NTP_TS"]]
    got, off = oracle_py.ipfix_basic(r, 0)
    for i, g in enumerate(gold["MK_NTP_TS"]):
        o = int(off[i]) + 33  # FLOW_START after end reason, bytes x2, packets x2
        assert bytes(got[o:o + 8]).hex() == g[2]


@pytest.mark.parametrize("n,share6,mtu", [(0, 0.5, 1458), (1, 0.0, 1458), (17, 0.0, 1458), (18, 0.0, 1458),
                                          (13, 1.0, 1458), (14, 1.0, 1458), (30, 0.3, 1458), (1000, 0.4, 1458),
                                          (777, 0.5, 9000), (500, 0.5, 125), (300, 0.1, 1500)])
def test_oracle_message_stream_structure(n, share6, mtu):
    """Every message of the oracle's stream is well formed and <= mtu, the template message
    comes once and first, sequence numbers count the records of earlier data messages, and the
    records decode back to the input."""
    rng = np.random.default_rng(n)
    recs = _random_records(n, seed=n)
    recs["ip_version"] = np.where(rng.random(n) < share6, 6, 4)
    x = oracle_py.ipfix_exporter(odid=42, dir_bit_field=5, export_time=1_700_000_000, mtu=mtu)
    b, nm = oracle_py.ipfix_export(x, recs)
    if n == 0:
        assert len(b) == 0 and nm == 0 and x.templates_sent == 0
        return
    msgs, tmpl, got, where, dirs = ipfixdec.decode(b)
    assert len(msgs) == nm and x.templates_sent == 1 and x.sequence == n
    assert msgs[0]["sets"][0][0] == 2 and all(s[0] != 2 for m in msgs[1:] for s in m["sets"])
    seq = 0
    for m in msgs:  # the template message is not bounded by mtu (create_template_packet :671-728)
        assert (m["length"] <= mtu or m["sets"][0][0] == 2) and m["odid"] == 42 and m["export_time"] == 1_700_000_000
        assert m["sequence"] == seq
        seq += m["records"]
    assert dirs == {5}
    assert ipfixdec.basic_view(got) == ipfixdec.basic_view(recs)
    # a second call: no template message, the sequence continues
    b2, _ = oracle_py.ipfix_export(x, recs[:3])
    m2, _, _, _, _ = ipfixdec.decode(b2, tmpl)
    assert all(s[0] != 2 for m in m2 for s in m["sets"]) and m2[0]["sequence"] == n


@pytest.mark.gpu
@pytest.mark.parametrize("n,share6,mtu", [(1, 0.0, 1458), (17, 0.0, 1458), (18, 0.0, 1458), (14, 1.0, 1458),
                                          (30, 0.3, 1458), (1000, 0.4, 1458), (777, 0.5, 9000), (500, 0.5, 125),
                                          (50_000, 0.2, 1458), (300_000, 0.5, 1500)])
def test_device_messages_equal_oracle(n, share6, mtu):
    """ipxg_ipfix_export (records fed v4-first, formatted and packed on the device) is byte
    for byte the oracle exporter over the same record order, across two calls (exporter state
    carried: templates once, sequence numbers continue)."""
    from ipfixprobe_amd import Engine
    rng = np.random.default_rng(n + 1)
    recs = _random_records(n, seed=n + 1)
    recs["ip_version"] = np.where(rng.random(n) < share6, 6, 4)
    with Engine() as e:
        xd = e.ipfix_exporter(odid=9, dir_bit_field=3, export_time=1_600_000_123, mtu=mtu)
        xo = oracle_py.ipfix_exporter(odid=9, dir_bit_field=3, export_time=1_600_000_123, mtu=mtu)
        for part in (recs, recs[: n // 3]):
            got, gm = e.ipfix_export(xd, part)
            want, wm = oracle_py.ipfix_export(xo, _v4_first(part))
            assert gm == wm and len(got) == len(want)
            assert bytes(got) == bytes(want)
            assert (xd.sequence, xd.templates_sent) == (xo.sequence, xo.templates_sent)


@pytest.mark.gpu
def test_poll_ipfix_messages_from_flow_cache():
    """A capture through the engine, exported as IPFIX messages straight from the device export
    buffer: the decoded records are the oracle's flow records (basic fields)."""
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(seed=21, n_flows=400, n_pkts=8000).batch()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    with Engine() as e:
        e.submit(arena, desc)
        e.finish()
        x = e.ipfix_exporter(odid=1, export_time=77)
        b, nrec, nm = e.poll_ipfix_messages(x)
        assert e.pending() == 0
    msgs, _, got, _, _ = ipfixdec.decode(b)
    assert nrec == len(want) == len(got) and nm == len(msgs)
    w = want.copy()
    w["end_reason"] = got["end_reason"][0]  # reasons differ by design (FORCED vs sweep), see flowcmp
    g = got.copy()
    g["end_reason"] = w["end_reason"][0]
    assert ipfixdec.basic_view(g) == ipfixdec.basic_view(w)


@pytest.mark.gpu
def test_poll_ipfix_messages_after_partial_poll():
    """After a partial ipxg_poll_exports the IPv6 export count no longer covers the pending
    records: the message layer counts them itself, and the stream still decodes to them."""
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(seed=22, n_flows=300, n_pkts=6000, v6_share=0.5).batch()
    with Engine() as e:
        e.submit(arena, desc)
        e.finish()
        n = e.pending()
        out = np.zeros(7, dtype=FLOW_DTYPE)
        import ctypes
        from ipfixprobe_amd import engine as eng_mod
        got = ctypes.c_size_t()
        eng_mod.lib().ipxg_poll_exports(e.handle, out.ctypes.data, 7, ctypes.byref(got))
        x = e.ipfix_exporter()
        b, nrec, nm = e.poll_ipfix_messages(x)
    assert got.value == 7 and nrec == n - 7
    msgs, _, recs, _, _ = ipfixdec.decode(b)
    assert len(recs) == n - 7


class _DevBytes:
    """__cuda_array_interface__ over n bytes of device memory (the engine's message buffer)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}


@pytest.mark.gpu
def test_device_messages_beside_a_batch_in_flight():
    """ipxg_device_ipfix_messages called with an asynchronous batch in flight (its k_fin_list not
    launched yet) formats the exports of the batches completed before it on the engine's
    formatting stream, beside that batch's kernels, without completing it; the batch's tail
    joins the formatting before it appends exports.  Over two steps the device streams carry the
    host message path's records, sizes and message sequence (exporter state carried; the export
    order within a step is not fixed -- workgroups reserve their export slots by atomics), with
    the first stream consumed while the second step's batch runs, and the two alternating buffers
    keep the first stream intact while the second is formatted."""
    import torch
    from ipfixprobe_amd import Engine
    a1, d1 = synth.flow_stream(seed=31, n_flows=600, n_pkts=12000).batch()
    a2, d2 = synth.flow_stream(seed=32, n_flows=700, n_pkts=12000, v6_share=0.3).batch()
    with Engine() as e:
        x = e.ipfix_exporter(odid=4, export_time=99)
        e.submit(a1, d1)
        e.finish()
        want1, _, _ = e.poll_ipfix_messages(x)
        e.submit(a2, d2, asynchronous=True)
        e.finish()
        want2, _, _ = e.poll_ipfix_messages(x)
    with Engine() as e:
        x = e.ipfix_exporter(odid=4, export_time=99)
        e.submit(a1, d1)
        e.finish()
        e.submit(a2, d2, asynchronous=True)  # in flight: its tail is launched by the next call
        p1, nb1, nr1, _ = e.device_ipfix_messages(x)
        e.finish()  # the tail joins the formatting of stream 1
        p2, nb2, nr2, _ = e.device_ipfix_messages(x)
        assert p1 != p2  # (alternating buffers: stream 1 is still valid here)
        torch.cuda.ExternalStream(e.ipfix_stream()).synchronize()
        got1 = torch.as_tensor(_DevBytes(p1, nb1), device="cuda").cpu().numpy().tobytes()
        got2 = torch.as_tensor(_DevBytes(p2, nb2), device="cuda").cpu().numpy().tobytes()
        assert e.pending() == 0
    assert len(got1) == len(want1) and len(got2) == len(want2)
    gm1, t1, gr1, _, _ = ipfixdec.decode(got1)
    wm1, _, wr1, _, _ = ipfixdec.decode(want1)
    gm2, _, gr2, _, _ = ipfixdec.decode(got2, t1)
    wm2, _, wr2, _, _ = ipfixdec.decode(want2, t1)
    assert nr1 == len(gr1) == len(wr1) > 500 and nr2 == len(gr2) == len(wr2) > 600
    assert ipfixdec.basic_view(gr1) == ipfixdec.basic_view(wr1)
    assert ipfixdec.basic_view(gr2) == ipfixdec.basic_view(wr2)
    assert [m["sequence"] for m in gm1 + gm2] == [m["sequence"] for m in wm1 + wm2]
