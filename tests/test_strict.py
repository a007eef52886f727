"""Strict mode (strict=true): the reference's own table -- 2^s records in
lines of 2^l, move to front, FLOW_END_NO_RES eviction with insertion at the middle and the
per-packet sweep (cache.cpp:322-523) -- replayed on the device (ipxg_strict.hip).  Every field
of every record is compared with the oracle's NHTFlowCache restatement, end_reason included,
at table sizes where lines overflow (NO_RES evictions) and the sweep exports idle records, and
the export statistics (end reasons, FlowRecordStats buckets) must be equal."""
import os
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil
import synth
from test_oracle_synth import PKT_BUCKETS

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference")
FIELDS = flowcmp.CONTRACT_FIELDS + ["end_reason"]
END = ["end_inactive", "end_active", "end_eof", "end_forced", "end_no_res", "total_exported"]


def _oracle_kw(params):
    kw = {}
    for tok in filter(None, params.split(";")):
        k, _, v = tok.partition("=")
        key = {"s": "cache_exp", "l": "line_exp", "a": "active", "i": "inactive", "fs": "frag_size",
               "ft": "frag_timeout"}.get(k)
        if key:
            kw[key] = int(v)
        elif k == "S":
            kw["split_biflow"] = True
        elif k == "fe":
            kw["frag_enable"] = v == "true"
    return kw


def test_oracle_no_res_regime_reached():
    """The parity cases below really evict: the oracle at s=8 exports NO_RES records."""
    arena, desc = synth.flow_stream(seed=31, n_flows=600, n_pkts=6000).batch()
    _, st = oracle_py.run_capture(arena, desc, 1, cache_exp=8, line_exp=4)
    assert st["end_no_res"] > 100 and st["end_inactive"] > 0


def _check(arena, desc, params, batch=None, dl=1, expire=None):
    from ipfixprobe_amd import Engine
    with Engine("strict=true;" + params, datalink=dl) as e:
        n = len(desc)
        step = batch or n
        for k in range(0, n, step):
            e.submit(arena, np.ascontiguousarray(desc[k:k + step]))
            if expire is not None:
                e.expire(expire(k))
        e.finish()
        got = e.poll()
        gst = e.stats()
    c = oracle_py.OracleCache(**_oracle_kw(params))
    for k in range(0, len(desc), batch or len(desc)):
        c.run(arena, np.ascontiguousarray(desc[k:k + (batch or len(desc))]), dl)
        if expire is not None:
            c.export_expired(expire(k))
    c.finish()
    want = c.take()
    wst = c.stats()
    c.close()
    d = flowcmp.diff(got, want, fields=FIELDS)
    assert not d, d
    for k in END + PKT_BUCKETS + ["fragmented_packets", "fragments_filled", "parsed_packets", "keyless_packets"]:
        assert gst[k] == wst[k], (k, gst[k], wst[k])
    return got, gst


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [None, 1000, 777])
@pytest.mark.parametrize("params", ["s=8", "s=7;l=2", "s=12;l=4;i=5;a=20", "s=8;S", "s=8;l=0", "s=8;l=1",
                                    "s=8;ft=1;fs=7", "s=6;l=3;a=60"])
def test_strict_stream_parity(params, batch):
    arena, desc = synth.flow_stream(seed=31, n_flows=600, n_pkts=6000, v6_share=0.3, vlan_share=0.2).batch()
    _, gst = _check(arena, desc, params, batch)
    if params.startswith(("s=8", "s=7", "s=6")):
        assert gst["end_no_res"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("wgs", ["0", "2", "8", "32"])
@pytest.mark.parametrize("params", ["s=8", "s=12;l=4;i=5;a=20", "s=8;S", "s=7;l=2", "s=20"])
def test_strict_multi_workgroup_parity(monkeypatch, params, wgs):
    """The replay on several workgroups of one XCD (IPXG_STRICT_WGS per XCD; sc1 table reads,
    agent-scope scheduler; the default is 12) or on one workgroup (0): the same records, end
    reasons and statistics as the oracle."""
    monkeypatch.setenv("IPXG_STRICT_WGS", wgs)
    arena, desc = synth.flow_stream(seed=41, n_flows=900, n_pkts=20000, v6_share=0.3, vlan_share=0.2).batch()
    _check(arena, desc, params, batch=6000)


@pytest.mark.gpu
def test_strict_multi_workgroup_watchdog(monkeypatch):
    """One flow on several workgroups: one chain, every other lane waits (progress-based bound)."""
    monkeypatch.setenv("IPXG_STRICT_WGS", "8")
    monkeypatch.setenv("IPXG_STRICT_SPIN_MAX", "4096")
    arena, desc = synth.flow_stream(seed=36, n_flows=1, n_pkts=50000, frag=False).batch()
    got, _ = _check(arena, desc, "s=10")
    assert len(got) >= 1


@pytest.mark.gpu
def test_strict_expire_is_one_sweep_step():
    """ipxg_expire in strict mode is the reference's export_expired(now): one step of the
    sweep cursor (cache.cpp:508-523), interleaved with the batches."""
    arena, desc = synth.flow_stream(seed=32, n_flows=300, n_pkts=5000).batch()
    ts = desc["ts_sec"]
    _check(arena, desc, "s=10;i=5", batch=250, expire=lambda k: int(ts[min(k + 249, len(ts) - 1)]) + 3)


@pytest.mark.gpu
def test_strict_fuzz_corpus():
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=33))
    _check(arena, desc, "s=11")


@pytest.mark.gpu
def test_strict_large_table():
    """2^16 lines (past the per-line LDS counters of the first replay; the DAG scheduler has no
    line limit): a stream whose flows spread over the table, every record still bit-exact."""
    arena, desc = synth.flow_stream(seed=35, n_flows=4000, n_pkts=30000, v6_share=0.2).batch()
    _check(arena, desc, "s=20", batch=7000)


@pytest.mark.gpu
def test_strict_one_hot_line():
    """Every packet of one flow (a chain of dependent events on one line) plus a few others."""
    arena, desc = synth.flow_stream(seed=34, n_flows=3, n_pkts=20000, frag=False).batch()
    _check(arena, desc, "s=6")


@pytest.mark.gpu
def test_strict_single_flow_watchdog(monkeypatch):
    """One flow only: the whole batch is one dependent chain run serially by one lane while the
    other 767 lanes wait.  The replay's watchdog is progress-based (it restarts whenever any
    packet finishes), so a short bound (IPXG_STRICT_SPIN_MAX, 4096 polling rounds: well under a
    millisecond, against the chain's ~0.1 s) must not give up on valid input."""
    monkeypatch.setenv("IPXG_STRICT_SPIN_MAX", "4096")
    arena, desc = synth.flow_stream(seed=36, n_flows=1, n_pkts=100000, frag=False).batch()
    got, _ = _check(arena, desc, "s=10")
    assert len(got) >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["basic", "vlan", "mqtt", "http", "quic"])
def test_strict_reproduces_reference_golden(name):
    """At the reference's own defaults (s=17, l=4) the engine in strict mode gives the golden
    output of the reference run (the same check as the oracle's, tests/test_oracle_golden.py)."""
    from ipfixprobe_amd import run_capture
    from test_oracle_golden import PAIRS, _columns
    dl, pk = pcaputil.read_capture(os.path.join(REF, PAIRS[name] + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    recs, _ = run_capture(arena, desc, datalink=dl, params="strict=true")
    cols = _columns(name)
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name), cols))
    assert Counter(pcaputil.format_records(recs, cols)) == gold


@pytest.mark.gpu
def test_strict_rejects_what_it_does_not_replay():
    from ipfixprobe_amd import Engine, IpxgError
    for bad in ("strict=true;l=5", "strict=true;s=29;l=4", "strict=true;ingest=atomic", "strict=true;ps=true"):
        with pytest.raises(IpxgError):
            Engine(bad)
    import plugins_py
    with Engine("strict=true;s=10") as e:
        with pytest.raises(IpxgError):
            e.add_plugin(plugins_py.DnsFlush().struct)
