"""Device parity on synthetic inputs the fixtures do not reach: a parser fuzz corpus over
every encapsulation, and multi-flow streams that trigger each split rule of
put_pkt_recursive (cache.cpp:431-472), the fragmentation cache, table growth and expiry,
cut into batches so that carried-in flow state crosses batch boundaries."""
import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil
import synth
from test_oracle_synth import PKT_BUCKETS

pytestmark = pytest.mark.gpu


def oracle_kwargs(params):
    kw = {"cache_exp": 20}
    for tok in filter(None, params.split(";")):
        k, _, v = tok.partition("=")
        if k == "a":
            kw["active"] = int(v)
        elif k == "i":
            kw["inactive"] = int(v)
        elif k == "S":
            kw["split_biflow"] = True
        elif k == "fe":
            kw["frag_enable"] = v == "true"
        elif k == "ft":
            kw["frag_timeout"] = int(v)
        elif k == "fs":
            kw["frag_size"] = int(v)
    return kw


@pytest.fixture(scope="module")
def engines():
    from ipfixprobe_amd import Engine
    cache = {}

    def get(dl):
        if dl not in cache:
            cache[dl] = Engine(datalink=dl)
        return cache[dl]
    yield get
    for e in cache.values():
        e.close()


def _cmp_parse(e, arena, desc, dl):
    got = e.parse(arena, desc)
    want, beyond = oracle_py.parse_batch(arena, desc, dl)
    bad = []
    for i in range(len(desc)):
        if beyond[i]:
            continue
        fields = pcaputil.PARSED_DTYPE.names if want[i]["valid"] else ("valid",)
        for f in fields:
            if not np.array_equal(got[i][f], want[i][f]):
                bad.append((i, f, got[i][f], want[i][f]))
    return bad, want


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_parse_fuzz_ethernet(engines, seed):
    corpus = synth.fuzz_corpus(20000, seed=seed)
    arena, desc = synth.to_batch(corpus)
    bad, want = _cmp_parse(engines(1), arena, desc, 1)
    assert not bad, bad[:10]
    assert want["valid"].sum() > 10000  # the corpus really exercises valid chains


@pytest.mark.parametrize("dl", [113, 276, 12])
def test_parse_fuzz_linktypes(engines, dl):
    rng = np.random.default_rng(dl)
    frames = []
    for _ in range(4000):
        et, l3 = synth._l3(rng)
        if dl == 113:
            f = synth.sll(l3, et, hatype=int(rng.integers(0, 3)))
        elif dl == 276:
            f = synth.sll2(l3, et, hatype=int(rng.integers(0, 3)))
        else:
            f = l3 if et in (0x0800, 0x86DD) and rng.random() < 0.9 else bytes(rng.integers(0, 256, 40, dtype=np.uint8))
        cl = len(f) if rng.random() < 0.9 else int(rng.integers(0, len(f) + 1))
        frames.append((f[:cl], cl, len(f)))
    arena, desc = synth.to_batch(frames)
    bad, _ = _cmp_parse(engines(dl), arena, desc, dl)
    assert not bad, bad[:10]


def test_parse_unaligned_offsets(engines):
    corpus = synth.fuzz_corpus(3000, seed=9)
    arena, desc = synth.to_batch(corpus)
    # shift every frame by 1..15 bytes: the byte-wise staging path
    pk = []
    big = np.zeros(len(arena) + 16 * len(desc) + 64, dtype=np.uint8)
    off = 0
    nd = desc.copy()
    for i, d in enumerate(desc):
        off += 1 + (i % 15)
        o, c = int(d["offset"]), int(d["caplen"])
        big[off: off + c] = arena[o: o + c]
        nd[i]["offset"] = off
        off += int(d["caplen"])
    bad, _ = _cmp_parse(engines(1), big[: off + 16], nd, 1)
    assert not bad, bad[:10]
    del pk


STREAMS = [
    dict(seed=7, n_flows=300, n_pkts=6000, params=""),
    dict(seed=8, n_flows=30, n_pkts=6000, params="", long_gap_share=0.0005),  # active timeouts
    dict(seed=9, n_flows=60, n_pkts=5000, params="a=20;i=5"),
    dict(seed=10, n_flows=200, n_pkts=5000, params="S"),
    dict(seed=11, n_flows=200, n_pkts=5000, params="fe=false"),
    dict(seed=12, n_flows=100, n_pkts=4000, params="i=1"),  # every flow on the sequential path
    dict(seed=13, n_flows=150, n_pkts=5000, params="ft=1;fs=7", v6_share=0.5, vlan_share=0.4),
]


def _stream(case):
    kw = {k: v for k, v in case.items() if k != "params"}
    return synth.flow_stream(**kw).batch()


def _with(params, extra):
    return ";".join(x for x in (params, extra) if x)


@pytest.mark.parametrize("walk", ["", "walk=wide"])
@pytest.mark.parametrize("batch", [None, 1, 37, 1000])
@pytest.mark.parametrize("ci", range(len(STREAMS)))
def test_stream_parity(ci, batch, walk):
    """walk "": the engine's choice per batch (narrow first, wide after a batch of mixed shapes);
    walk=wide: k_bin walks every header chain in LDS from the first batch."""
    from ipfixprobe_amd import run_capture
    case = STREAMS[ci]
    arena, desc = _stream(case)
    want, wst = oracle_py.run_capture(arena, desc, 1, **oracle_kwargs(case["params"]))
    assert wst["end_no_res"] == 0
    got, gst = run_capture(arena, desc, params=_with(case["params"], walk), batch=batch)
    d = flowcmp.diff(got, want)
    assert not d, d
    assert gst["fragmented_packets"] == wst["fragmented_packets"]
    assert gst["fragments_filled"] == wst["fragments_filled"]
    # FlowRecordStats (cache.cpp:601-616): the records are equal, so are their packet buckets
    assert [gst[k] for k in PKT_BUCKETS] == [wst[k] for k in PKT_BUCKETS]
    assert sum(gst[k] for k in PKT_BUCKETS) == gst["total_exported"] == len(got)


def test_stream_reasons_and_counts():
    """Every record the oracle closes by a split rule (EOF / INACTIVE / ACTIVE) is closed
    by the engine too; only records still open at the end differ in reason (FORCED vs the
    sweep's INACTIVE)."""
    from ipfixprobe_amd import run_capture
    case = STREAMS[1]
    arena, desc = _stream(case)
    want, wst = oracle_py.run_capture(arena, desc, 1, **oracle_kwargs(case["params"]))
    got, gst = run_capture(arena, desc, params=case["params"])
    assert gst["end_active"] == wst["end_active"] > 0
    assert gst["end_eof"] >= 1
    assert len(got) == len(want)


def test_expire_exports_everything_idle():
    from ipfixprobe_amd import Engine
    case = STREAMS[0]
    arena, desc = _stream(case)
    want, _ = oracle_py.run_capture(arena, desc, 1, **oracle_kwargs(case["params"]))
    with Engine() as e:
        e.submit_all(arena, desc, 500)
        e.expire(int(desc["ts_sec"][-1]) + 31)
        mid = e.poll()
        assert e.stats()["flows_in_cache"] == 0
        e.finish()
        rest = e.poll()
    assert len(rest) == 0
    assert set(np.unique(mid["end_reason"])) <= {1, 3}
    d = flowcmp.diff(mid, want)
    assert not d, d


def test_table_growth_and_deferral():
    """Start at 2^16 slots and push 200k new flows in one batch: probes overflow, the table
    is rebuilt mid-batch and the deferred packets re-applied."""
    from ipfixprobe_amd import run_capture
    rng = np.random.default_rng(5)
    frames = []
    for i in range(200_000):
        f = synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) +
                      synth.ipv4(synth.ip4(0x0A000000 + i), synth.ip4(0xC0A80001), 17,
                                 synth.udp(int(rng.integers(1024, 65536)), 53)))
        frames.append((f, len(f), len(f)))
    frames += frames[:50_000]  # second packets of the first 50k flows
    arena, desc = synth.to_batch(frames)
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=22)
    got, st = run_capture(arena, desc, params="s=16")
    assert st["table_rehashes"] >= 1
    d = flowcmp.diff(got, want)
    assert not d, d


def test_nonmonotonic_conserves_packets():
    """Out-of-order timestamps are outside the parity contract (the reference's sweep then
    depends on table positions); the engine must still account for every packet."""
    from ipfixprobe_amd import run_capture
    arena, desc = _stream(STREAMS[0])
    d2 = desc.copy()
    rng = np.random.default_rng(1)
    j = rng.choice(len(d2), 300, replace=False)
    d2["ts_sec"][j] -= rng.integers(0, 100, 300).astype(np.uint32)
    got, st = run_capture(arena, d2)
    keyed = st["parsed_packets"] - st["keyless_packets"]
    assert int(got["src_packets"].sum() + got["dst_packets"].sum()) == keyed
    assert st["complex_flows"] > 0


def test_bench_size_parity(monkeypatch):
    """The bench workload itself (10M 64 B packets, 100k biflows) against the oracle, through
    the bench's exact engine and step: its configuration (bench.engine_params: s=18, binned
    ingest, walk=auto), the batch submitted asynchronously from the device with the finish right
    behind it (the fused finish in k_fin_list), three steps in a row on the same engine (the
    partition sizing and the walk choice come from the previous step from the second on).  Then
    the same with the streamed reduce (IPXG_STREAM=1, round 6: k_reduce_stream folding k_bin's
    records while k_bin runs -- an A/B knob, off by default), from its second step on."""
    import torch

    import bench
    flows = bench.gen_flows(100_000, 0, 1, 1234)
    frames, desc = bench.build_batch(flows, 10_000_000, 1234, torch.device("cuda", 0))
    torch.cuda.synchronize()
    dn = desc.cpu().numpy().view(pcaputil.DESC_DTYPE)
    want, wst = oracle_py.run_capture(frames.cpu().numpy(), dn, 1, cache_exp=21)
    assert len(want) == 100_000 and wst["end_no_res"] == 0
    from ipfixprobe_amd import Engine
    with Engine(bench.engine_params(100_000)) as e:
        assert e.cfg.cache_exp == 18
        for step in range(3):
            e.submit(frames, desc, device=True, asynchronous=True, wait_producer=False)
            e.finish()
            got = e.poll()
            d = flowcmp.diff(got, want)
            assert not d, (step, d)
        assert e.stats()["complex_flows"] == 0
    monkeypatch.setenv("IPXG_STREAM", "1")
    with Engine(bench.engine_params(100_000)) as e:
        for step in range(3):
            e.submit(frames, desc, device=True, asynchronous=True, wait_producer=False)
            e.finish()
            got = e.poll()
            d = flowcmp.diff(got, want)
            assert not d, ("streamed", step, d)


# ---- the binned ingest's fast and fallback paths (ipxg_ingest.hip) -------------------------
NOFRAG = [
    dict(seed=14, n_flows=300, n_pkts=6000, params="", frag=False),
    dict(seed=15, n_flows=60, n_pkts=5000, params="a=20;i=5", frag=False),
    dict(seed=16, n_flows=200, n_pkts=5000, params="S", frag=False, v6_share=0.5),
]


@pytest.mark.parametrize("batch", [None, 1, 37, 1000])
@pytest.mark.parametrize("ci", range(len(NOFRAG)))
def test_stream_parity_no_fragments(ci, batch):
    """Without fragments k_reduce finalises the flows itself (no table scan)."""
    from ipfixprobe_amd import run_capture
    case = NOFRAG[ci]
    arena, desc = _stream(case)
    want, wst = oracle_py.run_capture(arena, desc, 1, **oracle_kwargs(case["params"]))
    got, _ = run_capture(arena, desc, params=case["params"], batch=batch)
    d = flowcmp.diff(got, want)
    assert not d, d


def test_fused_finalize_skips_table_scan():
    from ipfixprobe_amd import Engine
    arena, desc = _stream(NOFRAG[0])
    want, _ = oracle_py.run_capture(arena, desc, 1, **oracle_kwargs(""))
    with Engine() as e:
        e.profile(True)
        e.submit(arena, desc)
        tm = e.timing()
        e.finish()
        got = e.poll()
        st = e.stats()
    assert tm["reduce_launches"] == 1 and tm["finalize_launches"] == 0, tm
    assert st["spilled_packets"] == 0
    d = flowcmp.diff(got, want)
    assert not d, d


def _udp_batch(rng, flow_of_pkt, n_flows, reverse_share=0.5):
    sip = (10 << 24) + np.arange(n_flows, dtype=np.int64)
    dip = np.full(n_flows, (192 << 24) | (168 << 16) | 1, dtype=np.int64)
    sp = 1024 + (np.arange(n_flows, dtype=np.int64) * 7919) % 60000
    dp = 1 + (np.arange(n_flows, dtype=np.int64) % 1000)
    rev = rng.random(len(flow_of_pkt)) < reverse_share
    f = flow_of_pkt
    return synth.udp_frames(np.where(rev, dip[f], sip[f]), np.where(rev, sip[f], dip[f]),
                            np.where(rev, dp[f], sp[f]), np.where(rev, sp[f], dp[f]))


def test_elephant_flow_aggregated_per_tile():
    """Half of 200k packets in one biflow: each k_bin tile folds the elephant's ~1000 packets
    into one aggregate record (tile aggregation, first batch), so its partition's segments do
    not overflow; the records match the oracle."""
    from ipfixprobe_amd import run_capture
    rng = np.random.default_rng(21)
    n, F = 200_000, 5000
    fop = np.where(rng.random(n) < 0.5, 0, rng.integers(1, F, n))
    arena, desc = _udp_batch(rng, fop, F)
    want, wst = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got, st = run_capture(arena, desc, params="s=16")
    assert st["aggregated_packets"] >= n // 2 - 2000 and st["spilled_packets"] == 0
    d = flowcmp.diff(got, want)
    assert not d, d


@pytest.mark.parametrize("agg", ["0", "1"])
def test_elephant_flow_spill_path(monkeypatch, agg):
    """The same elephant with the segments forced small (IPXG_TILE_AGG / IPXG_PART_BITS tuning
    knobs are read per batch): records that do not fit their segment spill to device atomics
    (packet records, or whole aggregates) and the records still match the oracle."""
    from ipfixprobe_amd import Engine
    rng = np.random.default_rng(23)
    n, F = 200_000, 5000
    fop = np.where(rng.random(n) < 0.5, 0, rng.integers(1, F, n))
    arena, desc = _udp_batch(rng, fop, F)
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    monkeypatch.setenv("IPXG_TILE_AGG", agg)
    monkeypatch.setenv("IPXG_PART_BITS", "8")
    with Engine("s=16") as e:
        e.submit(arena, desc[:1000])  # first batch: the knob takes effect from the next one
        e.submit(arena, desc[1000:])
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["spilled_packets"] > 0 if agg == "0" else st["aggregated_packets"] > 0
    d = flowcmp.diff(got, want)
    assert not d, d


def test_partition_estimate_too_small_overflows_lds():
    """A first batch of 10 flows makes the engine size the next batch's partitions for 10
    flows; the next batch brings 300k new flows: k_reduce's LDS tables overflow (spill),
    the table overflows (deferral, growth), and every record must still match."""
    from ipfixprobe_amd import Engine
    rng = np.random.default_rng(22)
    F = 300_010
    fop = np.concatenate([np.arange(1000) % 10, 10 + rng.permutation(300_000)])
    arena, desc = _udp_batch(rng, fop, F)
    want, wst = oracle_py.run_capture(arena, desc, 1, cache_exp=22)
    with Engine() as e:
        e.submit(arena, desc[:1000])
        e.submit(arena, desc[1000:])
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["spilled_packets"] > 0 and st["table_rehashes"] >= 1
    d = flowcmp.diff(got, want)
    assert not d, d


@pytest.mark.parametrize("walk", ["narrow", "wide"])
@pytest.mark.parametrize("seed", [31, 32])
def test_flows_fuzz_corpus(seed, walk):
    """The parser fuzz corpus through the whole ingest against the oracle's flow records and
    parser counters: walk=narrow (k_bin's register fast path for plain Eth/IPv4/UDP|TCP frames,
    k_bin_slow's LDS walk for everything else) and walk=wide (k_bin walks every chain in LDS)."""
    from ipfixprobe_amd import run_capture
    corpus = synth.fuzz_corpus(20000, seed=seed)
    arena, desc = synth.to_batch(corpus)
    want, wst = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got, gst = run_capture(arena, desc, params="walk=" + walk)
    if walk == "wide":
        assert gst["walked_packets"] > 0
    d = flowcmp.diff(got, want)
    assert not d, d
    for k in ("seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets", "ipv6_packets",
              "tcp_packets", "udp_packets", "vlan_packets", "keyless_packets"):
        assert gst[k] == wst[k], k


@pytest.mark.parametrize("at", [1, 63, 64, 256, 2047, 2048, 2048 * 5 + 192])
def test_nonmonotonic_detected_at_wave_and_tile_boundaries(at):
    """One timestamp going backwards, at a lane / wave / tile boundary of k_bin: the batch is
    handled on the order-preserving path (every flow complex) and matches the oracle."""
    from ipfixprobe_amd import run_capture
    rng = np.random.default_rng(41)
    arena, desc = _udp_batch(rng, rng.integers(0, 50, 12000), 50)  # no order-dependent flows
    d2 = desc.copy()
    d2["ts_sec"][at] = d2["ts_sec"][at - 1] - 1  # before its predecessor
    want, _ = oracle_py.run_capture(arena, d2, 1, cache_exp=20)
    got, st = run_capture(arena, d2)
    assert st["complex_flows"] > 0
    d = flowcmp.diff(got, want)
    assert not d, d
    _, st0 = run_capture(arena, desc)
    assert st0["complex_flows"] == 0


def _edge_frames():
    """IPv6 extension chains (8- and 16-byte headers, the types the register walk takes and
    others), IPv4-in-GRE (optional fields, inner IPv6 / MPLS, IP options, fragments) and MPLS
    stacks of 1-3 labels over IPv4 / IPv6 with UDP / TCP, each
    also truncated at every caplen from 50 bytes: the shapes at the border of k_bin's wide
    register walk, where a frame either parses in registers or falls back to the LDS walk."""
    mac = b"\x02\0\0\0\0\x01", b"\x02\0\0\0\0\x02"
    a6, b6 = bytes(range(16)), bytes(range(16, 32))
    a4, b4 = b"\x0a\0\0\x01", b"\x0a\0\0\x02"
    out = []
    k = 0
    for chain in ((0,), (60,), (43,), (0, 60), (0, 43), (60, 60), (0, 60, 43), (44,), (51,), (135,)):
        for xlen in (0, 1):
            for l4 in ("udp", "tcp", "tcp_ts"):
                k += 1
                body = (synth.udp(1000 + k, 443) if l4 == "udp" else
                        synth.tcp(1000 + k, 443, 0x12, options=b"\x01\x01\x08\x0a" + b"\0" * 8 if l4 == "tcp_ts" else b""))
                proto = 17 if l4 == "udp" else 6
                ext = b""
                for j in range(len(chain) - 1, -1, -1):
                    nxt = chain[j + 1] if j + 1 < len(chain) else proto
                    ln = xlen if j == 0 else 0
                    ext = bytes([nxt, ln]) + b"\0" * (6 + 8 * ln) + ext
                out.append(synth.eth(*mac, 0x86DD) + synth.ipv6(a6, b6, chain[0], ext + body))
    for ihl in (5, 6):
        for flags in ((False, False, False), (True, False, False), (False, True, False), (False, False, True),
                      (True, True, False), (False, True, True), (True, True, True)):
            for inner in ("v4udp", "v4tcp", "v4tcp_ts", "v4frag", "v6udp", "mpls"):
                k += 1
                if inner.startswith("v4"):
                    l4 = (synth.udp(2000 + k, 53) if inner in ("v4udp", "v4frag") else
                          synth.tcp(2000 + k, 80, 0x02, options=b"\x01\x01\x08\x0a" + b"\0" * 8 if inner == "v4tcp_ts" else b""))
                    pay = synth.ipv4(a4, b4, 6 if "tcp" in inner else 17, l4, mf=1 if inner == "v4frag" else 0,
                                     ident=k)
                    pt = 0x0800
                elif inner == "v6udp":
                    pay, pt = synth.ipv6(a6, b6, 17, synth.udp(2000 + k, 53)), 0x86DD
                else:
                    pay, pt = synth.mpls([16], synth.ipv4(a4, b4, 17, synth.udp(2000 + k, 53))), 0x8847
                out.append(synth.eth(*mac, 0x0800) +
                           synth.ipv4(b"\xc0\0\0\x01", b"\xc0\0\0\x02", 47, synth.gre(pay, pt, *flags), ihl=ihl,
                                      df=1, ident=k))
    for n in (1, 2, 3):  # MPLS stacks (IPv6 under three labels: UDP in the window, TCP past it)
        for inner in ("v4udp", "v4tcp", "v6udp", "v6tcp", "v6tcp_ts"):
            k += 1
            l4 = (synth.udp(3000 + k, 443) if inner.endswith("udp") else
                  synth.tcp(3000 + k, 443, 0x10, options=b"\x01\x01\x08\x0a" + b"\0" * 8 if inner == "v6tcp_ts" else b""))
            proto = 17 if inner.endswith("udp") else 6
            ip = synth.ipv4(a4, b4, proto, l4) if inner.startswith("v4") else synth.ipv6(a6, b6, proto, l4)
            out.append(synth.eth(*mac, 0x8847) + synth.mpls([16 + j for j in range(n)], ip))
    frames = []
    for f in out:
        f = synth.pad(f)
        frames.append((f, len(f), len(f)))
        for cl in range(50, len(f)):
            frames.append((f[:cl], cl, len(f)))
    return frames


@pytest.mark.parametrize("walk", ["", "walk=wide"])
@pytest.mark.parametrize("frag", [True, False])
@pytest.mark.parametrize("agg", ["1", "0"])
def test_wide_walk_ext_and_gre_edges(walk, frag, agg, monkeypatch):
    """IPv6 extension headers and IPv4-in-GRE at the border of k_bin's register walk (untagged
    IPv6 + one to three 8-byte extension headers, IPv4 + GRE + IPv4): flow records
    and parser counters equal the oracle's, truncated copies included.  agg=0: k_bin without
    tile aggregation from the first batch on, whose wide walk reads the 96-byte window."""
    from ipfixprobe_amd import run_capture
    monkeypatch.setenv("IPXG_TILE_AGG", agg)
    arena, desc = synth.to_batch(_edge_frames())
    want, wst = oracle_py.run_capture(arena, desc, 1, cache_exp=20, frag_enable=frag)
    got, gst = run_capture(arena, desc, params=";".join(x for x in (walk, "" if frag else "fe=false") if x))
    if walk:
        assert gst["walked_packets"] > 0
    d = flowcmp.diff(got, want)
    assert not d, d
    for k in ("seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets", "ipv6_packets",
              "tcp_packets", "udp_packets", "vlan_packets", "keyless_packets"):
        assert gst[k] == wst[k], k


@pytest.mark.parametrize("asynchronous", [False, True])
def test_expire_idle_floor(asynchronous, monkeypatch):
    """ipxg_expire after every batch of a stream whose flows go idle at different times: the engine
    keeps a floor under every live record's last-seen time (k_expire's last scan), and an expire at a
    time when no record can be idle yet scans nothing.  Each poll equals the same engine's without
    the floor (IPXG_NO_IDLE_FLOOR: every expire scans) -- with synchronous host batches and with
    asynchronous device batches (the expire then runs guarded behind the batch in flight).  A batch
    whose timestamps go backwards drops the floor.  (The expire times run ahead of the packets, so
    the records are not the no-expire oracle's; the expire semantics themselves are pinned by the
    stream parity tests.)"""
    import torch
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(seed=101, n_flows=500, n_pkts=12000, frag=False).batch()
    desc = desc.copy()
    i = np.arange(len(desc))
    desc["ts_sec"] = 1_700_000_000 + i // 100  # 120 s: flows go idle one after another
    desc["ts_usec"] = (i % 100) * 1000
    desc["ts_sec"][7000:7100] -= 5  # one batch steps back in time
    da = torch.from_numpy(np.ascontiguousarray(arena)).cuda() if asynchronous else None

    def run(no_floor):
        monkeypatch.setenv("IPXG_NO_IDLE_FLOOR", "1" if no_floor else "0")
        polls, keep = [], []
        with Engine() as e:
            for s in range(0, len(desc), 1000):
                part = desc[s:s + 1000]
                now = int(part["ts_sec"].max())
                if asynchronous:
                    dd = torch.from_numpy(np.ascontiguousarray(part).view(np.uint8).reshape(-1)).cuda()
                    keep.append(dd)
                    e.submit(da, dd, device=True, asynchronous=True)
                else:
                    e.submit(arena, part)
                for t in (now - 1, now, now + 3):  # (repeated: the later ones often find nothing idle)
                    e.expire(t)
                polls.append(e.poll())
            e.finish()
            polls.append(e.poll())
        return polls

    with_floor, without = run(False), run(True)
    for k, (a, b) in enumerate(zip(with_floor, without)):
        d = flowcmp.diff(a, b)
        assert not d, "poll %d: %s" % (k, d)
    assert sum(len(g) for g in with_floor[:-1]) > 100  # flows did go idle along the way
