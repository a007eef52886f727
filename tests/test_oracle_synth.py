"""CPU: the oracle on the synthetic corpora (conservation laws; the corpora really reach
the code paths the GPU tests compare)."""
import numpy as np

import oracle_py
import synth


def test_fuzz_corpus_reaches_every_encapsulation():
    arena, desc = synth.to_batch(synth.fuzz_corpus(20000, seed=3))
    p, beyond = oracle_py.parse_batch(arena, desc)
    v = p[p["valid"] == 1]
    et = set(v["ethertype"].tolist())
    assert {0x0800, 0x86DD, 0x8847, 0x8848, 0x8864} <= et
    assert (v["vlan_id"] != 0).sum() > 100
    assert ((v["frag_off"] != 0) | (v["more_fragments"] != 0)).sum() > 100
    assert (v["tcp_options"] != 0).sum() > 100
    assert beyond.sum() < 500


def test_stream_conserves_packets_and_splits():
    arena, desc = synth.flow_stream(seed=8, n_flows=30, n_pkts=6000, long_gap_share=0.0005).batch()
    recs, st = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    assert int(recs["src_packets"].sum() + recs["dst_packets"].sum()) == st["parsed_packets"] - st["keyless_packets"]
    assert st["end_active"] > 0 and st["end_inactive"] > 0 and st["end_eof"] > 0
    assert st["fragments_filled"] > 0 and st["end_no_res"] == 0
    assert np.all(recs["time_last_sec"] >= recs["time_first_sec"])


PKT_BUCKETS = ["flows_1_packet", "flows_2_5_packets", "flows_6_10_packets", "flows_11_20_packets",
               "flows_21_50_packets", "flows_51_plus_packets"]


def record_buckets(recs):
    """update_flow_record_stats (cache.cpp:601-616) over exported records."""
    n = recs["src_packets"].astype(np.int64) + recs["dst_packets"].astype(np.int64)
    edges = [(1, 1), (2, 5), (6, 10), (11, 20), (21, 50)]
    out = [int(((n >= lo) & (n <= hi)).sum()) for lo, hi in edges]
    return out + [len(n) - sum(out)]


def test_flow_record_stats_buckets():
    """FlowRecordStats: every exported record counted once, by its packet total."""
    arena, desc = synth.flow_stream(seed=8, n_flows=30, n_pkts=6000, long_gap_share=0.0005).batch()
    recs, st = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got = [st[k] for k in PKT_BUCKETS]
    assert got == record_buckets(recs)
    assert sum(got) == st["total_exported"] == len(recs)
    assert got[0] > 0 and got[-1] > 0
