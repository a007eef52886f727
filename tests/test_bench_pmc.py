"""bench.py's roofline.traffic comes only from a PMC summary of a run of the same shape (VERDICT r5
item 4): tools/pmc_summary.py writes the profiled run's workload, packets per launch and offset form
into the summary's "_meta"; pmc_traffic takes a summary only when they match the bench run, and the
kernel's most-dispatched template variant in it (the steady state), and names that entry."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_pmc_traffic_matches_the_run_shape():
    import bench
    got = bench.pmc_traffic("k_bin", "udp64", 10_000_000, "bytes")
    assert got is not None
    path, nbytes, variant, calls = got
    with open(path) as f:
        js = json.load(f)
    meta = js["_meta"]
    assert (meta["workload"], meta["packets_per_launch"], meta["offsets"]) == ("udp64", 10_000_000, "bytes")
    v = js[variant]
    assert v["calls"] == calls and calls == max(e["calls"] for k, e in js.items()
                                                if k != "_meta" and "k_bin<" in k)
    rd = 128 * v["TCC_EA0_RDREQ_128B_sum"] + 64 * v["TCC_EA0_RDREQ_64B_sum"] + 32 * v["TCC_EA0_RDREQ_32B_sum"]
    assert abs(nbytes - (rd + 1024 * v["WRITE_SIZE"])) < 1.0
    # another batch size or offset form: no summary of that shape, no traffic
    assert bench.pmc_traffic("k_bin", "udp64", 5_000_000, "bytes") is None
    assert bench.pmc_traffic("k_bin", "quic", 5_000_000, "bytes") is None
    q = bench.pmc_traffic("k_bin", "quic", 10_000_000, "units")
    assert q is not None and "true>" in q[2]  # (the G64 variant: unit offsets)


def test_pmc_summary_meta_from_a_bench_line(tmp_path):
    import pmc_summary
    line = {"metric": "m", "value": 1.0, "config": {"name": "imix", "offsets": "units",
                                                     "packets_per_gpu_per_step": 100_000_005, "batches_per_step": 7}}
    p = tmp_path / "pmc_imix_FETCH_SIZE.json"
    p.write_text("noise on stdout\n" + json.dumps(line) + "\n")
    assert pmc_summary.bench_meta(str(p)) == {"workload": "imix", "offsets": "units", "packets_per_launch": 14_285_715,
                                              "bench_line": "pmc_imix_FETCH_SIZE.json"}
