"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_<TAG>/*/run_counter_collection.csv) into
{kernel: {counter: mean value per dispatch}} -- the steady-state dispatches only (the first
dispatch of each kernel is the warm-up, sized before the engine knew the flow count).

  python3 tools/pmc_summary.py <pmc dir> [<out.json> [<bench line of one pass>]]

With a bench line (the JSON bench.py printed under the profiler) the summary gets a "_meta" entry:
the workload's name, its packets per launch (per batch) and its descriptor offsets -- bench.py's
pmc_traffic takes a summary's traffic only for a run of that same shape."""
import collections
import csv
import glob
import json
import os
import sys


def summarise(pmc_dir):
    out = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "*", "run_counter_collection.csv"))):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "ipxg" not in k:
                continue
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            steady = v[1:] if len(v) > 1 else v
            out[k][c] = sum(steady) / len(steady)
            out[k]["calls"] = max(out[k].get("calls", 0), len(v))
    return dict(out)


def bench_meta(line_file):
    with open(line_file) as f:
        lines = [x for x in f.read().splitlines() if x.startswith("{")]
    cfg = json.loads(lines[-1])["config"]
    return {"workload": cfg["name"], "offsets": cfg.get("offsets", "bytes"),
            "packets_per_launch": cfg["packets_per_gpu_per_step"] // max(cfg["batches_per_step"], 1),
            "bench_line": os.path.basename(line_file)}


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    if len(sys.argv) > 3:
        s["_meta"] = bench_meta(sys.argv[3])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(s, f, indent=1, sort_keys=True)
    for k, v in sorted(s.items()):
        print(k, v if k == "_meta" else {c: round(x) for c, x in sorted(v.items())})
