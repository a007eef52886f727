"""Summarise rocprofv3 PMC passes (gpurun_out/pmc_<TAG>/*/run_counter_collection.csv) into
{kernel: {counter: mean value per dispatch}} -- the steady-state dispatches only (the first
dispatch of each kernel is the warm-up, sized before the engine knew the flow count)."""
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


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(s, f, indent=1, sort_keys=True)
    for k, v in sorted(s.items()):
        print(k, {c: round(x) for c, x in sorted(v.items())})
