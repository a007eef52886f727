"""Summarise bench.py JSON lines: value, ms per step, k_bin average, stage times, verify.
Usage: python tools/bline.py <file.json> ..."""
import json
import sys

for f in sys.argv[1:]:
    try:
        lines = [x for x in open(f).read().splitlines() if x.startswith("{")]
        d = json.loads(lines[-1])
    except (OSError, IndexError, ValueError) as ex:
        print("%s: no line (%s)" % (f, type(ex).__name__))
        continue
    r = d["roofline"]
    print("%s: %.1f Mpkt/s  %.4f ms/step  %s %.4f ms (frac %.3f)  step_frac %.3f  stages %s  verify %s" % (
        f, d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], r["step_frac"],
        d.get("stage_ms_per_step"), d.get("verify")))
