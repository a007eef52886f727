"""The timeline of the last steps of a bench.py run from a rocprofv3 kernel trace
(run_kernel_trace.csv): each step's kernels with their durations and the idle gaps before them,
to see where a step's wall time goes besides the kernels (launch gaps, host round trips).

  python3 tools/trace_gaps.py <run_kernel_trace.csv> [first_kernel_of_step] [steps]"""
import csv
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("ipxg::", "")[:34]


def main(path, first="fillBuffer", steps=3):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(starts) < steps + 1:
        print("not enough steps")
        return
    for s0, s1 in zip(starts[-steps - 1:-1], starts[-steps:]):
        t0 = int(rows[s0]["Start_Timestamp"])
        prev_end = None
        busy = 0
        print("step at %d (%.1f us to the next)" % (s0, (int(rows[s1]["Start_Timestamp"]) - t0) / 1e3))
        for r in rows[s0:s1]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (st - prev_end) / 1e3 if prev_end else 0.0
            busy += en - st
            print("  +%8.1f us  gap %6.1f  %-36s %8.1f us" % ((st - t0) / 1e3, gap, short(r["Kernel_Name"]),
                                                            (en - st) / 1e3))
            prev_end = en
        print("  kernels %.1f us of %.1f" % (busy / 1e3, (int(rows[s1]["Start_Timestamp"]) - t0) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fillBuffer", int(sys.argv[3]) if len(sys.argv) > 3 else 3)
