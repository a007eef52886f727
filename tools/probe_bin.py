"""Per-phase shader clocks of k_bin on the bench batch (library built with -DIPXG_PROBE:
IPXG_TUNING=1 IPXG_LIB=ipfixprobe_amd/variants/probe.so python3 tools/probe_bin.py)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ipfixprobe_amd import Engine
    dev = torch.device("cuda", 0)
    flows = bench.gen_flows(100_000, 0, 1, 1234)
    frames, desc = bench.build_batch(flows, 10_000_000, 1234, dev)
    eng = Engine("s=%d" % int(math.ceil(math.log2(2 * 100_000))))
    eng.profile(True)
    for _ in range(3):
        eng.submit(frames, desc, device=True)
        eng.finish()
        eng.clear_exports()
    pc = eng.probe_counters()
    tm = eng.timing()
    waves = 2048 * 4
    names = ["tile start", "packet loop", "emit", "slow flush"]
    tot = sum(int(x) for x in pc[:4])
    for k, nme in enumerate(names):
        print("%-12s %12.0f cycles/wave  %5.1f %%" % (nme, int(pc[k]) / waves, 100.0 * int(pc[k]) / max(tot, 1)))
    print("k_bin avg %.4f ms" % (tm["ingest_ms"] / tm["ingest_launches"]))
    blocks = 256  # k_reduce workgroups (partitions) of the bench batch
    for k, nme in ((4, "red: prefix+zero"), (5, "red: aggregate"), (6, "red: merge+list")):
        print("%-18s %10.0f cycles/workgroup" % (nme, int(pc[k]) / blocks))
    print("k_reduce avg %.4f ms" % (tm["reduce_ms"] / max(tm["reduce_launches"], 1)))
    waves = blocks * 16
    print("red aggregate: wait for records %10.0f cycles/wave, fold %10.0f cycles/wave"
          % (int(pc[12]) / waves, int(pc[13]) / waves))


if __name__ == "__main__":
    main()
