"""Per-phase shader clocks of k_reduce (and k_bin) on a batch of a configs[2] / configs[4] mix
(library built with -DIPXG_PROBE: IPXG_TUNING=1 IPXG_LIB=ipfixprobe_amd/variants/probe.so
python3 tools/probe_reduce.py quic|imix)."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main(name):
    import torch
    import synthgen
    import bench
    from ipfixprobe_amd import Engine
    dev = torch.device("cuda", 0)
    n = 5_000_000 if name == "quic" else 10_000_000
    mix = synthgen.Mix(name, 1_000_000, seed=1234, zipf=1.1 if name == "imix" else None)
    gen = synthgen.Generator(mix, dev, seed=1234)
    batches = [gen.batch(k * n, n) for k in range(4)]
    torch.cuda.synchronize()
    eng = Engine(bench.engine_params(1_000_000))
    eng.profile(True)
    for fr, de in batches:
        eng.submit(fr, de, device=True)
    pc = eng.probe_counters()
    tm = eng.timing()
    st = eng.stats()
    flows = st["flows_in_cache"]
    bits = 0
    while (1200 << bits) < flows and bits < 11:
        bits += 1
    P = 1 << bits
    print("%s: %d packets per batch, %d flows in cache, ~%d partitions (k_reduce workgroups)" % (name, n, flows, P))
    for k, nme in ((4, "red: prefix+zero"), (5, "red: aggregate"), (6, "red: merge+list")):
        print("%-18s %12.0f cycles/workgroup" % (nme, int(pc[k]) / P))
    print("k_reduce avg %.4f ms, k_fin_list avg %.4f ms" % (tm["reduce_ms"] / max(tm["reduce_launches"], 1),
                                                          tm["fin_ms"] / max(tm["reduce_launches"], 1)))
    print("red aggregate: wait for records %12.0f, fold %12.0f cycles/wave" % (int(pc[12]) / (P * 16), int(pc[13]) / (P * 16)))
    eng.close()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "quic")
