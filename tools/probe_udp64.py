"""Per-phase shader clocks of k_bin and k_reduce on the configs[1] batch (10M 64 B UDP packets,
100k flows; the control block is cleared per batch, so the counters are the last batch's; library
built with -DIPXG_PROBE:
  tools/variants.sh probe "-DIPXG_PROBE"
  IPXG_TUNING=1 IPXG_LIB=ipfixprobe_amd/variants/probe.so python3 tools/probe_udp64.py)."""
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
    fr, de = bench.build_batch(flows, 10_000_000, 1234, dev)
    torch.cuda.synchronize()
    eng = Engine(bench.engine_params(100_000))
    for _ in range(3):  # warm: partition sizing from the previous batch
        eng.submit(fr, de, device=True)
        eng.finish()
        eng.clear_exports()
    eng.profile(True)
    reps = 5
    for _ in range(reps):
        eng.submit(fr, de, device=True)
        eng.finish()
        eng.clear_exports()
    pc = [int(x) for x in eng.probe_counters()]
    tm = eng.timing()
    P, grid = 256, 512
    for k, nme in ((0, "bin: tile start"), (1, "bin: packet loop"), (2, "bin: emit"), (3, "bin: slow flush")):
        print("%-18s %12.0f cycles/workgroup-launch" % (nme, pc[k] / grid / 4))
    for k, nme in ((4, "red: prefix+zero"), (5, "red: aggregate"), (6, "red: merge+list")):
        print("%-18s %12.0f cycles/workgroup" % (nme, pc[k] / P))
    fin_blocks = (100_000 + 255) // 256  # (k_fin_list: one lane per listed flow)
    for k, nme in ((12, "fin: image"), (13, "fin: finalize"), (14, "fin: export"), (15, "fin: counts")):
        print("%-18s %12.0f cycles/workgroup (thread 0)" % (nme, pc[k] / fin_blocks))
    print("k_bin avg %.4f ms, k_reduce avg %.4f ms, k_fin_list avg %.4f ms" % (
        tm["ingest_ms"] / max(tm["ingest_launches"], 1), tm["reduce_ms"] / max(tm["reduce_launches"], 1),
        tm["fin_ms"] / max(tm["reduce_launches"], 1)))
    eng.close()


if __name__ == "__main__":
    main()
