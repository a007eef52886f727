"""Per-phase shader clocks of k_bin_slow on the configs[4] (quic) mix (library built with
-DIPXG_PROBE: IPXG_LIB=ipfixprobe_amd/variants/probe.so python3 tools/probe_slow.py [workload])."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ipfixprobe_amd import Engine
    wl_name = sys.argv[1] if len(sys.argv) > 1 else "quic"
    dev = torch.device("cuda", 0)
    args = types.SimpleNamespace(workload=wl_name, flows=1_000_000, seed=1234, zipf=None, packets=5_000_000,
                                 batches=2, mode="cold", warmup=0, steps=1, shard=None)
    wl = bench.make_workload(args, 0, 1, dev, 0)
    eng = Engine("s=21")
    eng.profile(True)
    for rep in range(3):
        for fr, de in wl.batches:
            eng.submit(fr, de, device=True)
        pc = eng.probe_counters()  # the last batch
        eng.finish()
        eng.clear_exports()
    st = eng.stats()
    tm = eng.timing()
    lanes_pk = int(pc[11])  # packets summed over every wave's lane 0
    print("slow packets share %.3f" % (st["slow_path_packets"] / max(st["parsed_packets"], 1)))
    tot = sum(int(x) for x in pc[8:11])
    for k, nme in ((8, "loads (issue->arrival)"), (9, "stage+parse+rank"), (10, "aggregate+emit")):
        print("%-24s %14.0f cycles summed over waves  %5.1f %%  %8.0f cycles per packet per wave"
              % (nme, int(pc[k]), 100.0 * int(pc[k]) / max(tot, 1), int(pc[k]) / max(lanes_pk, 1)))
    print("k_bin_slow avg %.4f ms, k_bin avg %.4f ms" % (tm["ingest_slow_ms"] / max(tm["ingest_launches"], 1),
                                                          tm["ingest_ms"] / max(tm["ingest_launches"], 1)))
    names = ["tile start", "packet loop", "emit", "slow flush"]
    for k, nme in enumerate(names):
        print("k_bin %-12s %14.0f cycles summed over waves" % (nme, int(pc[k])))
    for k, nme in ((4, "prefix+zero"), (5, "aggregate"), (6, "merge+list")):
        print("k_reduce %-12s %14.0f cycles summed over workgroups" % (nme, int(pc[k])))
    print("k_reduce avg %.4f ms, k_fin_list avg %.4f ms" % (tm["reduce_ms"] / max(tm["reduce_launches"], 1),
                                                        tm["fin_ms"] / max(tm["reduce_launches"], 1)))


if __name__ == "__main__":
    main()
