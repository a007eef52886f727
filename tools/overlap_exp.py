"""Timing experiment (round 6): does the GPU overlap one batch's flow-state kernels (k_reduce,
k_fin_list) with the next batch's k_bin when they sit on different HIP streams?

Runs the udp64 step (submit + finish, cold table) K times on one engine, then K times
alternating between two independent engines (each with its own stream and buffers), and prints
ms per step for each.  The second form is what a pipelined engine could reach at best.
Usage: python tools/overlap_exp.py [steps] [engine counts, e.g. 1,2,1,2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import torch
    from ipfixprobe_amd import Engine
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    args = argparse.Namespace(workload="udp64", shard=None, flows=100_000, seed=1234, mode="cold",
                              packets=10_000_000, offset16=False)
    dev = torch.device("cuda", 0)
    wl = bench.make_workload(args, 0, 1, dev, 0)
    fr, de = wl.batches[0]
    torch.cuda.synchronize()
    engs = [Engine(bench.engine_params(wl.flows), device_id=0) for _ in range(2)]

    def step(e):
        e.submit(fr, de, device=True, asynchronous=True, wait_producer=False)
        e.finish()
        e.clear_exports()

    modes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (1, 2, 1, 2)
    for n_eng in modes:
        for k in range(4):
            step(engs[k % n_eng])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            step(engs[k % n_eng])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        print("engines %d: %.4f ms/step  %.1f Mpkt/s" % (n_eng, dt * 1e3, 10e6 / dt / 1e6), flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
