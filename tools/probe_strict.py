"""Scheduler counters of the strict replay (k_strict_walk) on the bench's strict workload
(udp64 through the reference's table, s=17) -- library built with -DIPXG_PROBE:
IPXG_TUNING=1 IPXG_LIB=ipfixprobe_amd/variants/probe.so python3 tools/probe_strict.py [S]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main(s_exp):
    import torch
    import bench
    from ipfixprobe_amd import Engine
    dev = torch.device("cuda", 0)
    flows = bench.gen_flows(100_000, 0, 1, 1234)
    fr, de = bench.build_batch(flows, 10_000_000, 1234, dev)
    torch.cuda.synchronize()
    eng = Engine("strict=true;s=%d" % s_exp)
    t0 = time.perf_counter()
    eng.submit(fr, de, device=True)
    dt = time.perf_counter() - t0
    pc = [int(x) for x in eng.probe_counters()]
    n = int(de.numel()) // 16
    wgs = int(os.environ.get("IPXG_STRICT_WGS", "0") or 0)
    waves = 12 * max(1, wgs)  # (several workgroups: an upper bound -- those of one XCD take part)
    rounds, body, lanes, backlog, tbody, tall, sweeps, unfilled = pc[:8]
    print("strict s=%d: %d packets, submit %.1f ms (%.1f Mpkt/s)" % (s_exp, n, dt * 1e3, n / dt / 1e6))
    print("per wave: rounds %.0f, rounds with packets %.0f; lanes per such round %.1f" %
          (rounds / waves, body / waves, lanes / max(body, 1)))
    print("queue backlog per such round %.1f; due-but-unfilled lane rounds per wave %.0f" %
          (backlog / max(body, 1), unfilled / waves))
    print("clocks per wave: body %.0f of %.0f (%.0f%%); per body round %.0f" %
          (tbody / waves, tall / waves, 100.0 * tbody / max(tall, 1), tbody / max(body, 1)))
    print("packets with a sweep event: %d (%.2f%%)" % (sweeps, 100.0 * sweeps / n))
    ph = pc[8:12]
    print("body phases per round (clocks): fields %.0f, strict_packet %.0f, store drain %.0f, hand-off %.0f" %
          tuple(x / max(body, 1) for x in ph))
    eng.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 17)
