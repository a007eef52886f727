"""Debug: per-batch stat deltas of the engine on the imix mix at several batch sizes."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools", "synth"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
import synthgen
from ipfixprobe_amd import Engine

mix = synthgen.Mix("imix", 1_000_000, seed=1234, zipf=1.1)
gen = synthgen.Generator(mix, torch.device("cuda", 0), seed=1234)
for n in (10_000_000,):
    with Engine("s=21") as e:
        prev = e.stats()
        for k in range(10):
            fr, de = gen.batch(k * n, n)
            torch.cuda.synchronize()
            e.submit(fr, de, device=True)
            st = e.stats()
            d = {key: st[key] - prev[key] for key in ("seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets",
                                                    "ipv6_packets", "tcp_packets", "udp_packets", "slow_path_packets",
                                                    "spilled_packets", "keyless_packets")}
            print(n, k, d, "arena", fr.numel(), flush=True)
            prev = st
            del fr, de
            f, _, _, _, _ = synthgen.host_plan(gen, k * n, n)
        e.finish()
        recs = e.poll()
        print("records", len(recs), "pkts", int(recs["src_packets"].sum() + recs["dst_packets"].sum()), e.stats())
