"""The process-plugin step of configs[2] / configs[4] with the reference's OWN plugins
(oracle/_ref/libref_plugins.so: dns, http, tls, quic compiled unmodified behind the adapter)
against the bench's native stand-ins, same workload, same engine: the host walk's ms per step
with the real plugins -- their enrichment included (TLS/QUIC ClientHello parsing, QUIC's
AES-GCM Initial decryption) -- which bench.py cannot time (it may load nothing under oracle/).

  python3 tools/real_plugins_walk.py imix|quic [steps] [stand-in|reference]   -> one JSON line per plugin set

Test/measurement tooling only (loads oracle/_ref)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))


def main(name, steps, kinds=("stand-in", "reference")):
    import torch
    import bench
    import synthgen
    import test_ref_plugins
    from ipfixprobe_amd import Engine
    from ipfixprobe_amd.engine import StdPlugin
    dev = torch.device("cuda", 0)
    # the bench's default step shapes since ABI 8 (16-byte unit offsets: imix 7 x 14.3M, quic 2 x 10M);
    # IPXG_RPW_BYTES=1: the byte-offset shapes of round 4 (imix 10 x 10M, quic 4 x 5M)
    units = not os.environ.get("IPXG_RPW_BYTES")
    if units:
        n, nb = (14_285_715, 7) if name == "imix" else (10_000_000, 2)
    else:
        n, nb = (10_000_000, 10) if name == "imix" else (5_000_000, 4)
    names = ["dns", "http", "tls"] if name == "imix" else ["quic"]
    mix = synthgen.Mix(name, 1_000_000, seed=1234, zipf=1.1 if name == "imix" else None)
    gen = synthgen.Generator(mix, dev, seed=1234)
    batches = [gen.batch(k * n, n, offset16=units) for k in range(nb)]
    torch.cuda.synchronize()
    for kind in kinds:
        pls = [StdPlugin(p) if kind == "stand-in" else test_ref_plugins.RefPlugin(p) for p in names]
        with Engine(bench.engine_params(1_000_000)) as e:
            for p in pls:
                e.add_plugin(p.struct)

            def step():
                for fr, de in batches:
                    e.submit(fr, de, device=True, asynchronous=True, wait_producer=False, offset16=units)
                e.finish()
                e.clear_exports()  # (the real plugins' exported Flow objects are left to the process)

            step()  # warm-up
            e.profile(True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            tm = e.timing()
        print(json.dumps({"workload": name, "plugins": names, "kind": kind, "packets_per_step": n * nb,
                          "batches_per_step": nb, "offsets": "units" if units else "bytes",
                          "ms_per_step": round(dt * 1e3, 2), "Mpkts_per_s": round(n * nb / dt / 1e6, 1),
                          "host_walk_ms_per_step": round(tm["plugin_ms"] / steps, 2),
                          "walked_flows_per_step": round(tm["plugin_flows"] / steps),
                          "walked_packets_per_step": round(tm["plugin_packets"] / steps)}), flush=True)
        del pls


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "imix", int(sys.argv[2]) if len(sys.argv) > 2 else 2,
         tuple(sys.argv[3:]) or ("stand-in", "reference"))
