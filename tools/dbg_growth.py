"""Debug helper: the table-growth scenario of tests/test_gpu_semantics.py with stats printed."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
import synth, oracle_py, flowcmp
from ipfixprobe_amd import run_capture

rng = np.random.default_rng(5)
frames = []
for i in range(200_000):
    f = synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) +
                  synth.ipv4(synth.ip4(0x0A000000 + i), synth.ip4(0xC0A80001), 17,
                             synth.udp(int(rng.integers(1024, 65536)), 53)))
    frames.append((f, len(f), len(f)))
frames += frames[:50_000]
arena, desc = synth.to_batch(frames)
want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=22)
for params in sys.argv[1:] or ["s=16", "s=22"]:
    got, st = run_capture(arena, desc, params=params)
    print(params, {k: v for k, v in st.items() if v})
    d = flowcmp.diff(got, want)
    print("  diff:", d[:300] if d else "none")
