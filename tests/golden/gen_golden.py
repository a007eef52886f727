"""Regenerates tests/golden/xxh64_vectors.json.

Hashes come from python xxhash 3.8.1 (an implementation independent of both the oracle and
the device code) and, when the reference tree is present, are cross-checked against the
reference's own xxhash.c compiled into oracle/_ref/libxxhash_ref.so.  Keys cover the two
flow-key sizes (16 B IPv4, 40 B IPv6, cache.hpp:29-46), the 40 B fragmentation key
(fragmentationKeyData.hpp:49-82) and assorted lengths across the XXH64 code paths.
"""
import ctypes
import json
import os

import numpy as np
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    rng = np.random.default_rng(20261015)
    ref = None
    p = os.path.join(ROOT, "oracle", "_ref", "libxxhash_ref.so")
    if os.path.exists(p):
        ref = ctypes.CDLL(p)
        ref.XXH64.restype = ctypes.c_uint64
        ref.XXH64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    vecs = []
    lengths = [16] * 24 + [40] * 24 + list(range(0, 72, 3)) + [96, 200]
    for n in lengths:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0,) if n in (16, 40) else (0, 7):
            h = xxhash.xxh64_intdigest(b, seed)
            if ref is not None:
                buf = ctypes.create_string_buffer(b, max(n, 1))
                assert ref.XXH64(buf, n, seed) == h
            vecs.append({"key": b.hex(), "seed": seed, "hash": "%016x" % h})
    with open(os.path.join(HERE, "xxh64_vectors.json"), "w") as f:
        json.dump(vecs, f, indent=0)
    print("wrote %d vectors (reference xxhash.c cross-check: %s)" % (len(vecs), ref is not None))


if __name__ == "__main__":
    main()
