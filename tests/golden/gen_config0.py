"""Writes the BASELINE.json configs[0] fixture: tests/golden/config0_udp64.pcap, a classic
(microsecond) pcap of 1000 Ethernet/IPv4/UDP frames of 64 bytes (tot_len 50) over 100 biflows
(each packet picks a flow and a direction at random, 1 ms apart), and
tests/golden/config0_udp64.csv, the oracle's flow records for it in the reference functional
tests' basic-column text form (the oracle is pinned by the reference's own goldens,
tests/test_oracle_golden.py).  Deterministic (seed 1234)."""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def frames(n=1000, flows=100, seed=1234):
    rng = np.random.default_rng(seed)
    sip = (10 << 24) + rng.integers(1, 1 << 24, flows)
    dip = (192 << 24) + (168 << 16) + rng.integers(1, 1 << 16, flows)
    sp = rng.integers(1024, 65536, flows)
    dp = rng.integers(1, 1024, flows)
    out = []
    t0 = 1_700_000_000 * 1_000_000
    for i in range(n):
        f = int(rng.integers(0, flows))
        rev = bool(rng.integers(0, 2))
        a, b = (dip[f], sip[f]) if rev else (sip[f], dip[f])
        pa, pb = (dp[f], sp[f]) if rev else (sp[f], dp[f])
        cm = bytes([2, 0, 0, 0, 0, f])
        sm = bytes([4, 0, 0, 0, 0, f])
        eth = (cm + sm if rev else sm + cm) + b"\x08\x00"
        udp = struct.pack(">HHHH", int(pa), int(pb), 30, 0) + bytes(22)
        ip = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 50, i & 0xFFFF, 0x4000, 64, 17, 0, struct.pack(">I", int(a)),
                         struct.pack(">I", int(b)))
        fr = eth + ip + udp
        assert len(fr) == 64
        t = t0 + i * 1000
        out.append((t // 1_000_000, t % 1_000_000, fr))
    return out


def write_pcap(path, pk):
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for s, us, fr in pk:
            f.write(struct.pack("<IIII", s, us, len(fr), len(fr)) + fr)


def main():
    import oracle_py  # noqa: E402  (tests/ on the path)
    import pcaputil
    pk = frames()
    pcap = os.path.join(HERE, "config0_udp64.pcap")
    write_pcap(pcap, pk)
    dl, rd = pcaputil.read_capture(pcap)
    arena, desc = pcaputil.to_batch(rd)
    recs, st = oracle_py.run_capture(arena, desc, dl, cache_exp=17)
    assert st["end_no_res"] == 0 and len(recs) == 100
    with open(os.path.join(HERE, "config0_udp64.csv"), "w") as f:
        for line in sorted(pcaputil.format_records(recs)):
            f.write(line + "\n")
    print("wrote %s (%d packets) and %d flow records" % (pcap, len(pk), len(recs)))


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(os.path.dirname(HERE)))
    main()
