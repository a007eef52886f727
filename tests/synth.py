"""Synthetic packet crafting for parity tests (test infrastructure).

Builders for every header the reference parser walks (parser.cpp): Ethernet with 802.1Q /
802.1ad stacks, TRILL, MPLS (+EoMPLS), PPPoE, GRE (C/K/S options), IPv4 (options,
fragments), IPv6 (+hop-by-hop/dest/routing/fragment/AH/MH extension headers), TCP (options),
UDP, ICMP, Linux SLL/SLL2 and raw IP link types.  `fuzz_corpus` mixes them with random
truncation and byte corruption; `flow_stream` builds monotonic multi-flow streams that
exercise the cache's split rules (cache.cpp:431-472) and the fragmentation cache.
"""
import struct

import numpy as np


def mac(i):
    return bytes([0x02, 0, (i >> 24) & 0xFF, (i >> 16) & 0xFF, (i >> 8) & 0xFF, i & 0xFF])


def eth(dst, src, ethertype, vlans=()):
    b = dst + src
    for tpid, tci in vlans:
        b += struct.pack(">HH", tpid, tci)
    return b + struct.pack(">H", ethertype)


def ipv4(src, dst, proto, payload, ihl=5, frag_off=0, mf=0, df=0, ident=0, ttl=64, tos=0,
         tot_len=None, options=b""):
    opts = options.ljust((ihl - 5) * 4, b"\0")[: max(0, (ihl - 5) * 4)]
    tl = tot_len if tot_len is not None else 20 + len(opts) + len(payload)
    fo = (frag_off & 0x1FFF) | (0x2000 if mf else 0) | (0x4000 if df else 0)
    hdr = struct.pack(">BBHHHBBH4s4s", 0x40 | (ihl & 0xF), tos, tl & 0xFFFF, ident & 0xFFFF, fo,
                      ttl, proto, 0, src, dst)
    return hdr + opts + payload


def ipv6(src, dst, nxt, payload, hlim=64, tc=0, flow=0, plen=None):
    vtf = (6 << 28) | ((tc & 0xFF) << 20) | (flow & 0xFFFFF)
    pl = plen if plen is not None else len(payload)
    return struct.pack(">IHBB", vtf, pl & 0xFFFF, nxt, hlim) + src + dst + payload


def ext_hdr(nxt, body_len8=0, fill=0):
    """Hop-by-hop / dest-options / routing / MH style: (len + 1) * 8 bytes."""
    n = (body_len8 + 1) * 8
    return bytes([nxt, body_len8]) + bytes([fill]) * (n - 2)


def ah_hdr(nxt, length):
    """AH: the reference skips (len << 2) - 2 bytes (parser.cpp:382)."""
    n = max(2, (length << 2) - 2)
    return bytes([nxt, length]) + b"\0" * (n - 2)


def frag6_hdr(nxt, off=0, m=0, ident=0):
    return struct.pack(">BBHI", nxt, 0, ((off & 0x1FFF) << 3) | (1 if m else 0), ident)


def tcp(sport, dport, flags, options=b"", doff=None, seq=1, ack=0, win=1024, payload=b""):
    d = doff if doff is not None else 5 + (len(options) + 3) // 4
    opts = options.ljust(max(0, (d - 5) * 4), b"\0")[: max(0, (d - 5) * 4)]
    return struct.pack(">HHIIBBHHH", sport, dport, seq, ack, (d & 0xF) << 4, flags, win, 0, 0) + opts + payload


def udp(sport, dport, payload=b""):
    return struct.pack(">HHHH", sport, dport, 8 + len(payload), 0) + payload


def icmp(t=8, c=0):
    return struct.pack(">BBHI", t, c, 0, 0) + b"\0" * 8


def mpls(labels, inner):
    out = b""
    for k, lab in enumerate(labels):
        bos = 1 if k == len(labels) - 1 else 0
        out += struct.pack(">I", ((lab & 0xFFFFF) << 12) | (bos << 8) | 64)
    return out + inner


def pppoe(inner, proto=0x0021, code=0, sid=1):
    return struct.pack(">BBHH", 0x11, code, sid, len(inner) + 2) + struct.pack(">H", proto) + inner


def gre(inner, ptype, c=False, k=False, s=False):
    flags = (0x8000 if c else 0) | (0x2000 if k else 0) | (0x1000 if s else 0)
    opt = b"\0\0\0\0" * (int(c) + int(k) + int(s))
    return struct.pack(">HH", flags, ptype) + opt + inner


def trill(inner_eth, op_len=0):
    b0 = (op_len >> 2) & 0x7  # op_len1 in bits 0-2 of byte 0 (LE bitfield, headers.hpp:232)
    b1 = (op_len & 0x3) << 6
    return bytes([b0, b1]) + b"\0\0\0\0" + b"\0" * (op_len * 4) + inner_eth


def sll(inner, proto, hatype=1, addr=b"\x02\x00\x00\x00\x00\x01"):
    return struct.pack(">HHH", 0, hatype, 6) + addr.ljust(8, b"\0") + struct.pack(">H", proto) + inner


def sll2(inner, proto, hatype=1, addr=b"\x02\x00\x00\x00\x00\x01"):
    return struct.pack(">HHIHBB", proto, 0, 3, hatype, 0, 6) + addr.ljust(8, b"\0") + inner


def ip4(i):
    return struct.pack(">I", i & 0xFFFFFFFF)


def ip6(i):
    return b"\x20\x01\x0d\xb8" + struct.pack(">IQ", 0, i & 0xFFFFFFFFFFFFFFFF)


def pad(frame, n=60):
    return frame + b"\0" * max(0, n - len(frame))


# ---- parser fuzz corpus -------------------------------------------------------------------
def _l4(rng, proto):
    if proto == 6:
        kinds = [b"\x02\x04\x05\xb4", b"\x01", b"\x03\x03\x07", b"\x04\x02", b"\x08\x0a" + b"\x11" * 8,
                 b"\x00", b"\x1e\x06\x01\x02\x03\x04", bytes([rng.integers(0, 256), 0])]
        opts = b"".join(kinds[int(rng.integers(0, len(kinds)))] for _ in range(int(rng.integers(0, 4))))
        doff = None if rng.random() < 0.85 else int(rng.integers(0, 16))
        return tcp(int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), int(rng.integers(0, 256)),
                   opts[:40], doff=doff, payload=b"x" * int(rng.integers(0, 20)))
    if proto == 17:
        return udp(int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), b"y" * int(rng.integers(0, 20)))
    if proto == 1:
        return icmp()
    return b"z" * int(rng.integers(0, 30))


def _l3(rng, depth=0):
    """Returns (ethertype, bytes) of a random L3 chain."""
    r = rng.random()
    proto = [6, 17, 1, 58, 132, 47][int(rng.integers(0, 6))] if depth < 2 else [6, 17][int(rng.integers(0, 2))]
    if r < 0.45 or depth >= 2:
        if proto == 47 and depth < 2:
            et, inner = _l3(rng, depth + 1)
            pt = {0x0800: 0x0800, 0x86DD: 0x86DD, 0x8847: 0x8847, 0x8864: 0x8864}.get(et, 0x6558)
            if rng.random() < 0.1:
                pt = 0x1234
            g = gre(inner, pt, c=rng.random() < 0.3, k=rng.random() < 0.3, s=rng.random() < 0.3)
            return 0x0800, ipv4(ip4(int(rng.integers(0, 1 << 32))), ip4(int(rng.integers(0, 1 << 32))), 47, g)
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(0, 16))
        fo = 0 if rng.random() < 0.85 else int(rng.integers(0, 8))
        mf = int(rng.random() < 0.1)
        return 0x0800, ipv4(ip4(int(rng.integers(0, 1 << 32))), ip4(int(rng.integers(0, 1 << 32))), proto,
                            _l4(rng, proto), ihl=ihl, frag_off=fo, mf=mf, ident=int(rng.integers(0, 65536)))
    if r < 0.75:
        chain = []
        for _ in range(int(rng.integers(0, 4))):
            chain.append([0, 60, 43, 44, 51, 135][int(rng.integers(0, 6))])
        body = _l4(rng, proto if proto != 47 else 6)
        nxt = proto if proto != 47 else 6
        for t in reversed(chain):
            if t == 44:
                body = frag6_hdr(nxt, off=int(rng.integers(0, 3)), m=int(rng.random() < 0.5),
                                 ident=int(rng.integers(0, 1 << 32))) + body
            elif t == 51:
                body = ah_hdr(nxt, int(rng.integers(0, 6))) + body
            elif t == 135:
                body = ext_hdr(59 if rng.random() < 0.5 else nxt, int(rng.integers(0, 2))) + body
            else:
                body = ext_hdr(nxt, int(rng.integers(0, 3))) + body
            nxt = t
        return 0x86DD, ipv6(ip6(int(rng.integers(0, 1 << 62))), ip6(int(rng.integers(0, 1 << 62))), nxt, body)
    if r < 0.88:
        et, inner = _l3(rng, depth + 1)
        labels = [int(rng.integers(0, 1 << 20)) for _ in range(int(rng.integers(1, 4)))]
        if rng.random() < 0.2:  # EoMPLS: control word + Ethernet (parser.cpp:622-631)
            inner = b"\0\0\0\0" + eth(mac(1), mac(2), et) + inner
        return 0x8847 if rng.random() < 0.7 else 0x8848, mpls(labels, inner)
    et, inner = _l3(rng, depth + 1)
    proto = {0x0800: 0x0021, 0x86DD: 0x0057}.get(et, 0x0021)
    code = 0 if rng.random() < 0.9 else 7
    return 0x8864, pppoe(inner, proto=proto, code=code)


def fuzz_frame(rng):
    r = rng.random()
    vl = []
    if r < 0.3:
        for k in range(int(rng.integers(1, 4))):
            vl.append((0x88A8 if (k == 0 and rng.random() < 0.4) else 0x8100, int(rng.integers(0, 65536))))
    et, l3 = _l3(rng)
    if rng.random() < 0.04:
        et, l3 = int(rng.integers(0, 65536)), b"q" * 40
    frame = eth(mac(int(rng.integers(0, 1 << 30))), mac(int(rng.integers(0, 1 << 30))), et, vl) + l3
    if rng.random() < 0.05:
        frame = eth(mac(7), mac(8), 0x22F3) + trill(frame, op_len=int(rng.integers(0, 4)))
    if rng.random() < 0.1:  # byte corruption in the header area
        b = bytearray(frame)
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, min(len(b), 80)))] = int(rng.integers(0, 256))
        frame = bytes(b)
    return frame


def fuzz_corpus(n, seed=1):
    """List of (frame_bytes, caplen, wirelen) with random truncation."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        f = pad(fuzz_frame(rng))
        wl = len(f)
        cl = wl if rng.random() < 0.8 else int(rng.integers(0, wl + 1))
        out.append((f[:cl], cl, wl))
    return out


def to_batch(frames, t0=1_600_000_000, dt_us=1):
    """frames: [(bytes, caplen, wirelen)] or [(bytes, caplen, wirelen, sec, usec)]."""
    pk = []
    for i, fr in enumerate(frames):
        if len(fr) == 5:
            b, cl, wl, s, us = fr
        else:
            b, cl, wl = fr
            t = t0 * 1_000_000 + i * dt_us
            s, us = divmod(t, 1_000_000)
        pk.append((s, us, cl, wl, b))
    import pcaputil
    return pcaputil.to_batch(pk)


# ---- cache-semantics streams ---------------------------------------------------------------
class Stream:
    """Accumulates timestamped frames; time advances monotonically."""

    def __init__(self, t0=1_600_000_000):
        self.t = t0 * 1_000_000
        self.frames = []

    def add(self, frame, gap_us=1):
        self.t += gap_us
        f = pad(frame)
        s, us = divmod(self.t, 1_000_000)
        self.frames.append((f, len(f), len(f), s, us))

    def batch(self):
        return to_batch(self.frames)


def flow_stream(seed=7, n_flows=300, n_pkts=6000, v6_share=0.2, vlan_share=0.1, frag=True,
                long_gap_share=0.003):
    """Mixed TCP/UDP/ICMP biflows with SYN/FIN/RST sequences, idle gaps past the inactive
    timeout, flows outliving the active timeout, fragments, and symmetric keys."""
    rng = np.random.default_rng(seed)
    st = Stream()
    flows = []
    for f in range(n_flows):
        v6 = rng.random() < v6_share
        a = ip6(f * 2 + 1) if v6 else ip4(0x0A000000 + f * 2 + 1)
        b = ip6(f * 2 + 2) if v6 else ip4(0xC0A80000 + f * 2 + 2)
        if rng.random() < 0.02:
            b = a  # symmetric key when ports are equal too
        proto = [6, 6, 17, 17, 1][int(rng.integers(0, 5))]
        sp, dp = int(rng.integers(1024, 65536)), int(rng.integers(1, 1024))
        if a == b:
            dp = sp
        vlan = [(0x8100, int(rng.integers(1, 4095)))] if rng.random() < vlan_share else []
        flows.append((v6, a, b, proto, sp, dp, vlan))
    for i in range(n_pkts):
        v6, a, b, proto, sp, dp, vlan = flows[int(rng.integers(0, n_flows))]
        rev = rng.random() < 0.45
        s, d = (b, a) if rev else (a, b)
        ps, pd = (dp, sp) if rev else (sp, dp)
        if proto == 6:
            fl = [0x10, 0x18, 0x10, 0x02, 0x12, 0x01, 0x11, 0x04, 0x10][int(rng.integers(0, 9))]
            l4 = tcp(ps, pd, fl, options=b"\x02\x04\x05\xb4" if fl & 2 else b"")
        elif proto == 17:
            l4 = udp(ps, pd, b"u" * int(rng.integers(0, 30)))
        else:
            l4 = icmp()
        et = 0x86DD if v6 else 0x0800
        if frag and not v6 and rng.random() < 0.03:  # a fragmented datagram in 2-3 pieces
            ident = int(rng.integers(0, 65536))
            whole = l4 + b"f" * 40
            st.add(eth(mac(1), mac(2), et, vlan) + ipv4(s, d, proto, whole[:24], mf=1, ident=ident))
            st.add(eth(mac(1), mac(2), et, vlan) + ipv4(s, d, proto, whole[24:48], frag_off=3, mf=1, ident=ident),
                   gap_us=int(rng.integers(1, 5_000_000)))
            st.add(eth(mac(1), mac(2), et, vlan) + ipv4(s, d, proto, whole[48:], frag_off=6, ident=ident))
            continue
        l3 = ipv6(s, d, proto if proto != 1 else 58, l4) if v6 else ipv4(s, d, proto, l4)
        r = rng.random()
        if r < long_gap_share:
            gap = int(rng.integers(30_000_000, 90_000_000))  # past the default inactive timeout
        elif r < 0.03:
            gap = int(rng.integers(1_000_000, 8_000_000))
        else:
            gap = int(rng.integers(1, 20_000))
        st.add(eth(mac(3 if rev else 4), mac(4 if rev else 3), et, vlan) + l3, gap_us=gap)
    return st


# ---- vectorised 64 B UDP frames (large synthetic batches) ------------------------------------
def udp_frames(sip, dip, sport, dport, t0=1_600_000_000, dt_us=1, smac=None, dmac=None):
    """numpy arrays of per-packet IPv4 addresses / UDP ports -> (arena, desc) of 64 B
    Ethernet/IPv4/UDP frames (tot_len 50), one frame per 64 B slot, timestamps t0 + i*dt_us."""
    import pcaputil
    n = len(sip)
    fr = np.zeros((n, 64), dtype=np.uint8)

    def put(col, val, nbytes):
        val = np.asarray(val, dtype=np.uint64)
        for q in range(nbytes):
            fr[:, col + q] = (val >> np.uint64(8 * (nbytes - 1 - q))) & np.uint64(0xFF)

    put(0, 0x020000000001 if dmac is None else dmac, 6)
    put(6, 0x020000000002 if smac is None else smac, 6)
    fr[:, 12] = 0x08
    fr[:, 14] = 0x45
    fr[:, 17] = 50
    fr[:, 22] = 64
    fr[:, 23] = 17
    put(26, sip, 4)
    put(30, dip, 4)
    put(34, sport, 2)
    put(36, dport, 2)
    fr[:, 39] = 30
    desc = np.zeros(n, dtype=pcaputil.DESC_DTYPE)
    t = np.uint64(t0) * np.uint64(1_000_000) + np.arange(n, dtype=np.uint64) * np.uint64(dt_us)
    desc["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(64)
    desc["caplen"] = 64
    desc["wirelen"] = 64
    desc["ts_sec"] = t // np.uint64(1_000_000)
    desc["ts_usec"] = t % np.uint64(1_000_000)
    return fr.reshape(-1), desc
