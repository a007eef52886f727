"""Synthetic packet mixes of BASELINE.json's configs, generated on the GPU (bench and test
infrastructure; not part of the engine).

  udp64  configs[1]: 64 B Ethernet/IPv4/UDP (bench.py builds this one itself)
  imix   configs[2]: IMIX 64/594/1518 B at 7:4:1, Zipf(1.1) flow popularity, a TCP/UDP mix with
         TCP timestamp options on most TCP flows, TLS (443) / HTTP (80) / DNS (53) payload
         prefixes so L7 plugins have something to see, 11 % IPv6, 3 % 802.1Q
  quic   configs[4]: QUIC-heavy variable-length mix: 60 % UDP/443 QUIC (long-header Initial
         >= 1200 B datagrams and short-header packets), 40 % encapsulations the parser walks
         (802.1Q, QinQ, MPLS 1-3 labels, IPv6 + 1-3 extension headers, PPPoE, GRE)

Frame layouts are assembled here with the byte offsets of every per-flow / per-packet field;
tools/synth/ipxg_synth.hip stamps flows and packets into them on the device (one RNG stream per
global packet index, so a batch is reproducible on its own).  Timestamps are monotonic at a
virtual line rate (dt_ns per packet): no flow of these mixes reaches the inactive or active
timeout, and there is no FIN/RST, so flow records equal distinct biflows per batch sequence.
"""
import ctypes
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libipxg_synth.so")

LAYOUT_DTYPE = np.dtype([
    ("tmpl", "u1", (192,)), ("hdr_len", "<u2"), ("addr_len", "<u2"), ("sip_off", "<u2"), ("dip_off", "<u2"),
    ("sport_off", "<u2"), ("dport_off", "<u2"), ("tcp_flags_off", "<u2"), ("vlan_off", "<u2"),
    ("patch_off", "<u2", (4,)), ("patch_bias", "<u2", (4,)), ("size_mode", "<u2"), ("l7_off", "<u2"),
    ("min_len", "<u2"), ("alt_len", "<u2"), ("alt", "u1", (8,)), ("blob_len", "<u2"), ("pad", "<u2", (7,)),
])
FLOW_DTYPE = np.dtype([("sip", "u1", (16,)), ("dip", "u1", (16,)), ("sport", "<u2"), ("dport", "<u2"),
                       ("layout", "<u2"), ("vlan", "<u2"), ("mac_id", "<u4"), ("opening", "<u4")])
assert LAYOUT_DTYPE.itemsize == 256 and FLOW_DTYPE.itemsize == 48

SIZE_IMIX, SIZE_QUIC, SIZE_64 = 0, 1, 2

TLS_HELLO = bytes.fromhex("160301020001") + bytes.fromhex("0001fc0303") + bytes(range(32))
HTTP_GET = b"GET /index.html HTTP/1.1\r\nHost: www.example.com\r\nAccept: */*\r\n\r\n"
DNS_QUERY = struct.pack(">HHHHHH", 0x1234, 0x0100, 1, 0, 0, 0) + b"\x07example\x03com\x00" + struct.pack(">HH", 1, 1)
QUIC_INITIAL = (b"\xc3" + struct.pack(">I", 1) + b"\x08" + bytes(range(8)) + b"\x08" + bytes(range(8, 16)) +
                b"\x00" + b"\x44\xb0" + b"\x00\x00\x00\x01")
TCP_TS = b"\x01\x01\x08\x0a" + struct.pack(">II", 0x01020304, 0)
# what established flows carry where an opening flow has its first message
TLS_APPDATA = bytes.fromhex("1703030200")      # TLS application data record header
HTTP_BODY = b"\x1f\x8b\x08\x00data"           # (gzip) body bytes -- no method, no status line


def build_layout(ip=4, l4="udp", dport=0, vlan=0, mpls=0, pppoe=False, gre=False, ext=(), tcp_opts=b"",
                 l7=b"", size_mode=SIZE_IMIX, alt=b""):
    """One frame layout -> (LAYOUT_DTYPE record, server port).  vlan: 0 none, 1 802.1Q, 2 QinQ."""
    b = bytearray(b"\0" * 12)
    rec = np.zeros(1, dtype=LAYOUT_DTYPE)[0]
    patches = []
    vlan_off = 0
    if vlan:
        if vlan == 2:
            b += struct.pack(">HH", 0x88A8, 0x0064)
            vlan_off = 14
            b += struct.pack(">HH", 0x8100, 0x00C8)
        else:
            b += struct.pack(">HH", 0x8100, 0x0064)
            vlan_off = 14
    ip_et = 0x0800 if ip == 4 else 0x86DD
    if mpls:
        b += struct.pack(">H", 0x8847)
        for k in range(mpls):
            b += struct.pack(">I", ((1000 + k) << 12) | ((1 if k == mpls - 1 else 0) << 8) | 64)
    elif pppoe:
        b += struct.pack(">H", 0x8864)
        po = len(b)
        b += struct.pack(">BBHH", 0x11, 0, 7, 0) + struct.pack(">H", 0x0021 if ip == 4 else 0x0057)
        patches.append((po + 4, po + 6))
    elif gre:
        b += struct.pack(">H", 0x0800)
        oo = len(b)
        b += struct.pack(">BBHHHBBH4s4s", 0x45, 0, 0, 0, 0, 64, 47, 0, bytes([198, 51, 100, 1]),
                         bytes([198, 51, 100, 2]))
        patches.append((oo + 2, oo))
        b += struct.pack(">HH", 0x2000, ip_et) + struct.pack(">I", 42)  # key present
    else:
        b += struct.pack(">H", ip_et)
    proto = 6 if l4 == "tcp" else 17
    ipo = len(b)
    if ip == 4:
        b += struct.pack(">BBHHHBBH4s4s", 0x45, 0, 0, 0, 0x4000, 64, proto, 0, b"\0" * 4, b"\0" * 4)
        patches.append((ipo + 2, ipo))
        sip_off, dip_off, alen = ipo + 12, ipo + 16, 4
    else:
        nxt = ext[0] if ext else proto
        b += struct.pack(">IHBB", 6 << 28, 0, nxt, 64) + b"\0" * 32
        patches.append((ipo + 4, ipo + 40))
        sip_off, dip_off, alen = ipo + 8, ipo + 24, 16
        for k, t in enumerate(ext):
            n2 = ext[k + 1] if k + 1 < len(ext) else proto
            b += bytes([n2, 0]) + b"\0" * 6  # hop-by-hop / dest-options / routing: 8 bytes
    l4o = len(b)
    flags_off = 0
    if l4 == "tcp":
        opts = tcp_opts.ljust((len(tcp_opts) + 3) // 4 * 4, b"\0")
        doff = 5 + len(opts) // 4
        b += struct.pack(">HHIIBBHHH", 0, 0, 1, 0, doff << 4, 0x10, 1024, 0, 0) + opts
        flags_off = l4o + 13
    else:
        b += struct.pack(">HHHH", 0, 0, 0, 0)
        patches.append((l4o + 4, l4o))
    l7o = len(b)
    b += l7
    assert len(b) <= 192 and len(patches) <= 4
    rec["tmpl"][:len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    rec["hdr_len"] = len(b)
    rec["addr_len"] = alen
    rec["sip_off"], rec["dip_off"] = sip_off, dip_off
    rec["sport_off"], rec["dport_off"] = l4o, l4o + 2
    rec["tcp_flags_off"] = flags_off
    rec["vlan_off"] = vlan_off
    for k, (o, bias) in enumerate(patches):
        rec["patch_off"][k] = o
        rec["patch_bias"][k] = bias
    rec["size_mode"] = size_mode
    rec["l7_off"] = l7o
    rec["min_len"] = max(len(b), 60)
    rec["alt_len"] = len(alt)
    rec["alt"][:len(alt)] = np.frombuffer(alt, dtype=np.uint8)
    return rec, dport


# (share, layout kwargs).  dport 0 = a random well-known port per flow.
MIXES = {
    "imix": [
        (0.30, dict(ip=4, l4="tcp", dport=443, tcp_opts=TCP_TS, l7=TLS_HELLO, alt=TLS_APPDATA)),
        (0.15, dict(ip=4, l4="tcp", dport=80, tcp_opts=TCP_TS, l7=HTTP_GET, alt=HTTP_BODY)),
        (0.10, dict(ip=4, l4="tcp", dport=0)),
        (0.15, dict(ip=4, l4="udp", dport=53, l7=DNS_QUERY)),
        (0.15, dict(ip=4, l4="udp", dport=0)),
        (0.08, dict(ip=6, l4="tcp", dport=443, tcp_opts=TCP_TS, l7=TLS_HELLO, alt=TLS_APPDATA)),
        (0.04, dict(ip=6, l4="udp", dport=53, l7=DNS_QUERY)),
        (0.03, dict(ip=4, l4="tcp", dport=443, vlan=1, tcp_opts=TCP_TS, l7=TLS_HELLO, alt=TLS_APPDATA)),
    ],
    "quic": [
        (0.45, dict(ip=4, l4="udp", dport=443, l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.15, dict(ip=6, l4="udp", dport=443, l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.06, dict(ip=4, l4="udp", dport=443, vlan=1, l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.05, dict(ip=4, l4="tcp", dport=443, vlan=2, tcp_opts=TCP_TS, l7=TLS_HELLO, alt=TLS_APPDATA)),
        (0.03, dict(ip=4, l4="udp", dport=443, mpls=1, l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.03, dict(ip=4, l4="tcp", dport=443, mpls=2, tcp_opts=TCP_TS)),
        (0.02, dict(ip=6, l4="udp", dport=0, mpls=3)),
        (0.04, dict(ip=6, l4="udp", dport=443, ext=(0,), l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.03, dict(ip=6, l4="tcp", dport=443, ext=(0, 60), tcp_opts=TCP_TS)),
        (0.03, dict(ip=6, l4="udp", dport=0, ext=(0, 43, 60))),
        (0.04, dict(ip=4, l4="tcp", dport=80, pppoe=True, tcp_opts=TCP_TS, l7=HTTP_GET, alt=HTTP_BODY)),
        (0.02, dict(ip=6, l4="udp", dport=53, pppoe=True, l7=DNS_QUERY)),
        (0.03, dict(ip=4, l4="udp", dport=443, gre=True, l7=QUIC_INITIAL, size_mode=SIZE_QUIC)),
        (0.02, dict(ip=6, l4="tcp", dport=443, gre=True, tcp_opts=TCP_TS)),
    ],
}


_INITIAL = []


def quic_initial():
    """A complete QUIC client Initial datagram (the UDP payload of the reference's own QUIC test
    capture, tests/functional/inputs/quic_initial-sample.pcap, copied into tests/golden/reference:
    draft-29, 1330 bytes, one CRYPTO frame holding a TLS ClientHello).  The configs[4] mix's opening
    flows carry it as their long-header packets, so the reference's QUIC plugin decrypts a real
    Initial (RFC 9001 initial secrets from its DCID) on every one of them, as on live traffic -- a
    template with an undecryptable payload was never detected by it (quic_parser.cpp
    quic_set_server_port needs the parsed ClientHello)."""
    if not _INITIAL:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests"))
        import pcaputil
        dl, pk = pcaputil.read_capture(os.path.join(os.path.dirname(os.path.dirname(HERE)), "tests", "golden",
                                                    "reference", "quic_initial-sample.pcap"))
        fr = bytes(pk[0][4])
        et = struct.unpack(">H", fr[12:14])[0]
        assert et == 0x86DD and fr[14 + 6] == 17  # IPv6 / UDP
        udp = fr[54:]
        _INITIAL.append(udp[8:8 + struct.unpack(">H", udp[4:6])[0] - 8])
    return _INITIAL[0]


class Mix:
    """Layouts + flow table (+ Zipf CDF) of one mix, on the host.

    Connections being opened vs established (what the process plugins see): an opening flow's
    packets carry its protocol's first message (TLS ClientHello, HTTP request line, QUIC
    long-header Initial); an established flow's carry later traffic (TLS application data, HTTP
    body bytes, QUIC short headers).  With Zipf popularity the opening flows are the least
    popular `open_share` of the flows (short connections; the popular ones are long-lived and
    mid-connection), and DNS flows -- a query and its answer per flow -- rank last of all; with
    uniform popularity a random `open_share` of the flows is opening."""

    def __init__(self, name, n_flows, seed=1234, zipf=None, open_share=None):
        spec = MIXES[name]
        self.name = name
        self.zipf = zipf
        rng = np.random.default_rng(seed)
        recs = [build_layout(**kw) for _, kw in spec]
        self.layouts = np.array([r for r, _ in recs], dtype=LAYOUT_DTYPE)
        # QUIC layouts: the opening flows' long headers are a real client Initial (quic_initial)
        self.blob = None
        quic = np.array([kw.get("l7") == QUIC_INITIAL and kw.get("size_mode") == SIZE_QUIC for _, kw in spec])
        if quic.any():
            self.blob = np.frombuffer(quic_initial(), dtype=np.uint8)
            self.layouts["blob_len"][quic] = len(self.blob)
        shares = np.array([s for s, _ in spec], dtype=np.float64)
        shares /= shares.sum()
        F = int(n_flows)
        lay = rng.choice(len(spec), size=F, p=shares).astype(np.uint16)
        fl = np.zeros(F, dtype=FLOW_DTYPE)
        fl["layout"] = lay
        v6 = self.layouts["addr_len"][lay] == 16
        # IPv4 addresses in the first 4 bytes (client 10/8, server 172.16/12); IPv6 2001:db8::/32
        c4 = (10 << 24) | rng.integers(0, 1 << 24, F, dtype=np.int64)
        s4 = (172 << 24) | (16 << 16) | rng.integers(0, 1 << 20, F, dtype=np.int64)
        for col, v in (("sip", c4), ("dip", s4)):
            a = np.zeros((F, 16), dtype=np.uint8)
            for q in range(4):
                a[:, q] = (v >> (24 - 8 * q)) & 0xFF
            hi = rng.integers(0, 1 << 62, F, dtype=np.int64)
            a6 = np.zeros((F, 16), dtype=np.uint8)
            a6[:, 0:4] = [0x20, 0x01, 0x0d, 0xb8]
            a6[:, 4] = 1 if col == "sip" else 2
            for q in range(8):
                a6[:, 8 + q] = (hi >> (56 - 8 * q)) & 0xFF
            a[v6] = a6[v6]
            fl[col] = a
        fl["sport"] = rng.integers(1024, 65536, F)
        dp = np.array([kw.get("dport", 0) for _, kw in spec], dtype=np.int64)[lay]
        rnd = rng.integers(1, 1024, F)
        fl["dport"] = np.where(dp == 0, rnd, dp)
        fl["vlan"] = rng.integers(1, 4095, F)
        fl["mac_id"] = np.arange(F, dtype=np.uint32)
        self.flows = fl
        self.cdf = None
        self.rank_flow = None
        if zipf:
            w = np.arange(1, F + 1, dtype=np.float64) ** (-float(zipf))
            c = np.cumsum(w)
            c /= c[-1]
            # 2^64 - 2048: the largest float64 below 2^64 (the last entry is set to 2^64 - 1)
            self.cdf = np.floor(c * 18446744073709549568.0).astype(np.uint64)
            self.cdf[-1] = np.uint64(0xFFFFFFFFFFFFFFFF)
            dns = np.isin(lay, [k for k, (_, kw) in enumerate(spec) if kw.get("l7") == DNS_QUERY])
            # rank -> flow: the other flows in random order, then the DNS flows (the least popular)
            self.rank_flow = np.concatenate([rng.permutation(np.nonzero(~dns)[0]),
                                             rng.permutation(np.nonzero(dns)[0])]).astype(np.uint32)
            share = 0.3 if open_share is None else open_share
            fl["opening"][self.rank_flow[int(F * (1.0 - share)):]] = 1
        else:
            share = 1.0 / 16 if open_share is None else open_share
            fl["opening"] = rng.random(F) < share


    def restrict(self, keep):
        """Keep only the flows `keep` (indices; one rank's flow-hash shard): their popularity
        order is kept (Zipf over the kept flows, in the order the full mix ranked them), and
        with it which are opening and where the DNS flows rank."""
        keep = np.asarray(keep, dtype=np.int64)
        if self.rank_flow is not None:
            pos = np.empty(len(self.flows), dtype=np.int64)
            pos[self.rank_flow] = np.arange(len(self.flows))
            keep = keep[np.argsort(pos[keep], kind="stable")]  # in rank order
        self.flows = self.flows[keep]
        if self.cdf is not None:
            F = len(self.flows)
            w = np.arange(1, F + 1, dtype=np.float64) ** (-float(self.zipf))
            c = np.cumsum(w)
            c /= c[-1]
            self.cdf = np.floor(c * 18446744073709549568.0).astype(np.uint64)
            self.cdf[-1] = np.uint64(0xFFFFFFFFFFFFFFFF)
            self.rank_flow = np.arange(F, dtype=np.uint32)


class _Params(ctypes.Structure):
    _fields_ = [("layouts", ctypes.c_void_p), ("flows", ctypes.c_void_p), ("cdf", ctypes.c_void_p),
                ("rank_flow", ctypes.c_void_p), ("seed", ctypes.c_uint64), ("first_idx", ctypes.c_uint64),
                ("t0_ns", ctypes.c_uint64), ("nflows", ctypes.c_uint32), ("n", ctypes.c_uint32),
                ("dt_ns", ctypes.c_uint32), ("fwd_q16", ctypes.c_uint32), ("syn_q16", ctypes.c_uint32),
                ("psh_q16", ctypes.c_uint32), ("blob", ctypes.c_void_p), ("oshift", ctypes.c_uint32)]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        import torch  # noqa: F401  (bind to torch's HIP runtime, as ipfixprobe_amd.engine does)
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("tools/synth/libipxg_synth.so not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.synth_plan.argtypes = [ctypes.POINTER(_Params), vp, vp, vp]
        L.synth_write.argtypes = [ctypes.POINTER(_Params), vp, vp, vp, vp, vp]
        assert L.synth_layout_size() == LAYOUT_DTYPE.itemsize and L.synth_flow_size() == FLOW_DTYPE.itemsize
        _LIB = L
    return _LIB


class Generator:
    """A mix resident on one GPU; batch() generates packets [first, first + n) of its stream."""

    def __init__(self, mix, device, seed=1234, t0_ns=1_700_000_000 * 10**9, dt_ns=100, fwd_share=0.55,
                 syn_share=0.005, psh_share=0.045):
        import torch
        self.mix, self.device, self.seed, self.t0_ns, self.dt_ns = mix, device, seed, t0_ns, dt_ns
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(device)  # noqa: E731
        self.d_layouts = up(mix.layouts)
        self.d_flows = up(mix.flows)
        self.d_cdf = up(mix.cdf) if mix.cdf is not None else None
        self.d_rank = up(mix.rank_flow) if mix.rank_flow is not None else None
        self.d_blob = up(mix.blob) if mix.blob is not None else None
        self.q16 = [int(round(x * 65536)) for x in (fwd_share, syn_share, psh_share)]

    def _params(self, first, n):
        p = _Params()
        p.layouts = self.d_layouts.data_ptr()
        p.flows = self.d_flows.data_ptr()
        p.cdf = self.d_cdf.data_ptr() if self.d_cdf is not None else None
        p.rank_flow = self.d_rank.data_ptr() if self.d_rank is not None else None
        p.seed, p.first_idx, p.t0_ns = self.seed, first, self.t0_ns
        p.nflows, p.n, p.dt_ns = len(self.mix.flows), n, self.dt_ns
        p.fwd_q16, p.syn_q16, p.psh_q16 = self.q16
        p.blob = self.d_blob.data_ptr() if self.d_blob is not None else None
        return p

    def batch(self, first, n, offset16=False):
        """(arena uint8, desc uint8 [n * 16]) device tensors of packets [first, first + n).
        offset16: descriptor offsets in 16-byte units (IPXG_BATCH_OFFSET16, arenas past 4 GiB)."""
        import torch
        stream = torch.cuda.current_stream(self.device).cuda_stream
        p = self._params(first, n)
        p.oshift = 4 if offset16 else 0
        plan = torch.empty(n * 16, dtype=torch.uint8, device=self.device)
        alen = torch.empty(n, dtype=torch.int64, device=self.device)
        if lib().synth_plan(ctypes.byref(p), plan.data_ptr(), alen.data_ptr(), stream):
            raise RuntimeError("synth_plan failed")
        off, total = place(alen, torch)
        if total + 64 >= (1 << 36 if offset16 else 1 << 32):
            raise ValueError("batch arena %d B exceeds the descriptor offset range" % total)
        arena = torch.zeros(total + 64, dtype=torch.uint8, device=self.device)
        desc = torch.empty(n * 16, dtype=torch.uint8, device=self.device)
        if lib().synth_write(ctypes.byref(p), plan.data_ptr(), off.data_ptr(), arena.data_ptr(), desc.data_ptr(),
                             stream):
            raise RuntimeError("synth_write failed")
        del plan, alen, off
        return arena, desc


def place(alen, xp):
    """Frame placement in the arena (the producer's choice: the batch format takes any offsets).
    Frames longer than 64 bytes start on a 128-byte line (the region they share is laid out in
    128-byte multiples), so a header walk's head (<= 128 bytes) is one line, not two; frames of
    <= 64 bytes pack two to a line in a region of their own after it -- as NIC DMA into
    line-aligned receive buffers from two pools by size would place them.  alen = the frames'
    64-byte-rounded lengths in packet order (numpy or torch); returns (offsets, arena bytes)."""
    big = alen > 64
    abig = xp.where(big, (alen + 127) // 128 * 128, xp.zeros_like(alen))
    asmall = xp.where(big, xp.zeros_like(alen), xp.full_like(alen, 64))
    ebig = xp.cumsum(abig, 0) if xp is not np else np.cumsum(abig)
    esmall = xp.cumsum(asmall, 0) if xp is not np else np.cumsum(asmall)
    nbig = ebig[-1] if alen.shape[0] else 0
    off = xp.where(big, ebig - abig, nbig + esmall - asmall)
    total = (int(nbig) + int(esmall[-1])) if alen.shape[0] else 0
    return off, total


def alg_bytes(desc_np):
    """SURVEY 8(d) algorithmic bytes: min(caplen, 128) + 16 per packet."""
    return int(np.minimum(desc_np["caplen"].astype(np.int64), 128).sum()) + 16 * len(desc_np)


# ---- host restatement of the two kernels (the generator's own check, and CPU tests) --------
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def host_plan(gen, first, n):
    """k_synth_plan restated with numpy: (flow id, direction, frame length, long header, TCP flags)."""
    mix = gen.mix
    g = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r0 = _mix64(np.uint64(gen.seed) ^ (g * np.uint64(0xD1B54A32D192ED03)))
        r1 = _mix64(r0 ^ np.uint64(0x5851F42D4C957F2D))
    F = len(mix.flows)
    if mix.cdf is not None:
        f = np.searchsorted(mix.cdf, r0, side="right").astype(np.int64)
        f = np.minimum(f, F - 1)
    else:
        f = (((r0 >> np.uint64(32)) * np.uint64(F)) >> np.uint64(32)).astype(np.int64)
    if mix.rank_flow is not None:
        f = mix.rank_flow[f].astype(np.int64)
    L = mix.layouts[mix.flows["layout"][f].astype(np.int64)]
    u = (r1 & np.uint64(0xFFFF)).astype(np.int64)
    dirn = (((r1 >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.int64) >= gen.q16[0]).astype(np.int64)
    s12 = ((((r1 >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64) * 12) >> 16)
    lng = mix.flows["opening"][f] != 0
    mode = L["size_mode"].astype(np.int64)
    imix = np.where(s12 < 7, 64, np.where(s12 < 11, 594, 1518))
    ini = np.maximum(L["blob_len"].astype(np.int64), 1200)
    quic = np.where(lng, L["l7_off"].astype(np.int64) + ini, np.where(s12 < 6, 80, 1350))
    ln = np.where(mode == 0, imix, np.where(mode == 1, quic, 64))
    lng = lng & (mode == 1)
    ln = np.maximum(ln, L["min_len"].astype(np.int64))
    syn, psh = gen.q16[1], gen.q16[2]
    flags = np.where(u < syn, 0x02, np.where(u < syn + psh, 0x18, 0x10))
    return f, dirn, ln, lng, flags


def host_batch(gen, first, n):
    """k_synth_plan + k_synth_write restated with numpy: (arena uint8, desc DESC_DTYPE)."""
    mix = gen.mix
    f, dirn, ln, lng, flags = host_plan(gen, first, n)
    L = mix.layouts[mix.flows["layout"][f].astype(np.int64)]
    g = np.arange(first, first + n, dtype=np.uint64)
    alen = (ln + 63) & ~63
    off, total = place(alen, np)
    off = off.astype(np.int64)
    arena = np.zeros(total + 64, dtype=np.uint8)
    import pcaputil
    desc = np.zeros(n, dtype=pcaputil.DESC_DTYPE)
    t = np.uint64(gen.t0_ns) + g * np.uint64(gen.dt_ns)
    us = t // np.uint64(1000)
    desc["offset"] = off
    desc["caplen"] = ln
    desc["wirelen"] = ln
    desc["ts_sec"] = us // np.uint64(1000000)
    desc["ts_usec"] = us % np.uint64(1000000)
    fl = mix.flows
    for i in range(n):
        lay = L[i]
        h = bytearray(lay["tmpl"].tobytes())
        fi = f[i]
        d = dirn[i]
        a, b = (fl["dip"][fi], fl["sip"][fi]) if d else (fl["sip"][fi], fl["dip"][fi])
        al = int(lay["addr_len"])
        h[lay["sip_off"]:lay["sip_off"] + al] = a[:al].tobytes()
        h[lay["dip_off"]:lay["dip_off"] + al] = b[:al].tobytes()
        sp, dp = int(fl["sport"][fi]), int(fl["dport"][fi])
        h[lay["sport_off"]:lay["sport_off"] + 2] = struct.pack(">H", dp if d else sp)
        h[lay["dport_off"]:lay["dport_off"] + 2] = struct.pack(">H", sp if d else dp)
        m = int(fl["mac_id"][fi])
        cm = bytes([2, 0, (m >> 24) & 255, (m >> 16) & 255, (m >> 8) & 255, m & 255])
        sm = bytes([4]) + cm[1:]
        h[0:6], h[6:12] = (cm, sm) if d else (sm, cm)
        if lay["vlan_off"]:
            vo = int(lay["vlan_off"])
            tci = ((h[vo] << 8) | h[vo + 1]) & 0xF000
            h[vo:vo + 2] = struct.pack(">H", tci | (int(fl["vlan"][fi]) & 0xFFF))
        for k in range(4):
            if lay["patch_off"][k]:
                o = int(lay["patch_off"][k])
                h[o:o + 2] = struct.pack(">H", (int(ln[i]) - int(lay["patch_bias"][k])) & 0xFFFF)
        if lay["tcp_flags_off"]:
            h[lay["tcp_flags_off"]] = int(flags[i])
        if lay["size_mode"] == 1 and not lng[i]:
            h[lay["l7_off"]] = 0x43
        if not fl["opening"][fi]:
            o = int(lay["l7_off"])
            h[o:o + int(lay["alt_len"])] = lay["alt"][:int(lay["alt_len"])].tobytes()
        hl = min(int(lay["hdr_len"]), int(ln[i]))
        arena[off[i]:off[i] + hl] = np.frombuffer(bytes(h[:hl]), dtype=np.uint8)
        if lng[i] and int(lay["blob_len"]) and mix.blob is not None:  # the Initial over the template
            o = off[i] + int(lay["l7_off"])
            arena[o:o + len(mix.blob)] = mix.blob
    return arena, desc
