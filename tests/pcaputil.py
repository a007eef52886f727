"""Test-side capture tools: a small pure-Python pcap/pcapng reader and the UniRec logger
text format the reference's functional tests compare against.

The reader is deliberately independent of the product's C++ reader (libipxg
ipxg_capture_load) so each can check the other.  Timestamp handling follows libpcap as the
reference's pcap plugin sees it (pcap.cpp:54-70): microsecond precision, nanosecond
sources scaled down by integer division, pcapng if_tsresol honoured.
"""
import datetime
import socket
import struct

import numpy as np

DLT_EN10MB = 1
DLT_RAW = 12
DLT_LINUX_SLL = 113
DLT_LINUX_SLL2 = 276

_LINKTYPE_TO_DLT = {1: DLT_EN10MB, 101: DLT_RAW, 12: DLT_RAW, 14: DLT_RAW,
                    113: DLT_LINUX_SLL, 276: DLT_LINUX_SLL2}

DESC_DTYPE = np.dtype([("offset", "<u4"), ("caplen", "<u2"), ("wirelen", "<u2"),
                       ("ts_sec", "<u4"), ("ts_usec", "<u4")])
assert DESC_DTYPE.itemsize == 16

FLOW_DTYPE = np.dtype([
    ("flow_hash", "<u8"),
    ("time_first_sec", "<u4"), ("time_first_usec", "<u4"),
    ("time_last_sec", "<u4"), ("time_last_usec", "<u4"),
    ("src_bytes", "<u8"), ("dst_bytes", "<u8"),
    ("src_packets", "<u4"), ("dst_packets", "<u4"),
    ("src_tcp_flags", "u1"), ("dst_tcp_flags", "u1"), ("ip_version", "u1"), ("ip_proto", "u1"),
    ("src_port", "<u2"), ("dst_port", "<u2"),
    ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)),
    ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)),
    ("vlan_id", "<u2"), ("end_reason", "u1"), ("reserved0", "u1"), ("reserved", "u1", (8,)),
    ("ext", "<u8"), ("reserved2", "u1", (8,)),
])
assert FLOW_DTYPE.itemsize == 128

PARSED_DTYPE = np.dtype([
    ("valid", "u1"), ("ip_version", "u1"), ("ip_proto", "u1"), ("tcp_flags", "u1"),
    ("ethertype", "<u2"), ("ip_len", "<u2"), ("src_port", "<u2"), ("dst_port", "<u2"),
    ("frag_off", "<u2"), ("more_fragments", "u1"), ("ip_ttl", "u1"),
    ("vlan_id", "<u4"), ("frag_id", "<u4"), ("mpls_top", "<u4"), ("tcp_mss", "<u4"),
    ("tcp_options", "<u8"),
    ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,)),
    ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)),
    ("ip_tos", "u1"), ("ip_flags", "u1"), ("tcp_window", "<u2"),
    ("tcp_seq", "<u4"), ("tcp_ack", "<u4"),
    ("hash_fwd", "<u8"), ("hash_inv", "<u8"),
    ("payload_off", "<u2"), ("payload_len", "<u2"), ("reserved2", "<u4"),
])
assert PARSED_DTYPE.itemsize == 120

# include/ipxg.h ipxg_vlan_stats (VlanStats, parser-stats.hpp:126-160), test-side restatement
VLAN_STATS_DTYPE = np.dtype([("ipv4_packets", "<u8"), ("ipv6_packets", "<u8"), ("ipv4_bytes", "<u8"),
                             ("ipv6_bytes", "<u8"), ("tcp_packets", "<u8"), ("udp_packets", "<u8"),
                             ("total_packets", "<u8"), ("total_bytes", "<u8"),
                             ("hist_packets", "<u8", (10,)), ("hist_bytes", "<u8", (10,))])
VLAN_IDS = 4096

# ipxg_stats field order (include/ipxg.h), all uint64
STATS_FIELDS = [
    "seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets", "ipv6_packets",
    "tcp_packets", "udp_packets", "mpls_packets", "pppoe_packets", "trill_packets",
    "vlan_packets", "ipv4_bytes", "ipv6_bytes", "end_inactive", "end_active", "end_eof",
    "end_forced", "end_no_res", "flows_in_cache", "total_exported", "keyless_packets",
    "fragmented_packets", "fragments_filled", "complex_flows", "table_capacity",
    "table_rehashes", "batches", "spilled_packets", "slow_path_packets",
    "aggregated_packets", "walked_packets", "flows_1_packet", "flows_2_5_packets", "flows_6_10_packets",
    "flows_11_20_packets", "flows_21_50_packets", "flows_51_plus_packets",
]


def _read_pcap(d, big):
    e = ">" if big else "<"
    magic = struct.unpack(e + "I", d[:4])[0]
    nano = magic == 0xA1B23C4D
    linktype = struct.unpack(e + "I", d[20:24])[0] & 0x0FFFFFFF
    pkts = []
    o = 24
    while o + 16 <= len(d):
        s, frac, cl, wl = struct.unpack(e + "IIII", d[o:o + 16])
        o += 16
        us = frac // 1000 if nano else frac
        pkts.append((s, us, cl, wl, d[o:o + cl]))
        o += cl
    return _LINKTYPE_TO_DLT.get(linktype, linktype), pkts


def _read_pcapng(d):
    pkts = []
    ifaces = []  # (dlt, units_per_second)
    o = 0
    e = "<"
    while o + 12 <= len(d):
        btype = struct.unpack(e + "I", d[o:o + 4])[0]
        if btype == 0x0A0D0D0A:
            bom = d[o + 8:o + 12]
            e = "<" if bom == b"\x4d\x3c\x2b\x1a" else ">"
            ifaces = []
        blen = struct.unpack(e + "I", d[o + 4:o + 8])[0]
        body = d[o + 8:o + blen - 4]
        if btype == 1:  # IDB
            lt = struct.unpack(e + "H", body[0:2])[0]
            res = 1000000
            p = 8
            while p + 4 <= len(body):
                code, olen = struct.unpack(e + "HH", body[p:p + 4])
                if code == 0:
                    break
                if code == 9 and olen >= 1:
                    v = body[p + 4]
                    res = (2 ** (v & 0x7F)) if (v & 0x80) else 10 ** v
                p += 4 + ((olen + 3) & ~3)
            ifaces.append((_LINKTYPE_TO_DLT.get(lt, lt), res))
        elif btype == 6:  # EPB
            iid, th, tl, cl, wl = struct.unpack(e + "IIIII", body[:20])
            t = (th << 32) | tl
            res = ifaces[iid][1]
            sec, frac = divmod(t, res)
            if res != 1000000:
                dec = res == 10 ** (len(str(res)) - 1)
                frac = frac // (res // 1000000) if (dec and res > 1000000) else frac * 1000000 // res
            pkts.append((sec, frac, cl, wl, body[20:20 + cl]))
        elif btype == 3:  # SPB
            wl = struct.unpack(e + "I", body[:4])[0]
            pkts.append((0, 0, wl, wl, body[4:4 + wl]))
        o += blen
    dlt = ifaces[0][0] if ifaces else DLT_EN10MB
    return dlt, pkts


def read_capture(path):
    """Return (datalink, [(sec, usec, caplen, wirelen, bytes), ...])."""
    d = open(path, "rb").read()
    magic_le = struct.unpack("<I", d[:4])[0]
    if magic_le in (0xA1B2C3D4, 0xA1B23C4D):
        return _read_pcap(d, False)
    if magic_le in (0xD4C3B2A1, 0x4D3CB2A1):
        return _read_pcap(d, True)
    if magic_le == 0x0A0D0D0A:
        return _read_pcapng(d)
    raise ValueError("unknown capture format: %s" % path)


def to_batch(pkts, align=16):
    """Pack frames into (arena uint8, desc DESC_DTYPE) with aligned offsets; lengths are
    truncated to 16 bits exactly as the pcap plugin hands them to parse_packet."""
    desc = np.zeros(len(pkts), dtype=DESC_DTYPE)
    off = 0
    offs = []
    for i, (s, us, cl, wl, b) in enumerate(pkts):
        offs.append(off)
        off += (len(b) + align - 1) // align * align
    arena = np.zeros(max(off, align), dtype=np.uint8)
    for i, (s, us, cl, wl, b) in enumerate(pkts):
        arena[offs[i]:offs[i] + len(b)] = np.frombuffer(b, dtype=np.uint8)
        desc[i] = (offs[i], cl & 0xFFFF, wl & 0xFFFF, s, us)
    return arena, desc


# ---- UniRec logger text (reference tests/functional/scripts/run_test.sh) ----------------
def _ip(rec, which):
    b = bytes(rec[which])
    if rec["ip_version"] == 4:
        return socket.inet_ntop(socket.AF_INET, b[:4])
    return socket.inet_ntop(socket.AF_INET6, b)


def _mac(m):
    return ":".join("%02x" % x for x in bytes(m))


def _time(sec, usec):
    t = datetime.datetime.fromtimestamp(int(sec), datetime.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%S") + ".%06d" % int(usec)


BASIC_COLUMNS = ["DST_IP", "SRC_IP", "BYTES", "BYTES_REV", "LINK_BIT_FIELD", "TIME_FIRST",
                 "TIME_LAST", "DST_MAC", "SRC_MAC", "PACKETS", "PACKETS_REV", "DST_PORT",
                 "SRC_PORT", "DIR_BIT_FIELD", "PROTOCOL", "TCP_FLAGS", "TCP_FLAGS_REV"]


def basic_fields(rec):
    """The basic UniRec columns of one flow record, keyed by column name."""
    return {
        "DST_IP": _ip(rec, "dst_ip"), "SRC_IP": _ip(rec, "src_ip"),
        "BYTES": str(int(rec["src_bytes"])), "BYTES_REV": str(int(rec["dst_bytes"])),
        "LINK_BIT_FIELD": "0",
        "TIME_FIRST": _time(rec["time_first_sec"], rec["time_first_usec"]),
        "TIME_LAST": _time(rec["time_last_sec"], rec["time_last_usec"]),
        "DST_MAC": _mac(rec["dst_mac"]), "SRC_MAC": _mac(rec["src_mac"]),
        "PACKETS": str(int(rec["src_packets"])), "PACKETS_REV": str(int(rec["dst_packets"])),
        "DST_PORT": str(int(rec["dst_port"])), "SRC_PORT": str(int(rec["src_port"])),
        "DIR_BIT_FIELD": "0", "PROTOCOL": str(int(rec["ip_proto"])),
        "TCP_FLAGS": str(int(rec["src_tcp_flags"])),
        "TCP_FLAGS_REV": str(int(rec["dst_tcp_flags"])),
        "VLAN_ID": str(int(rec["vlan_id"])),
    }


def format_records(recs, columns=BASIC_COLUMNS):
    return [",".join(basic_fields(r)[c] for c in columns) for r in recs]


def read_golden(path, columns=BASIC_COLUMNS):
    """Project a reference golden output onto `columns`.  Fixed-size UniRec fields precede
    the variable ones (strings/bytes/arrays), so the first len(fixed) comma fields are
    unambiguous."""
    lines = open(path).read().splitlines()
    header = lines[-1].split(",")
    names = [h.split(" ", 1)[1] for h in header]
    types = [h.split(" ", 1)[0] for h in header]
    nfixed = 0
    for t in types:
        if t in ("string", "bytes") or t.endswith("*"):
            break
        nfixed += 1
    idx = [names.index(c) for c in columns]
    assert max(idx) < nfixed
    out = []
    for ln in lines[:-1]:
        f = ln.split(",", nfixed)
        out.append(",".join(f[i] for i in idx))
    return out
