"""The oracle (CPU restatement, oracle/ipxg_oracle.c) against the reference's own golden
outputs: tests/functional/outputs/* produced by ipfixprobe from tests/functional/inputs/*
(copied unchanged under tests/golden/reference/).  This pins the oracle before any GPU
result is compared with it."""
import ctypes
import os
from collections import Counter

import numpy as np
import pytest
import xxhash

import oracle_py
import pcaputil

REF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference")

# golden output -> capture, per reference tests/functional/CMakeLists.txt:14-35
PAIRS = {
    "basic": "mixed", "basicplus": "http", "bstats": "bstats", "dns": "dns", "dnssd": "dnssd",
    "http": "http", "idpcontent": "idpcontent", "mqtt": "mqtt", "netbios": "netbios",
    "ovpn": "ovpn", "passivedns": "dns", "phists": "mixed", "pstats": "mixed",
    "quic": "quic_initial-sample", "smtp": "smtp", "ssadetector": "ovpn", "ssdp": "ssdp",
    "tls": "tls", "vlan": "vlan", "wg": "wg", "sip": "sip", "rtsp": "rtsp", "ntp": "ntp",
    "nettisa": "mixed",
}
# basic columns identical to the reference output (no process plugin changes flow boundaries)
EQUAL = ["basic", "basicplus", "dnssd", "http", "idpcontent", "mqtt", "phists", "pstats",
         "quic", "ssdp", "vlan"]
# golden basic columns are a sub-multiset (the plugin test keeps only flows it matched)
SUBSET = ["bstats", "nettisa", "ovpn", "smtp", "ssadetector", "tls"]
# dns, passivedns, ntp, sip, rtsp, wg, netbios: plugins return FLOW_FLUSH(_WITH_REINSERT)
# (dns.cpp:127, ntp.cpp:86, sip.cpp:91, rtsp.cpp:121, wg.cpp:94 ...) or unirec emits one row
# per extension -- outside the core path, not compared.


def _columns(name):
    return pcaputil.BASIC_COLUMNS + (["VLAN_ID"] if name == "vlan" else [])


def _run(capture):
    dl, pk = pcaputil.read_capture(os.path.join(REF, capture + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    recs, st = oracle_py.run_capture(arena, desc, dl)
    return recs, st


@pytest.mark.parametrize("name", EQUAL)
def test_oracle_equals_reference_golden(name):
    recs, st = _run(PAIRS[name])
    cols = _columns(name)
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name), cols))
    mine = Counter(pcaputil.format_records(recs, cols))
    assert mine == gold
    assert st["end_no_res"] == 0


@pytest.mark.parametrize("name", SUBSET)
def test_oracle_superset_of_plugin_golden(name):
    recs, _ = _run(PAIRS[name])
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", name)))
    mine = Counter(pcaputil.format_records(recs))
    assert not (gold - mine)


def test_mixed_parser_counters():
    # mixed.pcap: 205 frames, 48 ARP frames are dropped by parse_packet (unknown ethertype)
    recs, st = _run("mixed")
    assert st["seen_packets"] == 205
    assert st["parsed_packets"] == 157
    assert st["unknown_packets"] == 48
    assert sum(int(r["src_packets"]) + int(r["dst_packets"]) for r in recs) == 157


def _ref_xxh64():
    path = os.path.join(os.path.dirname(REF), "..", "..", "oracle", "_ref", "libxxhash_ref.so")
    path = os.path.normpath(path)
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    L.XXH64.restype = ctypes.c_uint64
    L.XXH64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    return L


def test_xxh64_vectors():
    """oracle_xxh64 == python xxhash 3.8.1 == the reference's own xxhash.c (oracle/_ref)."""
    rng = np.random.default_rng(1234)
    ref = _ref_xxh64()
    for n in list(range(0, 80)) + [100, 128, 255, 1000]:
        for seed in (0, 1, 0xFFFFFFFFFFFFFFFF):
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            want = xxhash.xxh64_intdigest(b, seed)
            assert oracle_py.xxh64(b, seed) == want
            if ref is not None:
                buf = ctypes.create_string_buffer(b, max(n, 1))
                assert ref.XXH64(buf, n, seed) == want


def test_xxh64_golden_file(golden_dir):
    """Committed vectors (tests/golden/xxh64_vectors.json, made by gen_golden.py)."""
    import json
    with open(os.path.join(golden_dir, "xxh64_vectors.json")) as f:
        vecs = json.load(f)
    for v in vecs:
        assert oracle_py.xxh64(bytes.fromhex(v["key"]), v["seed"]) == int(v["hash"], 16)
