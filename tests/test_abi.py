"""CPU-side checks of the boundary: libipxg loads and exports every symbol include/ipxg.h
declares, the struct layouts agree with the header, option strings parse like the
reference's CacheOptParser, and the C++ capture reader agrees with the test reader."""
import ctypes
import os
import re

import numpy as np
import pytest

import pcaputil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "tests", "golden", "reference")


def _header_functions(name="ipxg.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(ipxg_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from ipfixprobe_amd import engine
    L = engine.lib()
    funcs = _header_functions()
    assert len(funcs) >= 20
    for f in funcs:
        assert hasattr(L, f), f
    assert set(engine.EXPORTED_SYMBOLS) <= set(funcs)


def test_stdplugins_library_exports_its_header():
    """libipxg_stdplugins.so (the native stand-in process plugins) exports every function
    include/ipxg_stdplugins.h declares, and the plugin struct is ABI 2's (masked prefixes,
    follow_packets appended)."""
    from ipfixprobe_amd import engine
    L = ctypes.CDLL(engine.STD_LIB_PATH)
    funcs = _header_functions("ipxg_stdplugins.h")
    assert funcs == ["ipxg_std_plugin", "ipxg_std_plugin_calls", "ipxg_std_plugin_free"]
    for f in funcs:
        assert hasattr(L, f), f
    assert ctypes.sizeof(engine.Plugin) == 664  # = sizeof(ipxg_plugin), gcc x86-64 (ABI 7: follow_bytes fills the padding)
    p = engine.StdPlugin("quic")
    assert p.struct.masked == 1 and p.struct.prefix_mask[0][0] == 0x80 and p.struct.follow_packets == 30
    with pytest.raises(engine.IpxgError):
        engine.StdPlugin("nope")


def test_struct_layouts_match_header_and_test_restatement():
    from ipfixprobe_amd import engine
    assert engine.DESC_DTYPE == pcaputil.DESC_DTYPE and engine.DESC_DTYPE.itemsize == 16
    assert engine.FLOW_DTYPE == pcaputil.FLOW_DTYPE and engine.FLOW_DTYPE.itemsize == 128
    assert engine.PARSED_DTYPE == pcaputil.PARSED_DTYPE and engine.PARSED_DTYPE.itemsize == 120
    assert ctypes.sizeof(engine.Config) == 48
    assert engine.STATS_FIELDS == pcaputil.STATS_FIELDS
    assert engine.VLAN_STATS_DTYPE == pcaputil.VLAN_STATS_DTYPE and engine.VLAN_STATS_DTYPE.itemsize == 224
    assert engine.PORT_STAT_DTYPE.itemsize == 16


def test_config_defaults_and_options():
    from ipfixprobe_amd import IpxgError, make_config
    c = make_config()
    assert (c.cache_exp, c.line_exp, c.active_s, c.inactive_s, c.split_biflow, c.frag_enable,
            c.frag_size, c.frag_timeout_s) == (17, 4, 300, 30, 0, 1, 10007, 3)
    c = make_config("size=20;line=3;active=60;inactive=10;split;frag-enable=false;frag-size=7;frag-timeout=1")
    assert (c.cache_exp, c.line_exp, c.active_s, c.inactive_s, c.split_biflow, c.frag_enable,
            c.frag_size, c.frag_timeout_s) == (20, 3, 60, 10, 1, 0, 7, 1)
    c = make_config("s;22;a;5")  # value as the next token (options.cpp:128-135)
    assert (c.cache_exp, c.active_s) == (22, 5)
    c = make_config("dev=3;batch=4096;dlt=LINUX_SLL")
    assert (c.device_id, c.batch_pkts, c.datalink) == (3, 4096, 113)
    assert make_config("walk=wide").flags == 0x2 and make_config("walk=narrow").flags == 0x4
    assert make_config("ps=true").flags == 0x8 and make_config("parser-stats=true;ps=false").flags == 0
    assert make_config("walk=wide;walk=auto").flags == 0 and make_config("ingest=atomic;walk=wide").flags == 0x3
    assert make_config("strict=true").flags == 0x10 and make_config("strict=true;strict=false").flags == 0
    for bad in ("s=3", "s=31", "x=1", "fe=yes", "fs=0", "a=", "batch=0", "walk=deep", "ps=1", "strict=1"):
        with pytest.raises(IpxgError):
            make_config(bad)


@pytest.mark.parametrize("name", sorted(f[:-5] for f in os.listdir(REF) if f.endswith(".pcap")))
def test_capture_reader_matches_test_reader(name):
    from ipfixprobe_amd import load_capture
    arena, desc, dl = load_capture(os.path.join(REF, name + ".pcap"))
    dl2, pk = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
    a2, d2 = pcaputil.to_batch(pk)
    assert dl == dl2
    assert np.array_equal(desc, d2)
    assert np.array_equal(arena[: len(a2)], a2)


def test_no_gpu_fails_loudly():
    """Without a GPU the product refuses to run (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ipfixprobe_amd import Engine, IpxgError
    with pytest.raises(IpxgError):
        Engine()


def _pcapng(path, tsresol, stamps):
    """A little-endian pcapng: SHB, one Ethernet IDB with if_tsresol = tsresol (None: no
    option), one EPB per raw timestamp in `stamps` (a 60-byte frame each)."""
    import struct

    def block(bt, body):
        body = body + b"\0" * ((4 - len(body) % 4) % 4)
        n = 12 + len(body)
        return struct.pack("<II", bt, n) + body + struct.pack("<I", n)

    out = block(0x0A0D0D0A, struct.pack("<IHHq", 0x1A2B3C4D, 1, 0, -1))
    opts = b""
    if tsresol is not None:
        opts = struct.pack("<HH", 9, 1) + bytes([tsresol]) + b"\0\0\0" + struct.pack("<HH", 0, 0)
    out += block(1, struct.pack("<HHI", 1, 0, 65535) + opts)
    frame = bytes(12) + b"\x08\x00" + bytes(46)
    for t in stamps:
        out += block(6, struct.pack("<IIIII", 0, t >> 32, t & 0xFFFFFFFF, len(frame), len(frame)) + frame)
    with open(path, "wb") as f:
        f.write(out)


@pytest.mark.parametrize("tsresol,unit", [(None, 10**6), (9, 10**9), (3, 10**3), (0x94, 2**20), (0x8A, 2**10),
                                          (0xBF, 2**63)])
def test_pcapng_tsresol_conversion(tmp_path, tsresol, unit):
    """if_tsresol as libpcap converts it: a decimal resolution finer than 1 us divides by the
    power of ten, anything else scales frac * 10^6 / resolution (binary 2^-20 was
    left unscaled)."""
    from ipfixprobe_amd import load_capture
    stamps = [unit - 1, unit, unit + unit // 2 + 1, 3 * unit + 12345 % unit if unit < 2**62 else unit + 7]
    p = str(tmp_path / "t.pcapng")
    _pcapng(p, tsresol, stamps)
    _, desc, _ = load_capture(p)
    _, pk = pcaputil.read_capture(p)
    want = [(t // unit, (t % unit) * 10**6 // unit) for t in stamps]
    assert [(int(d["ts_sec"]), int(d["ts_usec"])) for d in desc] == want
    assert [(k[0], k[1]) for k in pk] == want
    assert all(u < 10**6 for _, u in want)


@pytest.mark.parametrize("tsresol", [20, 64, 0x7F, 0xC0, 0xFF])
def test_pcapng_tsresol_out_of_range_is_rejected(tmp_path, tsresol):
    """A resolution of 10^20 or 2^64 and beyond does not fit 64 bits: the reader rejects the
    capture (IPXG_EIO) instead of dividing by zero / shifting out of range."""
    from ipfixprobe_amd import IpxgError, load_capture
    p = str(tmp_path / "t.pcapng")
    _pcapng(p, tsresol, [123456789])
    with pytest.raises(IpxgError):
        load_capture(p)
