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


def _header_functions():
    src = open(os.path.join(ROOT, "include", "ipxg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(ipxg_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from ipfixprobe_amd import engine
    L = engine.lib()
    funcs = _header_functions()
    assert len(funcs) >= 20
    for f in funcs:
        assert hasattr(L, f), f
    assert set(engine.EXPORTED_SYMBOLS) <= set(funcs)


def test_struct_layouts_match_header_and_test_restatement():
    from ipfixprobe_amd import engine
    assert engine.DESC_DTYPE == pcaputil.DESC_DTYPE and engine.DESC_DTYPE.itemsize == 16
    assert engine.FLOW_DTYPE == pcaputil.FLOW_DTYPE and engine.FLOW_DTYPE.itemsize == 128
    assert engine.PARSED_DTYPE == pcaputil.PARSED_DTYPE and engine.PARSED_DTYPE.itemsize == 112
    assert ctypes.sizeof(engine.Config) == 48
    assert engine.STATS_FIELDS == pcaputil.STATS_FIELDS


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
    for bad in ("s=3", "s=31", "x=1", "fe=yes", "fs=0", "a=", "batch=0"):
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
