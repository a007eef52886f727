"""Device parity: the HIP path (libipxg through its C-ABI) against the oracle and the
reference's golden outputs.  Integer work, so the bar is bit-exact."""
import json
import os
import subprocess
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py
import pcaputil

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.path.join(HERE, "golden", "reference")
ROOT = os.path.dirname(HERE)
CAPTURES = sorted(f[:-5] for f in os.listdir(REF) if f.endswith(".pcap"))


@pytest.fixture(scope="module")
def eng():
    from ipfixprobe_amd import Engine
    e = Engine()
    yield e
    e.close()


def _load(name):
    dl, pk = pcaputil.read_capture(os.path.join(REF, name + ".pcap"))
    arena, desc = pcaputil.to_batch(pk)
    return dl, arena, desc


def test_xxh64_device_golden(eng, golden_dir):
    with open(os.path.join(golden_dir, "xxh64_vectors.json")) as f:
        vecs = json.load(f)
    for keylen in sorted({len(v["key"]) // 2 for v in vecs}):
        for seed in (0, 7):
            sel = [v for v in vecs if len(v["key"]) // 2 == keylen and v["seed"] == seed]
            if not sel:
                continue
            keys = np.frombuffer(b"".join(bytes.fromhex(v["key"]) for v in sel), dtype=np.uint8)
            got = eng.xxh64(keys if keylen else np.zeros(0, np.uint8), keylen, seed) if keylen else None
            if keylen == 0:
                continue
            want = np.array([int(v["hash"], 16) for v in sel], dtype=np.uint64)
            assert np.array_equal(got, want), keylen


PARSE_FIELDS = [n for n in pcaputil.PARSED_DTYPE.names]


def _parse_cmp(eng, arena, desc, dl):
    from ipfixprobe_amd import Engine
    e = Engine(datalink=dl) if dl != 1 else eng
    got = e.parse(arena, desc)
    want, beyond = oracle_py.parse_batch(arena, desc, dl)
    if e is not eng:
        e.close()
    bad = []
    for i in range(len(desc)):
        if beyond[i]:
            continue  # the reference reads past caplen here (undefined behaviour)
        for f in PARSE_FIELDS:
            if f == "valid" or want[i]["valid"]:
                if not np.array_equal(got[i][f], want[i][f]):
                    bad.append((i, f, got[i][f], want[i][f]))
    return bad, int(beyond.sum())


@pytest.mark.parametrize("name", CAPTURES)
def test_parse_fixture(eng, name):
    dl, arena, desc = _load(name)
    bad, _ = _parse_cmp(eng, arena, desc, dl)
    assert not bad, bad[:10]


@pytest.mark.parametrize("batch", [None, 1, 7, 64])
@pytest.mark.parametrize("name", CAPTURES)
def test_flows_fixture(name, batch):
    from ipfixprobe_amd import run_capture
    dl, arena, desc = _load(name)
    want, wst = oracle_py.run_capture(arena, desc, dl)
    got, gst = run_capture(arena, desc, datalink=dl, batch=batch)
    assert wst["end_no_res"] == 0
    d = flowcmp.diff(got, want)
    assert not d, d
    for k in ("seen_packets", "parsed_packets", "unknown_packets", "ipv4_packets", "ipv6_packets",
              "tcp_packets", "udp_packets", "vlan_packets"):
        assert gst[k] == wst[k], k


@pytest.mark.parametrize("mode", [[], ["-q", "7"], ["--mbuf"], ["--mbuf", "-q", "32"]])
def test_basic_golden_through_probe_cli(mode):
    """The C++ host path end to end: ipxg_probe (the raw-ingest input plugin "pcapraw" ->
    input_storage_worker blocks -> GpuFlowCache::put_pkt -> finish) reproduces the reference's
    outputs/basic for mixed.pcap; --mbuf: every block as a DPDK rx burst of mbufs through the
    burst adapter (rawinput.hpp burst_to_block, dpdk.cpp:196-225)."""
    exe = os.path.join(ROOT, "ipfixprobe_amd", "ipxg_probe")
    out = subprocess.run([exe, "-i", os.path.join(REF, "mixed.pcap")] + mode, check=True,
                         stdout=subprocess.PIPE, text=True, timeout=120).stdout
    got = Counter(out.splitlines())
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", "basic")))
    assert got == gold


@pytest.mark.parametrize("mode", [[], ["--mbuf"]])
def test_vlan_golden_through_probe_cli(mode):
    exe = os.path.join(ROOT, "ipfixprobe_amd", "ipxg_probe")
    out = subprocess.run([exe, "-i", os.path.join(REF, "vlan.pcap"), "-o", "csv-vlan"] + mode, check=True,
                         stdout=subprocess.PIPE, text=True, timeout=120).stdout
    cols = pcaputil.BASIC_COLUMNS[:13] + ["VLAN_ID"] + pcaputil.BASIC_COLUMNS[13:]
    gold = Counter(pcaputil.read_golden(os.path.join(REF, "outputs", "vlan"), cols))
    assert Counter(out.splitlines()) == gold


@pytest.mark.parametrize("name", ["http", "quic", "mqtt"])
def test_probe_cli_raw_and_mbuf_inputs_match_oracle(name):
    """Other reference captures (one Linux-SLL, nanosecond) through both raw inputs: the basic
    columns of every record equal the oracle's."""
    from test_oracle_golden import PAIRS
    exe = os.path.join(ROOT, "ipfixprobe_amd", "ipxg_probe")
    path = os.path.join(REF, PAIRS[name] + ".pcap")
    dl, pk = pcaputil.read_capture(path)
    arena, desc = pcaputil.to_batch(pk)
    want, _ = oracle_py.run_capture(arena, desc, dl)
    for mode in ([], ["--mbuf"]):
        out = subprocess.run([exe, "-i", path] + mode, check=True, stdout=subprocess.PIPE, text=True,
                             timeout=120).stdout
        assert Counter(out.splitlines()) == Counter(pcaputil.format_records(want)), mode
