"""BASELINE.json configs[0]: a 1k-packet 64 B UDP pcap through the whole plumbing -- the
capture reader, the gpucache storage plugin, and IPFIX output (the reference's pcap input +
cache + ipfix output pipeline).  The fixture and its expected flow records are made by
tests/golden/gen_config0.py (the expected records come from the oracle, itself pinned by the
reference's functional-test goldens)."""
import os
import subprocess

import numpy as np
import pytest

import ipfixdec
import oracle_py
import pcaputil

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PCAP = os.path.join(HERE, "golden", "config0_udp64.pcap")
GOLD = os.path.join(HERE, "golden", "config0_udp64.csv")
PROBE = os.path.join(ROOT, "ipfixprobe_amd", "ipxg_probe")


def _gold():
    with open(GOLD) as f:
        return sorted(line.rstrip("\n") for line in f)


def test_fixture_is_the_config_and_matches_oracle():
    dl, pk = pcaputil.read_capture(PCAP)
    assert dl == 1 and len(pk) == 1000
    assert all(p[2] == 64 and p[3] == 64 for p in pk)  # caplen == wirelen == 64
    arena, desc = pcaputil.to_batch(pk)
    recs, st = oracle_py.run_capture(arena, desc, dl)  # the reference's default cache size
    assert st["end_no_res"] == 0 and st["udp_packets"] == 1000
    assert sorted(pcaputil.format_records(recs)) == _gold()


@pytest.mark.gpu
def test_config0_pcap_to_csv_through_probe():
    out = subprocess.run([PROBE, "-i", PCAP], check=True, stdout=subprocess.PIPE, text=True, timeout=120).stdout
    assert sorted(out.splitlines()) == _gold()


@pytest.mark.gpu
def test_config0_pcap_to_ipfix_through_probe(tmp_path):
    """pcap -> ipxg_probe (GpuFlowCache) -> IPFIX messages formatted on the device: the stream
    decodes to the expected flow records, and it is byte for byte what the reference exporter
    (oracle restatement of IPFIXExporter) emits for those records in the stream's order."""
    path = str(tmp_path / "out.ipfix")
    subprocess.run([PROBE, "-i", PCAP, "-o", "ipfix:" + path, "--odid", "7", "--export-time", "1700000100"],
                   check=True, timeout=120)
    data = np.fromfile(path, dtype=np.uint8)
    msgs, tmpl, recs, where, dirs = ipfixdec.decode(data)
    assert len(recs) == 100 and msgs[0]["sets"][0][0] == 2
    assert all(m["odid"] == 7 and m["export_time"] == 1700000100 and m["length"] <= 1458 for m in msgs[1:])
    recs["end_reason"] = 4  # FORCED at finish; the golden text form has no end reason
    assert sorted(pcaputil.format_records(recs)) == _gold()
    want, nm = oracle_py.ipfix_export(oracle_py.ipfix_exporter(odid=7, export_time=1700000100), recs)
    assert nm == len(msgs) and bytes(want) == bytes(data)
