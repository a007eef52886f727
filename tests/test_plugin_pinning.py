"""The bench's process-plugin stand-ins (ipfixprobe_amd/host/ipxg_stdplugins.c: the flush / claim
decisions of dns.cpp, http.cpp, tls.cpp and quic.cpp restated in C -- bench.py may not load
anything under oracle/) pinned to the reference's own plugins (oracle/_ref/libref_plugins.so:
their unmodified sources behind the adapter) on the workload mixes, not only on the golden
captures: over the same 600k packets of the configs[2] IMIX mix (dns, http,
tls) and of the configs[4] QUIC mix (quic), the oracle with the stand-ins and the oracle with
the real plugins give the same records -- the plugins' flushes set the flow boundaries -- and the
same set of flows carrying an extension (the flows a plugin claimed, which the bridge keeps on
the host walk).  CPU only: the packets come from the generator's host restatement
(synthgen.host_batch, which test_gpu_workloads pins to the device generator byte for byte)."""
import os
import sys
from collections import Counter

import numpy as np
import pytest

import flowcmp
import oracle_py

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_plugins.so")

PLUGINS = {"imix": ("dns", "http", "tls"), "quic": ("quic",)}  # bench.py --plugins config


class _G:
    """synthgen.Generator's parameters without a device (host_batch reads only these)."""

    def __init__(self, mix, seed=1234):
        self.mix, self.seed, self.t0_ns, self.dt_ns = mix, seed, 1_700_000_000 * 10**9, 100
        self.q16 = [int(round(x * 65536)) for x in (0.55, 0.005, 0.045)]


def _run(arena, desc, plugins):
    c = oracle_py.OracleCache(cache_exp=22)
    for p in plugins:
        c.add_plugin(p.struct)
    c.run(arena, desc, 1)
    c.finish()
    recs = c.take()
    st = c.stats()
    c.close()
    return recs, st


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref/libref_plugins.so not built")
@pytest.mark.parametrize("name", sorted(PLUGINS))
def test_stand_ins_decide_like_reference_plugins_on_mix(name):
    import synthgen
    import test_ref_plugins
    from ipfixprobe_amd.engine import StdPlugin
    mix = synthgen.Mix(name, 1_000_000, seed=1234, zipf=1.1 if name == "imix" else None)
    arena, desc = synthgen.host_batch(_G(mix), 0, 600_000)
    std = [StdPlugin(p) for p in PLUGINS[name]]
    a, ast = _run(arena, desc, std)
    ref = [test_ref_plugins.RefPlugin(p) for p in PLUGINS[name]]
    b, bst = _run(arena, desc, ref)
    claimed_ref = Counter(flowcmp.rec_key(r) for r in b[b["ext"] != 0])
    test_ref_plugins.take_texts(b)  # (releases the real plugins' Flow objects)
    assert ast["end_no_res"] == 0 and bst["end_no_res"] == 0
    d = flowcmp.diff(a, b)  # flush boundaries: every record (contract fields) equal
    assert not d, d
    claimed_std = Counter(flowcmp.rec_key(r) for r in a[a["ext"] != 0])
    assert claimed_std == claimed_ref
    assert len(claimed_ref) > 1000, len(claimed_ref)  # the mix gives the plugins flows to claim
