"""IPXG_BATCH_ASYNC: ipxg_submit of a device batch returns with the kernels enqueued; the next
call completes the batch (ipxg_finish runs speculatively behind it, held back on the device
by its guard when the batch needs the host).  Records must equal the synchronous path's
and the oracle's in every case: plain batches, batches that need the host (fragments,
deferrals, non-monotonic time, complex flows), and every entry point after an async batch."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))

import flowcmp  # noqa: E402
import oracle_py  # noqa: E402
import synth  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev(arena, desc):
    import torch
    a = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    d = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8).reshape(-1)).cuda()
    torch.cuda.synchronize()
    return a, d


def _run_async(arena, desc, params="", batch=None, poll_between=False):
    from ipfixprobe_amd import Engine
    a, _ = _dev(arena, desc)
    out = []
    with Engine(params) as e:
        n = len(desc)
        step = batch or n
        keep = []
        for s in range(0, n, step):
            _, d = _dev(arena, desc[s: s + step])
            keep.append(d)
            e.submit(a, d, device=True, asynchronous=True)
            if poll_between:
                out.append(e.poll())
        e.finish()
        out.append(e.poll())
        st = e.stats()
    return np.concatenate(out), st


CASES = [
    dict(seed=31, n_flows=200, n_pkts=5000, frag=False),                  # the fused fast path
    dict(seed=32, n_flows=150, n_pkts=5000, frag=True),                   # fragments: held
    dict(seed=33, n_flows=100, n_pkts=4000, frag=False, v6_share=0.5, vlan_share=0.4),
]


@pytest.mark.parametrize("batch", [None, 700])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_async_batches_match_oracle(ci, batch):
    arena, desc = synth.flow_stream(**CASES[ci]).batch()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got, _ = _run_async(arena, desc, batch=batch)
    d = flowcmp.diff(got, want)
    assert not d, d


def test_async_with_polls_between_batches():
    arena, desc = synth.flow_stream(seed=34, n_flows=120, n_pkts=4000, frag=False).batch()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got, _ = _run_async(arena, desc, batch=500, poll_between=True)
    d = flowcmp.diff(got, want)
    assert not d, d


def test_async_finish_held_by_complex_flows():
    """i=1: every flow goes through the sequential path (complex), so the guard must hold
    the speculative k_finish back."""
    arena, desc = synth.flow_stream(seed=35, n_flows=80, n_pkts=3000, frag=False).batch()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20, inactive=1)
    got, st = _run_async(arena, desc, params="i=1")
    assert st["complex_flows"] > 0
    d = flowcmp.diff(got, want)
    assert not d, d


def _growth_capture():
    rng = np.random.default_rng(6)
    frames = []
    for i in range(60_000):
        f = synth.pad(synth.eth(synth.mac(1), synth.mac(2), 0x0800) +
                      synth.ipv4(synth.ip4(0x0A000000 + i), synth.ip4(0xC0A80001), 17,
                                 synth.udp(int(rng.integers(1024, 65536)), 53)))
        frames.append((f, len(f), len(f)))
    return synth.to_batch(frames)


def test_async_table_growth():
    """A batch that outgrows the table (deferred packets, rehash) right before finish: behind a
    first batch whose flows are still live, so the finish cannot be folded into the batch's
    tail and the 60k flows need slots in the 2^14 table."""
    from ipfixprobe_amd import Engine
    arena, desc = _growth_capture()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    a, _ = _dev(arena, desc)
    with Engine("s=14") as e:
        _, d1 = _dev(arena, desc[:1000])
        _, d2 = _dev(arena, desc[1000:])
        e.submit(a, d1, device=True, asynchronous=True)
        e.submit(a, d2, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["table_rehashes"] >= 1
    d = flowcmp.diff(got, want)
    assert not d, d


def test_async_fused_finish_needs_no_slots():
    """The same 60k flows as one asynchronous batch into an empty 2^14 table, finished at once:
    the finish is folded into the batch's tail, which exports each new flow without a slot --
    no deferral, no table growth -- and the records are the oracle's."""
    arena, desc = _growth_capture()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    got, st = _run_async(arena, desc, params="s=14")
    assert st["table_rehashes"] == 0
    d = flowcmp.diff(got, want)
    assert not d, d


def test_async_then_expire_stats_and_sync_submit():
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(seed=36, n_flows=100, n_pkts=3000, frag=False).batch()
    half = len(desc) // 2
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    a, d1 = _dev(arena, desc[:half])
    with Engine() as e:
        e.submit(a, d1, device=True, asynchronous=True)
        st = e.stats()  # completes the batch
        assert st["parsed_packets"] == half
        e.submit(arena, desc[half:])  # a synchronous host batch after it
        e.finish()
        got = e.poll()
    d = flowcmp.diff(got, want)
    assert not d, d


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_async_host_batches_double_buffered(ci, pinned):
    """Host batches with IPXG_BATCH_ASYNC: each copied into one of two device staging slots on
    the copy stream while the previous batch is in the kernels.  Every batch is a separate
    host array (kept alive until the next call, as the contract asks)."""
    import torch
    from ipfixprobe_amd import Engine
    arena, desc = synth.flow_stream(**CASES[ci]).batch()
    want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    step = 600
    keep = []
    with Engine() as e:
        for s in range(0, len(desc), step):
            d = np.ascontiguousarray(desc[s:s + step])
            if pinned:
                a_h = torch.from_numpy(np.ascontiguousarray(arena)).pin_memory()
                d_h = torch.from_numpy(d.view(np.uint8).reshape(-1)).pin_memory()
            else:
                a_h, d_h = np.ascontiguousarray(arena), d
            keep.append((a_h, d_h))
            e.submit(a_h, d_h, asynchronous=True)
        e.finish()
        got = e.poll()
    d = flowcmp.diff(got, want)
    assert not d, d
