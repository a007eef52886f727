"""Fronts launched ahead (round 5): ipxg_submit of a device batch behind a batch or ipxg_finish whose
control block the host has not read launches its k_bin / k_bin_slow first, gated on that block
(Params::gate_mode): when the pending batch needs the host (fragments, complex flows, deferrals)
the gated kernels return at once and the front is launched again after the host's work.  ipxg_finish
returns without waiting; the next call completes it, and ipxg_clear_exports behind it drops its
exports when it completes.  Records must equal the oracle's whichever way the gate goes."""
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


def _steps():
    """Six independent steps: plain, fragments (its completion needs the host: the next step's
    front launched ahead finds the gate closed), v6/VLAN, plain, fragments, plain."""
    out = []
    for k in range(6):
        a, d = synth.flow_stream(seed=60 + k, n_flows=150 + 20 * k, n_pkts=3000 + 400 * k,
                                 frag=k in (1, 4)).batch()
        out.append((a, d))
    return out


@pytest.mark.parametrize("clear_every", [0, 2])
def test_cold_steps_back_to_back(clear_every):
    """The bench's cold step (submit async device batch, finish, clear / poll) repeated with
    different batches: every polled step's records are exactly that batch's oracle records; a
    cleared step leaves nothing behind in the next poll."""
    from ipfixprobe_amd import Engine
    steps = _steps()
    dev = [_dev(a, d) for a, d in steps]
    with Engine() as e:
        for k, ((a, d), (da, dd)) in enumerate(zip(steps, dev)):
            e.submit(da, dd, device=True, asynchronous=True)
            e.finish()
            if clear_every and k % clear_every == 0:
                e.clear_exports()
                continue
            got = e.poll()
            want, _ = oracle_py.run_capture(a, d, 1, cache_exp=20)
            diff = flowcmp.diff(got, want)
            assert not diff, "step %d: %s" % (k, diff)
        st = e.stats()
    assert st["batches"] == len(steps)


def test_cleared_finish_that_needs_the_host():
    """i=1: every flow is complex, so the fused finish leaves them and its completion exports
    them through the sequential path and k_finish -- after ipxg_clear_exports was called
    behind it; those exports are dropped too, and the next step's are intact."""
    from ipfixprobe_amd import Engine
    (a1, d1), (a2, d2) = [synth.flow_stream(seed=70 + k, n_flows=90, n_pkts=2500, frag=False).batch()
                          for k in range(2)]
    want, _ = oracle_py.run_capture(a2, d2, 1, cache_exp=20, inactive=1)
    da1, dd1 = _dev(a1, d1)
    da2, dd2 = _dev(a2, d2)
    with Engine("i=1") as e:
        e.submit(da1, dd1, device=True, asynchronous=True)
        e.finish()
        e.clear_exports()
        e.submit(da2, dd2, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["complex_flows"] > 0
    diff = flowcmp.diff(got, want)
    assert not diff, diff


def test_order_check_across_batches_ahead():
    """A batch whose first packet is earlier than the previous batch's last one: the order check
    of a front launched ahead reads the previous timestamp from the pending batch's control block
    (Params::prev_dev) -- the batch goes to the sequential path and the records are the oracle's
    (which replays the packets in the given order)."""
    a, d = synth.flow_stream(seed=80, n_flows=120, n_pkts=4000, frag=False).batch()
    d = d.copy()
    # batch 2 (packets 1000..1999) starts 5 s before batch 1 ends
    d["ts_sec"][1000:2000] -= 5
    want, _ = oracle_py.run_capture(a, d, 1, cache_exp=20)
    from ipfixprobe_amd import Engine
    da, _ = _dev(a, d)
    keep = []
    with Engine() as e:
        for s in range(0, len(d), 1000):
            _, dd = _dev(a, d[s:s + 1000])
            keep.append(dd)
            e.submit(da, dd, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["complex_flows"] > 0
    diff = flowcmp.diff(got, want)
    assert not diff, diff


def test_no_ahead_knob_gives_the_same_records(monkeypatch):
    """IPXG_NO_AHEAD=1 / IPXG_SYNC_FINISH=1 (A/B knobs): the same records as the default path."""
    from ipfixprobe_amd import Engine
    steps = _steps()[:3]
    outs = []
    for env in ({}, {"IPXG_NO_AHEAD": "1", "IPXG_SYNC_FINISH": "1"}):
        for k in ("IPXG_NO_AHEAD", "IPXG_SYNC_FINISH"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        got = []
        with Engine() as e:
            for a, d in steps:
                da, dd = _dev(a, d)
                e.submit(da, dd, device=True, asynchronous=True)
                e.finish()
                got.append(e.poll())
        outs.append(got)
    for x, y in zip(*outs):
        diff = flowcmp.diff(x, y)
        assert not diff, diff


def _plain_then_mixed(seed):
    """Plain 64 B UDP frames (no slow-list packet: the next batch is launched without k_bin_slow),
    then a mixed stream (VLAN, IPv6, TCP options, fragments: slow-list packets), later in time."""
    rng = np.random.default_rng(seed)
    n = 3000
    sip = (10 << 24) + rng.integers(0, 150, n)
    dip = (192 << 24) + (168 << 16) + rng.integers(0, 40, n)
    a1, d1 = synth.udp_frames(sip, dip, rng.integers(1024, 1100, n), rng.integers(1, 30, n), t0=1_599_999_000)
    a2, d2 = synth.flow_stream(seed=seed, n_flows=120, n_pkts=3000, frag=True).batch()
    d2 = d2.copy()
    d2["offset"] += len(a1)
    return np.concatenate([a1, a2]), np.concatenate([d1, d2]), len(d1)


@pytest.mark.parametrize("mode", ["sync", "async", "finish"])
def test_slow_pass_skipped_then_needed(mode):
    """A batch launched without k_bin_slow (the previous batch listed no slow packet) whose k_bin
    does list some: k_reduce and k_fin_list return at once (BatchCtl::slow_redo) and the host runs
    k_bin_slow, k_reduce and k_fin_list again -- synchronous, asynchronous, and folded into a
    finish.  Records equal the oracle's; the redo is counted."""
    from ipfixprobe_amd import Engine
    arena, desc, k = _plain_then_mixed(91)
    if mode == "finish":  # two independent steps
        want = np.concatenate([oracle_py.run_capture(arena, desc[:k], 1, cache_exp=20)[0],
                               oracle_py.run_capture(arena, desc[k:], 1, cache_exp=20)[0]])
    else:
        want, _ = oracle_py.run_capture(arena, desc, 1, cache_exp=20)
    with Engine() as e:
        if mode == "sync":
            e.submit(arena, desc[:k])
            e.submit(arena, desc[k:])
            e.finish()
            got = e.poll()
        else:
            da, d1 = _dev(arena, desc[:k])
            _, d2 = _dev(arena, desc[k:])
            e.submit(da, d1, device=True, asynchronous=True)
            if mode == "finish":
                e.finish()
                g1 = e.poll()
            e.submit(da, d2, device=True, asynchronous=True)
            e.finish()
            got = e.poll() if mode == "async" else np.concatenate([g1, e.poll()])
        tm = e.timing()
    assert tm["slow_redos"] >= 1
    diff = flowcmp.diff(got, want)
    assert not diff, diff


@pytest.mark.parametrize("poll_every", [0, 2])
def test_async_expire_between_batches(poll_every):
    """ipxg_expire(now) behind each asynchronous batch (the streaming step): enqueued right behind
    the batch's tail, guarded, completed by the next call.  Records equal the oracle's (an expired
    record's flow splits at its next packet there too); the live count the engine keeps from
    k_expire's exports (no table recount) equals what the final finish exports."""
    from ipfixprobe_amd import Engine
    a, d = synth.flow_stream(seed=95, n_flows=200, n_pkts=6000, long_gap_share=0.02, frag=False).batch()
    want, _ = oracle_py.run_capture(a, d, 1, cache_exp=20)
    da, _ = _dev(a, d)
    keep, out = [], []
    with Engine() as e:
        for k, s in enumerate(range(0, len(d), 1000)):
            _, dd = _dev(a, d[s:s + 1000])
            keep.append(dd)
            e.submit(da, dd, device=True, asynchronous=True)
            e.expire(int(d["ts_sec"][min(s + 999, len(d) - 1)]))
            if poll_every and k % poll_every == 0:
                out.append(e.poll())
        out.append(e.poll())
        live = e.stats()["flows_in_cache"]
        e.finish()
        rest = e.poll()
        st = e.stats()
    assert st["end_inactive"] > 0  # (the stream's idle gaps: expired mid-stream)
    assert len(rest) == live
    diff = flowcmp.diff(np.concatenate(out + [rest]), want)
    assert not diff, diff


def test_slow_pass_needed_after_cleared_finish():
    """a plain batch's finish, ipxg_clear_exports (no poll, so the next submit
    launches its front ahead, gated on the finish's block), then an asynchronous batch with slow-list
    packets (its k_bin runs without k_bin_slow behind it and flags slow_redo).  The redo's k_bin_slow
    must not inherit the front's gate: the finish's block was re-zeroed by then and read as "closed",
    so the redo wrote nothing and k_reduce folded stale slow columns.  Records equal the oracle's for
    the second step."""
    from ipfixprobe_amd import Engine
    arena, desc, k = _plain_then_mixed(93)
    want, _ = oracle_py.run_capture(arena, desc[k:], 1, cache_exp=20)
    da, d1 = _dev(arena, desc[:k])
    _, d2 = _dev(arena, desc[k:])
    with Engine() as e:
        e.submit(da, d1, device=True, asynchronous=True)
        e.finish()
        e.clear_exports()
        e.submit(da, d2, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        tm = e.timing()
    assert tm["slow_redos"] >= 1
    diff = flowcmp.diff(got, want)
    assert not diff, diff


def test_order_check_behind_expire_ahead():
    """a batch whose first packet is earlier than the previous batch's last one,
    submitted right behind an asynchronous ipxg_expire (its front launched ahead, gated on the
    expire): the order check continues from the previous batch's last timestamp, as without the
    expire, so the batch goes to the sequential path (complex flows) and the records are the
    oracle's.  (No idle flow in the stream: the expires export nothing, as the oracle's run has none.)"""
    a, d = synth.flow_stream(seed=81, n_flows=120, n_pkts=4000, long_gap_share=0.0, frag=False).batch()
    d = d.copy()
    d["ts_sec"] = d["ts_sec"][0] + (d["ts_sec"] - d["ts_sec"][0]) // 25  # (564 s -> 22 s: no flow idle 30 s)
    d["ts_sec"][2000:3000] -= 3  # batch 3 starts 3 s before batch 2 ends
    want, _ = oracle_py.run_capture(a, d, 1, cache_exp=20)
    from ipfixprobe_amd import Engine
    da, _ = _dev(a, d)
    keep = []
    with Engine() as e:
        for s in range(0, len(d), 1000):
            _, dd = _dev(a, d[s:s + 1000])
            keep.append(dd)
            e.submit(da, dd, device=True, asynchronous=True)
            e.expire(int(d["ts_sec"][s:s + 1000].max()))
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["complex_flows"] > 0
    assert st["end_inactive"] == 0
    diff = flowcmp.diff(got, want)
    assert not diff, diff


@pytest.mark.parametrize("ahead", [True, False])
def test_rehash_behind_a_front_ahead(monkeypatch, ahead):
    """a small table (s=10) that the pending batch's post_batch grows by the load-
    factor rehash while the next batch's front, launched ahead, is already queued (its k_bin's spills
    merged into the old table, its k_reduce then runs on the new one): records equal the oracle's,
    with and without fronts ahead (IPXG_NO_AHEAD)."""
    if not ahead:
        monkeypatch.setenv("IPXG_NO_AHEAD", "1")
    a, d = synth.flow_stream(seed=83, n_flows=3000, n_pkts=12000, frag=False).batch()
    want, _ = oracle_py.run_capture(a, d, 1, cache_exp=20)
    from ipfixprobe_amd import Engine
    da, _ = _dev(a, d)
    keep = []
    with Engine("s=10") as e:
        for s in range(0, len(d), 2000):
            _, dd = _dev(a, d[s:s + 2000])
            keep.append(dd)
            e.submit(da, dd, device=True, asynchronous=True)
        e.finish()
        got = e.poll()
        st = e.stats()
    assert st["table_capacity"] > 1 << 10
    diff = flowcmp.diff(got, want)
    assert not diff, diff


def test_fused_finish_closes_export_holes():
    """A fused finish (an asynchronous device batch into an empty table, finished at once) writes its
    exports in list order from the export count the host knows (no reservation per workgroup pass).
    Flows that turn complex -- a SYN after a FIN/RST, a gap past the inactive timeout -- leave their
    records as holes, which k_ex_compact closes before the records are handed out
    (ipxg_timing.ex_compactions).  Every workgroup's passes mix both kinds.  Four steps on one
    engine: the first two without a poll between them (the second starts past the first's
    records), the third's exports cleared: the polled records are exactly the oracle's."""
    from ipfixprobe_amd import Engine
    steps = [synth.flow_stream(seed=95 + k, n_flows=1500, n_pkts=8000, frag=False).batch() for k in range(4)]
    wants = [oracle_py.run_capture(a, d, 1, cache_exp=20)[0] for a, d in steps]
    with Engine() as e:
        for k, (a, d) in enumerate(steps):
            da, dd = _dev(a, d)
            e.submit(da, dd, device=True, asynchronous=True)
            e.finish()
            if k == 2:
                e.clear_exports()
            if k in (1, 3):
                got = e.poll()
                want = np.concatenate([wants[0], wants[1]]) if k == 1 else wants[3]
                diff = flowcmp.diff(got, want)
                assert not diff, "step %d: %s" % (k, diff)
                assert len(got) == len(want)
        st, tm = e.stats(), e.timing()
    assert st["complex_flows"] > 0
    assert tm["ex_compactions"] >= 3


def test_two_engines_in_turn():
    """bench.py's two_engines: cold steps alternating between two engines on one GPU (each its own
    stream and table), submitted without waiting -- each engine's polled records are exactly the
    oracle records of its steps."""
    from ipfixprobe_amd import Engine
    steps = _steps()
    dev = [_dev(a, d) for a, d in steps]
    wants = [oracle_py.run_capture(a, d, 1, cache_exp=20)[0] for a, d in steps]
    with Engine() as e0, Engine() as e1:
        engs = (e0, e1)
        for k, (da, dd) in enumerate(dev):
            engs[k % 2].submit(da, dd, device=True, asynchronous=True)
            engs[k % 2].finish()
        for r in range(2):
            got = engs[r].poll()
            want = np.concatenate([wants[k] for k in range(r, len(steps), 2)])
            diff = flowcmp.diff(got, want)
            assert not diff, "engine %d: %s" % (r, diff)
