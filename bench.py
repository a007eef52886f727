"""bench.py -- device-resident packet->biflow throughput on MI355X.

Workloads (BASELINE.json configs; `--workload`):
  udp64  configs[1] (default, the metric's config): per GPU, 10M synthetic 64 B
         Ethernet/IPv4/UDP frames (tot_len 50) over 100k distinct biflows (src 10/8, dst
         192.168/16, sport 1024-65535, dport 1-1023; each packet picks a direction at random).
         `--mode cold` (default): a step = ipxg_submit + ipxg_finish of the batch (every flow
         exported FORCED), timestamps 1 us apart.  `--mode stream`: a step = one batch of a
         continuing stream (timestamps 100 ns apart, batch k starts where k-1 ended), flows
         carried across batches, plus ipxg_expire(now) on the virtual clock -- the steady state.
  imix   configs[2]: IMIX 64/594/1518 B (7:4:1), Zipf(1.1) popularity over 1M flows, TCP (most
         with timestamp options) / UDP, TLS/HTTP/DNS payload prefixes, some IPv6 and 802.1Q
         (tools/synth); a step = 100M packets as 10 batches of 10M submitted back to back
         (flows carried across batches) + finish.  The TLS/HTTP/DNS process plugins run on the
         host above the C-ABI and are not part of this device measurement.
  quic   configs[4]: QUIC-heavy variable-length mix over 1M flows (60 % UDP/443 QUIC, 40 %
         802.1Q/QinQ/MPLS/IPv6-ext/PPPoE/GRE encapsulations; tools/synth); a step = 4 batches of
         5M + finish.
With N GPUs each rank owns a disjoint range of the canonical flow hash (the NIC-RSS analogue,
SURVEY 8(e)): every rank generates packets of its own flows only, so the data path has no
collective; at N > 1 the per-GPU export buffers are gathered to rank 0 over RCCL inside the step
(the path's only exchange).

Prints one JSON line (rank 0).  roofline.achieved = algorithmic bytes per launch of the dominant
ingest kernel (min(caplen, 128) + 16 B descriptor per packet, 80 B for 64 B frames)
/ its average duration from HIP events on the engine's stream; roofline.step = the same bytes
over the whole step (every kernel, the host round trips, the finish).  roofline.traffic is the
HBM bytes per launch of that kernel from the newest committed rocprofv3 PMC summary
(profiles/*/pmc_summary*.json for this workload, collected by tools/gpu_pmc.sh), or null.
"""
import argparse
import glob
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkts/s device-resident, 64B synthetic mix, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
DESC_NP = np.dtype([("offset", "<u4"), ("caplen", "<u2"), ("wirelen", "<u2"), ("ts_sec", "<u4"), ("ts_usec", "<u4")])


def gen_flows(F, rank, world, seed, device_id=0):
    """F distinct 64 B-UDP biflows whose canonical hash falls in this rank's range (hashed on
    this rank's GPU)."""
    from ipfixprobe_amd import Engine, shard
    rng = np.random.default_rng(seed)
    out = {k: [] for k in ("sip", "dip", "sport", "dport")}
    have = 0
    seen = set()
    with Engine(device_id=device_id) as e:
        while have < F:
            m = max(2 * (F - have) * world, 1024)
            sip = (10 << 24) | rng.integers(0, 1 << 24, m, dtype=np.uint64)
            dip = (192 << 24) | (168 << 16) | rng.integers(0, 1 << 16, m, dtype=np.uint64)
            sp = rng.integers(1024, 65536, m, dtype=np.uint64)
            dp = rng.integers(1, 1024, m, dtype=np.uint64)
            keys = np.zeros((m, 16), dtype=np.uint8)
            inv = np.zeros((m, 16), dtype=np.uint8)
            for k, (a, b, pa, pb) in ((keys, (sip, dip, sp, dp)), (inv, (dip, sip, dp, sp))):
                k[:, 0] = pa & 0xFF
                k[:, 1] = pa >> 8
                k[:, 2] = pb & 0xFF
                k[:, 3] = pb >> 8
                k[:, 4] = 17
                k[:, 5] = 4
                for q in range(4):  # addresses in network byte order
                    k[:, 6 + q] = (a >> (24 - 8 * q)) & 0xFF
                    k[:, 10 + q] = (b >> (24 - 8 * q)) & 0xFF
            hf = e.xxh64(keys.reshape(-1), 16)
            hi = e.xxh64(inv.reshape(-1), 16)
            own = shard.owner(shard.canonical(hf, hi), world)
            for j in np.nonzero(own == rank)[0]:
                t = (int(sip[j]), int(dip[j]), int(sp[j]), int(dp[j]))
                if t in seen or (t[1], t[0], t[3], t[2]) in seen:
                    continue
                seen.add(t)
                for key, v in zip(("sip", "dip", "sport", "dport"), t):
                    out[key].append(v)
                have += 1
                if have == F:
                    break
    return {k: np.array(v, dtype=np.int64) for k, v in out.items()}


def build_batch(flows, P, seed, device, dt_ns=1000, t0_pkt=0):
    """64 B frames (P, 64) uint8 and descriptors (P, 16) uint8, generated on the GPU; packet i
    is stamped 1_700_000_000 s + (t0_pkt + i) * dt_ns."""
    import torch
    F = len(flows["sip"])
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    fid = torch.randint(0, F, (P,), generator=g, device=device)
    rev = torch.randint(0, 2, (P,), generator=g, device=device).bool()
    t = {k: torch.as_tensor(v, device=device)[fid] for k, v in flows.items()}
    fmac = torch.arange(F, device=device, dtype=torch.int64)[fid]
    sip = torch.where(rev, t["dip"], t["sip"])
    dip = torch.where(rev, t["sip"], t["dip"])
    sp = torch.where(rev, t["dport"], t["sport"])
    dp = torch.where(rev, t["sport"], t["dport"])
    cmac = (0x02 << 40) | fmac  # client / server MACs per flow
    smac_c = (0x04 << 40) | fmac
    smac = torch.where(rev, smac_c, cmac)
    dmac = torch.where(rev, cmac, smac_c)
    fr = torch.zeros((P, 64), dtype=torch.uint8, device=device)

    def put(col, val, nbytes):
        for q in range(nbytes):
            fr[:, col + q] = ((val >> (8 * (nbytes - 1 - q))) & 0xFF).to(torch.uint8)

    put(0, dmac, 6)
    put(6, smac, 6)
    fr[:, 12] = 0x08
    fr[:, 14] = 0x45
    fr[:, 17] = 50  # IPv4 total length 50 = 20 + 8 + 22
    put(18, torch.arange(P, device=device, dtype=torch.int64) & 0xFFFF, 2)
    fr[:, 20] = 0x40  # DF
    fr[:, 22] = 64
    fr[:, 23] = 17
    put(26, sip, 4)
    put(30, dip, 4)
    put(34, sp, 2)
    put(36, dp, 2)
    fr[:, 39] = 30  # UDP length
    return fr.reshape(-1).contiguous(), stamp_desc(P, device, dt_ns, t0_pkt)


def stamp_desc(P, device, dt_ns, t0_pkt):
    """Descriptors of P consecutive 64 B frames, packet i at 1_700_000_000 s + (t0_pkt + i) * dt_ns."""
    import torch
    i = torch.arange(P, device=device, dtype=torch.int64)
    us = (t0_pkt + i) * dt_ns // 1000
    desc = torch.zeros((P, 4), dtype=torch.int32, device=device)
    desc[:, 0] = (i * 64).to(torch.int32)
    desc[:, 1] = 64 | (64 << 16)
    desc[:, 2] = (1_700_000_000 + us // 1_000_000).to(torch.int32)
    desc[:, 3] = (us % 1_000_000).to(torch.int32)
    return desc.reshape(-1).view(torch.uint8).contiguous()


class _DevArray:
    """Minimal __cuda_array_interface__ so torch can alias the engine's export buffer."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3}


class ExportGather:
    """The N > 1 step's only exchange (BASELINE.json configs[3]: "RCCL gather of per-GPU IPFIX
    export buffers over xGMI"): each rank's exports leave as the IPFIX message stream of its
    own observation domain (odid = rank), formatted on its GPU (ipxg_device_ipfix_messages,
    no host round trip), and move to rank 0 with shard.StreamGather on a side stream, behind
    the next step's kernels: exactly the stream bytes, point to point over RCCL, sized by the
    16-byte headers gathered the step before.  The engine's stream waits only for the copy of
    its message buffer."""

    def __init__(self, eng, rank, world, device):
        import torch
        from ipfixprobe_amd import shard
        self.eng, self.rank, self.world, self.device = eng, rank, world, device
        self.x = eng.ipfix_exporter(odid=rank, export_time=1_700_000_000)
        self.g = shard.StreamGather(rank, world, device)
        self.side = torch.cuda.Stream(device=device)
        self.eng_stream = torch.cuda.ExternalStream(eng.stream(), device=device)
        self.events = []
        self.fmt_stream = None
        self.host_s = 0.0  # host time inside step() (the engine's IPFIX planning + the stream hand-off)

    def produce(self):
        """The pending exports as the engine's IPFIX message stream, formatted on the engine's
        formatting stream (ipxg_device_ipfix_messages: beside the kernels of a batch submitted
        since); the hand-off waits for push_pending()."""
        import torch
        h0 = time.perf_counter()
        ptr, nb, nr, _ = self.eng.device_ipfix_messages(self.x)
        ready = torch.cuda.Event()
        if self.fmt_stream is None:  # (the engine's formatting stream exists from the first call)
            self.fmt_stream = torch.cuda.ExternalStream(self.eng.ipfix_stream(), device=self.device)
        ready.record(self.fmt_stream)
        self.pending = (ptr, nb, nr, self.eng.device_ipfix_counts(), ready)
        self.host_s += time.perf_counter() - h0

    def push_pending(self):
        """The produced stream to StreamGather on the side stream.  The bench calls it once the
        next step's kernels are enqueued, so this host work runs beside them.  No copy: the engine
        alternates two message buffers (ipxg_device_ipfix_messages), so this stream stays valid
        while the next one is formatted; its send happens in the next push, and the engine's
        stream waits for `copied` (recorded after that send) before it formats into this buffer
        again."""
        import torch
        if getattr(self, "pending", None) is None:
            return
        h0 = time.perf_counter()
        ptr, nb, nr, cptr, ready = self.pending
        self.pending = None
        src = torch.as_tensor(_DevArray(ptr, max(nb, 1)), device=self.device)
        counts = torch.as_tensor(_DevArray(cptr, 16), device=self.device).view(torch.int64)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        copied = torch.cuda.Event()
        self.side.wait_event(ready)
        with torch.cuda.stream(self.side):
            t0.record()
            self.g.push(src, nb, nr, copied=copied, counts=counts, copy=False)
            t1.record()
        self.eng_stream.wait_event(copied)
        self.events.append((t0, t1))
        self.host_s += time.perf_counter() - h0

    def step(self):
        self.produce()
        self.push_pending()

    def flush(self):
        """The last step's exports (their step() comes with a next step that does not follow),
        then the last exchange."""
        import torch
        if self.eng.pending():
            self.produce()
        self.push_pending()
        with torch.cuda.stream(self.side):
            self.g.flush()

    def device_ms(self, reset=True):
        """Side-stream time of the copies + exchanges (synchronise first)."""
        ms = sum(a.elapsed_time(b) for a, b in self.events)
        if reset:
            self.events = []
        return ms


# ---- CPU baseline ---------------------------------------------------------------
def host_cores():
    """nproc (honours the box's CPU share: OMP_NUM_THREADS / cgroup), the CPUs to pin to, the model."""
    try:
        n = int(subprocess.run(["nproc"], stdout=subprocess.PIPE, text=True, check=True).stdout.strip())
    except (OSError, ValueError, subprocess.CalledProcessError):
        n = os.cpu_count() or 1
    cpus = sorted(os.sched_getaffinity(0))[:n]
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, cpus, model


def cpu_baseline(arena_np, desc_np, canon_lo, flows, reps=3, label=""):
    """The oracle (oracle/ipxg_oracle.c, the reference path restated in C, gcc -O3) on the same
    packets, driven by oracle/cpu_baseline.c: one pinned pipeline thread per host core, each
    with its own cache over its shard of the packets -- the reference's scaling (one input
    thread + private NHTFlowCache per RSS queue, ipfixprobe.cpp:381-464); shards by the
    direction-symmetric canonical flow hash (the NIC's symmetric RSS, dpdkDevice.cpp:230-262;
    not timed).  Also one thread over the whole sample.  Median of `reps` each."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py
    n, cpus, model = host_cores()
    shard = ((canon_lo & np.uint64(0xFFFFFFFF)) * np.uint64(n) >> np.uint64(32)).astype(np.int64)
    s_all = min(30, int(math.ceil(math.log2(max(flows // n, 2)))) + 4)
    s_one = min(30, int(math.ceil(math.log2(max(flows, 2)))) + 4)
    multi, single = [], []
    nrec = no_res = 0
    for _ in range(reps):
        dt, nrec, no_res = oracle_py.bench_mt(arena_np, desc_np, shard, n, cpus, s_all)
        multi.append(dt)
    for _ in range(reps):
        dt1, rec1, nr1 = oracle_py.bench_mt(arena_np, desc_np, np.zeros(len(desc_np), np.int64), 1, cpus[:1], s_one)
        single.append(dt1)
    pk = len(desc_np)
    mt, st = float(np.median(multi)), float(np.median(single))
    return {"value": round(pk / mt / 1e6, 3), "unit": "Mpkts/s", "cores": n, "nproc": n, "cpu_model": model,
            "single_core": round(pk / st / 1e6, 3), "kind": "port",
            "sample": "%s%d packets x %d runs (median): oracle/ipxg_oracle.c (parse_packet + NHTFlowCache::"
                      "put_pkt + finish restated in C, gcc -O3) in oracle/cpu_baseline.c, %d pinned threads each "
                      "over its canonical-hash shard with its own cache (s=%d), %.3f s; single core: one thread, "
                      "s=%d, %.2f s; %d records, NO_RES %d"
                      % (label, pk, reps, n, s_all, mt, s_one, st, nrec, no_res)}


def canon_of(eng, arena_np, desc_np):
    """Canonical (direction-free) flow hash per packet from the device parser (RSS stand-in)."""
    from ipfixprobe_amd import shard
    out = np.zeros(len(desc_np), dtype=np.uint64)
    step = 2_000_000
    for s in range(0, len(desc_np), step):
        p = eng.parse(arena_np, desc_np[s:s + step])
        out[s:s + step] = shard.canonical(p["hash_fwd"], p["hash_inv"])
    return out


def pmc_traffic(kernel, workload, packets_per_launch, offsets):
    """HBM bytes per launch of `kernel` from the newest profiles/*/pmc_summary[_<workload>].json taken
    on a run of this shape: its "_meta" (tools/pmc_summary.py) names the same workload, packets per
    launch and descriptor offsets; of the kernel's template variants the one dispatched most often
    (the steady state of that run).  Bytes: the L2's fabric read requests by size
    (TCC_EA0_RDREQ_32B/64B/128B: 32, 64, 128 bytes each -- round 3 measured FETCH_SIZE = all requests x
    64 B while ~99.9 % of k_bin's are 128 B, i.e. FETCH_SIZE reads half, as MI355X_MICROARCH.md 'HBM'
    says) + WRITE_SIZE (KiB); summaries without the request sizes: FETCH_SIZE x 2 + WRITE_SIZE.
    Returns (path, bytes, variant, its dispatches) or None."""
    best = None
    name = "pmc_summary.json" if workload == "udp64" else "pmc_summary_%s.json" % workload
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", name))):
        try:
            with open(p) as f:
                js = json.load(f)
        except (OSError, ValueError):
            continue
        meta = js.get("_meta")
        if not meta or meta.get("workload") not in (workload, "udp64-" + workload) or \
                meta.get("packets_per_launch") != packets_per_launch \
                or meta.get("offsets") != offsets:
            continue  # (a summary of another batch size or offset form: not this run's kernel)
        found = None  # the template variant dispatched most often (the steady state)
        for kn, v in js.items():
            if kn == "_meta":
                continue
            if kn.split("::")[-1].split("<")[0] == kernel and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                if found is None or v.get("calls", 0) > found[0]:
                    if "TCC_EA0_RDREQ_128B_sum" in v:
                        rd = (128 * v["TCC_EA0_RDREQ_128B_sum"] + 64 * v.get("TCC_EA0_RDREQ_64B_sum", 0) +
                              32 * v.get("TCC_EA0_RDREQ_32B_sum", 0))
                    else:
                        rd = 2 * v["FETCH_SIZE"] * 1024.0
                    found = (v.get("calls", 0), rd + v["WRITE_SIZE"] * 1024.0, kn)
        if found is not None:
            best = (p, found[1], found[2], found[0])
    return best


def end_to_end_pipelined(eng, frames, desc, packets, nb=4):
    """PCIe-inclusive rate of the double-buffered ingest: nb copies of the batch in pinned host
    memory (timestamps shifted 1 s per copy, so flows carry across them), submitted with
    IPXG_BATCH_ASYNC -- batch k+1's H2D copy (copy stream) overlaps batch k's kernels -- then
    ipxg_finish and the D2H poll of every record."""
    import torch
    hosts = []
    for k in range(nb):
        d = desc.cpu().clone()
        dv = d.view(torch.int32).view(-1, 4)
        dv[:, 2] += k
        hosts.append((frames.cpu().pin_memory(), d.pin_memory()))

    def run():
        for hf, hd in hosts:
            eng.submit(hf, hd, asynchronous=True)
        eng.finish()
        return len(eng.poll())

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nrec = run()
    dt = time.perf_counter() - t0
    h2d = sum(hf.numel() + hd.numel() for hf, hd in hosts)
    return {"value": round(packets * nb / dt / 1e6, 2), "unit": "Mpkts/s", "ms_per_batch": round(dt / nb * 1e3, 3),
            "h2d_GBs_effective": round(h2d / dt / 1e9, 2), "batches": nb, "records": nrec,
            "path": "pinned host batches -> H2D on the copy stream into two staging slots, overlapped with the "
                    "previous batch's kernels -> finish -> D2H poll of the records"}


def end_to_end(eng, frames, desc, packets, reps=3):
    """PCIe-inclusive rate (never `value`): the same batch from pinned host memory through
    ipxg_submit (hipMemcpyAsync H2D of arena + descriptors, then the kernels), ipxg_finish and
    the D2H poll of every exported record, one batch after another (no overlap)."""
    import torch
    hf = frames.cpu().pin_memory()
    hd = desc.cpu().pin_memory()

    def one():
        eng.submit(hf, hd)
        eng.finish()
        return len(eng.poll())

    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nrec = 0
    for _ in range(reps):
        nrec = one()
    dt = time.perf_counter() - t0
    h2d = hf.numel() + hd.numel() * hd.element_size()
    return {"value": round(packets * reps / dt / 1e6, 2), "unit": "Mpkts/s",
            "ms_per_batch": round(dt / reps * 1e3, 3),
            "h2d_bytes_per_batch": h2d, "h2d_GBs_effective": round(h2d * reps / dt / 1e9, 2),
            "records_per_batch": nrec,
            "path": "pinned host batch -> H2D copy -> kernels -> finish -> D2H poll of the records, "
                    "batches back to back (no copy/compute overlap)"}


# ---- workloads -------------------------------------------------------------------------------------
def two_engines(eng, wl, args, local, step_on, steps, one_ms):
    """The same cold steps on two engines in turn, each with its own stream and table (two capture
    queues of one GPU, as the reference runs a cache per queue): step k+1's k_bin starts while step
    k's k_reduce / k_fin_list run on the other stream.  Every step starts from an empty table and is
    finished, so each step's records are the one-engine records (tests/test_gpu_ahead.py
    test_two_engines_in_turn).  Reported beside the line's value, which stays the one-engine rate."""
    import torch
    from ipfixprobe_amd import Engine
    eng.profile(0)
    e2 = Engine(engine_params(wl.flows, args.ingest, args.walk), device_id=local)
    try:
        engs = (eng, e2)
        for k in range(4):
            step_on(engs[k % 2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            step_on(engs[k % 2])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        e2.close()
    pk = sum(wl.packets[:wl.per_step])
    ms = dt / steps * 1e3
    return {"value": round(pk * steps / dt / 1e6, 2), "unit": "Mpkts/s", "ms_per_step": round(ms, 4),
            "steps": steps, "vs_one_engine": round(one_ms / ms, 4),
            "what": "the line's cold steps alternating between two engines (streams, tables): one step's "
                    "flow-state kernels overlap the next step's k_bin; records per step unchanged"}


def torch_int32():
    import torch
    return torch.int32


class Workload:
    """Device-resident batches and how a step walks them."""

    def __init__(self, name, batches, flows, per_step, finish, description):
        self.name, self.batches, self.flows = name, batches, flows
        self.per_step = per_step        # batches submitted per step
        self.finish = finish            # ipxg_finish at the end of each step
        self.description = description
        self.alg = [self._alg(d) for _, d in batches]
        self.packets = [d.numel() // 16 for _, d in batches]
        self.last_sec = [int(d[-16:].view(torch_int32())[2].item()) for _, d in batches]  # virtual clock

    @staticmethod
    def _alg(desc):
        import torch
        cl = desc.view(-1, 16)[:, 4:6].contiguous().view(torch.int16).to(torch.int64) & 0xFFFF
        return int(torch.clamp(cl, max=128).sum().item()) + 16 * desc.numel() // 16


def make_workload(args, rank, world, device, local):
    import torch
    if args.workload == "udp64":
        sr, sw = args.shard if args.shard else (rank, world)
        flows = gen_flows(args.flows, sr, sw, args.seed, device_id=local)
        if args.mode == "cold":
            fr, de = build_batch(flows, args.packets, args.seed + rank, device)
            desc = ("configs[1]: %d synthetic 64B Eth/IPv4/UDP packets over %d distinct biflows per GPU; step = "
                    "parse + XXH64 + biflow-cache update + finish (all flows exported)" % (args.packets, args.flows))
            return Workload("udp64", [(fr, de)], args.flows, 1, True, desc)
        # stream: one frame arena, one descriptor array per step with advancing timestamps
        fr, d0 = build_batch(flows, args.packets, args.seed + rank, device, dt_ns=100)
        nb = args.warmup + args.steps + min(args.steps, 10) + 1
        batches = [(fr, d0)] + [(fr, stamp_desc(args.packets, device, 100, k * args.packets)) for k in range(1, nb)]
        desc = ("configs[1] streaming: %d synthetic 64B Eth/IPv4/UDP packets per step over %d distinct biflows per "
                "GPU, 100 ns apart, flows carried across steps; step = parse + XXH64 + biflow-cache update of one "
                "batch + ipxg_expire(now)" % (args.packets, args.flows))
        return Workload("udp64-stream", batches, args.flows, 1, False, desc)
    sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
    import synthgen
    # the flow-hash-range shard this process generates: its torch.distributed rank, or one rank's
    # shard of an N-GPU job run alone on this GPU (--shard r/N: configs[3] at 1/N of its size)
    srank, sworld = args.shard if args.shard else (rank, world)
    mixname = "imix" if args.workload == "imix10m" else args.workload
    zipf = args.zipf if args.zipf is not None else (1.1 if mixname == "imix" else None)
    mix = synthgen.Mix(mixname, args.flows * sworld if sworld > 1 else args.flows, seed=args.seed, zipf=zipf)
    if sworld > 1:  # this rank's flows only (flow-hash-range shards, the NIC-RSS analogue)
        mix.restrict(rank_flows(mix, srank, sworld, local))
    gen = synthgen.Generator(mix, device, seed=args.seed + 7919 * srank)
    batches = [gen.batch(k * args.packets, args.packets, offset16=args.offset16) for k in range(args.batches)]
    torch.cuda.synchronize()
    cfg = {"imix": "configs[2]", "quic": "configs[4]", "imix10m": "configs[3]"}[args.workload]
    if args.shard:
        cfg += " shard %d/%d (one rank's slice of the %d-GPU job: %d of its %d flows, %d of its %d packets per step)" % (
            srank, sworld, sworld, len(mix.flows), args.flows * sworld, args.packets * args.batches,
            args.packets * args.batches * sworld)
    desc = ("%s: %s mix, %d packets per GPU per step (%d batches of %d, flows carried across batches) over %d "
            "flows%s; step = parse + XXH64 + biflow-cache update of every batch + finish"
            % (cfg, mixname, args.packets * args.batches, args.batches, args.packets, len(mix.flows),
               " (Zipf %.2f popularity)" % zipf if zipf else " (uniform popularity)"))
    if args.offset16:
        desc += "; descriptor offsets in 16-byte units (IPXG_BATCH_OFFSET16)"
    wl = Workload(args.workload, batches, len(mix.flows), args.batches, True, desc)
    wl.gen = gen
    return wl


def flow_owners(mix, world, local=0, hasher=None):
    """The rank (of world) owning each flow of the mix by its canonical hash (shard.owner).
    hasher(keys, keylen) -> XXH64 per key: the engine's (ipxg_xxh64_batch on GPU `local`) by
    default; the CPU tests pass the oracle's."""
    from ipfixprobe_amd import Engine, shard
    F = len(mix.flows)
    owner = np.zeros(F, dtype=np.int64)
    e = None
    if hasher is None:
        e = Engine(device_id=local)
        hasher = e.xxh64
    try:
        for s in range(0, F, 1 << 20):
            sub = mix.flows[s:s + (1 << 20)]
            owner[s:s + len(sub)] = shard.owner(flow_canon(hasher, mix, sub), world)
    finally:
        if e is not None:
            e.close()
    return owner


def rank_flows(mix, rank, world, local, hasher=None):
    """Indices of the mix's flows whose canonical hash this rank owns."""
    return np.nonzero(flow_owners(mix, world, local, hasher) == rank)[0]


def flow_canon(hasher, mix, fl):
    """Canonical hash of each flow of a synthetic mix from its packed keys (cache.hpp:29-46);
    hasher(keys, keylen) -> XXH64 per key (Engine.xxh64, or the oracle's on the CPU)."""
    from ipfixprobe_amd import shard
    lay = mix.layouts[fl["layout"].astype(np.int64)]
    v6 = lay["addr_len"] == 16
    proto = np.where(lay["tcp_flags_off"] > 0, 6, 17).astype(np.uint8)
    out = np.zeros(len(fl), dtype=np.uint64)
    for is6, klen in ((False, 16), (True, 40)):
        sel = np.nonzero(v6 == is6)[0]
        if not len(sel):
            continue
        al = 16 if is6 else 4
        kf = np.zeros((len(sel), klen), dtype=np.uint8)
        ki = np.zeros((len(sel), klen), dtype=np.uint8)
        f = fl[sel]
        vl = np.where(lay["vlan_off"][sel] > 0, f["vlan"], 0).astype(np.uint16)
        for k, (a, b, pa, pb) in ((kf, (f["sip"], f["dip"], f["sport"], f["dport"])),
                                  (ki, (f["dip"], f["sip"], f["dport"], f["sport"]))):
            k[:, 0:2] = pa.astype("<u2").view(np.uint8).reshape(-1, 2)
            k[:, 2:4] = pb.astype("<u2").view(np.uint8).reshape(-1, 2)
            k[:, 4] = proto[sel]
            k[:, 5] = 6 if is6 else 4
            k[:, 6:6 + al] = a[:, :al]
            k[:, 6 + al:6 + 2 * al] = b[:, :al]
            k[:, 6 + 2 * al:8 + 2 * al] = vl.view(np.uint8).reshape(-1, 2)
        out[sel] = shard.canonical(hasher(kf.reshape(-1), klen), hasher(ki.reshape(-1), klen))
    return out


def engine_params(flows, ingest="binned", walk="auto"):
    """The bench's engine: a table of >= 2 x flows slots (2^16 at least), the binned ingest, the
    header walk chosen per batch."""
    return "s=%d;ingest=%s;walk=%s" % (max(16, int(math.ceil(math.log2(2 * flows)))), ingest, walk)


def launch_ranks(n):
    """Start N ranks of this very command line under torch.distributed.run (one process per GPU,
    rendezvous on 127.0.0.1) as a child process and return its exit code.  The parent has made no
    GPU call (nothing here initialises HIP), and it never execs: it waits for the child."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the box's driver)
    return subprocess.run(cmd, env=env).returncode


def cpu_selftest(args):
    """The N > 1 plumbing without a GPU (gloo): every rank pushes, per step, a stream of a
    different pseudo-random size and content through shard.StreamGather; rank 0 checks that it
    received every rank's every stream byte for byte, and that the bytes it received are exactly
    the streams' (no padding), then prints one JSON line."""
    import torch
    import torch.distributed as dist
    from ipfixprobe_amd import shard
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")

    def stream(r, k):
        g = np.random.default_rng(1000 * r + k)
        n = int(g.integers(0, 5000)) if (r + k) % 5 else 0  # some empty streams
        return g.integers(0, 256, n, dtype=np.uint8), n // 81

    g = shard.StreamGather(rank, world, "cpu")
    steps = args.steps or 5
    sent = expect = 0
    bad = []
    for k in range(steps):
        b, nr = stream(rank, k)
        g.push(torch.from_numpy(b.copy()), len(b), nr)
        sent += len(b)
        if rank == 0 and k > 0:  # the previous step's streams arrived in this push
            for r, t, rec in g.last:
                want, wn = stream(r, k - 1)
                if not np.array_equal(t.numpy(), want) or rec != wn:
                    bad.append((k - 1, r))
    g.flush()
    if rank == 0:
        for r, t, rec in g.last:
            want, wn = stream(r, steps - 1)
            if not np.array_equal(t.numpy(), want) or rec != wn:
                bad.append((steps - 1, r))
        expect = sum(len(stream(r, k)[0]) for r in range(world) for k in range(steps))
        print(json.dumps({"selftest": "stream-gather", "n_ranks": world, "steps": steps,
                          "received_bytes": g.received_bytes, "expected_bytes": expect,
                          "header_bytes": g.header_bytes, "mismatches": bad}))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 1 if bad or (rank == 0 and g.received_bytes != expect) else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="udp64", choices=["udp64", "imix", "quic", "imix10m"],
                    help="udp64 = configs[1], imix = configs[2], imix10m = configs[3] (per GPU: 1/N of 1G packets "
                         "over 10M flows), quic = configs[4]")
    ap.add_argument("--shard", default=None, metavar="R/N",
                    help="generate only rank R's flow-hash shard of an N-GPU job, on this one GPU (configs[3]'s "
                         "per-GPU slice without the other N-1 GPUs)")
    ap.add_argument("--mode", default="cold", choices=["cold", "stream"], help="udp64 only")
    ap.add_argument("--packets", type=int, default=None, help="packets per batch")
    ap.add_argument("--offsets", default="auto", choices=["auto", "units", "bytes"],
                    help="synthetic mixes: descriptor offsets in 16-byte units (IPXG_BATCH_OFFSET16: batch arenas "
                         "past 4 GiB, so a step's packets in fewer, larger batches) or in bytes (arenas <= 4 GiB); "
                         "auto = units for imix / quic / imix10m")
    ap.add_argument("--batches", type=int, default=None, help="batches per step (imix / quic)")
    ap.add_argument("--flows", type=int, default=None)
    ap.add_argument("--zipf", type=float, default=None)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check one step's records against the oracle")
    ap.add_argument("--ingest", default="binned", choices=["binned", "atomic"])
    ap.add_argument("--walk", default="auto", choices=["auto", "wide", "narrow"],
                    help="k_bin's header walk (auto: chosen per batch from the previous batch's mix)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive (host batch) rate")
    ap.add_argument("--no-two-engines", action="store_true",
                    help="skip the two-engine rate of the cold steps (two_engines in the line)")
    ap.add_argument("--strict", type=int, default=None, metavar="S",
                    help="strict mode with the reference's table of 2^S records (S=17: its default): "
                         "its evictions and sweep replayed exactly (ipxg_strict.hip)")
    ap.add_argument("--plugins", default=None,
                    help="process plugins through the bridge (native stand-ins, include/ipxg_stdplugins.h): a "
                         "comma list of dns,http,tls,quic, or 'config' for the workload's own (configs[2]: "
                         "dns,http,tls; configs[4]: quic)")
    ap.add_argument("--walk-threads", type=int, default=0,
                    help="threads of the plugin flows' host walk (0: the host's threads, at most 16)")
    ap.add_argument("--gather", action="store_true",
                    help="run the N > 1 step's export exchange (IPFIX streams to rank 0, shard.StreamGather) at any "
                         "N, world size 1 included: its cost on one GPU")
    ap.add_argument("--prof-every", type=int, default=8,
                    help="HIP events around k_bin / k_bin_slow on one timed batch of every N (roofline.avg_launch_ms)")
    ap.add_argument("--cpu-selftest", action="store_true",
                    help="no GPU: the N-rank launcher and the export exchange over gloo with synthetic streams "
                         "(tests/test_launcher.py)")
    args = ap.parse_args()
    # --gpus N: one process per GPU.  Under torchrun (the driver's N > 1 runs) WORLD_SIZE is set
    # and must equal N; run directly with N > 1, bench.py starts the N ranks itself.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: WORLD_SIZE=%s but --gpus %d\n" % (env_world, args.gpus))
        sys.exit(2)
    if args.cpu_selftest:
        sys.exit(cpu_selftest(args))
    if args.shard:
        a, b = (int(x) for x in args.shard.split("/"))
        if not 0 <= a < b:
            ap.error("--shard R/N needs 0 <= R < N")
        args.shard = (a, b)
    # imix10m: configs[3] = 1G IMIX packets over 10M flows on 8 GPUs -> per GPU 125M packets over 1.25M flows.
    # The mixes' steps in batches as large as the arena allows: with byte offsets a batch's arena stays within
    # 4 GiB (quic 4 x 5M, imix 10 x 10M, imix10m 13 x 9,615,385); with 16-byte unit offsets (ABI 8) up to the
    # engine's 16M-packet batch (quic 2 x 10M, imix 7 x 14,285,715, imix10m 9 x 13,888,889): the flow-state
    # passes (k_reduce, k_fin_list) run once per batch over the flows it touches, so fewer batches cost less
    # (with process plugins too: imix + dns/http/tls 2.43-2.49 -> 3.01-3.12 Gpkt/s, quic + quic 0.43-0.47 ->
    # 0.53-0.56, each pair on one box -- profiles/r05/plugin_offsets_ab.txt)
    args.offset16 = args.workload != "udp64" and args.offsets != "bytes"
    if args.offset16:
        dflt = {"udp64": (10_000_000, 1, 100_000, 3000), "imix": (14_285_715, 7, 1_000_000, 5),
                "quic": (10_000_000, 2, 1_000_000, 10), "imix10m": (13_888_889, 9, 1_250_000, 3)}[args.workload]
    else:
        dflt = {"udp64": (10_000_000, 1, 100_000, 3000), "imix": (10_000_000, 10, 1_000_000, 5),
                "quic": (5_000_000, 4, 1_000_000, 10), "imix10m": (9_615_385, 13, 1_250_000, 3)}[args.workload]
    args.packets = args.packets or dflt[0]
    args.batches = args.batches or dflt[1]
    args.flows = args.flows or dflt[2]
    # (stream mode keeps one descriptor array per step: 160 MB each at 10M packets)
    args.steps = args.steps or (50 if args.workload == "udp64" and args.mode == "stream" else dflt[3])

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from ipfixprobe_amd import Engine
    wl = make_workload(args, rank, world, device, local)
    torch.cuda.synchronize()
    if args.strict is not None:
        wl.description += "; strict mode: the reference's table of 2^%d records in 16-way lines" % args.strict
        eng = Engine("strict=true;s=%d" % args.strict, device_id=local)
    else:
        eng = Engine(engine_params(wl.flows, args.ingest, args.walk), device_id=local)
    plugins = []
    if args.plugins:
        from ipfixprobe_amd.engine import StdPlugin
        names = args.plugins.split(",") if args.plugins != "config" else \
            {"imix": ["dns", "http", "tls"], "imix10m": ["dns", "http", "tls"], "quic": ["quic"]}.get(args.workload, [])
        plugins = [StdPlugin(nm) for nm in names]
        eng.set_walk_threads(args.walk_threads)
        for pl in plugins:
            eng.add_plugin(pl.struct)
        wl.description += "; process plugins %s through the bridge (native stand-ins)" % ",".join(names)
    cursor = [0]
    gather = ExportGather(eng, rank, world, device) if world > 1 or args.gather else None

    def step_on(e):
        # with the gather: the previous step's exports are formatted (ipxg_device_ipfix_messages on
        # the engine's formatting stream) and handed to the gather right after this step's first
        # batch is submitted, beside its k_bin -- the tail of the batch joins the formatting
        if wl.finish:
            for k in range(wl.per_step):
                fr, de = wl.batches[k]
                # back to back; finish right behind (the batches were synchronised after generation)
                e.submit(fr, de, device=True, asynchronous=True, wait_producer=False, offset16=args.offset16)
                if k == 0 and gather is not None:
                    gather.step()
            e.finish()
        else:
            fr, de = wl.batches[cursor[0]]
            cursor[0] += 1
            e.submit(fr, de, device=True, asynchronous=True, wait_producer=False)
            if gather is not None:
                gather.step()
            e.expire(wl.last_sec[cursor[0] - 1])  # the virtual clock: idle flows out (none idle here)
        if gather is None:
            e.clear_exports()

    def step():
        step_on(eng)

    for _ in range(args.warmup):
        step()
    verify = None
    if args.verify and rank == 0 and wl.finish:
        verify = verify_step(eng, wl, args.strict, args.offset16)
    # timed region: HIP events around the ingest kernels only (k_bin, k_bin_slow), on one batch of
    # every PROF_EVERY: each event record is a packet of its own on the engine's stream (~4-5 us of
    # GPU time, tools/gapbench), so events on every batch added ~13 us to every udp64 step; the
    # every-stage events come from a separate (untimed) pass below
    eng.profile(3, every=args.prof_every)
    if gather is not None:
        torch.cuda.synchronize()
        gather.device_ms()
        gather.host_s = 0.0
        rx0 = (gather.g.received_bytes, gather.g.header_bytes, gather.g.sent_bytes, gather.g.k)
    # the counters at the start of the timed region: the slow-path share below is the timed steps'
    # (the warmup's first batch runs the narrow walk, which leaves far more packets to the slow
    # pass than the wide walk the engine switches to after it -- engine totals from the start
    # attributed those to every timed k_bin_slow launch: VERDICT r3, the imix slow line)
    st0 = eng.stats()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    tm_in = eng.timing()
    st = eng.stats()
    gms = gather.device_ms() / args.steps if gather is not None else None
    ghost = gather.host_s * 1e3 / args.steps if gather is not None else None
    if gather is not None:  # per-step exchange volume over the timed steps (rank 0 received / this rank sent)
        gx = gather.g
        g_rx = (gx.received_bytes - rx0[0]) / args.steps
        g_hdr = (gx.header_bytes - rx0[1]) / args.steps
        g_tx = (gx.sent_bytes - rx0[2]) / max(gx.k - rx0[3], 1)
    eng.profile(1)  # stage breakdown (untimed)
    stage_steps = min(args.steps, 10)
    for _ in range(stage_steps):
        step()
    tm = eng.timing()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    pk_step = sum(wl.packets[:wl.per_step]) if wl.finish else wl.packets[0]
    alg_step = sum(wl.alg[:wl.per_step]) if wl.finish else wl.alg[0]
    plug = None
    if plugins:  # full caplen for the packets handed to process plugins
        alg_step += tm_in["plugin_extra_bytes"] / args.steps
        hw_ms = tm_in["plugin_ms"] / args.steps
        plug = {"names": [p.name for p in plugins],
                "walk_threads": args.walk_threads or "default (host threads, at most 16)",
                "host_walk": {"flows_per_step": round(tm_in["plugin_flows"] / args.steps),
                              "packets_per_step": round(tm_in["plugin_packets"] / args.steps),
                              "packet_share": round(tm_in["plugin_packets"] / args.steps / pk_step, 5),
                              "bytes_per_step": round(tm_in["plugin_bytes"] / args.steps),
                              # what crossed PCIe for the walk: frames (whole, or the plugins' byte
                              # budget past the headers -- ipxg_plugin.follow_bytes), packet / flow records
                              "d2h_bytes_per_step": round(tm_in["plugin_d2h_bytes"] / args.steps),
                              "ms_per_step": round(hw_ms, 3),
                              "share_of_step_time": round(hw_ms / (dt / args.steps * 1e3), 4),
                              # batches whose k_bin / k_bin_slow ran during the previous batch's walk
                              "overlapped_batches_per_step": round(tm_in["plugin_overlapped"] / args.steps, 2)},
                "hook_calls": {p.name: p.calls() for p in plugins},
                "what": "flows with a plugin's packet in a batch (device pre-classifier) are replayed on the host "
                        "through the hooks; ms_per_step = wall time of that host walk inside the step (pack, "
                        "D2H of the packets, hooks, write-back)"}
    total_pkts = pk_step * args.steps * world
    value = total_pkts / dt / 1e6
    launches = max(tm_in["ingest_launches"], 1)
    bin_ms = tm_in["ingest_ms"] / launches
    slow_ms = tm_in["ingest_slow_ms"] / launches
    alg_launch = alg_step / (wl.per_step if wl.finish else 1)
    kname = "k_bin" if args.ingest == "binned" else "k_ingest"
    if args.strict is not None:
        kname = "strict (prep + sort + k_strict_walk)"
        kms = dt / args.steps * 1e3 / wl.per_step  # the strict pipeline's kernels, one batch
    elif args.ingest == "binned" and slow_ms > bin_ms:
        kname, kms = "k_bin_slow", slow_ms
    else:
        kms = bin_ms
    achieved = alg_launch / (kms / 1e3) / 1e9 if kms > 0 else 0.0
    ingest_gbs = alg_launch / ((bin_ms + slow_ms) / 1e3) / 1e9 if bin_ms > 0 else 0.0
    step_ms = dt / args.steps * 1e3
    step_gbs = alg_step * world / (step_ms / 1e3) / 1e9
    pk_launch = pk_step // (wl.per_step if wl.finish else 1)
    offsets = "units" if args.offset16 else "bytes"
    pmc = pmc_traffic(kname, wl.name if wl.name != "udp64-stream" else "stream", pk_launch, offsets)
    # the slow pass (frames the register walks do not take) on its own: its packets per launch
    # from the engine's counter, their algorithmic bytes at the workload's mean per packet
    slow_share = (st["slow_path_packets"] - st0["slow_path_packets"]) / max(st["parsed_packets"] - st0["parsed_packets"], 1)
    slow_pk = slow_share * alg_launch / max(alg_step / pk_step, 1e-9)
    slow_line = None
    if slow_share > 0.001 and slow_ms > 0:
        sgbs = slow_pk * (alg_step / pk_step) / (slow_ms / 1e3) / 1e9
        slow_line = {"kernel": "k_bin_slow", "packets_per_launch": round(slow_pk), "avg_launch_ms": round(slow_ms, 4),
                     "Mpkts_per_s": round(slow_pk / (slow_ms / 1e3) / 1e6, 1), "achieved": round(sgbs, 1),
                     "frac": round(sgbs / HBM_PEAK_GBS, 4),
                     "what": "slow-list packets (the workload's mean algorithmic bytes per packet) / k_bin_slow's "
                             "average launch"}
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and args.workload == "udp64" and args.mode == "cold" and \
            args.strict is None:
        e2e = end_to_end(eng, wl.batches[0][0], wl.batches[0][1], wl.packets[0])
        e2e["pipelined"] = end_to_end_pipelined(eng, wl.batches[0][0], wl.batches[0][1], wl.packets[0])
    two = None
    if rank == 0 and world == 1 and wl.finish and gather is None and not plugins and args.strict is None and \
            not args.no_two_engines:
        two = two_engines(eng, wl, args, local, step_on, min(args.steps, 300), step_ms)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        fr, de = wl.batches[0]
        label = "the first batch of the workload, "
        if args.offset16:  # (the CPU port takes byte offsets: the batch's first packets regenerated so)
            fr, de = wl.gen.batch(0, min(wl.packets[0], 4_000_000))
            label = "the first %d packets of the workload (byte offsets), " % (de.numel() // 16)
        arena_np = fr.cpu().numpy()
        desc_np = de.cpu().numpy().view(DESC_NP)
        canon = canon_of(eng, arena_np, desc_np)
        cpu = cpu_baseline(arena_np, desc_np, canon, wl.flows, label=label)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpkts/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_ms, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (generated on device, seed %d)" % args.seed,
            "config": {"workload": wl.description, "name": wl.name,
                       "packets_per_gpu_per_step": pk_step, "flows_per_gpu": wl.flows, "offsets": offsets,
                       "batches_per_step": wl.per_step, "ingest": args.ingest,
                       "parallelism": "flow-hash-range shards x%d, RCCL gather of export buffers"
                                      % world if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": round(pmc[1]) if pmc else None,
                         "traffic_source": os.path.relpath(pmc[0], ROOT) if pmc else None,
                         # the summary entry it came from: the kernel's template variant and its
                         # dispatches in that run (the summary's _meta matched this run's shape)
                         "traffic_entry": {"kernel": pmc[2], "dispatches": pmc[3], "packets_per_launch": pk_launch,
                                           "offsets": offsets} if pmc else None,
                         "algorithmic_bytes_per_launch": alg_launch,
                         "algorithmic_bytes_per_packet": round(alg_step / pk_step, 2),
                         "avg_launch_ms": round(kms, 4),
                         "timed_launches": int(launches),
                         "events": "HIP events on the engine's stream around k_bin (and k_bin_slow) of one timed batch "
                                   "in every %d" % args.prof_every,
                         "ingest": {"kernels": "k_bin+k_bin_slow", "avg_ms": round(bin_ms + slow_ms, 4),
                                    "achieved": round(ingest_gbs, 1), "frac": round(ingest_gbs / HBM_PEAK_GBS, 4)},
                         "step": {"what": "algorithmic bytes of the step / the whole step (every kernel, host "
                                          "round trips, finish)",
                                  "achieved": round(step_gbs, 1), "frac": round(step_gbs / HBM_PEAK_GBS, 4)},
                         "step_frac": round(step_gbs / HBM_PEAK_GBS, 4),
                         "slow": slow_line},
            "stage_ms_per_step": {k: round(tm[k + "_ms"] / stage_steps, 4)
                                  for k in ("ingest", "ingest_slow", "reduce", "fin", "finalize", "slow",
                                            "finish")},
            "flows_exported_per_step": int(st["total_exported"] // max(st["batches"] // max(wl.per_step, 1), 1)),
            "slow_path_packets_share": round(slow_share, 4),
            "walked_packets_share": round((st["walked_packets"] - st0["walked_packets"]) /
                                          max(st["parsed_packets"] - st0["parsed_packets"], 1), 4),
            "e2e_pcie": e2e,
            "two_engines": two,
            "spilled_packets": int(st["spilled_packets"]),
            "complex_flows": int(st["complex_flows"]),
            "gather": {"what": "per-rank IPFIX stream (odid = rank) -> rank 0 over RCCL point to point, exactly "
                               "the stream bytes, sized by 16-byte headers gathered the step before; on a side "
                               "stream, overlapped with the next step",
                       "device_ms_per_step": round(gms, 4),
                       "host_ms_per_step": round(ghost, 4),
                       "rank0_receives_bytes_per_step": round(g_rx),
                       "header_bytes_per_step": round(g_hdr),
                       "rank0_stream_bytes_per_step": round(g_tx)} if gather is not None else None,
            "verify": verify,
            "cpu_baseline": cpu,
            "plugins": plug,
            "strict": {"cache_exp": args.strict, "end_no_res_per_step": int(st["end_no_res"] // max(st["batches"], 1))}
            if args.strict is not None else None,
        }
        print(json.dumps(line))
    if gather is not None:
        gather.flush()
        torch.cuda.synchronize()
    eng.close()
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def verify_step(eng, wl, strict=None, offset16=False):
    """One step of the workload against the oracle (the first batch only for multi-batch steps,
    in its own engine state): bit-exact flow records or the first differences."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import flowcmp
    import oracle_py
    fr, de = wl.batches[0]
    if offset16 and fr.numel() >= 1 << 32:
        return "not run: the oracle takes byte offsets (arena of %d bytes)" % fr.numel()
    eng.submit(fr, de, device=True, offset16=offset16)
    eng.finish()
    got = eng.poll()
    d = de.cpu().numpy().view(DESC_NP).copy()
    if offset16:
        d["offset"] *= 16
    s = strict if strict is not None else min(30, int(math.ceil(math.log2(2 * wl.flows))) + 2)
    want, _ = oracle_py.run_capture(fr.cpu().numpy(), d, 1, cache_exp=s)
    diff = flowcmp.diff(got, want, fields=flowcmp.CONTRACT_FIELDS + (["end_reason"] if strict is not None else []))
    return "%d records, %s" % (len(got), "bit-exact vs oracle" if not diff else diff[:500])


if __name__ == "__main__":
    main()
