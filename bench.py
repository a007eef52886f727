"""bench.py -- device-resident packet->biflow throughput on MI355X.

Workload (BASELINE.json configs[1]): per GPU, 10M synthetic 64 B Ethernet/IPv4/UDP frames
(tot_len 50) over 100k distinct biflows (src 10/8, dst 192.168/16, sport 1024-65535, dport
1-1023; each packet picks a direction at random), timestamps 1 us apart (10 s span, so no
inactive/active timeout fires).  A step is one pass of the hot path over that batch with
the frames already in HBM: ipxg_submit (parse + 2x XXH64 + biflow-table update) followed by
ipxg_finish (every flow exported FORCED into the device export buffer).  With N GPUs each
rank owns a disjoint range of the canonical flow hash (the NIC-RSS analogue),
so there is no collective in the data path; at N > 1 the per-GPU export buffers are gathered
to rank 0 over RCCL inside the step (the path's only exchange).

Prints one JSON line (rank 0).  roofline.achieved = algorithmic bytes per launch of the
dominant kernel k_bin (64 B frame + 16 B descriptor per packet) / its average
duration, timed with HIP events on the engine's stream; roofline.stage gives the same bytes
over the whole ingest (k_bin + k_bin_slow + k_reduce + k_fin_list).  roofline.traffic is the HBM bytes per k_bin launch
from the newest committed rocprofv3 PMC summary (profiles/*/pmc_summary.json, collected by
tools/gpu_pmc.sh), or null when none covers k_bin.
"""
import argparse
import glob
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkts/s device-resident, 64B synthetic mix, 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
ALG_BYTES_PER_PKT = 80  # 64 B frame + 16 B descriptor


def gen_flows(F, rank, world, seed, device_id=0):
    """F distinct biflows whose canonical hash falls in this rank's range (hashed on this
    rank's GPU)."""
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


def build_batch(flows, P, seed, device):
    """64 B frames (P, 64) uint8 and descriptors (P, 16) uint8, generated on the GPU."""
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
    i = torch.arange(P, device=device, dtype=torch.int64)
    desc = torch.zeros((P, 4), dtype=torch.int32, device=device)
    desc[:, 0] = (i * 64).to(torch.int32)
    desc[:, 1] = 64 | (64 << 16)
    desc[:, 2] = (1_700_000_000 + i // 1_000_000).to(torch.int32)
    desc[:, 3] = (i % 1_000_000).to(torch.int32)
    return fr.reshape(-1).contiguous(), desc.reshape(-1).view(torch.uint8).contiguous()


class _DevArray:
    """Minimal __cuda_array_interface__ so torch can alias the engine's export buffer."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 3}


def gather_exports(eng, rank, world, device):
    """RCCL gather of every rank's device export buffer into rank 0 (ipfixprobe_amd.shard)."""
    import torch
    from ipfixprobe_amd.shard import gather_records
    ptr, n = eng.device_exports()
    buf = torch.as_tensor(_DevArray(ptr, max(n, 1) * 128), device=device)
    out = gather_records(buf, n, rank, world, device)
    return 0 if out is None else out.numel() // 128


def cpu_baseline(frames, desc, flows_per_shard, threads=16, reps=3):
    """The oracle (CPU restatement of the reference path) on the same packets, one pipeline
    per core as the reference scales (one input thread + private NHTFlowCache per RSS queue,
    ipfixprobe.cpp:381-464): packets are dealt to `threads` shards by a symmetric hash of the
    IP pair (the NIC's symmetric RSS on IPs, dpdkDevice.cpp:230-262 -- not timed), each shard
    runs parse_packet + put_pkt + finish in its own thread (ctypes drops the GIL)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_py
    arena = frames.cpu().numpy()
    d = desc.cpu().numpy().view(np.uint8).view(
        np.dtype([("offset", "<u4"), ("caplen", "<u2"), ("wirelen", "<u2"),
                  ("ts_sec", "<u4"), ("ts_usec", "<u4")]))
    threads = max(1, min(threads, os.cpu_count() or 1))
    fr = arena.reshape(-1, 64)
    ip = lambda c: fr[:, c:c + 4].view(">u4").reshape(-1).astype(np.uint64)  # noqa: E731
    sym = (ip(26) ^ ip(30)) * np.uint64(0x9E3779B97F4A7C15)
    shard = ((sym >> np.uint64(40)) % np.uint64(threads)).astype(np.int64)
    parts = [np.ascontiguousarray(d[shard == k]) for k in range(threads)]
    s_exp = min(30, int(math.ceil(math.log2(max(flows_per_shard // threads, 2)))) + 4)
    caches = [oracle_py.OracleCache(cache_exp=s_exp) for _ in range(threads)]
    counts = [0] * threads

    def work(k):
        for _ in range(reps):
            caches[k].run(arena, parts[k], 1)
            caches[k].finish()
            counts[k] += len(caches[k].take())

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    no_res = sum(c.stats()["end_no_res"] for c in caches)
    for c in caches:
        c.close()
    pkts = len(d) * reps
    return {"value": round(pkts / dt / 1e6, 3), "unit": "Mpkts/s", "cores": threads, "kind": "port",
            "sample": "the bench batch (%d packets, %d flows) x%d passes through oracle/ipxg_oracle.c "
                      "(parse_packet + NHTFlowCache::put_pkt + finish restated in C, gcc -O2), "
                      "%d threads each owning a symmetric-IP-hash shard with its own cache (s=%d), "
                      "%.2f s wall; %d records, NO_RES evictions %d"
                      % (len(d), flows_per_shard, reps, threads, s_exp, dt, sum(counts), no_res)}


def pmc_traffic(kernel="k_bin"):
    """HBM bytes per launch of `kernel` from the newest profiles/*/pmc_summary.json:
    FETCH_SIZE (KiB; doubled -- gfx950 tallies wide streaming reads at half, MI355X_MICROARCH.md
    'HBM') + WRITE_SIZE (KiB), both per launch."""
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json"))):
        try:
            with open(p) as f:
                js = json.load(f)
        except (OSError, ValueError):
            continue
        for name, v in js.items():
            if name.split("::")[-1].split("<")[0] == kernel and "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                best = (p, (2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0)
    return best


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--flows", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check the records against the oracle")
    ap.add_argument("--ingest", default="binned", choices=["binned", "atomic"])
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive (host batch) rate")
    args = ap.parse_args()

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
    flows = gen_flows(args.flows, rank, world, args.seed, device_id=local)
    frames, desc = build_batch(flows, args.packets, args.seed + rank, device)
    torch.cuda.synchronize()
    eng = Engine("s=%d;ingest=%s" % (max(16, int(math.ceil(math.log2(2 * args.flows)))), args.ingest),
                 device_id=local)

    def step():
        eng.submit(frames, desc, device=True, asynchronous=True)  # finish follows right behind
        eng.finish()
        if world > 1:
            gather_exports(eng, rank, world, device)
        eng.clear_exports()

    for _ in range(args.warmup):
        step()
    if args.verify and rank == 0:
        eng.submit(frames, desc, device=True)
        eng.finish()
        got = eng.poll()
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import flowcmp
        import oracle_py
        d = desc.cpu().numpy().view(np.uint8).view(
            np.dtype([("offset", "<u4"), ("caplen", "<u2"), ("wirelen", "<u2"),
                      ("ts_sec", "<u4"), ("ts_usec", "<u4")]))
        want, _ = oracle_py.run_capture(frames.cpu().numpy(), d, 1, cache_exp=21)
        diff = flowcmp.diff(got, want)
        print("verify: %d records, %s" % (len(got), "bit-exact vs oracle" if not diff else diff),
              file=sys.stderr)
    # timed region: HIP events around the ingest kernel only (the roofline's launch time);
    # every-stage events cost ~35 us of host time per step, so the stage breakdown comes
    # from a separate pass below
    eng.profile(2)
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
    tm_bin = eng.timing()
    st = eng.stats()
    eng.profile(1)  # stage breakdown (untimed)
    for _ in range(min(args.steps, 10)):
        step()
    tm = eng.timing()
    stage_steps = min(args.steps, 10)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    total_pkts = args.packets * args.steps * world
    value = total_pkts / dt / 1e6
    bin_ms = tm_bin["ingest_ms"] / max(tm_bin["ingest_launches"], 1)
    red_ms = (tm["ingest_slow_ms"] + tm["reduce_ms"] + tm["fin_ms"]) / max(tm["reduce_launches"], 1)
    alg = ALG_BYTES_PER_PKT * args.packets
    achieved = alg / (bin_ms / 1e3) / 1e9 if bin_ms > 0 else 0.0
    stage = alg / ((bin_ms + red_ms) / 1e3) / 1e9 if bin_ms > 0 else 0.0
    kname = "k_bin" if args.ingest == "binned" else "k_ingest"
    pmc = pmc_traffic(kname)
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        e2e = end_to_end(eng, frames, desc, args.packets)
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(frames, desc, args.flows, threads=args.cpu_threads)
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mpkts/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (generated on device, seed %d)" % args.seed,
            "config": {"workload": "configs[1]: %d synthetic 64B Eth/IPv4/UDP packets over %d distinct "
                                   "biflows per GPU; step = parse + XXH64 + biflow-cache update + "
                                   "finish (all flows exported)" % (args.packets, args.flows),
                       "packets_per_gpu": args.packets, "flows_per_gpu": args.flows,
                       "ingest": args.ingest,
                       "parallelism": "flow-hash-range shards x%d, RCCL gather of export buffers"
                                      % world if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": round(pmc[1]) if pmc else None,
                         "traffic_source": os.path.relpath(pmc[0], ROOT) if pmc else None,
                         "algorithmic_bytes_per_launch": alg,
                         "avg_launch_ms": round(bin_ms, 4),
                         "stage": {"kernels": "k_bin+k_bin_slow+k_reduce+k_fin_list",
                                   "achieved": round(stage, 1),
                                   "frac": round(stage / HBM_PEAK_GBS, 4),
                                   "avg_ms": round(bin_ms + red_ms, 4)}},
            "stage_ms_per_step": {k: round(tm[k + "_ms"] / stage_steps, 4)
                                  for k in ("ingest", "ingest_slow", "reduce", "fin", "finalize", "slow",
                                            "finish")},
            "flows_exported_per_step": int(st["end_forced"] // max(st["batches"], 1)),
            "e2e_pcie": e2e,
            "spilled_packets": int(st["spilled_packets"]),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    eng.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
