// ipxg_kernels.hip -- the engine's table and slow-path kernels for gfx950 (the per-batch
// ingest, k_bin + k_reduce, is in ipxg_ingest.hip).
//
//   k_ingest<INGEST>   the atomic ingest mode (cfg flag IPXG_CFG_ATOMIC_INGEST, kept for A/B
//                      measurement): one lane per packet folds straight into the table with
//                      device atomics.  k_ingest<GATHER> collects the packets of complex flows.
//   k_frag_walk        fragments sorted by (bucket, index): one lane per bucket replays the
//                      reference's 4-entry ring in arrival order (fragmentationCache.cpp).
//   k_frag_accumulate  folds the port-resolved fragments into the table.
//   k_deferred         re-applies packets whose probe failed, after the table has grown.
//   k_finalize         full-table scan applying finalize_slot to every slot still holding
//                      batch accumulators (when k_reduce could not finalise them itself).
//   k_complex_*        complex flows only: gather their packets, sort by index, and replay
//                      put_pkt_recursive sequentially per flow (cache.cpp:330-491).
// Maintenance: k_expire (export_expired), k_finish (finish), k_rehash (table growth).
#include "ipxg_table.hpp"

namespace ipxg {

// Fold one parsed packet into its flow's batch accumulators with device atomics (the
// slow paths: fragments, deferred packets, and the atomic ingest mode).
__device__ __forceinline__ bool flow_accumulate(const TableView& t, const Params& p, const BatchView& b,
                                                const DevPkt& pk, uint32_t idx, uint32_t sec, uint32_t* new_keys) {
    uint64_t lo, hf;
    uint32_t cdir;
    canon<false>(pk, p, lo, cdir, hf);
    return merge_packet_atomic(t, lo, idx, pack_misc(pk, cdir, time_bucket(sec, b.base_sec, p.bucket_w)),
                               new_keys);
}

// ---- K1: ingest ------------------------------------------------------------------------
enum IngestMode { MODE_INGEST = 0, MODE_GATHER = 1 };

template <int MODE>
__global__ __launch_bounds__(IPXG_BLOCK) void k_ingest(BatchView b, Params p, TableView t, FragView f,
                                                       BatchCtl* ctl, uint32_t* deferred_list,
                                                       unsigned long long* stats, ComplexView cx) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    __shared__ uint32_t sc[ST_COUNT];
    const uint32_t tid = threadIdx.x;
    if (b.base_sec == BASE_FROM_DESC0) b.base_sec = b.n ? b.desc[0].ts_sec : 0;
    if (tid < ST_COUNT) sc[tid] = 0;
    __syncthreads();
    ParseCounts c = {};
    uint32_t keyless = 0, frags = 0;
    uint32_t* col = &win[tid];
    for (uint32_t base = blockIdx.x * IPXG_BLOCK; base < b.n; base += gridDim.x * IPXG_BLOCK) {
        const uint32_t i = base + tid;
        const bool act = i < b.n;
        ipxg_pkt_desc d = {0, 0, 0, 0, 0};
        if (act) d = b.desc[i];
        if (MODE == MODE_INGEST) {
            const uint64_t ts = ((uint64_t)d.ts_sec << 32) | d.ts_usec;
            uint64_t prev = (uint64_t)__shfl_up((unsigned long long)ts, 1);
            bool has_prev = i > 0 || p.prev_valid;
            if (lane_id() == 0) {
                if (i > 0 && act) {
                    ipxg_pkt_desc q = b.desc[i - 1];
                    prev = ((uint64_t)q.ts_sec << 32) | q.ts_usec;
                } else {
                    prev = ((uint64_t)p.prev_sec << 32) | p.prev_usec;
                }
            }
            if (act && has_prev && ts < prev) ctl->nonmono = 1;
            if (act && i == b.n - 1) {
                ctl->last_sec = d.ts_sec;
                ctl->last_usec = d.ts_usec;
            }
        }
        if (!act) continue;
        stage_frame(col, frame_ptr(b, d), d.caplen);
        LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
        DevPkt pk;
        if (!parse_frame<false>(S, d.caplen, p.dlt, pk, c)) continue;
        if (pk.ip_version != 4 && pk.ip_version != 6) {
            keyless++;
            continue;
        }
        const bool is_frag = p.frag_enable && (pk.frag_off || pk.more_fragments);
        if (MODE == MODE_INGEST) {
            if (is_frag) {
                frags++;
                uint32_t bucket = (uint32_t)(frag_key_hash(pk) % (uint64_t)p.frag_size);
                uint32_t pos = atomicAdd(&ctl->frag_count, 1u);
                f.list[pos] = ((uint64_t)bucket << 24) | i;
                continue;
            }
            if (!flow_accumulate(t, p, b, pk, i, d.ts_sec, &ctl->new_keys)) {
                uint32_t pos = atomicAdd(&ctl->deferred, 1u);
                deferred_list[pos] = i;
            }
        } else {  // MODE_GATHER: collect the packets of complex flows
            if (is_frag) apply_frag_ports(p, f, i, pk);
            uint64_t lo, hf;
            uint32_t cdir;
            canon<false>(pk, p, lo, cdir, hf);
            const int64_t rr = complex_rank_of(cx, lo);
            if (rr >= 0) {
                const uint32_t r = (uint32_t)rr;
                uint32_t pos = atomicAdd(&cx.cursor[r], 1u);
                cx.list[cx.seg[r] + pos] = ((uint64_t)r << 24) | i;
            }
        }
    }
    if (MODE == MODE_INGEST) {
        flush_counts(c, keyless, frags, sc);
        flush_block_stats(sc, stats);
    }
}

static inline uint32_t grid_for(uint32_t n, uint32_t maxg) {
    uint32_t g = (n + IPXG_BLOCK - 1) / IPXG_BLOCK;
    if (g > maxg) g = maxg;
    return g ? g : 1;
}

void launch_ingest(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                   BatchCtl* ctl, uint32_t* deferred_list, unsigned long long* stats) {
    ComplexView cx = {};
    hipLaunchKernelGGL(k_ingest<MODE_INGEST>, dim3(grid_for(b.n, 1024)), dim3(IPXG_BLOCK), 0, st, b, p,
                       t, f, ctl, deferred_list, stats, cx);
}


// ---- fragmentation cache -----------------------------------------------------------------
__device__ __forceinline__ void frag_words(const DevPkt& pk, uint64_t w[5]) {
    const uint32_t* s = pk.sip;
    const uint32_t* d = pk.dip;
    w[0] = (uint64_t)pk.ip_version | ((uint64_t)s[0] << 16) | ((uint64_t)(s[1] & 0xFFFF) << 48);
    w[1] = (uint64_t)(s[1] >> 16) | ((uint64_t)s[2] << 16) | ((uint64_t)(s[3] & 0xFFFF) << 48);
    w[2] = (uint64_t)(s[3] >> 16) | ((uint64_t)d[0] << 16) | ((uint64_t)(d[1] & 0xFFFF) << 48);
    w[3] = (uint64_t)(d[1] >> 16) | ((uint64_t)d[2] << 16) | ((uint64_t)(d[3] & 0xFFFF) << 48);
    w[4] = (uint64_t)(d[3] >> 16) | ((uint64_t)pk.frag_id << 16) | ((uint64_t)(pk.vlan_id & 0xFFFF) << 48);
}

// One lane per bucket segment of the (bucket, index)-sorted fragment list: replay the ring
// (FragmentationTable::insert/find, RingBuffer push_back with overwrite) in arrival order.
__global__ __launch_bounds__(256) void k_frag_walk(BatchView b, Params p, FragView f, uint32_t nfrag,
                                                   unsigned long long* stats) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nfrag) return;
    const uint32_t bucket = (uint32_t)(f.sorted[j] >> 24);
    if (j > 0 && (uint32_t)(f.sorted[j - 1] >> 24) == bucket) return;
    FragEntry* E = f.ent + (size_t)bucket * 4;
    uint32_t cnt = f.cnt[bucket];
    uint32_t filled = 0;
    for (uint32_t k = j; k < nfrag && (uint32_t)(f.sorted[k] >> 24) == bucket; ++k) {
        const uint32_t idx = (uint32_t)(f.sorted[k] & 0xFFFFFF);
        ipxg_pkt_desc d = b.desc[idx];
        GlobalSrc g{frame_ptr(b, d), d.caplen};
        ParseCounts dummy = {};
        DevPkt pk;
        parse_frame<false>(g, d.caplen, p.dlt, pk, dummy);
        uint64_t w[5];
        frag_words(pk, w);
        uint32_t ports = ((uint32_t)pk.src_port << 16) | pk.dst_port;
        if (!pk.frag_off && pk.more_fragments) {  // first fragment: insert
            if (cnt == 4) {
                for (int e = 0; e < 3; ++e) E[e] = E[e + 1];
                cnt = 3;
            }
            FragEntry& e = E[cnt++];
            for (int q = 0; q < 5; ++q) e.kw[q] = w[q];
            e.sport = pk.src_port;
            e.dport = pk.dst_port;
            e.sec = d.ts_sec;
            e.usec = d.ts_usec;
        } else {
            for (int e = (int)cnt - 1; e >= 0; --e) {
                const FragEntry& x = E[e];
                if (x.kw[0] != w[0] || x.kw[1] != w[1] || x.kw[2] != w[2] || x.kw[3] != w[3] || x.kw[4] != w[4])
                    continue;
                // packet.ts > data.timestamp + timeout (timevalUtils.hpp:27-47)
                uint64_t ls = (uint64_t)x.sec + p.frag_timeout_s, lu = x.usec;
                if (lu >= 1000000) {
                    ls++;
                    lu -= 1000000;
                }
                bool later = (d.ts_sec == ls) ? (d.ts_usec > lu) : (d.ts_sec > ls);
                if (!later) {
                    ports = ((uint32_t)x.sport << 16) | x.dport;
                    filled++;
                }
                break;
            }
        }
        f.ports[idx] = ports;
    }
    f.cnt[bucket] = cnt;
    if (filled) atomicAdd(&stat_row(stats)[ST_FRAG_FILLED], (unsigned long long)filled);
}

void launch_frag_walk(hipStream_t st, const BatchView& b, const Params& p, FragView f, uint32_t nfrag,
                      unsigned long long* stats) {
    hipLaunchKernelGGL(k_frag_walk, dim3((nfrag + 255) / 256), dim3(256), 0, st, b, p, f, nfrag, stats);
}

__global__ __launch_bounds__(256) void k_frag_accumulate(BatchView b, Params p, TableView t, FragView f,
                                                         uint32_t nfrag, BatchCtl* ctl,
                                                         uint32_t* deferred_list) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nfrag) return;
    if (b.base_sec == BASE_FROM_DESC0) b.base_sec = b.desc[0].ts_sec;
    const uint32_t idx = (uint32_t)(f.list[j] & 0xFFFFFF);
    DevPkt pk;
    ipxg_pkt_desc d;
    if (!reparse<false>(b, p, f, idx, pk, d)) return;
    // a non-first fragment never passed parse_tcp_hdr / parse_udp_hdr (no TopPorts count), but
    // the ports the cache gave it put it into a flow whose count includes it: take it back out
    if (t.port_cnt && pk.frag_off && (pk.ip_proto == 6 || pk.ip_proto == 17) && (pk.src_port || pk.dst_port)) {
        unsigned long long* a = t.port_cnt + (pk.ip_proto == 17 ? 65536 : 0);
        atomicAdd(a + pk.src_port, ~0ull);  // -1
        atomicAdd(a + pk.dst_port, ~0ull);
    }
    if (!flow_accumulate(t, p, b, pk, idx, d.ts_sec, &ctl->new_keys)) {
        uint32_t pos = atomicAdd(&ctl->deferred, 1u);
        deferred_list[pos] = idx;
    }
}

void launch_frag_accumulate(hipStream_t st, const BatchView& b, const Params& p, TableView t,
                            FragView f, uint32_t nfrag, BatchCtl* ctl, uint32_t* deferred_list) {
    hipLaunchKernelGGL(k_frag_accumulate, dim3((nfrag + 255) / 256), dim3(256), 0, st, b, p, t, f, nfrag,
                       ctl, deferred_list);
}

// Re-apply packets whose probe failed before the table was grown.
__global__ __launch_bounds__(256) void k_deferred(BatchView b, Params p, TableView t, FragView f,
                                                  const uint32_t* in_list, uint32_t n_in, BatchCtl* ctl,
                                                  uint32_t* out_list) {
    uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_in) return;
    if (b.base_sec == BASE_FROM_DESC0) b.base_sec = b.desc[0].ts_sec;
    const uint32_t idx = in_list[j];
    DevPkt pk;
    ipxg_pkt_desc d;
    if (!reparse<false>(b, p, f, idx, pk, d)) return;
    if (!flow_accumulate(t, p, b, pk, idx, d.ts_sec, &ctl->new_keys)) {
        uint32_t pos = atomicAdd(&ctl->deferred, 1u);
        out_list[pos] = idx;
    }
}

void launch_deferred(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                     const uint32_t* in_list, uint32_t n_in, BatchCtl* ctl, uint32_t* out_list) {
    hipLaunchKernelGGL(k_deferred, dim3((n_in + 255) / 256), dim3(256), 0, st, b, p, t, f, in_list, n_in,
                       ctl, out_list);
}

// Re-apply deferred tile aggregates (3 slots each) after the table has grown.
__global__ __launch_bounds__(256) void k_deferred_agg(TableView t, const uint4* in_list, uint32_t n_in, BatchCtl* ctl,
                                                      uint4* out_list) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_in) return;
    const uint4 s0 = in_list[3 * (size_t)j], s1 = in_list[3 * (size_t)j + 1], s2 = in_list[3 * (size_t)j + 2];
    if (!merge_agg_probe(t, agg_decode(s0, s1, s2), &ctl->new_keys)) defer_agg(&ctl->agg_deferred, out_list, s0, s1, s2);
}

void launch_deferred_agg(hipStream_t st, TableView t, const uint4* in_list, uint32_t n_in, BatchCtl* ctl,
                         uint4* out_list) {
    hipLaunchKernelGGL(k_deferred_agg, dim3((n_in + 255) / 256), dim3(256), 0, st, t, in_list, n_in, ctl, out_list);
}

// ---- K3: finalize (full-table scan; the fast path finalises inside k_reduce) -------------
__global__ __launch_bounds__(256) void k_finalize(BatchView b, Params p, TableView t, FragView f,
                                                  ExportView ex, BatchCtl* ctl, unsigned long long* stats,
                                                  uint32_t cap) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    __shared__ uint32_t sc[ST_COUNT];
    __shared__ uint32_t cnt[4];  // keys, live, complex, exported
    if (threadIdx.x < ST_COUNT) sc[threadIdx.x] = 0;
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t keys = 0, live_n = 0, cx_n = 0, ex_n = 0;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < cap; s += gridDim.x * blockDim.x) {
        const HotSlot h = t.hot(s);
        bool do_export = false;
        uint8_t reason = 0;
        RecW er;
        if (h.key != 0) {
            keys++;
            const bool was_live = h.state & SLOT_LIVE;
            if (h.last1 == 0 || (h.state & SLOT_COMPLEX)) {  // untouched, or already decided
                if (was_live) live_n++;
            } else {
                const FinResult fr = finalize_slot<true>(b, p, t, f, s, h, p.force_complex != 0,
                                                         &win[threadIdx.x], er);
                if (fr.status == FIN_COMPLEX) {
                    cx_n++;
                    if (was_live) live_n++;
                } else {
                    live_n++;
                    do_export = fr.do_export;
                    reason = fr.reason;
                }
            }
        }
        uint32_t pos = wave_append(ex.count, do_export);
        if (do_export) {
            store_export_w(ex, pos, er, reason);
            ex_n++;
        }
        count_exports_wave(sc, do_export, er, reason);
        count_v6_exports(ex, do_export && rw_ipver(er) == 6);
    }
    wave_add_lds(&cnt[0], keys);
    wave_add_lds(&cnt[1], live_n);
    wave_add_lds(&cnt[2], cx_n);
    wave_add_lds(&cnt[3], ex_n);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (cnt[0]) atomicAdd(&ctl->keys, cnt[0]);
        if (cnt[1]) atomicAdd(&ctl->live, cnt[1]);
        if (cnt[2]) atomicAdd(&ctl->complex_count, cnt[2]);
        if (cnt[3]) atomicAdd(&ctl->exported, cnt[3]);
    }
    flush_block_stats(sc, stats);
}

static inline uint32_t table_grid(uint32_t cap) {
    uint32_t g = (cap + 255) / 256;
    return g > 2048 ? 2048 : g;
}

void launch_finalize(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                     ExportView ex, BatchCtl* ctl, unsigned long long* stats) {
    const uint32_t cap = t.mask + 1;
    hipLaunchKernelGGL(k_finalize, dim3(table_grid(cap)), dim3(256), 0, st, b, p, t, f, ex, ctl, stats, cap);
}

// ---- complex flows: sequential replay of put_pkt_recursive ------------------------------
// Each complex flow gets a rank and a segment of its packet count.  A workgroup scans a
// contiguous range of at most CXR_SPAN slots, lists its complex ones in LDS, and takes ranks and
// packet positions for all of them with ONE atomic on the {ranks, packets} counter (a returning
// atomic per lane, then per wave, on that one word serialised: ~10^5 complex flows per batch of
// the configs[2] mix with its plugins, 0.37 ms per batch at one atomic per wave).
constexpr uint32_t CXR_SPAN = 4096;  // slots per workgroup (LDS list: 8 bytes per entry)
__global__ __launch_bounds__(256) void k_complex_rank(TableView t, ComplexView cx, BatchCtl* ctl, uint32_t cap,
                                                      uint32_t span, uint32_t ncx) {
    __shared__ uint32_t l_slot[CXR_SPAN], l_npk[CXR_SPAN];
    __shared__ uint32_t l_n, scan_s[256 / 64 + 1];
    __shared__ unsigned long long l_base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) l_n = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * span, s1 = min(cap, s0 + span);
    for (uint32_t s = s0 + tid; s < s1; s += 256) {
        const uint64_t key = t.hot(s).key;
        const uint32_t st = t.hot(s).state;
        if (key == 0 || !(st & SLOT_COMPLEX)) continue;
        const uint64_t a0 = t.hot(s).acc[0], a1 = t.hot(s).acc[1];
        const uint32_t k = atomicAdd(&l_n, 1u);
        l_slot[k] = s;
        l_npk[k] = (uint32_t)(a0 >> 40) + (uint32_t)(a1 >> 40);
    }
    __syncthreads();
    const uint32_t n = l_n;
    if (n == 0) return;  // (uniform)
    // packets: thread tid sums entries [tid * per, +per), a block scan gives each range's offset
    const uint32_t per = (n + 255) / 256, k0 = min(n, tid * per), k1 = min(n, k0 + per);
    uint32_t sum = 0;
    for (uint32_t k = k0; k < k1; ++k) sum += l_npk[k];
    uint32_t tot;
    uint32_t off = block_exclusive_scan<256>(sum, scan_s, &tot);
    if (tid == 0) l_base = atomicAdd((unsigned long long*)&ctl->cx_alloc, ((unsigned long long)n << 32) | tot);
    __syncthreads();
    const uint32_t r0 = (uint32_t)(l_base >> 32), p0 = (uint32_t)l_base;
    if (r0 + n > ncx) {  // more complex slots than the finalisers counted (guard; the host reports it)
        if (tid == 0) atomicOr(&ctl->guard, 1u);
        return;
    }
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t sl = l_slot[k], npk = l_npk[k], r = r0 + k;
        t.slot_rank[sl] = r;
        cx.slot_of[r] = sl;
        cx.seg[r] = p0 + off;
        cx.len[r] = npk;
        cx.cursor[r] = 0;
        off += npk;
        const uint64_t key = t.hot(sl).key;
        uint32_t e = (uint32_t)key & cx.kmask;  // >= 2 entries per complex flow: terminates
        while (atomicCAS(&cx.keys[e], 0ull, (unsigned long long)key) != 0ull) e = (e + 1) & cx.kmask;
        cx.key_rank[e] = r;
        if (cx.bloom) atomicOr(&cx.bloom[((uint32_t)key >> 5) & cx.bmask], 1u << ((uint32_t)key & 31u));
    }
}

void launch_complex_rank(hipStream_t st, TableView t, ComplexView cx, BatchCtl* ctl, uint32_t cap, uint32_t ncx) {
    // at least 2048 workgroups, at most CXR_SPAN slots each
    uint32_t g = std::max<uint32_t>(std::min<uint32_t>(2048, (cap + 255) / 256), (cap + CXR_SPAN - 1) / CXR_SPAN);
    const uint32_t span = ((cap + g - 1) / g + 255) & ~255u;
    g = (cap + span - 1) / span;
    hipLaunchKernelGGL(k_complex_rank, dim3(g ? g : 1), dim3(256), 0, st, t, cx, ctl, cap, span, ncx);
}

__global__ __launch_bounds__(64) void k_complex_walk(BatchView b, Params p, TableView t, FragView f,
                                                     ComplexView cx, uint32_t nranks, ExportView ex,
                                                     BatchCtl* ctl, unsigned long long* stats) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nranks) return;
    const uint32_t s = cx.slot_of[r];
    const HotSlot h = t.hot(s);
    if (h.state & SLOT_HOST) return;  // a process plugin's flow: the host walks it (plugin_walk)
    bool live = h.state & SLOT_LIVE;
    if (!live) atomicAdd(&ctl->cx_new_live, 1u);  // the slot ends the walk live
    ipxg_flow_record rec;
    if (live) rec = tbl_rec(t, s);
    const uint32_t seg = cx.seg[r], len = cx.len[r];
    const uint32_t I = p.inactive_s, A = p.active_s;
    uint32_t n_ex = 0;
    for (uint32_t k = 0; k < len; ++k) {
        const uint32_t idx = (uint32_t)(cx.sorted[seg + k] & 0xFFFFFF);
        DevPkt pk;
        ipxg_pkt_desc d;
        reparse<true>(b, p, f, idx, pk, d);
        uint64_t lo, hf;
        uint32_t cdir;
        canon(pk, p, lo, cdir, hf);
        bool dsrc = true;
        if (live) {  // cache.cpp:428-472
            dsrc = p.split_biflow || hf == rec.flow_hash;  // cache.cpp:428 (the record may be the host walk's)
            const uint8_t flw = dsrc ? rec.src_tcp_flags : rec.dst_tcp_flags;
            uint8_t reason = 0;
            if ((pk.tcp_flags & 0x02) && (flw & 0x05)) reason = IPXG_FLOW_END_EOF;
            else if ((int64_t)d.ts_sec - (int64_t)rec.time_last_sec >= (int64_t)I) reason = export_reason(rec);
            else if ((int64_t)d.ts_sec - (int64_t)rec.time_first_sec >= (int64_t)A) reason = IPXG_FLOW_END_ACTIVE;
            if (reason) {
                uint32_t pos = atomicAdd(ex.count, 1u);
                store_export(ex, pos, rec, reason);
                if (ex.count6 && rec.ip_version == 6) atomicAdd(ex.count + 2, 1u);
                atomicAdd(&stat_row(stats)[ST_END_INACTIVE + reason - 1], 1ull);
                atomicAdd(&stat_row(stats)[ST_PKTS_1 + pkts_bucket((uint64_t)rec.src_packets + rec.dst_packets)], 1ull);
                n_ex++;
                live = false;
            }
        }
        if (!live) {
            rec_create(rec, pk, d, hf, cdir);
            rec.src_packets = 1;
            rec.src_bytes = pk.ip_len;
            if (pk.ip_proto == 6) rec.src_tcp_flags = pk.tcp_flags;
            live = true;
        } else {
            rec.time_last_sec = d.ts_sec;
            rec.time_last_usec = d.ts_usec;
            if (dsrc) {
                rec.src_packets++;
                rec.src_bytes += pk.ip_len;
                if (pk.ip_proto == 6) rec.src_tcp_flags |= pk.tcp_flags;
            } else {
                rec.dst_packets++;
                rec.dst_bytes += pk.ip_len;
                if (pk.ip_proto == 6) rec.dst_tcp_flags |= pk.tcp_flags;
            }
        }
    }
    tbl_put_rec(t, s, rec);
    clear_slot(&t.hot(s), h.key, SLOT_LIVE);
    count_flow_ports(t, rec, len);  // every packet of the walk: the flow's ports
    if (n_ex) atomicAdd(&ctl->exported, n_ex);
}

void launch_complex_walk(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                         ComplexView cx, uint32_t nranks, ExportView ex, BatchCtl* ctl,
                         unsigned long long* stats) {
    hipLaunchKernelGGL(k_complex_walk, dim3((nranks + 63) / 64), dim3(64), 0, st, b, p, t, f, cx, nranks,
                       ex, ctl, stats);
}

// ---- maintenance: export_expired / finish / rehash / count ------------------------------
constexpr uint32_t SCAN_PER_THREAD = 1;  // slots per thread in the export scans (more made the
                                         // cold-record loads wait on the previous export stores)

static inline uint32_t scan_grid(uint32_t cap) {
    const uint32_t per = 256 * SCAN_PER_THREAD;
    return (cap + per - 1) / per;
}

// Export every live record idle for >= inactive seconds at `now` (export_expired,
// cache.cpp:508-523, over the whole table).  Slots [blk*256*SCAN_PER_THREAD, ...); one
// export-buffer reservation per block (a single counter saturates at ~88 returning
// atomics/us: MI355X_MICROARCH.md "dequeue").
// A finish or expire enqueued right behind a batch whose control block the host has not read
// must not run when the batch left work for the host (fragments, deferred packets or
// finalise-list entries, the table scan, complex flows, a slow pass to run again) or when the
// export buffer might not hold every live record; every workgroup decides alike from fields the
// kernel does not change, workgroup 0 reports it (guard->hold).
__device__ __forceinline__ bool guard_holds(BatchCtl* guard, uint32_t ex_before, uint32_t live_before, uint32_t cap) {
    const bool hold = guard->frag_count || guard->deferred || guard->agg_deferred || guard->pending ||
                      guard->complex_count || guard->fin_deferred || guard->slow_redo ||
                      (uint64_t)ex_before + guard->exported + live_before + guard->new_live > cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) guard->hold = hold ? 1u : 0u;
    return hold;
}

__global__ __launch_bounds__(256) void k_expire(Params p, TableView t, uint32_t cap, int64_t now,
                                                ExportView ex, unsigned long long* stats, BatchCtl* guard,
                                                uint32_t* expired, uint32_t ex_before, uint32_t live_before,
                                                int64_t floor, uint32_t* tls_inv) {
    __shared__ uint32_t scratch[8];
    __shared__ uint32_t sc[ST_COUNT];
    __shared__ uint32_t bbase;
    __shared__ uint32_t tmin;
    if (guard && guard_holds(guard, ex_before, live_before, ex.cap)) return;
    // no live record can be idle: each one's time_last_sec is at least the floor, later than
    // now - inactive (the batch in front of a guarded expire kept the order: no older packet)
    if (floor != IDLE_FLOOR_NONE && now - (int64_t)p.inactive_s < floor && !(guard && guard->nonmono)) return;
    if (threadIdx.x < ST_COUNT) sc[threadIdx.x] = 0;
    if (threadIdx.x == 0) tmin = 0xFFFFFFFFu;
    const uint32_t base = blockIdx.x * 256 * SCAN_PER_THREAD;
    uint32_t mask = 0, c = 0, my_min = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_PER_THREAD; ++j) {
        const uint32_t s = base + j * 256 + threadIdx.x;
        if (s >= cap) continue;
        const uint64_t key = t.hot(s).key;
        const uint32_t state = t.hot(s).state;
        if (key == 0 || !(state & SLOT_LIVE)) continue;
        const uint32_t tls = t.line[s].head[RW_TLS];
        if (now - (int64_t)tls >= (int64_t)p.inactive_s) {
            // the record leaves with its plugin extensions: nothing is followed any more (a
            // FOLLOW bit left behind kept the dead slot through every rehash and sent the key's
            // next packets to the host walk)
            t.hot(s).state = state & ~(SLOT_LIVE | SLOT_FOLLOW);
            mask |= 1u << j;
            c++;
        } else {
            my_min = min(my_min, tls);
        }
    }
    if (tls_inv) {  // the least time_last_sec left live: wave minimum, one LDS atomic per wave
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) my_min = min(my_min, (uint32_t)__shfl_xor((int)my_min, o));
        if ((threadIdx.x & 63) == 0 && my_min != 0xFFFFFFFFu) atomicMin(&tmin, my_min);
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<256>(c, scratch, &total);  // (its barriers: tmin complete)
    if (tls_inv && threadIdx.x == 0) {  // ~min as a maximum (1: scanned, none left); most blocks find
                                        // a larger value already there and add no atomic
        const uint32_t v = tmin == 0xFFFFFFFFu ? 1u : max(~tmin, 2u);
        if (v > __hip_atomic_load(tls_inv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(tls_inv, v);
    }
    if (threadIdx.x == 0) bbase = total ? atomicAdd(ex.count, total) : 0;
    if (threadIdx.x == 0 && total && expired) atomicAdd(expired, total);
    __syncthreads();
    uint32_t pos = bbase + off;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_PER_THREAD; ++j) {
        const bool mine = mask >> j & 1;
        RecW rec;
        uint8_t reason = 0;
        if (mine) {
            rec = tbl_load_rec(t, base + j * 256 + threadIdx.x);
            reason = export_reason_w(rec);
            store_export_w(ex, pos++, rec, reason);
        }
        count_exports_wave(sc, mine, rec, reason);
        count_v6_exports(ex, mine && rw_ipver(rec) == 6);
    }
    flush_block_stats(sc, stats);
}

void launch_expire(hipStream_t st, const Params& p, TableView t, uint32_t cap, int64_t now,
                   ExportView ex, unsigned long long* stats, BatchCtl* guard, uint32_t* expired,
                   uint32_t ex_before, uint32_t live_before, int64_t floor, uint32_t* tls_inv) {
    hipLaunchKernelGGL(k_expire, dim3(scan_grid(cap)), dim3(256), 0, st, p, t, cap, now, ex, stats, guard, expired,
                       ex_before, live_before, floor, tls_inv);
}

// Export every live record as FLOW_END_FORCED (finish, cache.cpp:276-288) and empty the
// table (every occupied slot it scans is zeroed).
// guard != nullptr: a finish enqueued right behind a batch before the host has read the
// batch's control block (guard_holds); when it holds, the host completes the batch and finishes
// again.
// FIN_SCAN_THREADS slots per workgroup: one reservation of export records per workgroup, a
// returning atomic on the one counter (~11 ns each when they queue: MI355X_MICROARCH.md "fanin") --
// at 256 slots per workgroup a 2^21-slot table made 8192 of them.  1024: configs[4]'s finish 140 ->
// 136 us (the reservations mostly overlap the scan's loads; profiles/r06/finish_ab.txt).
#ifndef IPXG_FINISH_THREADS
#define IPXG_FINISH_THREADS 1024
#endif
constexpr uint32_t FIN_SCAN_THREADS = IPXG_FINISH_THREADS;
__global__ __launch_bounds__(FIN_SCAN_THREADS) void k_finish(TableView t, uint32_t cap, ExportView ex,
                                                unsigned long long* stats, BatchCtl* guard, uint32_t ex_before,
                                                uint32_t live_before) {
    __shared__ uint32_t scratch[FIN_SCAN_THREADS / 64 + 1];
    __shared__ uint32_t bbase;
    __shared__ uint32_t pb[6];  // FlowRecordStats buckets of the block's exports
    if (guard && guard_holds(guard, ex_before, live_before, ex.cap)) return;
    const uint32_t base = blockIdx.x * FIN_SCAN_THREADS * SCAN_PER_THREAD;
    uint32_t mask = 0, c = 0;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_PER_THREAD; ++j) {
        const uint32_t s = base + j * FIN_SCAN_THREADS + threadIdx.x;
        if (s >= cap) continue;
        if (t.hot(s).key == 0) continue;  // an empty slot is all zero already
        if (t.hot(s).state & SLOT_LIVE) {
            mask |= 1u << j;
            c++;
        }
        uint4* z = reinterpret_cast<uint4*>(&t.hot(s));
        z[0] = z[1] = z[2] = z[3] = make_uint4(0, 0, 0, 0);
    }
    uint32_t total;
    const uint32_t off = block_exclusive_scan<FIN_SCAN_THREADS>(c, scratch, &total);
    if (threadIdx.x == 0) bbase = total ? atomicAdd(ex.count, total) : 0;
    if (threadIdx.x < 6) pb[threadIdx.x] = 0;
    __syncthreads();
    uint32_t pos = bbase + off;
#pragma unroll
    for (uint32_t j = 0; j < SCAN_PER_THREAD; ++j) {
        const bool mine = mask >> j & 1;
        RecW rec;
        if (mine) {
            rec = tbl_load_rec(t, base + j * FIN_SCAN_THREADS + threadIdx.x);
            store_export_w(ex, pos++, rec, IPXG_FLOW_END_FORCED);
        }
        {  // the FlowRecordStats buckets, one LDS atomic per wave and bucket present
            const uint32_t bk = mine ? pkts_bucket((uint64_t)rec.w[RW_SPK] + rec.w[RW_DPK]) : 0u;
#pragma unroll
            for (uint32_t q = 0; q < 6; ++q) {
                const unsigned long long m = __ballot(mine && bk == q);
                if ((threadIdx.x & 63) == 0 && m) atomicAdd(&pb[q], (uint32_t)__popcll(m));
            }
        }
        count_v6_exports(ex, mine && rw_ipver(rec) == 6);
    }
    __syncthreads();
    unsigned long long* const sh = stat_row(stats);
    if (threadIdx.x == 0 && total) atomicAdd(&sh[ST_END_FORCED], (unsigned long long)total);
    if (threadIdx.x < 6 && pb[threadIdx.x]) atomicAdd(&sh[ST_PKTS_1 + threadIdx.x], (unsigned long long)pb[threadIdx.x]);
}

// Copy a control block and the export counters into host-mapped memory, without a D2H copy
// command of its own: [ctl_words of the block][4 export words][sequence word].  seq != 0: the
// sequence word is written last, behind a system-scope fence of every lane's copies -- the host
// polls it instead of waiting for the stream to drain (work queued behind this kernel keeps
// running: ipxg_engine.cpp wait_seq).
__global__ __launch_bounds__(64) void k_publish(const uint32_t* ctl, const uint32_t* ex, uint32_t* dst,
                                                uint32_t ctl_words, uint32_t seq) {
    for (uint32_t i = threadIdx.x; i < ctl_words; i += 64) dst[i] = ctl[i];
    if (threadIdx.x < 4) dst[ctl_words + threadIdx.x] = ex[threadIdx.x];
    if (seq) {
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(&dst[ctl_words + 4], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void launch_publish(hipStream_t st, const uint32_t* ctl, const uint32_t* ex, uint32_t* dst, uint32_t ctl_words,
                    uint32_t seq) {
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, ctl, ex, dst, ctl_words, seq);
}

// Closes the holes a fused k_fin_list left in its export reservation (BatchCtl::ex_holes: flows that
// turned complex or found no slot).  A rare path -- those flows send the batch to the host's sequential
// path anyway -- so one workgroup walks [lo, hi) in 1024-record chunks: each chunk is read whole (the
// scan's barriers) before any of it is written, and every destination lies at or below its source, so
// the copy is in place and keeps the order.
__global__ __launch_bounds__(1024) void k_ex_compact(ExportView ex, uint32_t lo, uint32_t hi) {
    __shared__ uint32_t scan_s[1024 / 64 + 1];
    uint32_t out = lo;
    for (uint32_t base = lo; base < hi; base += 1024) {  // uniform
        const uint32_t k = base + threadIdx.x;
        RecW r;
        bool keep = false;
        if (k < hi) {
            r = rec_load_w(&ex.buf[k]);
            keep = ((r.w[RW_VLAN] >> 16) & 0xFF) != 0;
        }
        uint32_t tot;
        const uint32_t pos = block_exclusive_scan<1024>(keep ? 1u : 0u, scan_s, &tot);
        if (keep) rec_store_w(&ex.buf[out + pos], r);
        out += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) ex.count[0] = out;
}

void launch_ex_compact(hipStream_t st, ExportView ex, uint32_t lo, uint32_t hi) {
    hipLaunchKernelGGL(k_ex_compact, dim3(1), dim3(1024), 0, st, ex, lo, hi);
}

void launch_finish(hipStream_t st, TableView t, uint32_t cap, ExportView ex, unsigned long long* stats,
                   BatchCtl* guard, uint32_t ex_before, uint32_t live_before) {
    hipLaunchKernelGGL(k_finish, dim3((cap + FIN_SCAN_THREADS * SCAN_PER_THREAD - 1) / (FIN_SCAN_THREADS * SCAN_PER_THREAD)),
                       dim3(FIN_SCAN_THREADS), 0, st, t, cap, ex, stats, guard, ex_before, live_before);
}

__global__ __launch_bounds__(256) void k_rehash(TableView from, uint32_t from_cap, TableView to,
                                                uint32_t* fail) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < from_cap; s += gridDim.x * blockDim.x) {
        const HotSlot h = from.hot(s);
        if (h.key == 0) continue;
        if (!(h.state & (SLOT_LIVE | SLOT_COMPLEX | SLOT_HOST)) && h.last1 == 0) continue;  // dead slot
        uint32_t ns = (uint32_t)h.key & to.mask;
        bool ok = false;
        for (uint32_t probe = 0; probe <= to.mask; ++probe) {
            unsigned long long old = atomicCAS((unsigned long long*)&to.hot(ns).key, 0ull,
                                               (unsigned long long)h.key);
            if (old == 0) {
                ok = true;
                break;
            }
            ns = (ns + 1) & to.mask;
        }
        if (!ok) {
            atomicAdd(fail, 1u);
            continue;
        }
        HotSlot c = h;
        uint32_t* dst = reinterpret_cast<uint32_t*>(&to.hot(ns));
        const uint32_t* src = reinterpret_cast<const uint32_t*>(&c);
        for (int k = 2; k < 16; ++k) dst[k] = src[k];  // key already claimed
        tbl_store_rec(to, ns, tbl_load_rec(from, s));
    }
}

void launch_rehash(hipStream_t st, TableView from, uint32_t from_cap, TableView to, uint32_t* fail) {
    hipLaunchKernelGGL(k_rehash, dim3(table_grid(from_cap)), dim3(256), 0, st, from, from_cap, to, fail);
}

// ---- stateless entry points ------------------------------------------------------------------
__global__ __launch_bounds__(IPXG_BLOCK) void k_parse_batch(BatchView b, uint32_t dlt, ipxg_parsed_pkt* out) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    const uint32_t i = blockIdx.x * IPXG_BLOCK + threadIdx.x;
    if (i >= b.n) return;
    const ipxg_pkt_desc d = b.desc[i];
    uint32_t* col = &win[threadIdx.x];
    stage_frame(col, frame_ptr(b, d), d.caplen);
    LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
    DevPkt pk;
    ParseCounts c = {};
    const bool ok = parse_frame<true>(S, d.caplen, dlt, pk, c);
    ipxg_parsed_pkt o = to_parsed(pk, ok);
    out[i] = o;
}

void launch_parse_batch(hipStream_t st, const BatchView& b, uint32_t dlt, ipxg_parsed_pkt* out) {
    hipLaunchKernelGGL(k_parse_batch, dim3((b.n + IPXG_BLOCK - 1) / IPXG_BLOCK), dim3(IPXG_BLOCK), 0, st, b,
                       dlt, out);
}

__global__ __launch_bounds__(256) void k_xxh64(const uint8_t* keys, uint32_t keylen, uint32_t n, uint64_t seed,
                                               uint64_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* k = keys + (size_t)i * keylen;
    if (seed == 0 && keylen == 16) {
        uint64_t w0 = 0, w1 = 0;
        for (int q = 7; q >= 0; --q) {
            w0 = (w0 << 8) | k[q];
            w1 = (w1 << 8) | k[8 + q];
        }
        out[i] = xxh64_16(w0, w1);
    } else if (seed == 0 && keylen == 40) {
        uint64_t w[5] = {0, 0, 0, 0, 0};
        for (int j = 0; j < 5; ++j)
            for (int q = 7; q >= 0; --q) w[j] = (w[j] << 8) | k[8 * j + q];
        out[i] = xxh64_40(w[0], w[1], w[2], w[3], w[4]);
    } else {
        out[i] = xxh64_any(k, keylen, seed);
    }
}

void launch_xxh64(hipStream_t st, const uint8_t* keys, uint32_t keylen, uint32_t n, uint64_t seed,
                  uint64_t* out) {
    hipLaunchKernelGGL(k_xxh64, dim3((n + 255) / 256), dim3(256), 0, st, keys, keylen, n, seed, out);
}

// ---- parser side statistics (ps=true) ----------------------------------------------------
// Per packet of the batch, as parse_packet keeps them in ParserStats (parser-stats.hpp:126-201):
// VlanStats for the packet's VLAN id (parser.cpp:798: every valid packet, sizes = caplen), and
// the TopPorts increments the flow records cannot carry (count_flow_ports): a TCP segment
// dropped after parse_tcp_hdr read its ports, and TCP/UDP packets with both ports 0.
// Each lane sums its packets' VlanStats in registers while their VLAN id stays the same (one
// id for untagged traffic), then adds them to the block's LDS copy of that id (64 ids,
// direct-mapped; another id in the entry: straight to the device counters); the block adds
// its LDS copies to the device counters at the end.
constexpr uint32_t VS_EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ void vs_flush(uint32_t vid, const uint32_t (&acc)[VS_N], uint32_t* vkey,
                                         uint32_t (*vacc)[VS_N], unsigned long long* vlan_st) {
    if (vid == VS_EMPTY) return;
    const uint32_t e = vid & 63;
    const uint32_t k = atomicCAS(&vkey[e], VS_EMPTY, vid);
    if (k == VS_EMPTY || k == vid) {
#pragma unroll
        for (uint32_t q = 0; q < VS_N; ++q)
            if (acc[q]) atomicAdd(&vacc[e][q], acc[q]);
    } else {
#pragma unroll
        for (uint32_t q = 0; q < VS_N; ++q)
            if (acc[q]) atomicAdd(&vlan_st[(size_t)vid * VS_N + q], (unsigned long long)acc[q]);
    }
}

__global__ __launch_bounds__(256) void k_pstats(BatchView b, Params p, unsigned long long* pstat) {
    if (gated(p)) return;  // (a front launched ahead of the previous batch's completion: as k_bin)
    __shared__ uint32_t win[IPXG_WIN_DW * 256];
    __shared__ uint32_t vkey[64];
    __shared__ uint32_t vacc[64][VS_N];
    unsigned long long* const ports = pstat;
    unsigned long long* const vlan_st = pstat + PSTAT_PORTS;
    const uint32_t tid = threadIdx.x;
    if (tid < 64) vkey[tid] = VS_EMPTY;
    for (uint32_t q = tid; q < 64 * VS_N; q += 256) (&vacc[0][0])[q] = 0;
    __syncthreads();
    uint32_t cur = VS_EMPTY, acc[VS_N];
#pragma unroll
    for (uint32_t q = 0; q < VS_N; ++q) acc[q] = 0;
    const bool eth = p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB;
    for (uint32_t i = blockIdx.x * 256 + tid; i < b.n; i += gridDim.x * 256) {
        const ipxg_pkt_desc d = b.desc[i];
        DevPkt pk;
        ParseCounts dummy = {};
        bool ok = false, fast = false;
        if (eth && fast_shape(b, d)) {
            const uint4* fr = reinterpret_cast<const uint4*>(frame_ptr(b, d));
            fast = ok = parse_fast(fr[0], fr[1], fr[2], d.caplen, false, pk, dummy);
        }
        if (!fast) {
            stage_frame(&win[tid], frame_ptr(b, d), d.caplen);
            LdsFrame S{{&win[tid], {frame_ptr(b, d), d.caplen}}};
            ok = parse_frame<false>(S, d.caplen, p.dlt, pk, dummy);
        }
        if (pk.l4 && (ok ? (pk.src_port == 0 && pk.dst_port == 0) : pk.l4 == 6)) {  // rare
            unsigned long long* a = ports + (pk.l4 == 17 ? 65536 : 0);
            atomicAdd(a + pk.src_port, 1ull);
            atomicAdd(a + pk.dst_port, 1ull);
        }
        if (!ok) continue;
        const uint32_t vid = pk.vlan_id & 0xFFF;
        if (vid != cur) {
            vs_flush(cur, acc, vkey, vacc, vlan_st);
            cur = vid;
#pragma unroll
            for (uint32_t q = 0; q < VS_N; ++q) acc[q] = 0;
        }
        const uint32_t len = d.caplen;  // packet_len = caplen (parser.cpp:771), uint16_t
        const bool v4 = pk.ip_version == 4, v6 = pk.ip_version == 6;
        acc[0] += v4;
        acc[1] += v6;
        acc[2] += v4 ? len : 0;
        acc[3] += v6 ? len : 0;
        acc[4] += pk.ip_proto == 6;
        acc[5] += pk.ip_proto == 17;
        acc[6] += 1;
        acc[7] += len;
        const uint32_t bk = len <= 64 ? 0 : len < 128 ? 1 : len < 256 ? 2 : len < 512 ? 3 : len < 1024 ? 4
                          : len < 1518 ? 5 : len < 2048 ? 6 : len < 4096 ? 7 : len < 8192 ? 8 : 9;
#pragma unroll
        for (uint32_t q = 0; q < IPXG_SIZE_BUCKETS; ++q) {  // compile-time indices only
            acc[8 + q] += bk == q;
            acc[8 + IPXG_SIZE_BUCKETS + q] += bk == q ? len : 0;
        }
    }
    vs_flush(cur, acc, vkey, vacc, vlan_st);
    __syncthreads();
    for (uint32_t q = tid; q < 64 * VS_N; q += 256) {
        const uint32_t e = q / VS_N, f = q % VS_N;
        const uint32_t v = (&vacc[0][0])[q];
        if (v && vkey[e] != VS_EMPTY) atomicAdd(&vlan_st[(size_t)vkey[e] * VS_N + f], (unsigned long long)v);
    }
}

void launch_pstats(hipStream_t st, const BatchView& b, const Params& p, unsigned long long* pstat) {
    uint32_t g = (b.n + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_pstats, dim3(g ? g : 1), dim3(256), 0, st, b, p, pstat);
}

}  // namespace ipxg
