// ipxg_bridge.hip -- device side of the process-plugin bridge.
//
// The reference calls its process plugins' hooks from NHTFlowCache::put_pkt_recursive for
// every packet (processPlugin.hpp:59-108; call sites cache.cpp:330-491), and a hook may end the
// flow there (FLOW_FLUSH / FLOW_FLUSH_WITH_REINSERT, cache.cpp:290-320).  Plugins look at
// particular packets only (DNS: port 53, HTTP: request/response lines, ...), so:
//   k_classify      pre-classifies every packet of the batch against the registered plugins'
//                   rules (TCP/UDP ports, payload prefixes) and marks the flows of the matching
//                   packets SLOT_PLUGIN in the flow table, before the ingest;
//   (ingest)        such a flow is aggregated as usual, then finalize_slot turns it complex,
//                   and the complex path gathers and sorts its packets of the batch;
//   k_plugin_pack   lists the plugin flows among the complex ones with their slot images;
//   k_plugin_pkts   parses their packets (every field a hook reads, payload included) and
//   k_plugin_bytes  copies the frames out -- the host replays put_pkt_recursive for these
//                   flows through the hooks, in packet order (ipxg_engine.cpp, plugin_walk);
//   k_plugin_apply  writes the flows' final slot and record back.
// Flows with none of the plugins' packets in a batch never leave the device (the plugin
// contract: hooks are no-ops on the packets outside the rule).
#include "ipxg_table.hpp"

namespace ipxg {

typedef uint32_t bridge_u32x4 __attribute__((ext_vector_type(4)));

// The 16 payload bytes at byte p of a frame at a 16-byte aligned offset o (two aligned 16-byte
// buffer loads, re-based by p & 15; zeros past the arena)
__device__ __forceinline__ uint4 payload16(__amdgpu_buffer_rsrc_t arena, uint32_t o, uint32_t p) {
    const uint32_t a = o + (p & ~15u);
    const bridge_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(arena, a, 0, 0);
    const bridge_u32x4 y = __builtin_amdgcn_raw_buffer_load_b128(arena, a + 16u, 0, 0);
    const uint32_t d[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    const uint32_t q = (p >> 2) & 3u, sh = p & 3u;
    uint32_t o4[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)  // dwords q .. q + 4 (selects: no dynamic register index)
        o4[j] = q == 0 ? d[j] : q == 1 ? d[j + 1] : q == 2 ? d[j + 2] : d[j + 3];
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(o4[1], o4[0], sh);
    r.y = __builtin_amdgcn_alignbyte(o4[2], o4[1], sh);
    r.z = __builtin_amdgcn_alignbyte(o4[3], o4[2], sh);
    r.w = __builtin_amdgcn_alignbyte(o4[4], o4[3], sh);
    return r;
}

// One packet against the plugins' rules, k_classify's test: frames of the shapes k_bin's wide walk
// takes are parsed from an 80-byte register window (and their payload's first 16 bytes loaded for
// the prefix rules); the others by the general parser in the lane's LDS column.  true: a rule
// matched, lo its flow's key.
__device__ __forceinline__ bool classify_packet(const BatchView& b, const Params& p, const DevRule* rules,
                                                uint32_t nrules, __amdgpu_buffer_rsrc_t rs_arena, uint32_t* col,
                                                uint32_t i, uint64_t& lo) {
    const bool eth = p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB;
    const ipxg_pkt_desc d = b.desc[i];
    DevPkt pk;
    ParseCounts dummy = {};
    bool reg = false, hit = false;
    // (the register window by buffer loads with byte offsets; 16-byte units: the general parser)
    if (eth && !b.oshift && fast_shape(b, d) && (uint64_t)d.offset + 80u <= b.arena_lim) {
        uint32_t w[WIDE_DW];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const bridge_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs_arena, d.offset + 16u * k, 0, 0);
            w[4 * k] = x.x;
            w[4 * k + 1] = x.y;
            w[4 * k + 2] = x.z;
            w[4 * k + 3] = x.w;
        }
        bool ext = false;
        reg = parse_medium<true>(w, d.caplen, p.frag_enable, pk, dummy, ext);
        if (reg && (pk.l4 == 6 || pk.l4 == 17)) {
            const uint4 pw = payload16(rs_arena, d.offset, pk.payload_off);
            const uint32_t pd[4] = {pw.x, pw.y, pw.z, pw.w};
            auto pay = [&](uint32_t k) {  // (bytes at or past caplen read as 0, as in the LDS walk)
                const uint32_t dw = k >> 2;
                const uint32_t v = dw == 0 ? pd[0] : dw == 1 ? pd[1] : dw == 2 ? pd[2] : pd[3];
                return (uint32_t)pk.payload_off + k < d.caplen ? (v >> (8 * (k & 3))) & 0xFFu : 0u;
            };
            for (uint32_t r = 0; r < nrules && !hit; ++r) hit = rule_match(rules[r], pk, pay);
        }
    }
    if (!reg) {
        stage_frame(col, frame_ptr(b, d), d.caplen);
        LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
        if (!parse_frame<true>(S, d.caplen, p.dlt, pk, dummy)) return false;
        if (pk.ip_version != 4 && pk.ip_version != 6) return false;
        if (pk.frag_off) return false;  // no L4 header (its ports come from the fragmentation cache)
        auto pay = [&](uint32_t k) { return S.b(pk.payload_off + k); };
        for (uint32_t r = 0; r < nrules && !hit; ++r) hit = rule_match(rules[r], pk, pay);
    }
    if (!hit) return false;
    uint64_t hf;
    uint32_t cdir;
    canon<false>(pk, p, lo, cdir, hf);
    return true;
}

// A plugin flow's slot claimed (if new) and marked SLOT_PLUGIN before k_reduce folds the batch
__device__ __forceinline__ void mark_plugin_flow(const TableView& t, BatchCtl* ctl, uint64_t lo, uint32_t& claimed_n) {
    uint4 head;
    bool claimed;
    HotSlot* h = probe_insert(t, lo, head, claimed);
    if (!h) {
        atomicOr(&ctl->plugin_fail, 1u);  // table too full to mark the flow (host: error)
        return;
    }
    if (claimed) claimed_n++;
    atomicOr(&h->state, SLOT_PLUGIN);
}

// Pre-classification of every packet against the plugins' rules (when k_bin does not check them
// itself: Params::plug off) -- which parsed every frame before: 0.9 ms per 10M-packet batch of the
// configs[2] mix, more than k_bin.
__global__ __launch_bounds__(IPXG_BLOCK) void k_classify(BatchView b, Params p, TableView t, const DevRule* rules,
                                                         uint32_t nrules, BatchCtl* ctl) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    uint32_t* col = &win[threadIdx.x];
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    uint32_t claimed_n = 0;
    for (uint32_t i = blockIdx.x * IPXG_BLOCK + threadIdx.x; i < b.n; i += gridDim.x * IPXG_BLOCK) {
        uint64_t lo;
        if (classify_packet(b, p, rules, nrules, rs_arena, col, i, lo)) mark_plugin_flow(t, ctl, lo, claimed_n);
    }
    if (claimed_n) atomicAdd(&ctl->new_keys, claimed_n);
}

// Params::plug: the marks k_bin (register walk: hits with their key, packets whose prefix test
// lies past the window) and k_bin_slow (its TCP/UDP packets) listed, workgroup b's at
// marks[b * slow_stride ...]: hits marked, the rest classified from their frames.
__global__ __launch_bounds__(IPXG_BLOCK) void k_plugin_marks(BatchView b, Params p, TableView t, const DevRule* rules,
                                                             uint32_t nrules, BatchCtl* ctl, BinView bv) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    uint32_t* col = &win[threadIdx.x];
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    uint32_t claimed_n = 0;
    for (uint32_t g = blockIdx.x; g < bv.bin_grid; g += gridDim.x) {  // (block-uniform)
        const uint32_t n = min(bv.mark_cnt[g], bv.slow_stride);
        const uint4* m = bv.marks + (size_t)g * bv.slow_stride;
        for (uint32_t k = threadIdx.x; k < n; k += IPXG_BLOCK) {
            const uint4 e = m[k];
            const uint32_t kind = e.z >> 30, i = e.z & 0x3FFFFFFFu;
            uint64_t lo = ((uint64_t)e.y << 32) | e.x;
            if (kind == MARK_HIT || (i < b.n && classify_packet(b, p, rules, nrules, rs_arena, col, i, lo)))
                mark_plugin_flow(t, ctl, lo, claimed_n);
        }
    }
    if (claimed_n) atomicAdd(&ctl->new_keys, claimed_n);
}

void launch_plugin_marks(hipStream_t st, const BatchView& b, const Params& p, TableView t, const DevRule* rules,
                         uint32_t nrules, BatchCtl* ctl, const BinView& bv) {
    hipLaunchKernelGGL(k_plugin_marks, dim3(bv.bin_grid ? bv.bin_grid : 1), dim3(IPXG_BLOCK), 0, st, b, p, t, rules,
                       nrules, ctl, bv);
}

void launch_classify(hipStream_t st, const BatchView& b, const Params& p, TableView t, const DevRule* rules,
                     uint32_t nrules, BatchCtl* ctl) {
    uint32_t g = (b.n + IPXG_BLOCK - 1) / IPXG_BLOCK;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_classify, dim3(g ? g : 1), dim3(IPXG_BLOCK), 0, st, b, p, t, rules, nrules, ctl);
}

// The plugin flows among the ncx complex ones, put in the order the host walks them -- by their
// first packet in the batch -- and everything the walk reads laid out in that order, so the host
// streams through memory and splits the flows over its threads by contiguous ranges:
//   k_plugin_keys   key[r] = first packet index << 32 | rank for a plugin flow, PF_NONE otherwise
//   (radix sort of the keys, 56 bits)
//   k_plugin_pack   flow k of the sorted keys -> PluginFlow out[k], its packet count flen[k]
//   (exclusive scan of flen: the flows' first positions in the packet list)
//   k_plugin_idx    the packet list (batch indices, flows in order, each flow's in arrival order)
//                   and each listed packet's captured length (exclusive scan: byte offsets)
//   k_plugin_totals {plugin flows, packets, bytes} for the host
constexpr uint64_t PF_NONE = (1ull << 56) - 1;

__global__ __launch_bounds__(256) void k_plugin_keys(TableView t, ComplexView cx, uint32_t ncx, uint64_t* keys,
                                                     uint32_t* count) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= ncx) return;
    const bool host = (t.hot(cx.slot_of[r]).state & SLOT_HOST) != 0;
    keys[r] = host ? ((cx.sorted[cx.seg[r]] & 0xFFFFFFull) << 32) | r : PF_NONE;
    // one atomic per wave
    const uint64_t m = __ballot(host);
    if (m && threadIdx.x % 64 == (uint32_t)__builtin_ctzll(m)) atomicAdd(count, (uint32_t)__popcll(m));
}

__global__ __launch_bounds__(256) void k_plugin_pack(TableView t, ComplexView cx, const uint64_t* skeys, uint32_t ncx,
                                                     const uint32_t* count, PluginFlow* out, uint32_t* flen,
                                                     uint32_t* hstate, uint32_t* lflag) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k > ncx) return;
    if (k >= *count) {
        flen[k] = 0;  // (the scans' tails: first[k] = packets, lpos[k] = live flows for k >= flows)
        lflag[k] = 0;
        return;
    }
    const uint32_t r = (uint32_t)skeys[k];
    const uint32_t s = cx.slot_of[r];
    const HotSlot h = t.hot(s);
    PluginFlow f;
    f.slot = s;
    f.seg = cx.seg[r];
    f.len = cx.len[r];
    f.state = h.state;
    f.key = h.key;
    f.pad = 0;
    f.rec = tbl_rec(t, s);
    out[k] = f;
    flen[k] = f.len;
    hstate[k] = f.state;
    lflag[k] = (f.state & SLOT_LIVE) ? 1u : 0u;
}

// The records of the flows live before the walk, compacted (rec[lpos[k]]): the host gets the
// records it needs, not 160-byte images of every flow.
__global__ __launch_bounds__(256) void k_plugin_recs(const PluginFlow* flows, const uint32_t* count,
                                                     const uint32_t* lflag, const uint32_t* lpos,
                                                     ipxg_flow_record* recs) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= *count || !lflag[k]) return;
    recs[lpos[k]] = flows[k].rec;
}

// One wave per flow: its packets' batch indices and captured lengths at first[k] ...
__global__ __launch_bounds__(256) void k_plugin_idx(BatchView b, ComplexView cx, const PluginFlow* flows,
                                                    const uint32_t* count, const uint32_t* first, uint32_t* idx,
                                                    uint64_t* clen) {
    const uint32_t lane = threadIdx.x % 64;
    const uint32_t nf = *count;
    for (uint32_t k = (blockIdx.x * 256 + threadIdx.x) / 64; k < nf; k += gridDim.x * 4) {
        const uint32_t seg = flows[k].seg, len = flows[k].len, at = first[k];
        for (uint32_t j = lane; j < len; j += 64) {
            const uint32_t i = (uint32_t)(cx.sorted[seg + j] & 0xFFFFFFu);
            idx[at + j] = i;
            clen[at + j] = ((uint32_t)b.desc[i].caplen + 15u) & ~15u;  // (16-byte aligned frame starts)
        }
    }
}

__global__ void k_plugin_totals(const uint32_t* count, const uint32_t* first, const uint64_t* off,
                                const uint32_t* lpos, uint64_t* tot) {
    const uint32_t nf = *count, m = first[nf];
    tot[0] = nf;
    tot[1] = m;
    tot[2] = off[m];
    tot[3] = lpos[nf];
}

// Packet idx[k] (k < the walked packets): every field a hook reads (ipxg_parsed_pkt, FULL parse),
// its descriptor and its index, as one WalkPkt; with a byte budget, also the length of it that
// crosses to the host (clen[k], 16-byte rounded): the whole frame when a plugin's rule matches the
// packet (k_classify's test on the parsed packet), else its headers and `budget` payload bytes.
__global__ __launch_bounds__(IPXG_BLOCK) void k_plugin_pkts(BatchView b, Params p, FragView f, const uint32_t* idx,
                                                            const uint32_t* count, const uint32_t* first, WalkPkt* out,
                                                            const DevRule* rules, uint32_t nrules, uint32_t budget,
                                                            uint64_t* clen) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    const uint32_t k = blockIdx.x * IPXG_BLOCK + threadIdx.x;
    if (k >= first[*count]) return;
    const uint32_t i = idx[k];
    const ipxg_pkt_desc d = b.desc[i];
    uint32_t* col = &win[threadIdx.x];
    stage_frame(col, frame_ptr(b, d), d.caplen);
    LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
    DevPkt pk;
    ParseCounts c = {};
    const bool ok = parse_frame<true>(S, d.caplen, p.dlt, pk, c);
    if (budget) {
        // (an unparsed frame and a fragment -- its ports come from the fragmentation cache -- cross whole)
        bool full = !ok || pk.frag_off || pk.more_fragments;
        if (!full && (pk.ip_version == 4 || pk.ip_version == 6) && (pk.l4 == 6 || pk.l4 == 17)) {
            auto pay = [&](uint32_t j) { return S.b(pk.payload_off + j); };
            for (uint32_t r = 0; r < nrules && !full; ++r) full = rule_match(rules[r], pk, pay);
        }
        const uint32_t n = full ? d.caplen : min((uint32_t)d.caplen, (uint32_t)pk.payload_off + budget);
        clen[k] = (n + 15u) & ~15u;
    }
    if (ok) apply_frag_ports(p, f, i, pk);  // a fragment's ports from the fragmentation cache
    WalkPkt w;
    w.pk = to_parsed(pk, ok);
    w.d = d;
    w.idx = i;
    out[k] = w;
}

void launch_plugin_order(hipStream_t st, const BatchView& b, const Params& p, FragView f, TableView t, ComplexView cx,
                         uint32_t ncx, uint32_t npk, const PluginOrder& o) {
    hipLaunchKernelGGL(k_plugin_keys, dim3((ncx + 255) / 256), dim3(256), 0, st, t, cx, ncx, o.keys, o.count);
    size_t tb = o.temp_bytes;
    (void)sort_keys_u64(o.temp, tb, o.keys, o.skeys, ncx, 56, st);
    hipLaunchKernelGGL(k_plugin_pack, dim3((ncx + 1 + 255) / 256), dim3(256), 0, st, t, cx, o.skeys, ncx, o.count,
                       o.flows, o.flen, o.hstate, o.lflag);
    tb = o.temp_bytes;
    (void)exclusive_scan_u32(o.temp, tb, o.flen, o.first, ncx + 1, st);
    tb = o.temp_bytes;
    (void)exclusive_scan_u32(o.temp, tb, o.lflag, o.lpos, ncx + 1, st);
    hipLaunchKernelGGL(k_plugin_recs, dim3((ncx + 255) / 256), dim3(256), 0, st, o.flows, o.count, o.lflag, o.lpos,
                       o.recs);
    uint32_t g = (ncx + 3) / 4;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_plugin_idx, dim3(g ? g : 1), dim3(256), 0, st, b, cx, o.flows, o.count, o.first, o.idx,
                       o.clen);
    hipLaunchKernelGGL(k_plugin_pkts, dim3((npk + IPXG_BLOCK - 1) / IPXG_BLOCK), dim3(IPXG_BLOCK), 0, st, b, p, f,
                       o.idx, o.count, o.first, o.wpk, o.rules, o.nrules, o.budget, o.clen);
    tb = o.temp_bytes;
    (void)exclusive_scan_u64(o.temp, tb, o.clen, o.off, npk + 1, st);
    hipLaunchKernelGGL(k_plugin_totals, dim3(1), dim3(1), 0, st, o.count, o.first, o.off, o.lpos, o.tot);
}

// Scratch bytes launch_plugin_order needs for ncx flows / npk packets (radix sort + scans).
size_t plugin_order_temp(uint32_t ncx, uint32_t npk) {
    size_t a = 0, c = 0, d = 0;
    (void)sort_keys_u64(nullptr, a, nullptr, nullptr, ncx, 56, nullptr);
    (void)exclusive_scan_u32(nullptr, c, nullptr, nullptr, ncx + 1, nullptr);
    (void)exclusive_scan_u64(nullptr, d, nullptr, nullptr, npk + 1, nullptr);
    return std::max(a, std::max(c, d));
}

// Frame bytes of packet idx[k] to out + off[k], a wave per packet: 16-byte copies when the frame
// starts on 16 bytes (out + off[k] always does: k_plugin_idx rounds the lengths up), so the
// rounded-up tail is read from inside the arena; byte copies otherwise.  (A workgroup per packet
// with byte copies: the quic walk's 330 MB of frames per batch.)
__global__ __launch_bounds__(256) void k_plugin_bytes(BatchView b, const uint32_t* idx, const uint64_t* off,
                                                      uint32_t m, uint8_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6); k < m; k += gridDim.x * 4) {
        const ipxg_pkt_desc d = b.desc[idx[k]];
        const uint8_t* src = frame_ptr(b, d);
        uint8_t* dst = out + off[k];
        const uint32_t n16 = (uint32_t)((off[k + 1] - off[k]) >> 4);  // (the frame, or its budget)
        if (frame_aligned(b, d) && frame_off(b, d) + 16ull * n16 <= b.arena_len) {
            for (uint32_t j = lane; j < n16; j += 64)
                reinterpret_cast<uint4*>(dst)[j] = reinterpret_cast<const uint4*>(src)[j];
        } else {
            const uint32_t n = min((uint32_t)d.caplen, 16u * n16);
            for (uint32_t j = lane; j < n; j += 64) dst[j] = src[j];
        }
    }
}

void launch_plugin_bytes(hipStream_t st, const BatchView& b, const uint32_t* idx, const uint64_t* off, uint32_t m,
                         uint8_t* out) {
    const uint32_t g = (m + 3) / 4 < 4096 ? (m + 3) / 4 : 4096;
    hipLaunchKernelGGL(k_plugin_bytes, dim3(g ? g : 1), dim3(256), 0, st, b, idx, off, m, out);
}

// The host walk's result: flow k's new slot state (LIVE -- and FOLLOW while a plugin follows every
// packet of it -- or empty of records), and the records of the flows live after the walk
// (out_recs[j] for flow out_idx[j]).
__global__ __launch_bounds__(256) void k_plugin_apply(TableView t, const PluginFlow* flows, const uint32_t* state,
                                                      uint32_t n, BatchCtl* ctl) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    const uint32_t slot = flows[k].slot;
    if (slot > t.mask) {  // (guard: never, unless the flow images were overwritten)
        atomicOr(&ctl->guard, 4u);
        return;
    }
    clear_slot(&t.hot(slot), flows[k].key, state[k] & (SLOT_LIVE | SLOT_FOLLOW));
}

__global__ __launch_bounds__(256) void k_plugin_apply_recs(TableView t, const PluginFlow* flows, uint32_t nf,
                                                           const ipxg_flow_record* recs, uint32_t n, BatchCtl* ctl) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    ipxg_flow_record r = recs[j];
    uint32_t k;
    memcpy(&k, r.reserved2, 4);  // the flow's index, carried in the record's spare bytes
    memset(r.reserved2, 0, sizeof(r.reserved2));
    if (k >= nf || flows[k].slot > t.mask) {  // (guard: the host handed back a bad index)
        atomicOr(&ctl->guard, 4u);
        return;
    }
    tbl_put_rec(t, flows[k].slot, r);
}

void launch_plugin_apply(hipStream_t st, TableView t, const PluginFlow* flows, const uint32_t* state, uint32_t nf,
                         const ipxg_flow_record* recs, uint32_t nrec, BatchCtl* ctl) {
    if (nrec)
        hipLaunchKernelGGL(k_plugin_apply_recs, dim3((nrec + 255) / 256), dim3(256), 0, st, t, flows, nf, recs, nrec, ctl);
    hipLaunchKernelGGL(k_plugin_apply, dim3((nf + 255) / 256), dim3(256), 0, st, t, flows, state, nf, ctl);
}

// chunk blockIdx.y, 16-byte word (blockIdx.x * 256 + threadIdx.x) of its records
__global__ __launch_bounds__(256) void k_host_gather(HostChunks c, uint4* dst) {
    const uint32_t ch = blockIdx.y;
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= c.n[ch] * 8u) return;
    dst[(size_t)c.at[ch] * 8u + w] = c.src[ch][w];
}

void launch_host_gather(hipStream_t st, const HostChunks& c, ipxg_flow_record* dst) {
    if (!c.count || !c.max_n) return;
    hipLaunchKernelGGL(k_host_gather, dim3((c.max_n * 8u + 255) / 256, c.count), dim3(256), 0, st, c,
                       reinterpret_cast<uint4*>(dst));
}

}  // namespace ipxg
