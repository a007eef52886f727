// ipxg_strict.hip -- strict mode (strict=true): the reference's own flow table, bit for bit.
//
// NHTFlowCache (cache.cpp:322-523) keeps 2^s records in lines of L = 2^l (default 16): a packet
// looks for its flow in the line of XXH64(key), then in the line of XXH64(inverse key); a hit
// moves to the line's front; a miss takes the line's first empty position or, in a full line,
// evicts the last one (FLOW_END_NO_RES) and inserts at position L/2; after every keyed packet
// a sweep cursor exports the idle records of the next L/2 positions of the table.  The result
// depends on the order of every packet that touches a line, which is why the default engine
// (order-independent batch reductions into a growing table) is exact only while no line
// overflows.  This mode replays those rules exactly, on the device:
//
//   k_strict_prep1   parse (statistics), fragments listed for the fragmentation cache (the
//                    engine then replays it: k_frag_walk) and the keyed packets marked;
//   (scan)           keyed prefix -> each keyed packet's sweep step q (cursor = q * L/2);
//   k_strict_prep2   re-parse with the fragment ports: both hashes, the update fields and the
//                    record the packet would create (FlowRecord::create, cache.cpp:94-132);
//   k_strict_lb      per line, a lower bound of the time_last values it holds during the batch;
//   k_strict_events  a keyed packet is an event on up to three lines: its forward line, its
//                    inverse line and the line its sweep visits -- the last only when the sweep
//                    can export something there (its second minus the line's bound reaches the
//                    inactive timeout): a sweep that provably exports nothing orders nothing, and
//                    dropping those events cuts the DAG's depth about four-fold (the sweep cursor
//                    otherwise chains every line to the packet order);
//   (sort)           events by line, stably: each line's sequence of packets;
//   k_strict_dag     each event's successor on its line and whether it has a predecessor: the
//                    per-line orders form a DAG over the packets (edges from lower to higher
//                    index, at most three per packet);
//   k_strict_ready   each packet's in-degree; the packets with none start the ready queue;
//   k_strict_walk    the replay: the 1024 lanes of ONE workgroup take queue tickets in order; a
//                    lane runs its ticket's packet once the entry is filled, then decrements its
//                    successors' in-degrees and queues those that reach zero.  Every line sees
//                    exactly the reference's sequence of operations (a topological order of the
//                    DAG), packets touching disjoint lines proceed in parallel, and every lane
//                    works on whatever is ready (round-robin packet ownership left most lanes of
//                    a wave waiting on their one packet: 4 Mpkt/s).  One workgroup: its lanes
//                    share one L1 and LDS, so the hand-off between two packets of a line needs
//                    only workgroup-scope ordering (no cross-CU release/acquire).
// The state: records [line * L + slot], their hashes (FlowRecord::m_hash, 0 = empty) and per
// line the position -> slot permutation (4 bits per position) standing in for the
// reference's pointer array m_flow_table: moves and evictions rewrite one 64-bit word.
#include "ipxg_table.hpp"

#include <cstdlib>

namespace ipxg {

// ---- parse, statistics, fragments, keyed marks -------------------------------------------------
__global__ __launch_bounds__(IPXG_BLOCK) void k_strict_prep1(BatchView b, Params p, FragView f, BatchCtl* ctl,
                                                             unsigned long long* stats) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    __shared__ uint32_t sc[ST_COUNT];
    const uint32_t tid = threadIdx.x;
    if (tid < ST_COUNT) sc[tid] = 0;
    __syncthreads();
    ParseCounts c = {};
    uint32_t keyless = 0, frags = 0;
    uint32_t* col = &win[tid];
    for (uint32_t i = blockIdx.x * IPXG_BLOCK + tid; i < b.n; i += gridDim.x * IPXG_BLOCK) {
        const ipxg_pkt_desc d = b.desc[i];
        stage_frame(col, frame_ptr(b, d), d.caplen);
        LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
        DevPkt pk;
        if (!parse_frame<false>(S, d.caplen, p.dlt, pk, c)) continue;
        if (pk.ip_version != 4 && pk.ip_version != 6) {  // create_hash_key false
            keyless++;
            continue;
        }
        if (p.frag_enable && (pk.frag_off || pk.more_fragments)) {
            frags++;
            divert_fragment(pk, p, f, ctl, i);
        }
    }
    flush_counts(c, keyless, frags, sc);
    flush_block_stats(sc, stats);
}

// every keyed packet's update fields, the record it would create, and its keyed mark
__global__ __launch_bounds__(IPXG_BLOCK) void k_strict_prep2(BatchView b, Params p, FragView f, StrictPkt* sp,
                                                             ipxg_flow_record* crec, uint32_t* keyed,
                                                             uint32_t* ts_acc) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    uint32_t* col = &win[threadIdx.x];
    uint32_t inv_min = 0;  // ~(earliest keyed second seen by this lane)
    for (uint32_t i = blockIdx.x * IPXG_BLOCK + threadIdx.x; i < b.n; i += gridDim.x * IPXG_BLOCK) {
        DevPkt pk;
        ipxg_pkt_desc d;
        StrictPkt s = {};
        const bool ok = reparse_lds<true>(b, p, f, i, col, pk, d) && (pk.ip_version == 4 || pk.ip_version == 6);
        if (ok) {
            FlowKey kf, ki;
            build_keys(pk, kf, ki);
            s.h_fwd = key_hash(kf);
            s.h_inv = key_hash(ki);
            s.ts_sec = d.ts_sec;
            s.ts_usec = d.ts_usec;
            s.ip_len = pk.ip_len;
            s.tcp_flags = pk.tcp_flags;
            s.ip_proto = pk.ip_proto;
            ipxg_flow_record r;
            rec_create(r, pk, d, s.h_fwd, 0);
            r.src_packets = 1;  // FlowRecord::create, cache.cpp:96-126
            r.src_bytes = pk.ip_len;
            if (pk.ip_proto == 6) r.src_tcp_flags = pk.tcp_flags;
            crec[i] = r;
            inv_min = max(inv_min, ~d.ts_sec);
        }
        sp[i] = s;
        keyed[i] = ok ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o; o >>= 1) inv_min = max(inv_min, (uint32_t)__shfl_xor((int)inv_min, o));
    if ((threadIdx.x & 63) == 0 && inv_min) atomicMax(ts_acc, inv_min);
}

// Per line: a lower bound of every time_last it holds while this batch runs -- the least of its
// records' time_last now (0xFFFFFFFF: empty) and the batch's first second (every record the batch
// creates or updates takes a packet's second).  A sweep step at second t on a line with
// t - lb < inactive finds no idle record whatever ran before it: k_strict_events leaves it out
// of the DAG (the line's order does not involve it) and the replay skips it.
__global__ __launch_bounds__(256) void k_strict_lb(StrictView v) {
    const uint32_t line = blockIdx.x * 256 + threadIdx.x;
    if (line >= v.lines) return;
    const uint32_t L = 1u << v.line_bits;
    uint32_t m = ~v.lb[v.lines];
    const uint32_t* tp = v.tlast + (size_t)line * L;
    for (uint32_t r = 0; r < L; ++r) m = min(m, tp[r]);
    v.lb[line] = m;
}

// Lines of packet i's events: forward, inverse (not split, not the forward line), and the line
// its sweep visits (not one of those); NONE = no event.  Sweep step q = q_base + its rank
// among the keyed packets (qx).
__device__ __forceinline__ uint32_t sweep_line(const StrictView& v, uint64_t q) {
    const uint32_t half = (1u << v.line_bits) >> 1;
    return half ? (uint32_t)((q * half) & v.slot_mask) >> v.line_bits : STRICT_NONE;
}

// (s.sweep 0: the sweep step provably exports nothing, no event on its line)
__device__ __forceinline__ void strict_lines(const StrictView& v, const StrictPkt& s, uint64_t q, uint32_t split,
                                             uint32_t (&ln)[3]) {
    const uint32_t mask = v.slot_mask & ~((1u << v.line_bits) - 1u);
    ln[0] = (uint32_t)(s.h_fwd & mask) >> v.line_bits;
    ln[1] = split ? STRICT_NONE : (uint32_t)(s.h_inv & mask) >> v.line_bits;
    if (ln[1] == ln[0]) ln[1] = STRICT_NONE;
    ln[2] = s.sweep ? sweep_line(v, q) : STRICT_NONE;
    if (ln[2] == ln[0] || ln[2] == ln[1]) ln[2] = STRICT_NONE;
}

__global__ __launch_bounds__(256) void k_strict_events(StrictView v, StrictPkt* sp, const uint32_t* keyed,
                                                       const uint32_t* qx, uint32_t n, uint64_t q_base,
                                                       uint32_t split, uint32_t inactive, uint32_t* keys,
                                                       uint32_t* vals) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t ln[3] = {STRICT_NONE, STRICT_NONE, STRICT_NONE};
    if (keyed[i]) {
        StrictPkt s = sp[i];
        const uint64_t q = q_base + qx[i];
        const uint32_t sl = sweep_line(v, q);
        // the sweep's idle test (strict_sweep) against the line's lower bound of time_last
        s.sweep = sl != STRICT_NONE && (int64_t)s.ts_sec - (int64_t)v.lb[sl] >= (int64_t)inactive;
        sp[i].sweep = s.sweep;
        strict_lines(v, s, q, split, ln);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        keys[3 * i + j] = ln[j] == STRICT_NONE ? v.lines : ln[j];  // v.lines sorts after every line
        vals[3 * i + j] = 4 * i + j;
    }
}

// each event's successor on its line (STRICT_NONE: the line's last) and predecessor flag
__global__ __launch_bounds__(256) void k_strict_dag(const uint32_t* keys, const uint32_t* vals, uint32_t m,
                                                    uint32_t lines, uint32_t* succ, uint8_t* pred) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    if (e >= m) return;
    const uint32_t L = keys[e];
    if (L >= lines) return;
    const uint32_t v = vals[e];  // 4 * packet + event slot
    succ[v] = e + 1 < m && keys[e + 1] == L ? vals[e + 1] >> 2 : STRICT_NONE;
    pred[v] = e > 0 && keys[e - 1] == L ? 1 : 0;
}

// in-degrees (events with a predecessor); the keyed packets with none go to the ready queue
__global__ __launch_bounds__(256) void k_strict_ready(const uint32_t* keys, const uint8_t* pred, const uint32_t* keyed,
                                                      uint32_t n, uint32_t lines, uint32_t* indeg, uint32_t* queue,
                                                      uint32_t* q_count) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t d = 0;
    bool ready = false;
    if (i < n) {
#pragma unroll
        for (int j = 0; j < 3; ++j)
            if (keys[3 * i + j] < lines && pred[4 * i + j]) d++;
        indeg[i] = d;
        ready = keyed[i] && d == 0;
    }
    const uint32_t pos = wave_append(q_count, ready);
    if (ready) queue[pos] = i;
}

// ---- the line permutation ---------------------------------------------------------------------
__device__ __forceinline__ uint32_t nib(uint64_t perm, uint32_t j) { return (uint32_t)(perm >> (4 * j)) & 15u; }
__device__ __forceinline__ uint64_t below(uint32_t j) { return j >= 16 ? ~0ull : ((1ull << (4 * j)) - 1ull); }
// the record at position a moves to position b <= a; positions b..a-1 move up by one
__device__ __forceinline__ uint64_t perm_move(uint64_t perm, uint32_t a, uint32_t b) {
    const uint64_t r = nib(perm, a);
    const uint64_t keep = perm & ~(below(a + 1) & ~below(b));
    const uint64_t seg = perm & below(a) & ~below(b);
    return keep | (seg << 4) | (r << (4 * b));
}

// ---- table reads ------------------------------------------------------------------------------
// One workgroup (MW false): plain loads -- its lanes share one CU and its L1, and a lane's stores
// are visible to the next packet of the line once they have completed (s_waitcnt vmcnt(0)).
// Several workgroups on ONE XCD (MW true): the lanes of different CUs hand lines to each other, and
// a CU's L1 is never refreshed by another CU's stores: every read of the table is an sc1 load
// (L1 bypassed, served by the XCD's L2, which every participating CU shares and which every
// completed store has reached) -- buffer loads of 16 bytes over the hash, time_last and record
// arrays, 8-byte agent-scope loads of the line maps.  Nothing else is handed over between lanes.
typedef unsigned int strict_u32x4 __attribute__((ext_vector_type(4)));
constexpr int STRICT_SC1 = 16;  // buffer-load cache policy: sc1

template <bool MW>
struct TableIO;

template <>
struct TableIO<false> {
    StrictView v;
    __device__ __forceinline__ uint64_t perm(uint32_t line) const { return v.perm[line]; }
    __device__ __forceinline__ void hashes(uint32_t line, uint32_t L, uint64_t (&h)[16]) const {
        const uint64_t* hp = v.hash + (size_t)line * L;
#pragma unroll
        for (uint32_t r = 0; r < 16; ++r) h[r] = r < L ? hp[r] : 0;
    }
    __device__ __forceinline__ void tlasts(uint32_t line, uint32_t L, uint32_t (&t)[16]) const {
        const uint32_t* tp = v.tlast + (size_t)line * L;
#pragma unroll
        for (uint32_t r = 0; r < 16; ++r) t[r] = r < L ? tp[r] : 0xFFFFFFFFu;
    }
    __device__ __forceinline__ RecW rec(uint32_t slot) const { return rec_load_w(&v.rec[slot]); }
};

template <>
struct TableIO<true> {
    StrictView v;
    __amdgpu_buffer_rsrc_t rh, rt, rr;
    __device__ explicit TableIO(const StrictView& sv) : v(sv) {
        const uint32_t S = sv.slot_mask + 1;  // (the engine pads hash and time_last by 64 bytes)
        rh = __builtin_amdgcn_make_buffer_rsrc(sv.hash, 0, (int)(S * 8u + 64u), 0x00020000);
        rt = __builtin_amdgcn_make_buffer_rsrc(sv.tlast, 0, (int)(S * 4u + 64u), 0x00020000);
        rr = __builtin_amdgcn_make_buffer_rsrc(sv.rec, 0, (int)(S * 128u), 0x00020000);
    }
    __device__ __forceinline__ uint64_t perm(uint32_t line) const {
        return __hip_atomic_load(&v.perm[line], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ void hashes(uint32_t line, uint32_t L, uint64_t (&h)[16]) const {
        const uint32_t o = line * L * 8u;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            strict_u32x4 x = {0, 0, 0, 0};
            if (2 * k < L) x = __builtin_amdgcn_raw_buffer_load_b128(rh, o + 16 * k, 0, STRICT_SC1);
            h[2 * k] = ((uint64_t)x.y << 32) | x.x;
            h[2 * k + 1] = 2 * k + 1 < L ? ((uint64_t)x.w << 32) | x.z : 0;
        }
    }
    __device__ __forceinline__ void tlasts(uint32_t line, uint32_t L, uint32_t (&t)[16]) const {
        const uint32_t o = line * L * 4u;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            strict_u32x4 x = {~0u, ~0u, ~0u, ~0u};
            if (4 * k < L) x = __builtin_amdgcn_raw_buffer_load_b128(rt, o + 16 * k, 0, STRICT_SC1);
            t[4 * k] = x.x;
            t[4 * k + 1] = 4 * k + 1 < L ? x.y : 0xFFFFFFFFu;
            t[4 * k + 2] = 4 * k + 2 < L ? x.z : 0xFFFFFFFFu;
            t[4 * k + 3] = 4 * k + 3 < L ? x.w : 0xFFFFFFFFu;
        }
    }
    __device__ __forceinline__ RecW rec(uint32_t slot) const {
        RecW r;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const strict_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rr, slot * 128u + 16u * i, 0, STRICT_SC1);
            r.w[4 * i] = x.x;
            r.w[4 * i + 1] = x.y;
            r.w[4 * i + 2] = x.z;
            r.w[4 * i + 3] = x.w;
        }
        return r;
    }
};

struct LineImg {
    uint64_t perm;
    uint64_t h[16];  // by record slot
};

template <bool MW>
__device__ __forceinline__ void load_line(const TableIO<MW>& io, uint32_t line, LineImg& li) {
    const uint32_t L = 1u << io.v.line_bits;
    li.perm = io.perm(line);
    io.hashes(line, L, li.h);
}

// the position of record slot r (< L) in the line's map: the one nibble equal to r, found as the
// lowest zero nibble of perm ^ r...r (positions >= L forced non-zero)
__device__ __forceinline__ uint32_t pos_of(uint64_t perm, uint32_t r, uint32_t L) {
    const uint64_t x = (perm ^ (0x1111111111111111ull * r)) | ~below(L);
    const uint64_t z = (x - 0x1111111111111111ull) & ~x & 0x8888888888888888ull;
    return (uint32_t)__builtin_ctzll(z) >> 2;
}

// the record slots of the line whose hash is h (bit r = slot r)
__device__ __forceinline__ uint32_t match_slots(const LineImg& li, uint32_t L, uint64_t h) {
    uint32_t rm = 0;
#pragma unroll
    for (uint32_t r = 0; r < 16; ++r)
        if (r < L && li.h[r] == h) rm |= 1u << r;
    return rm;
}
// the position of a flow's record (h != 0: at most one record of a line has a given hash --
// a packet finds an existing record before it creates one), NO_POS when none
constexpr uint32_t NO_POS = 16;
__device__ __forceinline__ uint32_t match_first(const LineImg& li, uint32_t L, uint64_t h) {
    const uint32_t rm = match_slots(li, L, h);
    return rm ? pos_of(li.perm, __builtin_ctz(rm), L) : NO_POS;
}
// the lowest position whose slot is empty, NO_POS when the line is full
__device__ __forceinline__ uint32_t first_empty(const LineImg& li, uint32_t L) {
    const uint32_t rm = match_slots(li, L, 0);
    uint32_t pm = 0;
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
        if (j < L && ((rm >> nib(li.perm, j)) & 1u)) pm |= 1u << j;
    return pm ? __builtin_ctz(pm) : NO_POS;
}

// ---- the replay --------------------------------------------------------------------------------
struct WalkCtx {
    StrictView v;
    ExportView ex;
    uint32_t* sc;        // block counters (LDS)
    int32_t live;        // records created - exported (this lane)
    uint32_t inactive, active;
};

// export_flow (cache.cpp:262-274): the record leaves with its reason, its slot becomes empty
// (the record as 32 words in registers, RecW: through ipxg_flow_record's byte fields it lived
// in scratch memory)
__device__ __forceinline__ void strict_export(WalkCtx& w, uint32_t slot, const RecW& r, uint8_t reason) {
    const uint32_t pos = atomicAdd(w.ex.count, 1u);
    store_export_w(w.ex, pos, r, reason);
    if (w.ex.count6 && rw_ipver(r) == 6) atomicAdd(w.ex.count + 2, 1u);
    count_export_w(w.sc, r, reason);
    w.v.hash[slot] = 0;
    w.v.tlast[slot] = 0xFFFFFFFFu;
    w.live--;
}

// the sweep line's position -> slot map and its slots' time_last (prefetched with the packet's
// own lines when the sweep visits a third line)
struct SweepImg {
    uint64_t perm;
    uint32_t tl[16];
};
template <bool MW>
__device__ __forceinline__ void load_sweep(const TableIO<MW>& io, uint32_t line, SweepImg& si) {
    const uint32_t L = 1u << io.v.line_bits;
    si.perm = io.perm(line);
    io.tlasts(line, L, si.tl);
}

// export_expired (cache.cpp:508-523) at sweep step q: positions [q * L/2, +L/2) of the table.
// An empty slot's time_last is 0xFFFFFFFF, so it never tests idle; only the records that
// leave are read.  pre: the line's map and time_last as loaded before this packet's own update
// (valid when the sweep line is none of the packet's lookup lines).
template <bool MW>
__device__ void strict_sweep(WalkCtx& w, const TableIO<MW>& io, uint64_t q, int64_t ts, const SweepImg* pre = nullptr) {
    const StrictView& v = w.v;
    const uint32_t L = 1u << v.line_bits, half = L >> 1;
    const uint32_t at = (uint32_t)((q * half) & v.slot_mask);
    const uint32_t line = at >> v.line_bits, off = at & (L - 1u);
    SweepImg si;
    if (pre) si = *pre;
    else load_sweep(io, line, si);
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
        const uint32_t j = off + k;
        if (k >= half) break;
        const uint32_t r = nib(si.perm, j);
        uint32_t tl = si.tl[0];
#pragma unroll
        for (uint32_t x = 1; x < 16; ++x) tl = r == x ? si.tl[x] : tl;  // (selects: no indexed copy)
        if (ts - (int64_t)tl >= (int64_t)w.inactive) {
            const uint32_t slot = line * L + r;
            const RecW rec = io.rec(slot);
            strict_export(w, slot, rec, export_reason_w(rec));
        }
    }
}

// put_pkt_recursive (cache.cpp:330-491) for one keyed packet, its sweep included
template <bool MW>
__device__ void strict_packet(WalkCtx& w, const TableIO<MW>& io, const StrictPkt& s, const ipxg_flow_record* crec_i,
                              uint64_t q, uint32_t split) {
    const StrictView& v = w.v;
    const uint32_t L = 1u << v.line_bits, half = L >> 1;
    uint32_t ln[3];
    strict_lines(v, s, q, split, ln);
    const uint32_t lf = ln[0];
    const uint32_t li_line = split ? lf : (uint32_t)(s.h_inv & (v.slot_mask & ~(L - 1u))) >> v.line_bits;
    // The packet's lines are loaded together up front: the forward line, the inverse line (read
    // only when the forward search misses, about every other packet) and the line its sweep
    // visits -- no other packet touches them until this one is done (the DAG), so the images
    // stay valid until this packet changes them itself.
    LineImg F, I;
    SweepImg S;
    const bool pre_sweep = half && ln[2] != STRICT_NONE;
    load_line(io, lf, F);
    if (!split) load_line(io, li_line, I);
    if (pre_sweep) load_sweep(io, ln[2], S);
    for (int depth = 0; depth < 8; ++depth) {  // the recursion after an export (at most twice)
        if (depth) {  // an export changed the table: read the lines again
            load_line(io, lf, F);
            if (!split) load_line(io, li_line, I);
        }
        uint32_t line = lf, pos = 0;
        bool found = false, src = true;
        uint64_t perm = F.perm;
        pos = match_first(F, L, s.h_fwd);
        if (pos != NO_POS) {
            found = true;
        } else if (!split && (pos = match_first(I, L, s.h_inv)) != NO_POS) {
            found = true;
            src = false;
            line = li_line;
            perm = I.perm;
        }
        if (found) {  // move to the line's front (:375-391)
            perm = perm_move(perm, pos, 0);
            v.perm[line] = perm;
            pos = 0;
        } else {
            pos = first_empty(F, L);
            if (pos == NO_POS) {  // line full: the last position leaves (NO_RES), its slot re-enters at L/2 (:400-419)
                const uint32_t slot = lf * L + nib(perm, L - 1);
                const RecW ev = io.rec(slot);
                strict_export(w, slot, ev, IPXG_FLOW_END_NO_RES);
                perm = perm_move(perm, L - 1, half);
                v.perm[lf] = perm;
                pos = half;
            }
        }
        const uint32_t slot = line * L + nib(perm, pos);
        if (!found) {  // FlowRecord::create (:440-443)
            const RecW r = rec_load_w(crec_i);
            rec_store_w(&v.rec[slot], r);
            v.hash[slot] = s.h_fwd;
            v.tlast[slot] = r.w[RW_TLS];
            w.live++;
            break;
        }
        RecW r = io.rec(slot);
        const uint32_t flw = src ? rw_sflags(r) : rw_dflags(r);
        if ((s.tcp_flags & 0x02) && (flw & 0x05)) {  // SYN after FIN/RST (:431-438)
            strict_export(w, slot, r, IPXG_FLOW_END_EOF);
            continue;
        }
        if ((int64_t)s.ts_sec - (int64_t)r.w[RW_TLS] >= (int64_t)w.inactive) {  // :453-461
            strict_export(w, slot, r, export_reason_w(r));
            continue;
        }
        if ((int64_t)s.ts_sec - (int64_t)r.w[RW_TFS] >= (int64_t)w.active) {  // :464-472
            strict_export(w, slot, r, IPXG_FLOW_END_ACTIVE);
            continue;
        }
        r.w[RW_TLS] = s.ts_sec;  // FlowRecord::update (:134-152)
        r.w[RW_TLU] = s.ts_usec;
        const uint32_t fl = s.ip_proto == 6 ? s.tcp_flags : 0u;
        if (src) {
            r.w[RW_SPK]++;
            rw64_set(r, RW_SBYTES, rw64(r, RW_SBYTES) + s.ip_len);
            r.w[RW_FLAGS] |= fl;
        } else {
            r.w[RW_DPK]++;
            rw64_set(r, RW_DBYTES, rw64(r, RW_DBYTES) + s.ip_len);
            r.w[RW_FLAGS] |= fl << 8;
        }
        rec_store_w(&v.rec[slot], r);
        v.tlast[slot] = s.ts_sec;
        break;
    }
    // export_expired (:508-523): positions [q * L/2, +L/2) of the table, idle against this packet
    // (s.sweep 0: no record there can be idle, k_strict_lb)
    if (half && s.sweep) strict_sweep(w, io, q, (int64_t)s.ts_sec, pre_sweep ? &S : nullptr);
}

// The DAG scheduler of the file comment.  An idle lane holds one ticket (a queue position) and
// runs the ticket's packet once a predecessor (or k_strict_ready) has filled it.  A lane that sees
// no packet finish for p.spin_max polling rounds gives up and stops the replay (ctl->strict_fail;
// progress-based, so one long chain -- an elephant flow run serially by the lane that owns it --
// never trips it; the scheduler cannot deadlock -- the lowest unfinished packet is always running
// or queued at a position some lane's ticket reaches -- the bound guards engine bugs).
//
// MW false: ONE workgroup; the queue's head/tail and the done count live in LDS, hand-offs need
// workgroup-scope ordering only.
// MW true: the workgroups of ONE XCD (the first to arrive claims its XCD, the workgroups placed on
// any other XCD leave at once); head/tail/done/stop are agent-scope atomics in `g` (StrictSched),
// tickets and the done count are taken once per wave (one atomic for all its lanes), the table is
// read with sc1 loads (TableIO<true>), and a lane signals a successor (in-degree decrement, queue
// entry) only after its own table stores have completed (s_waitcnt vmcnt(0)) -- in the shared L2.
struct StrictSched {  // each counter on a 128-byte line of its own (its own L2 channel)
    uint32_t head, pad0[31];
    uint32_t tail, pad1[31];
    uint32_t done, pad2[31];
    uint32_t stop;
    uint32_t xcc;      // 1 + the XCD the replay runs on (0: not claimed yet)
    uint32_t members;  // workgroups that took part
    uint32_t pad3[29];
};

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}

template <bool MW, int LANES = STRICT_LANES>
__global__ __launch_bounds__(LANES) void k_strict_walk(StrictView v, Params p, const StrictPkt* sp,
                                                              const ipxg_flow_record* crec, const uint32_t* keyed,
                                                              const uint32_t* qx, const uint32_t* succ,
                                                              uint32_t* indeg, uint32_t* queue, uint32_t* sched,
                                                              uint32_t n, uint64_t q_base, ExportView ex,
                                                              BatchCtl* ctl, unsigned long long* stats) {
    __shared__ uint32_t head, tail, stop, done, member;
    __shared__ uint32_t sc[ST_COUNT];
    StrictSched* const g = reinterpret_cast<StrictSched*>(sched);  // MW: the shared scheduler state
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) {
        if constexpr (MW) {
            const uint32_t x = xcc_id() + 1u;
            const uint32_t prev = atomicCAS(&g->xcc, 0u, x);
            member = prev == 0u || prev == x;
            if (member) atomicAdd(&g->members, 1u);
        } else {
            head = 0;
            tail = *sched;  // (the ready count k_strict_ready left)
            stop = 0;
            done = 0;
            member = 1;
        }
    }
    if (tid < ST_COUNT) sc[tid] = 0;
    __syncthreads();
    if (!member) return;  // (uniform: a workgroup on another XCD)
    const uint32_t K = n ? qx[n - 1] + keyed[n - 1] : 0;  // keyed packets = tickets
    WalkCtx w{v, ex, sc, 0, p.inactive_s, p.active_s};
    const TableIO<MW> io{v};
    // A lane that makes a successor ready runs it next itself (the chain's hand-off costs no queue
    // round trip and no wait for another wave's poll); further ready successors are queued.  An
    // idle lane holds one ticket; every lane stops when all K keyed packets are done.
    constexpr uint32_t NO_TICKET = 0xFFFFFFFFu;
    uint32_t t = NO_TICKET, cur = STRICT_NONE, spins = 0, seen_done = 0;
    bool failed = false, fin = K == 0;
#ifdef IPXG_PROBE
    // per wave: loop rounds, rounds that ran packets, lanes that ran one in those, the queue's
    // backlog (tail - head) summed over those rounds, shader clocks in the packet body / in all,
    // packets whose sweep step stayed in the DAG, lanes whose ticket was due but not yet filled
    uint64_t pr_rounds = 0, pr_body = 0, pr_lanes = 0, pr_backlog = 0, pr_tbody = 0, pr_sweep = 0, pr_unfilled = 0;
    uint64_t pr_ph[4] = {0, 0, 0, 0};  // body phases: packet fields, strict_packet, store drain, hand-off
    const uint64_t pr_t0 = __builtin_readcyclecounter();
#endif
    while (__any(!fin)) {
        bool progressed = false;
#ifdef IPXG_PROBE
        pr_rounds++;
#endif
        if constexpr (MW) {  // tickets for the wave's idle lanes, one atomic for all of them
            const uint64_t need = __ballot(!fin && cur == STRICT_NONE && t == NO_TICKET);
            if (need) {
                const uint32_t leader = (uint32_t)__builtin_ctzll(need);
                uint32_t base = 0;
                if (lane == leader)
                    base = __hip_atomic_fetch_add(&g->head, (uint32_t)__popcll(need), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                base = __shfl(base, leader);
                if ((need >> lane) & 1ull) t = base + (uint32_t)__popcll(need & ((1ull << lane) - 1ull));
            }
        }
        if (!fin && cur == STRICT_NONE) {
            uint32_t tl;
            if constexpr (MW) {
                tl = __hip_atomic_load(&g->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (t == NO_TICKET) t = atomicAdd(&head, 1u);
                // poll the queue's LDS tail; the global entry is read only once it is due (lanes
                // polling global memory queued the working lanes' loads behind theirs)
                tl = __hip_atomic_load(&tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            const bool due = t < tl;
            const uint32_t pk = !due ? STRICT_NONE
                                : MW ? __hip_atomic_load(&queue[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : __hip_atomic_load(&queue[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (pk != STRICT_NONE) {
                cur = pk;
                t = NO_TICKET;
                spins = 0;
                if constexpr (!MW) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            } else {
#ifdef IPXG_PROBE
                if (due) pr_unfilled++;
#endif
                const uint32_t dn = MW ? __hip_atomic_load(&g->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : __hip_atomic_load(&done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t st = MW ? __hip_atomic_load(&g->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                       : __hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (dn >= K || st) {
                    fin = true;  // every packet done (this ticket is never filled), or a lane gave up
                } else if (dn != seen_done) {
                    seen_done = dn;  // the replay still makes progress (a long chain running on
                    spins = 0;       // other lanes): waiting is legitimate, the bound restarts
                } else if (++spins > p.spin_max) {
                    failed = true;  // no packet finished for STRICT_SPIN_MAX rounds: engine bug
                    if constexpr (MW) atomicOr(&g->stop, 1u);
                    else atomicOr(&stop, 1u);
                    fin = true;
                }
            }
        }
#ifdef IPXG_PROBE
        const uint64_t pr_act = __ballot(!fin && cur != STRICT_NONE);
        uint64_t pr_tb = 0;
        if (pr_act) {
            pr_body++;
            pr_lanes += __popcll(pr_act);
            const uint32_t tl = MW ? __hip_atomic_load(&g->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(&tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t hd = MW ? __hip_atomic_load(&g->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(&head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            pr_backlog += tl > hd ? tl - hd : 0;
            pr_tb = __builtin_readcyclecounter();
        }
#endif
        if (!fin && cur != STRICT_NONE) {
            const uint32_t pk = cur;
            const StrictPkt s = sp[pk];
            const uint64_t q = q_base + qx[pk];
            uint32_t nxt[3];  // the packet's successors, read with its fields (not after its update)
#pragma unroll
            for (int j = 0; j < 3; ++j) nxt[j] = succ[4 * pk + j];
#ifdef IPXG_PROBE
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint64_t ph1 = __builtin_readcyclecounter();
#endif
            strict_packet(w, io, s, crec + pk, q, p.split_biflow);
#ifdef IPXG_PROBE
            const uint64_t ph2 = __builtin_readcyclecounter();
#endif
            if constexpr (!MW) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's table stores are done
#ifdef IPXG_PROBE
            const uint64_t ph3 = __builtin_readcyclecounter();
#endif
            uint32_t ln[3];
            strict_lines(v, s, q, p.split_biflow, ln);
            cur = STRICT_NONE;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint32_t nx = ln[j] == STRICT_NONE ? STRICT_NONE : nxt[j];
                if (nx == STRICT_NONE) continue;
                const uint32_t before =
                    MW ? __hip_atomic_fetch_add(&indeg[nx], 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : __hip_atomic_fetch_add(&indeg[nx], 0xFFFFFFFFu, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (before == 1u) {
                    if (cur == STRICT_NONE) {
                        cur = nx;  // run it next, on this lane
                    } else if constexpr (MW) {
                        const uint32_t at = __hip_atomic_fetch_add(&g->tail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(&queue[at], nx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        const uint32_t at = atomicAdd(&tail, 1u);
                        __hip_atomic_store(&queue[at], nx, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
            if constexpr (!MW) atomicAdd(&done, 1u);
            progressed = true;
#ifdef IPXG_PROBE
            pr_sweep += s.sweep;
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const uint64_t ph4 = __builtin_readcyclecounter();
            if (lane == (uint32_t)__builtin_ctzll(pr_act)) {  // one lane per wave-round: the wave's phases
                pr_ph[0] += ph1 - pr_tb;
                pr_ph[1] += ph2 - ph1;
                pr_ph[2] += ph3 - ph2;
                pr_ph[3] += ph4 - ph3;
            }
#endif
        }
#ifdef IPXG_PROBE
        if (pr_act) pr_tbody += __builtin_readcyclecounter() - pr_tb;
#endif
        const uint64_t pm = __ballot(progressed);
        if constexpr (MW) {  // the wave's finished packets, one atomic
            if (pm && lane == (uint32_t)__builtin_ctzll(pm))
                __hip_atomic_fetch_add(&g->done, (uint32_t)__popcll(pm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!pm) {
            // nothing finished in this wave: a wave with no packet at all backs off longer (its
            // polls go to the L2 the working lanes wait on)
            if (MW && !__ballot(cur != STRICT_NONE)) __builtin_amdgcn_s_sleep(8);
            else __builtin_amdgcn_s_sleep(2);
        }
    }
    if (failed) atomicOr(&ctl->strict_fail, 1u);
    if (w.live) atomicAdd(&ctl->strict_live, w.live);
    flush_block_stats(sc, stats);
#ifdef IPXG_PROBE
    if ((tid & 63) == 0) {
        const uint64_t acc[8] = {pr_rounds, pr_body, pr_lanes, pr_backlog, pr_tbody, __builtin_readcyclecounter() - pr_t0, 0,
                                 pr_unfilled};
        for (int k = 0; k < 8; ++k) atomicAdd((unsigned long long*)&ctl->probe[k], (unsigned long long)acc[k]);
    }
    for (int o = 32; o; o >>= 1) pr_sweep += (uint64_t)__shfl_xor((unsigned long long)pr_sweep, o);
    if ((tid & 63) == 0) atomicAdd((unsigned long long*)&ctl->probe[6], (unsigned long long)pr_sweep);
    for (int k = 0; k < 4; ++k) {
        uint64_t x = pr_ph[k];
        for (int o = 32; o; o >>= 1) x += (uint64_t)__shfl_xor((unsigned long long)x, o);
        if ((tid & 63) == 0) atomicAdd((unsigned long long*)&ctl->probe[8 + k], (unsigned long long)x);
    }
#endif
}

// ipxg_expire in strict mode: one export_expired call (cache.cpp:508-523) at `now`, sweep step q
__global__ void k_strict_expire(StrictView v, Params p, uint64_t q, int64_t now, ExportView ex, BatchCtl* ctl,
                                unsigned long long* stats) {
    __shared__ uint32_t sc[ST_COUNT];
    if (threadIdx.x < ST_COUNT) sc[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        WalkCtx w{v, ex, sc, 0, p.inactive_s, p.active_s};
        strict_sweep(w, TableIO<false>{v}, q, now);
        if (w.live) atomicAdd(&ctl->strict_live, w.live);
    }
    flush_block_stats(sc, stats);
}

// finish (cache.cpp:276-288): every record FORCED, the table emptied
__global__ __launch_bounds__(256) void k_strict_finish(StrictView v, ExportView ex, BatchCtl* ctl,
                                                       unsigned long long* stats) {
    __shared__ uint32_t sc[ST_COUNT];
    if (threadIdx.x < ST_COUNT) sc[threadIdx.x] = 0;
    __syncthreads();
    WalkCtx w{v, ex, sc, 0, 0, 0};
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s <= v.slot_mask; s += gridDim.x * 256) {
        if (v.hash[s] == 0) continue;
        strict_export(w, s, rec_load_w(&v.rec[s]), IPXG_FLOW_END_FORCED);
    }
    if (w.live) atomicAdd(&ctl->strict_live, w.live);
    flush_block_stats(sc, stats);
}

// the identity permutation of every line, every record empty
__global__ __launch_bounds__(256) void k_strict_clear(StrictView v) {
    const uint32_t L = 1u << v.line_bits;
    uint64_t id = 0;
    for (uint32_t j = 0; j < L; ++j) id |= (uint64_t)j << (4 * j);
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s <= v.slot_mask; s += gridDim.x * 256) {
        v.hash[s] = 0;
        v.tlast[s] = 0xFFFFFFFFu;
        if (s < v.lines) v.perm[s] = id;
    }
}

// ---- launchers -----------------------------------------------------------------------------------
static uint32_t grid_for(uint32_t n, uint32_t block, uint32_t cap) {
    uint32_t g = (n + block - 1) / block;
    return g < 1 ? 1 : (g > cap ? cap : g);
}

void launch_strict_prep1(hipStream_t st, const BatchView& b, const Params& p, FragView f, BatchCtl* ctl,
                         unsigned long long* stats) {
    hipLaunchKernelGGL(k_strict_prep1, dim3(grid_for(b.n, IPXG_BLOCK, 2048)), dim3(IPXG_BLOCK), 0, st, b, p, f, ctl,
                       stats);
}

void launch_strict_prep2(hipStream_t st, const BatchView& b, const Params& p, FragView f, StrictPkt* sp,
                         ipxg_flow_record* crec, uint32_t* keyed, uint32_t* ts_acc) {
    hipLaunchKernelGGL(k_strict_prep2, dim3(grid_for(b.n, IPXG_BLOCK, 2048)), dim3(IPXG_BLOCK), 0, st, b, p, f, sp,
                       crec, keyed, ts_acc);
}

void launch_strict_lb(hipStream_t st, StrictView v) {
    hipLaunchKernelGGL(k_strict_lb, dim3((v.lines + 255) / 256), dim3(256), 0, st, v);
}

void launch_strict_events(hipStream_t st, StrictView v, StrictPkt* sp, const uint32_t* keyed, const uint32_t* qx,
                          uint32_t n, uint64_t q_base, uint32_t split, uint32_t inactive, uint32_t* keys,
                          uint32_t* vals) {
    hipLaunchKernelGGL(k_strict_events, dim3((n + 255) / 256), dim3(256), 0, st, v, sp, keyed, qx, n, q_base, split,
                       inactive, keys, vals);
}

void launch_strict_dag(hipStream_t st, const uint32_t* keys_sorted, const uint32_t* vals_sorted, uint32_t m,
                       const uint32_t* keys, const uint32_t* keyed, uint32_t n, uint32_t lines, uint32_t* succ,
                       uint8_t* pred, uint32_t* indeg, uint32_t* queue, uint32_t* q_count) {
    hipLaunchKernelGGL(k_strict_dag, dim3((m + 255) / 256), dim3(256), 0, st, keys_sorted, vals_sorted, m, lines, succ,
                       pred);
    hipLaunchKernelGGL(k_strict_ready, dim3((n + 255) / 256), dim3(256), 0, st, keys, pred, keyed, n, lines, indeg,
                       queue, q_count);
}

void launch_strict_walk(hipStream_t st, StrictView v, const Params& p, const StrictPkt* sp,
                        const ipxg_flow_record* crec, const uint32_t* keyed, const uint32_t* qx, const uint32_t* succ,
                        uint32_t* indeg, uint32_t* queue, uint32_t* sched, uint32_t n, uint64_t q_base,
                        ExportView ex, BatchCtl* ctl, unsigned long long* stats, uint32_t wgs_per_xcd) {
    static_assert(sizeof(StrictSched) == STRICT_SCHED_BYTES && offsetof(StrictSched, tail) == 4 * STRICT_SCHED_TAIL_WORD,
                  "scheduler block");
    // lanes per workgroup of the multi-workgroup replay: 256 (measured best at s=17: 12 x 256 per
    // XCD 114 Mpkt/s, 6 x 768 76); IPXG_STRICT_MW_LANES=128/768 for tuning
    static const char* lanes_env = std::getenv("IPXG_STRICT_MW_LANES");
    static const int lanes = lanes_env ? std::atoi(lanes_env) : 256;
    if (wgs_per_xcd && lanes == 128)  // 8 x wgs_per_xcd workgroups: those on the first XCD to arrive take part
        hipLaunchKernelGGL((k_strict_walk<true, 128>), dim3(8 * wgs_per_xcd), dim3(128), 0, st, v, p, sp, crec, keyed,
                           qx, succ, indeg, queue, sched, n, q_base, ex, ctl, stats);
    else if (wgs_per_xcd && lanes == 768)
        hipLaunchKernelGGL(k_strict_walk<true>, dim3(8 * wgs_per_xcd), dim3(STRICT_LANES), 0, st, v, p, sp, crec, keyed,
                           qx, succ, indeg, queue, sched, n, q_base, ex, ctl, stats);
    else if (wgs_per_xcd)
        hipLaunchKernelGGL((k_strict_walk<true, 256>), dim3(8 * wgs_per_xcd), dim3(256), 0, st, v, p, sp, crec, keyed,
                           qx, succ, indeg, queue, sched, n, q_base, ex, ctl, stats);
    else
        hipLaunchKernelGGL(k_strict_walk<false>, dim3(1), dim3(STRICT_LANES), 0, st, v, p, sp, crec, keyed, qx, succ,
                           indeg, queue, sched, n, q_base, ex, ctl, stats);
}

void launch_strict_expire(hipStream_t st, StrictView v, const Params& p, uint64_t q, int64_t now, ExportView ex,
                          BatchCtl* ctl, unsigned long long* stats) {
    hipLaunchKernelGGL(k_strict_expire, dim3(1), dim3(64), 0, st, v, p, q, now, ex, ctl, stats);
}

void launch_strict_finish(hipStream_t st, StrictView v, ExportView ex, BatchCtl* ctl, unsigned long long* stats) {
    hipLaunchKernelGGL(k_strict_finish, dim3(grid_for(v.slot_mask + 1, 256, 1024)), dim3(256), 0, st, v, ex, ctl,
                       stats);
}

void launch_strict_clear(hipStream_t st, StrictView v) {
    hipLaunchKernelGGL(k_strict_clear, dim3(grid_for(v.slot_mask + 1, 256, 1024)), dim3(256), 0, st, v);
}

}  // namespace ipxg
