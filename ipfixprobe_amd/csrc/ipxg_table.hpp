// ipxg_table.hpp -- device helpers shared by the ingest kernels (ipxg_ingest.hip) and the
// table kernels (ipxg_kernels.hip): wave/block counting, flow-table probing, the per-packet
// and per-aggregate merges into a slot's batch accumulators, flow-record construction
// (FlowRecord::create, cache.cpp:94-133) and the per-slot batch finalisation (the
// reference's split rules of put_pkt_recursive, cache.cpp:428-486, applied at the batch
// boundary from the recorded packet indices).
#pragma once

#include "ipxg_device.hpp"
#include "ipxg_kernels.hpp"

namespace ipxg {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// rank of the complex flow with canonical key lo, or -1
__device__ __forceinline__ int64_t complex_rank_of(const ComplexView& cx, uint64_t lo) {
    if (cx.bloom && !((cx.bloom[((uint32_t)lo >> 5) & cx.bmask] >> ((uint32_t)lo & 31u)) & 1u)) return -1;
    for (uint32_t e = (uint32_t)lo & cx.kmask;; e = (e + 1) & cx.kmask) {
        const unsigned long long k = cx.keys[e];
        if (k == lo) return cx.key_rank[e];
        if (k == 0ull) return -1;
    }
}

// Wave-aggregated append: one atomic per wave instead of one per lane.  Every lane of the
// wave must call it (convergent).
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, bool pred) {
    uint64_t m = __ballot(pred);
    if (m == 0) return 0;
    uint32_t lane = lane_id();
    uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    uint64_t below = lane ? (m & ((~0ull) >> (64 - lane))) : 0ull;
    return base + (uint32_t)__popcll(below);
}

// Exclusive prefix sum of v over a block of NT threads (NT a multiple of 64, <= 1024);
// *total receives the block sum.  `scratch` holds NT/64 + 1 words of LDS.  Contains
// __syncthreads(): every thread of the block must call it.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* scratch, uint32_t* total) {
    constexpr int NW = NT / 64;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) scratch[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int k = 0; k < NW; ++k) {
            uint32_t t = scratch[k];
            scratch[k] = s;
            s += t;
        }
        scratch[NW] = s;
    }
    __syncthreads();
    const uint32_t r = scratch[w] + x - v;
    *total = scratch[NW];
    __syncthreads();
    return r;
}

// ---- block statistics ---------------------------------------------------------------------
// Each counter summed over the wave first, then one LDS atomic per wave and non-zero counter:
// every lane's atomic on the same 15 LDS words serialised 64-fold per wave instruction.
__device__ __forceinline__ void flush_counts(const ParseCounts& c, uint32_t keyless, uint32_t frags,
                                             uint32_t* sc) {
    uint32_t v[15] = {c.seen, c.parsed, c.unknown, c.ipv4, c.ipv6, c.tcp, c.udp, c.mpls, c.pppoe, c.trill, c.vlan,
                      c.ipv4_bytes, c.ipv6_bytes, keyless, frags};
    constexpr uint32_t idx[15] = {ST_SEEN, ST_PARSED, ST_UNKNOWN, ST_IPV4, ST_IPV6, ST_TCP, ST_UDP, ST_MPLS, ST_PPPOE,
                                  ST_TRILL, ST_VLAN, ST_IPV4_BYTES, ST_IPV6_BYTES, ST_KEYLESS, ST_FRAGMENTED};
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        if (!__any(v[k] != 0)) continue;  // (wave-uniform)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
        if ((threadIdx.x & 63) == 0 && v[k]) atomicAdd(&sc[idx[k]], v[k]);
    }
}

// sc: ST_COUNT block-local counters in LDS; one device atomic per non-zero counter.
__device__ __forceinline__ void flush_block_stats(uint32_t* sc, unsigned long long* stats) {
    __syncthreads();
    if (threadIdx.x < ST_COUNT && sc[threadIdx.x])
        atomicAdd(&stat_row(stats)[threadIdx.x],
                  (unsigned long long)sc[threadIdx.x]);
}

// ---- canonical biflow hash --------------------------------------------------------------
// lo = min(XXH64(key), XXH64(key_inv)) identifies the biflow (the reference's identity is
// the 64-bit hash too, cache.cpp:84-92, looked up forward then inverse, :341-373); cdir is
// the packet's direction relative to lo; hf the forward hash (the record's flow_hash).
// The canonical direction of a packet: 1 when its (source address, source port) endpoint orders
// after its (destination address, destination port) one -- address words compared first (one for
// IPv4, four for IPv6), then ports; equal endpoints give 0.  Both directions of a biflow see the
// same canonical endpoint order, so the same canonical key.
__device__ __forceinline__ uint32_t canon_dir(const DevPkt& pk) {
    // (words compared most significant first as one 64-bit pair per step: no loop, no indexing)
    const bool v6 = pk.ip_version == 6;
    const uint64_t s0 = ((uint64_t)pk.sip[0] << 32) | (v6 ? pk.sip[1] : 0u);
    const uint64_t d0 = ((uint64_t)pk.dip[0] << 32) | (v6 ? pk.dip[1] : 0u);
    const uint64_t s1 = v6 ? ((uint64_t)pk.sip[2] << 32) | pk.sip[3] : 0ull;
    const uint64_t d1 = v6 ? ((uint64_t)pk.dip[2] << 32) | pk.dip[3] : 0ull;
    if (s0 != d0) return s0 > d0 ? 1u : 0u;
    if (s1 != d1) return s1 > d1 ? 1u : 0u;
    return pk.src_port > pk.dst_port ? 1u : 0u;
}

// The table key of a packet's flow: XXH64 of its canonical key (the forward key in canonical
// direction 0, the inverse key in direction 1) -- one hash per packet.  The reference finds a
// flow by either of its two hashes (cache.cpp:330-372: the forward hash, then the inverse one);
// a canonical key names the same biflow (barring 64-bit collisions, which the reference's own
// lookup shares).  The creator's forward hash (the record's flow_hash) is lo when the creator
// went in canonical direction 0, so `flow_hash != slot key` still tells the creator's direction
// (finalize_slot).  HF: also hf = XXH64(forward key) (record creation; a second hash only in
// canonical direction 1).  split_biflow: lo = hf, direction 0.
template <bool HF = true>
__device__ __forceinline__ void canon(const DevPkt& pk, const Params& p, uint64_t& lo, uint32_t& cdir,
                                      uint64_t& hf) {
    FlowKey kf, ki;
    build_keys(pk, kf, ki);
    if (p.split_biflow) {
        hf = lo = key_hash(kf);
        cdir = 0;
        return;
    }
    cdir = canon_dir(pk);
    lo = key_hash(cdir ? ki : kf);
    hf = lo;
    if (HF && cdir) hf = key_hash(kf);
}

__device__ __forceinline__ uint32_t time_bucket(uint32_t sec, uint32_t base, uint32_t w) {
    if (sec < base) return 31;
    uint32_t b = (sec - base) / w;
    return b > 30 ? 31 : b;
}

// Per-packet contribution packed into one word (also the bin record's 4th word):
// ip_len | tcp_flags << 16 | cdir << 24 | tcp << 25 | time bucket << 26.
__device__ __forceinline__ uint32_t pack_misc(const DevPkt& pk, uint32_t cdir, uint32_t tb) {
    return (uint32_t)pk.ip_len | ((uint32_t)pk.tcp_flags << 16) | (cdir << 24) |
           ((pk.ip_proto == 6 ? 1u : 0u) << 25) | (tb << 26);
}
__device__ __forceinline__ uint32_t misc_len(uint32_t m) { return m & 0xFFFF; }
__device__ __forceinline__ uint32_t misc_flags(uint32_t m) { return (m >> 16) & 0xFF; }
__device__ __forceinline__ uint32_t misc_dir(uint32_t m) { return (m >> 24) & 1; }
__device__ __forceinline__ bool misc_tcp(uint32_t m) { return (m >> 25) & 1; }
__device__ __forceinline__ uint32_t misc_tb(uint32_t m) { return (m >> 26) & 31; }

// The batch's first packet of a flow, as one max-reduced word: (~index & 0xFFFFFF) << 8 (the
// largest is the smallest index; indices are < 2^24 - 1, so a packet's key is never 0) and, in
// the low bits, what the boundary checks of put_pkt_recursive need of that packet without
// parsing it again: its SYN flag (cache.cpp:431) and its canonical direction (:428).
__device__ __forceinline__ uint32_t first_key(uint32_t idx, uint32_t m) {
    return ((~idx & 0xFFFFFFu) << 8) | (((misc_flags(m) >> 1) & 1u) << 1) | misc_dir(m);
}
__device__ __forceinline__ uint32_t first_idx(uint32_t fk) { return ~(fk >> 8) & 0xFFFFFFu; }
__device__ __forceinline__ bool first_syn(uint32_t fk) { return (fk & 2u) != 0; }
__device__ __forceinline__ uint32_t first_dir(uint32_t fk) { return fk & 1u; }

// ---- flow-table probing (open addressing, linear probing, capacity 2^k) ------------------
// Probe for (and if absent claim) the slot of canonical hash lo; nullptr after MAX_PROBE.
// One 16-byte load per probe returns the key together with first_n and tbits, so the
// caller can skip reductions that cannot change them.  A stale copy is harmless: a stale
// empty key falls through to the CAS (which returns the true owner), and stale first_n/tbits
// only cause a redundant atomic.  *claimed is set when this call took an empty slot.
__device__ __forceinline__ HotSlot* probe_insert(const TableView& t, uint64_t lo, uint4& head, bool& claimed) {
    uint32_t s = (uint32_t)lo & t.mask;
    claimed = false;
    for (uint32_t probe = 0; probe < MAX_PROBE; ++probe) {
        HotSlot* h = &t.hot(s);
        head = *reinterpret_cast<const uint4*>(h);
        uint64_t k = ((uint64_t)head.y << 32) | head.x;
        if (k == 0) {
            unsigned long long old = atomicCAS((unsigned long long*)&h->key, 0ull, (unsigned long long)lo);
            if (old == 0) {
                head = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), 0, 0);
                claimed = true;
                return h;
            }
            k = old;
            head.z = 0;  // unknown: force the reductions
            head.w = 0;
        }
        if (k == lo) return h;
        s = (s + 1) & t.mask;
    }
    return nullptr;
}

// probe_insert for a caller that needs the whole slot: each probe reads the 64-byte slot
// (one line), so a found slot needs no second read and a claimed one is known empty.  For
// k_reduce, whose workgroup is the only writer of its keys' slots in that kernel.
__device__ __forceinline__ HotSlot* probe_insert_full(const TableView& t, uint64_t lo, HotSlot& h, bool& claimed) {
    uint32_t s = (uint32_t)lo & t.mask;
    claimed = false;
    for (uint32_t probe = 0; probe < MAX_PROBE; ++probe) {
        HotSlot* p = &t.hot(s);
        h = *p;
        if (h.key == 0) {
            const unsigned long long old = atomicCAS((unsigned long long*)&p->key, 0ull, (unsigned long long)lo);
            if (old == 0) {
                h = HotSlot{};
                h.key = lo;
                claimed = true;
                return p;
            }
            if (old == lo) {  // inserted meanwhile by another path: read it again
                h = *p;
                return p;
            }
        } else if (h.key == lo) {
            return p;
        }
        s = (s + 1) & t.mask;
    }
    return nullptr;
}

__device__ __forceinline__ int64_t probe_find(const TableView& t, uint64_t lo) {
    uint32_t s = (uint32_t)lo & t.mask;
    for (uint32_t probe = 0; probe <= t.mask; ++probe) {
        uint64_t k = t.hot(s).key;
        if (k == lo) return s;
        if (k == 0) return -1;
        s = (s + 1) & t.mask;
    }
    return -1;
}

// Fold one packet (canonical hash lo, packet index idx, packed contribution m) into its
// slot's batch accumulators with device atomics (NHTFlowCache::put_pkt's update,
// cache.cpp:134-152, as order-independent reductions keyed by packet index).  Returns false
// when the probe failed (the caller defers the packet until the table has grown).
__device__ __forceinline__ bool merge_packet_atomic(const TableView& t, uint64_t lo, uint32_t idx, uint32_t m,
                                                    uint32_t* new_keys) {
    uint4 head;
    bool claimed;
    HotSlot* h = probe_insert(t, lo, head, claimed);
    if (!h) return false;
    if (claimed) atomicAdd(new_keys, 1u);
    const uint32_t cdir = misc_dir(m);
    atomicAdd((unsigned long long*)&h->acc[cdir], (1ull << 40) | (uint64_t)misc_len(m));
    atomicMax(&h->last1, idx + 1);
    const uint32_t fn = first_key(idx, m);
    if (head.z < fn) atomicMax(&h->first_n, fn);
    const uint32_t tb = 1u << misc_tb(m);
    if (!(head.w & tb)) atomicOr(&h->tbits, tb);
    const uint32_t fl = misc_flags(m);
    if (misc_tcp(m) && fl) {
        atomicOr(&h->tflags, fl << (8 * cdir));
        if (fl & 0x02) atomicMax(&h->syn1[cdir], idx + 1);
        if (fl & 0x05) atomicMax(&h->fin_n[cdir], ~idx);
    }
    return true;
}

// The accumulator half of a HotSlot, as a per-workgroup aggregate (k_reduce's LDS table).
struct FlowAgg {
    unsigned long long key;
    unsigned long long acc[2];
    uint32_t first_n, last1, tbits, tflags;
    uint32_t fin_n[2], syn1[2];
};
static_assert(sizeof(FlowAgg) == 56, "");

// plain merge of an aggregate into a slot image (commutative: sums, maxima, ORs)
__device__ __forceinline__ void agg_fold(HotSlot& h, const FlowAgg& a) {
    h.acc[0] += a.acc[0];
    h.acc[1] += a.acc[1];
    h.first_n = max(h.first_n, a.first_n);
    h.last1 = max(h.last1, a.last1);
    h.tbits |= a.tbits;
    h.tflags |= a.tflags;
    h.fin_n[0] = max(h.fin_n[0], a.fin_n[0]);
    h.fin_n[1] = max(h.fin_n[1], a.fin_n[1]);
    h.syn1[0] = max(h.syn1[0], a.syn1[0]);
    h.syn1[1] = max(h.syn1[1], a.syn1[1]);
}

// ---- tile aggregates (k_bin / k_bin_slow -> k_reduce) ------------------------------------
// A flow with >= TAGG_MIN packets in one k_bin tile travels as one aggregate of its packets
// instead of one 16-byte record per packet: three consecutive record slots in the partition
// segment, each marked with bit 31 of word w (a packet record's w = pack_misc() leaves bit 31
// clear) and its slot index in bits 29-30.  Fields (indices absolute in the batch):
//   s0 = {lo low, lo high, first | tflags dir0 << 24, last | first SYN, dir << 24 | MARK | 0 << 29}
//   s1 = {bytes0 | packets0 low 5 << 27, bytes1 | packets1 low 5 << 27, tbits,
//         packets0 >> 5 | (packets1 >> 5) << 7 | tflags dir1 << 14 | MARK | 1 << 29}
//   s2 = {syn1[0], syn1[1], fin1[0], fin1[1] | MARK | 2 << 29}   (index + 1, 0 = none)
// A tile has 2048 packets: packets <= 2048 (12 bits), bytes <= 2048 * 65535 < 2^27.
constexpr uint32_t AGG_MARK = 0x80000000u;
constexpr uint32_t TAGG_MIN = 3;  // below this, packet records are smaller than one aggregate

__device__ __forceinline__ bool rec_is_agg(const uint4& r) { return (r.w & AGG_MARK) != 0; }
__device__ __forceinline__ uint32_t rec_agg_slot(const uint4& r) { return (r.w >> 29) & 3; }

__device__ __forceinline__ void agg_encode(const FlowAgg& a, uint4& s0, uint4& s1, uint4& s2) {
    const uint32_t p0 = (uint32_t)(a.acc[0] >> 40), p1 = (uint32_t)(a.acc[1] >> 40);
    const uint32_t b0 = (uint32_t)(a.acc[0] & ACC_BYTES_MASK), b1 = (uint32_t)(a.acc[1] & ACC_BYTES_MASK);
    const uint32_t f1[2] = {a.fin_n[0] ? ~a.fin_n[0] + 1 : 0u, a.fin_n[1] ? ~a.fin_n[1] + 1 : 0u};
    s0 = make_uint4((uint32_t)a.key, (uint32_t)(a.key >> 32), first_idx(a.first_n) | ((a.tflags & 0xFF) << 24),
                    (a.last1 - 1) | ((a.first_n & 3u) << 24) | AGG_MARK);
    s1 = make_uint4(b0 | (p0 << 27), b1 | (p1 << 27), a.tbits,
                    (p0 >> 5) | ((p1 >> 5) << 7) | (((a.tflags >> 8) & 0xFF) << 14) | AGG_MARK | (1u << 29));
    s2 = make_uint4(a.syn1[0], a.syn1[1], f1[0], f1[1] | AGG_MARK | (2u << 29));
}

__device__ __forceinline__ FlowAgg agg_decode(const uint4& s0, const uint4& s1, const uint4& s2) {
    FlowAgg a;
    a.key = ((unsigned long long)s0.y << 32) | s0.x;
    const uint64_t p0 = (s1.x >> 27) | ((s1.w & 0x7F) << 5), p1 = (s1.y >> 27) | (((s1.w >> 7) & 0x7F) << 5);
    a.acc[0] = (p0 << 40) | (s1.x & 0x07FFFFFFu);
    a.acc[1] = (p1 << 40) | (s1.y & 0x07FFFFFFu);
    a.first_n = ((~s0.z & 0xFFFFFFu) << 8) | ((s0.w >> 24) & 3u);
    a.last1 = (s0.w & 0xFFFFFF) + 1;
    a.tbits = s1.z;
    a.tflags = (s0.z >> 24) | (((s1.w >> 14) & 0xFF) << 8);
    a.syn1[0] = s2.x;
    a.syn1[1] = s2.y;
    const uint32_t f0 = s2.z, f1 = s2.w & 0xFFFFFF;
    a.fin_n[0] = f0 ? ~(f0 - 1) : 0u;
    a.fin_n[1] = f1 ? ~(f1 - 1) : 0u;
    return a;
}

// atomic merge of an aggregate into a slot (when other workgroups may touch it too)
__device__ __forceinline__ void agg_merge_atomic(HotSlot* h, const FlowAgg& a) {
    if (a.acc[0]) atomicAdd((unsigned long long*)&h->acc[0], a.acc[0]);
    if (a.acc[1]) atomicAdd((unsigned long long*)&h->acc[1], a.acc[1]);
    atomicMax(&h->first_n, a.first_n);
    atomicMax(&h->last1, a.last1);
    if (a.tbits) atomicOr(&h->tbits, a.tbits);
    if (a.tflags) atomicOr(&h->tflags, a.tflags);
    for (int d = 0; d < 2; ++d) {
        if (a.fin_n[d]) atomicMax(&h->fin_n[d], a.fin_n[d]);
        if (a.syn1[d]) atomicMax(&h->syn1[d], a.syn1[d]);
    }
}

// probe/claim the aggregate's slot and merge it with device atomics; false when the probe
// failed (the caller defers the aggregate until the table has grown)
__device__ __forceinline__ bool merge_agg_probe(const TableView& t, const FlowAgg& a, uint32_t* new_keys) {
    uint4 head;
    bool claimed;
    HotSlot* h = probe_insert(t, a.key, head, claimed);
    if (!h) return false;
    if (claimed) atomicAdd(new_keys, 1u);
    agg_merge_atomic(h, a);
    return true;
}

// deferred aggregates: 3 record slots each, after the per-packet deferral list's counter
__device__ __forceinline__ void defer_agg(uint32_t* count, uint4* list, const uint4& s0, const uint4& s1,
                                          const uint4& s2) {
    const uint32_t pos = atomicAdd(count, 1u);
    list[3 * (size_t)pos] = s0;
    list[3 * (size_t)pos + 1] = s1;
    list[3 * (size_t)pos + 2] = s2;
}

// ---- flow record construction (FlowRecord::create/update, cache.cpp:94-152) ---------------
__device__ __forceinline__ void rec_create(ipxg_flow_record& r, const DevPkt& pk, const ipxg_pkt_desc& d,
                                           uint64_t hf, uint32_t cdir) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
    for (int k = 0; k < 32; ++k) w[k] = 0;
    r.flow_hash = hf;
    r.time_first_sec = r.time_last_sec = d.ts_sec;
    r.time_first_usec = r.time_last_usec = d.ts_usec;
    r.ip_version = pk.ip_version;
    r.ip_proto = pk.ip_proto;
    for (int k = 0; k < 4; ++k) {
        for (int q = 0; q < 4; ++q) {
            r.src_ip[4 * k + q] = (uint8_t)(pk.sip[k] >> (8 * q));
            r.dst_ip[4 * k + q] = (uint8_t)(pk.dip[k] >> (8 * q));
        }
    }
    const uint32_t m[3] = {pk.mac_lo, pk.mac_mid, pk.mac_hi};
    for (int q = 0; q < 6; ++q) {
        r.dst_mac[q] = (uint8_t)(m[q >> 2] >> (8 * (q & 3)));
        r.src_mac[q] = (uint8_t)(m[(q + 6) >> 2] >> (8 * ((q + 6) & 3)));
    }
    const uint8_t pr = pk.ip_proto;
    if (pr == 6 || pr == 17 || pr == 1 || pr == 58) {
        r.src_port = pk.src_port;
        r.dst_port = pk.dst_port;
    }
    r.vlan_id = (uint16_t)pk.vlan_id;
    r.reserved[0] = (uint8_t)cdir;  // creator's canonical direction (not exported)
}

__device__ __forceinline__ uint8_t export_reason(const ipxg_flow_record& r) {
    return ((r.src_tcp_flags | r.dst_tcp_flags) & 0x05) ? IPXG_FLOW_END_EOF : IPXG_FLOW_END_INACTIVE;
}

// ex.count[1] is raised if the host under-sized the buffer (reported as an error)
__device__ __forceinline__ void store_export(ExportView ex, uint32_t pos, const ipxg_flow_record& r,
                                             uint8_t reason) {
    if (pos >= ex.cap) {
        atomicOr(ex.count + 1, 1u);
        return;
    }
    ipxg_flow_record o = r;
    o.end_reason = reason;
    o.reserved0 = 0;
    for (int k = 0; k < 8; ++k) o.reserved[k] = 0;  // (ext: exported with the record)
    ex.buf[pos] = o;
}

// export_flow's statistics (cache.cpp:264-267) into a block's counters: end reason and
// FlowRecordStats bucket
__device__ __forceinline__ void count_export(uint32_t* sc, const ipxg_flow_record& r, uint8_t reason) {
    atomicAdd(&sc[ST_END_INACTIVE + reason - 1], 1u);
    atomicAdd(&sc[ST_PKTS_1 + pkts_bucket((uint64_t)r.src_packets + r.dst_packets)], 1u);
}

// ---- the flow record as 32 words in registers -----------------------------------------------
// Built or updated through ipxg_flow_record's byte fields, a record stayed in scratch memory
// (128 B per lane in k_fin_list, 84 B in k_finish); the per-flow finalise and export paths
// handle it as 32 words at compile-time indices instead (ipxg.h layout, little-endian).
struct RecW {
    uint32_t w[32];
};
enum RecWord : int {
    RW_HASH = 0, RW_TFS = 2, RW_TFU = 3, RW_TLS = 4, RW_TLU = 5, RW_SBYTES = 6, RW_DBYTES = 8, RW_SPK = 10,
    RW_DPK = 11,
    RW_FLAGS = 12,  // src_tcp_flags | dst_tcp_flags << 8 | ip_version << 16 | ip_proto << 24
    RW_PORTS = 13,  // src_port | dst_port << 16
    RW_SIP = 14, RW_DIP = 18,
    RW_MAC = 22,    // src_mac[6], dst_mac[6] over words 22..24
    RW_VLAN = 25,   // vlan_id | end_reason << 16 | reserved0 << 24
    RW_RSV = 26,    // reserved[8]: byte 0 = the creator's canonical direction while the flow lives
    RW_EXT = 28, RW_RSV2 = 30
};
static_assert(offsetof(ipxg_flow_record, time_first_sec) == 4 * RW_TFS && offsetof(ipxg_flow_record, src_bytes) == 4 * RW_SBYTES &&
              offsetof(ipxg_flow_record, src_packets) == 4 * RW_SPK && offsetof(ipxg_flow_record, src_tcp_flags) == 4 * RW_FLAGS &&
              offsetof(ipxg_flow_record, src_port) == 4 * RW_PORTS && offsetof(ipxg_flow_record, src_ip) == 4 * RW_SIP &&
              offsetof(ipxg_flow_record, dst_ip) == 4 * RW_DIP && offsetof(ipxg_flow_record, src_mac) == 4 * RW_MAC &&
              offsetof(ipxg_flow_record, vlan_id) == 4 * RW_VLAN && offsetof(ipxg_flow_record, reserved) == 4 * RW_RSV &&
              offsetof(ipxg_flow_record, ext) == 4 * RW_EXT && sizeof(ipxg_flow_record) == 128,
              "RecW word map");
__device__ __forceinline__ uint64_t rw64(const RecW& r, int k) { return ((uint64_t)r.w[k + 1] << 32) | r.w[k]; }
__device__ __forceinline__ void rw64_set(RecW& r, int k, uint64_t v) {
    r.w[k] = (uint32_t)v;
    r.w[k + 1] = (uint32_t)(v >> 32);
}
__device__ __forceinline__ uint32_t rw_sflags(const RecW& r) { return r.w[RW_FLAGS] & 0xFF; }
__device__ __forceinline__ uint32_t rw_dflags(const RecW& r) { return (r.w[RW_FLAGS] >> 8) & 0xFF; }
__device__ __forceinline__ uint32_t rw_ipver(const RecW& r) { return (r.w[RW_FLAGS] >> 16) & 0xFF; }
__device__ __forceinline__ uint32_t rw_proto(const RecW& r) { return r.w[RW_FLAGS] >> 24; }
__device__ __forceinline__ uint32_t rw_creator(const RecW& r) { return r.w[RW_RSV] & 0xFF; }
__device__ __forceinline__ RecW rec_load_w(const ipxg_flow_record* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    RecW r;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint4 v = q[i];
        r.w[4 * i] = v.x;
        r.w[4 * i + 1] = v.y;
        r.w[4 * i + 2] = v.z;
        r.w[4 * i + 3] = v.w;
    }
    return r;
}
// The record's first 64 bytes (words 0-15: flow hash, times, byte and packet counters, TCP flags,
// version/protocol, ports, the first word of src_ip) -- everything a continuing flow's batch reads
// and updates; the second half (addresses, MACs, VLAN, extension handle) is written once, when the
// record is created, and read again only when it is exported.
__device__ __forceinline__ void rec_load_head_w(const ipxg_flow_record* p, RecW& r) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = q[i];
        r.w[4 * i] = v.x;
        r.w[4 * i + 1] = v.y;
        r.w[4 * i + 2] = v.z;
        r.w[4 * i + 3] = v.w;
    }
}
__device__ __forceinline__ void rec_load_tail_w(const ipxg_flow_record* p, RecW& r) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 4; i < 8; ++i) {
        const uint4 v = q[i];
        r.w[4 * i] = v.x;
        r.w[4 * i + 1] = v.y;
        r.w[4 * i + 2] = v.z;
        r.w[4 * i + 3] = v.w;
    }
}
__device__ __forceinline__ void rec_store_head_w(ipxg_flow_record* p, const RecW& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = make_uint4(r.w[4 * i], r.w[4 * i + 1], r.w[4 * i + 2], r.w[4 * i + 3]);
}
__device__ __forceinline__ void rec_store_w(ipxg_flow_record* p, const RecW& r) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = make_uint4(r.w[4 * i], r.w[4 * i + 1], r.w[4 * i + 2], r.w[4 * i + 3]);
}
// the record of slot s in the table: its first half in the slot's line, its second in `tail`
__device__ __forceinline__ void tbl_load_head(const TableView& t, uint32_t s, RecW& r) {
    rec_load_head_w(reinterpret_cast<const ipxg_flow_record*>(t.line[s].head), r);
}
__device__ __forceinline__ void tbl_load_tail(const TableView& t, uint32_t s, RecW& r) {
    const uint4* q = reinterpret_cast<const uint4*>(t.tail + (size_t)s * REC_TAIL_WORDS);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = q[i];
        r.w[16 + 4 * i] = v.x;
        r.w[16 + 4 * i + 1] = v.y;
        r.w[16 + 4 * i + 2] = v.z;
        r.w[16 + 4 * i + 3] = v.w;
    }
}
__device__ __forceinline__ void tbl_store_head(const TableView& t, uint32_t s, const RecW& r) {
    rec_store_head_w(reinterpret_cast<ipxg_flow_record*>(t.line[s].head), r);
}
__device__ __forceinline__ void tbl_store_rec(const TableView& t, uint32_t s, const RecW& r) {
    tbl_store_head(t, s, r);
    uint4* q = reinterpret_cast<uint4*>(t.tail + (size_t)s * REC_TAIL_WORDS);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        q[i] = make_uint4(r.w[16 + 4 * i], r.w[16 + 4 * i + 1], r.w[16 + 4 * i + 2], r.w[16 + 4 * i + 3]);
}
__device__ __forceinline__ RecW tbl_load_rec(const TableView& t, uint32_t s) {
    RecW r;
    tbl_load_head(t, s, r);
    tbl_load_tail(t, s, r);
    return r;
}
__device__ __forceinline__ ipxg_flow_record tbl_rec(const TableView& t, uint32_t s) {
    const RecW w = tbl_load_rec(t, s);
    ipxg_flow_record r;
    memcpy(&r, &w, sizeof(r));
    return r;
}
__device__ __forceinline__ void tbl_put_rec(const TableView& t, uint32_t s, const ipxg_flow_record& r) {
    RecW w;
    memcpy(&w, &r, sizeof(w));
    tbl_store_rec(t, s, w);
}
__device__ __forceinline__ uint8_t export_reason_w(const RecW& r) {
    return ((rw_sflags(r) | rw_dflags(r)) & 0x05) ? IPXG_FLOW_END_EOF : IPXG_FLOW_END_INACTIVE;
}
// store_export / count_export on the word form
__device__ __forceinline__ void store_export_w(ExportView ex, uint32_t pos, const RecW& r, uint8_t reason) {
    if (pos >= ex.cap) {
        atomicOr(ex.count + 1, 1u);
        return;
    }
    RecW o = r;
    o.w[RW_VLAN] = (r.w[RW_VLAN] & 0xFFFF) | ((uint32_t)reason << 16);  // end_reason; reserved0 = 0
    o.w[RW_RSV] = o.w[RW_RSV + 1] = 0;                                  // reserved zero on export
    rec_store_w(&ex.buf[pos], o);
}
// A reserved export record left unfilled (k_fin_list's early reservation): all zero, so its end
// reason is 0, which no export has (k_ex_compact drops it)
__device__ __forceinline__ void store_export_hole(ExportView ex, uint32_t pos) {
    if (pos >= ex.cap) {
        atomicOr(ex.count + 1, 1u);
        return;
    }
    uint4* q = reinterpret_cast<uint4*>(&ex.buf[pos]);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void count_export_w(uint32_t* sc, const RecW& r, uint8_t reason) {
    atomicAdd(&sc[ST_END_INACTIVE + reason - 1], 1u);
    atomicAdd(&sc[ST_PKTS_1 + pkts_bucket((uint64_t)r.w[RW_SPK] + r.w[RW_DPK])], 1u);
}
// The same for a wave's exports (active lanes; convergent): one LDS atomic per reason and bucket
// present -- lanes exporting alike (a finish exports every record as FORCED) otherwise serialise
// on one LDS word.
__device__ __forceinline__ void count_exports_wave(uint32_t* sc, bool active, const RecW& r, uint32_t reason) {
    if (!__any(active)) return;  // (wave-uniform)
    const uint32_t bucket = active ? pkts_bucket((uint64_t)r.w[RW_SPK] + r.w[RW_DPK]) : 0u;
    const bool lead = (threadIdx.x & 63) == 0;
#pragma unroll
    for (uint32_t q = 1; q <= 5; ++q) {
        const unsigned long long m = __ballot(active && reason == q);
        if (lead && m) atomicAdd(&sc[ST_END_INACTIVE + q - 1], (uint32_t)__popcll(m));
    }
#pragma unroll
    for (uint32_t q = 0; q < 6; ++q) {
        const unsigned long long m = __ballot(active && bucket == q);
        if (lead && m) atomicAdd(&sc[ST_PKTS_1 + q], (uint32_t)__popcll(m));
    }
}
// v summed over the wave into one LDS word (convergent)
__device__ __forceinline__ void wave_add_lds(uint32_t* w, uint32_t v) {
    if (!__any(v != 0)) return;  // (wave-uniform)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(w, v);
}

// FlowRecord::create's fields (rec_create) into the word form
__device__ __forceinline__ void rec_create_w(RecW& r, const DevPkt& pk, const ipxg_pkt_desc& d, uint64_t hf,
                                             uint32_t cdir) {
#pragma unroll
    for (int k = 0; k < 32; ++k) r.w[k] = 0;
    rw64_set(r, RW_HASH, hf);
    r.w[RW_TFS] = r.w[RW_TLS] = d.ts_sec;
    r.w[RW_TFU] = r.w[RW_TLU] = d.ts_usec;
    r.w[RW_FLAGS] = ((uint32_t)pk.ip_version << 16) | ((uint32_t)pk.ip_proto << 24);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        r.w[RW_SIP + k] = pk.sip[k];
        r.w[RW_DIP + k] = pk.dip[k];
    }
    // frame bytes 0-5 = dst_mac, 6-11 = src_mac (mac_lo/mid/hi = bytes 0-11, little-endian)
    r.w[RW_MAC] = (pk.mac_mid >> 16) | (pk.mac_hi << 16);     // src_mac[0..3]
    r.w[RW_MAC + 1] = (pk.mac_hi >> 16) | (pk.mac_lo << 16);  // src_mac[4..5], dst_mac[0..1]
    r.w[RW_MAC + 2] = (pk.mac_lo >> 16) | (pk.mac_mid << 16); // dst_mac[2..5]
    const uint8_t pr = pk.ip_proto;
    if (pr == 6 || pr == 17 || pr == 1 || pr == 58) r.w[RW_PORTS] = (uint32_t)pk.src_port | ((uint32_t)pk.dst_port << 16);
    r.w[RW_VLAN] = (uint32_t)pk.vlan_id & 0xFFFF;
    r.w[RW_RSV] = cdir & 0xFF;  // creator's canonical direction (not exported)
}

// ex.count[2] counts the exported records that take the IPv6 basic template (the IPFIX message
// layout needs the split, ipxg_engine.cpp ipfix_plan).  Convergent: every lane of the wave.
__device__ __forceinline__ void count_v6_exports(ExportView ex, bool v6) {
    if (!ex.count6) return;  // uniform
    const uint64_t m = __ballot(v6);
    if (m && lane_id() == (uint32_t)__builtin_ctzll(m)) atomicAdd(ex.count + 2, (uint32_t)__popcll(m));
}

__device__ __forceinline__ void clear_slot(HotSlot* h, uint64_t key, uint32_t state) {
    HotSlot z = {};
    z.key = key;
    z.state = state;
    *h = z;
}

__device__ __forceinline__ void apply_frag_ports(const Params& p, const FragView& f, uint32_t idx,
                                                 DevPkt& pk) {
    if (p.frag_enable && (pk.frag_off || pk.more_fragments)) {
        uint32_t pp = f.ports[idx];
        pk.src_port = (uint16_t)(pp >> 16);
        pk.dst_port = (uint16_t)(pp & 0xFFFF);
    }
}

// a fragment for the fragmentation-cache path: (bucket << 24) | packet index
__device__ __forceinline__ void divert_fragment(const DevPkt& pk, const Params& p, const FragView& f, BatchCtl* ctl,
                                                uint32_t i) {
    const uint32_t bucket = (uint32_t)(frag_key_hash(pk) % (uint64_t)p.frag_size);
    const uint32_t pos = atomicAdd(&ctl->frag_count, 1u);
    f.list[pos] = ((uint64_t)bucket << 24) | i;
}

// ---- register parser for the common frame shape -------------------------------------------
// The common frame shape -- Ethernet (no VLAN tag), IPv4 with IHL 5, UDP or TCP without
// options -- read straight from its first 48 bytes in registers: exactly the fields, checks
// and counters parse_frame produces for such a frame (parse_eth_hdr parser.cpp:68-155,
// parse_ipv4_hdr :311-356, parse_tcp_hdr :469-543 with doff <= 5, parse_udp_hdr :552-573),
// without staging it in LDS.  Returns false for any other shape, a TCP header cut by caplen,
// or a fragment when the fragmentation cache is on: the caller then takes the general
// path.  c0..c2 = bytes 0..47, caplen >= 48.
__device__ __forceinline__ bool parse_fast(const uint4& c0, const uint4& c1, const uint4& c2, uint32_t caplen,
                                           bool frag_enable, DevPkt& p, ParseCounts& c) {
    if ((c0.w & 0xFFFF) != 0x0008) return false;          // ethertype 0x0800 at bytes 12-13
    if (((c0.w >> 16) & 0xFF) != 0x45) return false;      // version 4, IHL 5
    const uint32_t proto = c1.y >> 24;                     // byte 23
    if (proto == 47) return false;                         // GRE: the general parser recurses
    const uint32_t fo = bswap16(c1.y);                     // bytes 20-21
    const uint32_t frag_off = fo & 0x1FFF;
    if (frag_enable && (fo & 0x3FFF)) return false;        // a fragment: the fragmentation-cache path
    uint32_t ports = 0, flags = 0;
    if (frag_off == 0 && proto == 6) {
        if (caplen < 54) return false;                     // 20 > data_len: the general path drops it
        if (((c2.w >> 20) & 0xF) > 5) return false;        // TCP options: the general option walk
        flags = c2.w >> 24;                                // byte 47
    }
    if (frag_off == 0 && (proto == 6 || proto == 17)) ports = (c2.x >> 16) | (c2.y << 16);  // bytes 34-37
    p.ip_version = 4;
    p.ip_proto = (uint8_t)proto;
    p.tcp_flags = (uint8_t)flags;
    p.ethertype = 0x0800;
    p.ip_len = bswap16(c1.x);                              // bytes 16-17
    p.frag_id = bswap16(c1.x >> 16);                       // bytes 18-19
    p.frag_off = (uint16_t)frag_off;
    p.more_fragments = (fo & 0x2000) ? 1 : 0;
    p.src_port = bswap16(ports);
    p.dst_port = bswap16(ports >> 16);
    p.l4 = (frag_off == 0 && (proto == 6 || proto == 17)) ? (uint8_t)proto : 0;
    p.vlan_id = 0;
    p.sip[0] = (c1.z >> 16) | (c1.w << 16);                // bytes 26-29, memory order
    p.dip[0] = (c1.w >> 16) | (c2.x << 16);                // bytes 30-33
    p.sip[1] = p.sip[2] = p.sip[3] = 0;
    p.dip[1] = p.dip[2] = p.dip[3] = 0;
    c.seen++;
    c.parsed++;
    c.ipv4++;
    c.ipv4_bytes += caplen;
    if (frag_off == 0 && proto == 6) c.tcp++;
    if (frag_off == 0 && proto == 17) c.udp++;
    return true;
}

// a frame the register parser may take: 16-byte aligned in the arena, 48 bytes captured
__device__ __forceinline__ bool fast_shape(const BatchView& b, const ipxg_pkt_desc& d) {
    return frame_aligned(b, d) && d.caplen >= 48;
}

// ---- register parser for the shapes of the variable-length mixes --------------------------
// The wide walk (k_bin<., true>) loads a frame's first 80 bytes (WIDE_DW dwords) and parses
// the header chains that make up most of the configs[2] / configs[4] mixes straight from those
// registers: Ethernet with 0, 1 or 2 VLAN tags (outer 0x8100 / 0x88A8, inner 0x8100), then
// IPv4 with IHL 5 or IPv6 whose next header is TCP or UDP, then TCP without options or with the
// NOP,NOP,Timestamp block (doff 8, the option walk of parse_tcp_hdr succeeds on it whatever
// the timestamp bytes; with IPv6 only untagged, as its options end at byte 78), or UDP;
// untagged IPv6 may carry one or two 8-byte extension headers (two: UDP only), and untagged
// IPv4 may carry GRE with an inner IPv4 + UDP, or + option-less TCP (GRE with at most one
// optional field).
// Every header boundary of these chains sits at 2 mod 4 bytes,
// and the tags only shift the L3 header by whole dwords, so the window is re-based by 0, 1 or
// 2 dwords (two selects per dword) and every field is then read at a compile-time offset: no
// dynamic register indexing, no LDS.  The fields, checks and counters are those parse_frame
// gives such a frame (parse_eth_hdr parser.cpp:68-155, parse_ipv4_hdr :311-356,
// parse_ipv6_hdr :423-460, parse_tcp_hdr :469-543, parse_udp_hdr :552-573); any other shape,
// or any read the caplen checks would not cover, returns false and the frame takes the general
// parser (k_bin_slow).  *ext: the frame is not the plain shape parse_fast takes.
constexpr int WIDE_DW = 20;  // 80 bytes
constexpr int WIDE2_DW = 24; // 96 bytes: k_bin's wide walk without tile aggregation (its registers allow
                             // a sixth chunk): also IPv6 with three 8-byte extension headers (UDP) and
                             // IPv6 TCP behind one or two, timestamp options included

template <int O>
__device__ __forceinline__ uint32_t wle32(const uint32_t* w) {
    if constexpr (O % 4 == 0) return w[O / 4];
    else return __builtin_amdgcn_alignbyte(w[O / 4 + 1], w[O / 4], O % 4);
}
template <int O>
__device__ __forceinline__ uint32_t wb8(const uint32_t* w) { return (w[O / 4] >> (8 * (O % 4))) & 0xFF; }
template <int O>
__device__ __forceinline__ uint32_t wbe16(const uint32_t* w) { return bswap16(wle32<O>(w)); }

// PAY: also Packet::payload / payload_len as parse_frame<true> gives them (parser.cpp:780-797;
// the pre-classifier of the plugin bridge compares payload prefixes)
template <bool PAY = false, int WD = WIDE_DW>
__device__ __forceinline__ bool parse_medium(const uint32_t (&w)[WD], uint32_t caplen, bool frag_enable,
                                             DevPkt& p, ParseCounts& c, bool& ext) {
    static_assert(WD == WIDE_DW || WD == WIDE2_DW, "window");
    constexpr bool W2 = WD >= WIDE2_DW;
    // Ethernet + tags (parse_eth_hdr): only the outermost tag's VLAN id is kept
    uint32_t et = wbe16<12>(w), vlan = 0, S = 0;
    if (et == ETH_P_8021AD || et == ETH_P_8021Q) {
        vlan = wbe16<14>(w) & 0x0FFF;
        et = wbe16<16>(w);
        S = 1;
        if (et == ETH_P_8021Q) {
            et = wbe16<20>(w);
            S = 2;
            if (et == ETH_P_8021Q) return false;  // a third tag: the general walk
        }
    }
    // untagged MPLS (1-3 labels) and PPPoE sessions (process_mpls_stack :581-602 + process_mpls
    // :611-634, process_pppoe :643-671) shift the IP header by whole dwords too; the counters keep
    // the Ethernet ethertype (parse_packet counts IPv4/IPv6 by it, :798-805)
    uint32_t l3 = et;
    bool mpls = false, pppoe = false;
    if ((et == ETH_P_MPLS_UC || et == ETH_P_MPLS_MC) && S == 0) {
        // bottom of stack: bit 0 of a label's byte 2 (frame bytes 16, 20, 24)
        const uint32_t n = (wb8<16>(w) & 1) ? 1u : ((wb8<20>(w) & 1) ? 2u : ((wb8<24>(w) & 1) ? 3u : 0u));
        if (n == 0 || caplen < 14 + 4 * n + 1) return false;  // deeper stacks / past caplen: the general walk
        const uint32_t nib = (n == 1 ? wb8<18>(w) : (n == 2 ? wb8<22>(w) : wb8<26>(w))) >> 4;
        l3 = nib == 4 ? ETH_P_IP : (nib == 6 ? ETH_P_IPV6 : 0u);  // 0 (EoMPLS) or other: the general walk
        S = n;
        mpls = true;
    } else if (et == ETH_P_PPP_SES && S == 0) {
        if (caplen < 22 || wb8<15>(w) != 0) return false;  // code != 0 ends the reference's parse
        const uint32_t nh = wbe16<20>(w);
        l3 = nh == 0x0021 ? ETH_P_IP : (nh == 0x0057 ? ETH_P_IPV6 : 0u);
        S = 2;
        pppoe = true;
    }
    if (l3 != ETH_P_IP && l3 != ETH_P_IPV6) return false;
    // the window re-based so that the L3 header starts at byte 14 of v
    constexpr int VD = WD - 2;
    uint32_t v[VD];
    // masks rather than a select the compiler could fold into a dynamic index of w (which
    // would put w on the stack)
    const uint32_t m0 = 0u - (S == 0), m1 = 0u - (S == 1), m2 = 0u - (S == 2), m3 = 0u - (S == 3);
#pragma unroll
    for (int k = 3; k < VD; ++k)
        v[k] = (w[k] & m0) | (w[k + 1] & m1) | (w[k + 2] & m2) | (k + 3 < WD ? w[k + 3] & m3 : 0u);
    v[0] = v[1] = v[2] = 0;
    // untagged IPv4 (IHL 5) -> GRE -> IPv4 (parse_ipv4_hdr :320-326, parse_gre :256-302): the
    // outer header sets no field; the inner one starts 6 dwords later plus one per optional
    // field (checksum, key, sequence number) -- with two or three, only its UDP ports fit
    bool gre = false;
    uint32_t gopt = 0;
    if (l3 == ETH_P_IP && S == 0 && wb8<23>(w) == 47) {
        const uint32_t gf = wbe16<34>(w);
        if (wb8<14>(w) != 0x45 || wbe16<36>(w) != ETH_P_IP) return false;
        gopt = ((gf & GRE_CHECKSUM) ? 1u : 0u) + ((gf & GRE_KEY) ? 1u : 0u) + ((gf & GRE_SEQNUM) ? 1u : 0u);
        const uint32_t g0 = 0u - (gopt == 0), g1 = 0u - (gopt == 1), g2 = 0u - (gopt == 2), g3 = 0u - (gopt == 3);
#pragma unroll
        for (int k = 3; k < VD; ++k)
            v[k] = (k + 6 < WD ? w[k + 6] & g0 : 0u) | (k + 7 < WD ? w[k + 7] & g1 : 0u) |
                   (k + 8 < WD ? w[k + 8] & g2 : 0u) | (k + 9 < WD ? w[k + 9] & g3 : 0u);
        gre = true;
    }
    const uint32_t o3 = 14 + 4 * S + (gre ? 24u + 4u * gopt : 0u);  // the L3 offset in the frame
    uint32_t proto, o4, frag_off = 0, xh = 0;
    if (l3 == ETH_P_IP) {
        if (caplen < o3 + 20) return false;
        if (wb8<14>(v) != 0x45) return false;          // IHL 5 (options: the general walk)
        proto = wb8<23>(v);
        if (proto == 47) return false;                 // GRE (in GRE: the general walk)
        const uint32_t fo = wbe16<20>(v);
        frag_off = fo & 0x1FFF;
        if (frag_enable && (fo & 0x3FFF)) return false;  // the fragmentation-cache path
        p.ip_version = 4;
        p.ip_len = (uint16_t)wbe16<16>(v);
        p.frag_id = wbe16<18>(v);
        p.frag_off = (uint16_t)frag_off;
        p.more_fragments = (fo & 0x2000) ? 1 : 0;
        p.sip[0] = wle32<26>(v);
        p.dip[0] = wle32<30>(v);
        p.sip[1] = p.sip[2] = p.sip[3] = 0;
        p.dip[1] = p.dip[2] = p.dip[3] = 0;
        o4 = o3 + 20;
    } else {
        if (caplen < o3 + 40) return false;
        proto = wb8<20>(v);
        // untagged only: up to two 8-byte hop-by-hop / routing / destination-options headers
        // (length byte 0), the walk of skip_ipv6_ext_hdrs parser.cpp:365-412 for those types; its
        // data-length checks are implied by the L4 caplen checks below
        if (proto == 0 || proto == 43 || proto == 60) {
            if (S != 0 || wb8<55>(w) != 0) return false;
            const uint32_t p1 = wb8<54>(w);
            if (p1 == 0 || p1 == 43 || p1 == 60) {
                if (wb8<63>(w) != 0) return false;
                proto = wb8<62>(w);
                xh = 2;
                if constexpr (W2) {  // a third (the 96-byte window)
                    if (proto == 0 || proto == 43 || proto == 60) {
                        if (wb8<71>(w) != 0) return false;
                        proto = wb8<70>(w);
                        xh = 3;
                    }
                }
            } else {
                proto = p1;
                xh = 1;
            }
        }
        if (proto != 6 && proto != 17) return false;   // other extension headers (or another L4)
        if (xh == (W2 ? 3u : 2u) && proto == 6) return false;  // its TCP header would end past the window
        if (S == 3 && proto == 6) return false;         // under 3 MPLS labels: UDP fits, TCP does not
        p.ip_version = 6;
        p.ip_len = (uint16_t)(wbe16<18>(v) + 40);
        p.frag_id = 0;
        p.frag_off = 0;
        p.more_fragments = 0;
        p.sip[0] = wle32<22>(v);
        p.sip[1] = wle32<26>(v);
        p.sip[2] = wle32<30>(v);
        p.sip[3] = wle32<34>(v);
        p.dip[0] = wle32<38>(v);
        p.dip[1] = wle32<42>(v);
        p.dip[2] = wle32<46>(v);
        p.dip[3] = wle32<50>(v);
        o4 = o3 + 40 + 8 * xh;
    }
    const bool v6 = l3 == ETH_P_IPV6;
    uint32_t ports = 0, flags = 0, l4h = 0;
    bool tcp_opt = false;
    if (frag_off == 0 && proto == 6) {
        if (caplen < o4 + 20 || gopt > 1) return false;  // (past the window)
        uint32_t w3 = v6 ? (xh ? wle32<74>(w) : wle32<66>(v)) : wle32<46>(v);  // L4 bytes 12..15
        if constexpr (W2) w3 = xh == 2 ? wle32<82>(w) : w3;
        const uint32_t doff = (w3 & 0xFF) >> 4;
        l4h = 4 * doff;
        if (doff > 5) {
            if (gre || (v6 && (S != 0 || (!W2 && xh)))) return false;  // the options would end past the window
            uint32_t opt = v6 ? wle32<74>(w) : wle32<54>(v);  // L4 bytes 20..23
            if constexpr (W2) opt = v6 ? (xh == 2 ? wle32<90>(w) : (xh ? wle32<82>(w) : opt)) : opt;
            if (doff != 8 || opt != 0x0A080101u || caplen < o4 + 32) return false;
            tcp_opt = true;
        }
        flags = (w3 >> 8) & 0xFF;
        ports = v6 ? (xh == 2 ? wle32<70>(w) : (xh ? wle32<62>(w) : wle32<54>(v))) : wle32<34>(v);
    } else if (frag_off == 0 && proto == 17) {
        if (caplen < o4 + 8) return false;
        ports = v6 ? (xh == 2 ? wle32<70>(w) : (xh ? wle32<62>(w) : wle32<54>(v))) : wle32<34>(v);
        if constexpr (W2) ports = xh == 3 ? wle32<78>(w) : ports;
        l4h = 8;
    }
    if constexpr (PAY) {  // parser.cpp:780-797 in its uint16_t arithmetic (l4 offset o4 != l3 offset)
        const uint32_t ipl = v6 ? ((uint32_t)p.ip_len - 40u - 8u * xh) & 0xFFFF : ((uint32_t)p.ip_len - 20u) & 0xFFFF;
        const uint32_t off = o4 + l4h;
        uint32_t pkt_len = caplen;
        if (o4 + ipl < 64) pkt_len = (o4 + ipl) & 0xFFFF;
        uint32_t plen = (ipl - l4h) & 0xFFFF;
        if (plen + off > pkt_len) plen = (pkt_len - off) & 0xFFFF;
        p.payload_off = (uint16_t)off;
        p.payload_len = (uint16_t)plen;
    }
    p.ip_proto = (uint8_t)proto;
    p.tcp_flags = (uint8_t)flags;
    p.ethertype = (uint16_t)et;
    p.src_port = bswap16(ports);
    p.dst_port = bswap16(ports >> 16);
    p.l4 = (frag_off == 0 && (proto == 6 || proto == 17)) ? (uint8_t)proto : 0;
    p.vlan_id = vlan;
    ext = S != 0 || v6 || tcp_opt || gre;
    c.seen++;
    c.parsed++;
    const uint32_t e4 = et == ETH_P_IP ? 1u : 0u, e6 = et == ETH_P_IPV6 ? 1u : 0u;  // branch-free (see parse_frame)
    c.ipv6 += e6;
    c.ipv6_bytes += e6 ? caplen : 0u;
    c.ipv4 += e4;
    c.ipv4_bytes += e4 ? caplen : 0u;
    c.mpls += mpls ? 1u : 0u;
    c.pppoe += pppoe ? 1u : 0u;
    c.tcp += (frag_off == 0 && proto == 6) ? 1u : 0u;
    c.udp += (frag_off == 0 && proto == 17) ? 1u : 0u;
    c.vlan += vlan ? 1u : 0u;
    return true;
}

// DevPkt (FULL parse) -> the C-ABI's ipxg_parsed_pkt, flow-key hashes included
__device__ __forceinline__ ipxg_parsed_pkt to_parsed(const DevPkt& pk, bool ok) {
    ipxg_parsed_pkt o;
    uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
    for (int k = 0; k < (int)(sizeof(o) / 4); ++k) ow[k] = 0;
    o.valid = ok;
    o.ip_version = pk.ip_version;
    o.ip_proto = pk.ip_proto;
    o.tcp_flags = pk.tcp_flags;
    o.ethertype = pk.ethertype;
    o.ip_len = pk.ip_len;
    o.src_port = pk.src_port;
    o.dst_port = pk.dst_port;
    o.frag_off = pk.frag_off;
    o.more_fragments = pk.more_fragments;
    o.ip_ttl = pk.ip_ttl;
    o.vlan_id = pk.vlan_id;
    o.frag_id = pk.frag_id;
    o.mpls_top = pk.mpls_top;
    o.tcp_mss = pk.tcp_mss;
    o.tcp_options = pk.tcp_options;
    for (int k = 0; k < 4; ++k)
        for (int q = 0; q < 4; ++q) {
            o.src_ip[4 * k + q] = (uint8_t)(pk.sip[k] >> (8 * q));
            o.dst_ip[4 * k + q] = (uint8_t)(pk.dip[k] >> (8 * q));
        }
    const uint32_t m[3] = {pk.mac_lo, pk.mac_mid, pk.mac_hi};
    for (int q = 0; q < 6; ++q) {
        o.dst_mac[q] = (uint8_t)(m[q >> 2] >> (8 * (q & 3)));
        o.src_mac[q] = (uint8_t)(m[(q + 6) >> 2] >> (8 * ((q + 6) & 3)));
    }
    o.ip_tos = pk.ip_tos;
    o.ip_flags = pk.ip_flags;
    o.tcp_window = pk.tcp_window;
    o.tcp_seq = pk.tcp_seq;
    o.tcp_ack = pk.tcp_ack;
    if (ok && (pk.ip_version == 4 || pk.ip_version == 6)) {
        FlowKey kf, ki;
        build_keys(pk, kf, ki);
        o.hash_fwd = key_hash(kf);
        o.hash_inv = key_hash(ki);
    }
    if (ok) {
        o.payload_off = pk.payload_off;
        o.payload_len = pk.payload_len;
    }
    return o;
}

// ---- header staging into LDS ------------------------------------------------------------
// Stage the first min(caplen, IPXG_WIN) bytes of a frame into this lane's LDS column,
// zero-masked past caplen, plus one zero chunk so straddling reads see zeros.
__device__ __forceinline__ void stage_frame(uint32_t* col, const uint8_t* f, uint32_t cap) {
    const uint32_t nbytes = cap < IPXG_WIN ? cap : IPXG_WIN;
    const uint32_t nch = (nbytes + 15) >> 4;
    constexpr int NCH = IPXG_WIN / 16;
    if (((uintptr_t)f & 15) == 0) {
        uint4 v[NCH];
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            v[ch] = make_uint4(0, 0, 0, 0);
            if ((uint32_t)ch < nch) v[ch] = *reinterpret_cast<const uint4*>(f + 16 * ch);
        }
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            if ((uint32_t)ch > nch) break;
            uint32_t w[4] = {v[ch].x, v[ch].y, v[ch].z, v[ch].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                int b0 = 16 * ch + 4 * k;
                int valid = (int)cap - b0;
                uint32_t m = valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
                col[(4 * ch + k) * IPXG_BLOCK] = w[k] & m;
            }
        }
    } else {  // unaligned frame: byte loads (correct for any offset)
        for (uint32_t dw = 0; dw < 4 * (nch + (nch < NCH ? 1 : 0)); ++dw) {
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t o = dw * 4 + k;
                if (o < nbytes) w |= (uint32_t)f[o] << (8 * k);
            }
            col[dw * IPXG_BLOCK] = w;
        }
    }
}

// LDS window with caplen guard (bytes >= caplen read as 0).
struct LdsFrame {
    LdsWin w;
    __device__ __forceinline__ uint32_t b(uint32_t o) const { return o < w.g.cap ? w.b(o) : 0u; }
    __device__ __forceinline__ uint32_t le32(uint32_t o) const { return o < w.g.cap ? w.le32(o) : 0u; }
};

// ---- re-parse of one packet -------------------------------------------------------------
// straight from HBM (byte loads)
template <bool FULL>
__device__ __forceinline__ bool reparse(const BatchView& b, const Params& p, const FragView& f,
                                        uint32_t idx, DevPkt& pk, ipxg_pkt_desc& d) {
    d = b.desc[idx];
    GlobalSrc g{frame_ptr(b, d), d.caplen};
    ParseCounts dummy = {};
    if (!parse_frame<FULL>(g, d.caplen, p.dlt, pk, dummy)) return false;
    apply_frag_ports(p, f, idx, pk);
    return true;
}

// header bytes staged into this lane's LDS column with 16-byte loads (the column stride is
// IPXG_BLOCK dwords)
template <bool FULL>
__device__ __forceinline__ bool reparse_lds(const BatchView& b, const Params& p, const FragView& f,
                                            uint32_t idx, uint32_t* col, DevPkt& pk, ipxg_pkt_desc& d) {
    d = b.desc[idx];
    ParseCounts dummy = {};
    if ((p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB) && fast_shape(b, d)) {  // the common shape: registers only
        const uint4* fr = reinterpret_cast<const uint4*>(frame_ptr(b, d));
        const uint4 c0 = fr[0], c1 = fr[1], c2 = fr[2];
        if (parse_fast(c0, c1, c2, d.caplen, p.frag_enable, pk, dummy)) {
            if (FULL) {  // parse_eth_hdr's MAC copy; the rest of the FULL-only fields stay zero
                pk.mac_lo = c0.x;
                pk.mac_mid = c0.y;
                pk.mac_hi = c0.z;
                pk.mpls_top = pk.tcp_seq = pk.tcp_ack = pk.tcp_mss = 0;
                pk.tcp_options = 0;
                pk.tcp_window = 0;
                pk.ip_ttl = pk.ip_tos = pk.ip_flags = 0;
            }
            apply_frag_ports(p, f, idx, pk);
            return true;
        }
        // the wide register walk (k_bin's: tags, MPLS, PPPoE, IPv6, GRE, TCP timestamps) on the
        // 80-byte head -- the creators of the configs[2]/[4] mixes' flows, before the LDS walk
        if (frame_off(b, d) + 16u * 5 <= b.arena_len) {
            const uint4 z = make_uint4(0, 0, 0, 0);  // (chunks past caplen read as 0, as k_bin's loads)
            const uint4 c3 = 48u < d.caplen ? fr[3] : z, c4 = 64u < d.caplen ? fr[4] : z;
            const uint32_t w[WIDE_DW] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y,
                                         c2.z, c2.w, c3.x, c3.y, c3.z, c3.w, c4.x, c4.y, c4.z, c4.w};
            bool ext = false;
            if (parse_medium(w, d.caplen, p.frag_enable, pk, dummy, ext)) {
                if (FULL) {
                    pk.mac_lo = c0.x;
                    pk.mac_mid = c0.y;
                    pk.mac_hi = c0.z;
                    pk.mpls_top = pk.tcp_seq = pk.tcp_ack = pk.tcp_mss = 0;
                    pk.tcp_options = 0;
                    pk.tcp_window = 0;
                    pk.ip_ttl = pk.ip_tos = pk.ip_flags = 0;
                }
                apply_frag_ports(p, f, idx, pk);
                return true;
            }
        }
    }
    stage_frame(col, frame_ptr(b, d), d.caplen);
    LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
    if (!parse_frame<FULL>(S, d.caplen, p.dlt, pk, dummy)) return false;
    apply_frag_ports(p, f, idx, pk);
    return true;
}

// ---- TopPorts from the flow records (ps=true) ----------------------------------------------
// Every packet of a TCP/UDP flow passed parse_tcp_hdr / parse_udp_hdr with the flow's two
// ports (in one order or the other), so TopPorts' per-packet increments (parser.cpp:484-485,
// 563-564) sum to `packets` on each of the flow's ports -- two device atomics per flow and
// batch instead of two per packet.  The packets this misses or over-counts are corrected one
// by one where they are seen (k_pstats: TCP segments dropped after their ports were read, and
// TCP/UDP packets with both ports 0, whose flows are skipped here because non-first fragments
// share them; k_frag_accumulate: non-first fragments given ports by the fragmentation cache).
__device__ __forceinline__ void count_flow_ports(const TableView& t, const ipxg_flow_record& r, uint32_t packets) {
    if (!t.port_cnt || !packets || (r.ip_proto != 6 && r.ip_proto != 17) || (r.src_port == 0 && r.dst_port == 0))
        return;
    unsigned long long* a = t.port_cnt + (r.ip_proto == 17 ? 65536 : 0);
    atomicAdd(a + r.src_port, (unsigned long long)packets);
    atomicAdd(a + r.dst_port, (unsigned long long)packets);
}

__device__ __forceinline__ void count_flow_ports_w(const TableView& t, const RecW& r, uint32_t packets) {
    const uint32_t pr = rw_proto(r), sp = r.w[RW_PORTS] & 0xFFFF, dp = r.w[RW_PORTS] >> 16;
    if (!t.port_cnt || !packets || (pr != 6 && pr != 17) || (sp == 0 && dp == 0)) return;
    unsigned long long* a = t.port_cnt + (pr == 17 ? 65536 : 0);
    atomicAdd(a + sp, (unsigned long long)packets);
    atomicAdd(a + dp, (unsigned long long)packets);
}

// ---- per-slot batch finalisation ----------------------------------------------------------
enum FinStatus : uint32_t { FIN_DONE = 1, FIN_COMPLEX = 2 };
struct FinResult {
    uint32_t status;   // FIN_DONE / FIN_COMPLEX
    bool created;      // the slot held no live record before (a record was created)
    bool do_export;    // the open record was closed at the batch boundary (er, reason)
    bool fin_export;   // fuse: the completed record (er) is exported FORCED and the slot emptied
    uint8_t reason;
};

// h = the slot's complete batch image (key, accumulators, state) with h.last1 != 0.
// Applies the reference's SYN-after-FIN/RST, inactive and active checks at the batch's first
// packet of the flow (cache.cpp:431-472) -- from that packet's SYN flag and direction carried
// in h.first_n and its descriptor's timestamp -- and decides whether a split could fall
// strictly inside the batch (a SYN after a FIN/RST in the same direction, a gap >= inactive --
// detected conservatively as an empty inactive/2 bucket between busy ones --, or the active
// limit inside the batch).  If so the slot is marked complex (k_complex_walk replays the
// flow's packets sequentially); otherwise the accumulators are folded into the record and the
// slot cleared.  Only a flow that starts a record here (new, or split at the boundary)
// re-parses its first packet (FlowRecord::create's fields, cache.cpp:94-133).  Writes the slot
// (and its cold record) back.
// LDSW: stage the creator's headers in the lane's LDS column `col` (else byte loads).
// fuse (a finish follows, k_fin_list's fused mode; only on a table that held no live record
// before the batch, so no boundary export can coincide): the completed record goes to er
// (fin_export) instead of the table, and the slot is emptied.  One record out per slot either
// way, so the caller holds one record, not two (two were kept in scratch).
// slot_clean: the slot in memory holds only {key, state} (k_reduce listed its merged image
// without writing it back, and no packet of the batch was accumulated into it directly): a
// continuing flow whose state does not change then leaves the slot untouched.
// A continuing flow reads and writes only the first half of its record (rec_load_head_w); the
// creator's canonical direction comes from its flow hash (FlowRecord::create keys the record by
// the creating packet's forward hash, cache.cpp:84-92: it is the slot's canonical key iff the
// creator went in canonical direction 0 -- the rule rec_create_w / the host walk store in
// reserved[0]), so the second half is read only for an export.
// tmax: the batch's latest second when its timestamps are known not to decrease (the caller's
// batch was not flagged non-monotonic), else TMAX_UNKNOWN.  A continuing flow then reads its first
// packet's descriptor only when the batch reaches an inactive or active boundary of its record
// (the checks below cannot fire otherwise): one random 128-byte line less per flow on the 1M-flow
// mixes, where most flows continue.
constexpr uint32_t TMAX_UNKNOWN = 0xFFFFFFFFu;
// s = FIN_NO_SLOT: a new flow finalised without a table slot (k_fin_list's fused finish into a
// table empty before the batch: the record leaves at once); a flow that turns out complex is
// returned with FIN_COMPLEX and nothing written -- the caller claims its slot then.
constexpr uint32_t FIN_NO_SLOT = 0xFFFFFFFFu;
template <bool LDSW>
__device__ __forceinline__ FinResult finalize_slot(const BatchView& b, const Params& p, const TableView& t,
                                                   const FragView& f, uint32_t s, const HotSlot& h,
                                                   bool force_cx, uint32_t* col, RecW& er, bool fuse = false,
                                                   bool slot_clean = false, uint32_t tmax = TMAX_UNKNOWN) {
    FinResult res = {FIN_DONE, false, false, false, 0};
    const uint32_t first = first_idx(h.first_n), last = h.last1 - 1;
    const bool live = h.state & SLOT_LIVE;
    RecW rec;
    if (live) tbl_load_head(t, s, rec);
    ipxg_pkt_desc df;
    bool have_df = false;
    if (!live || tmax == TMAX_UNKNOWN) {
        df = b.desc[first];
        have_df = true;
    }
    const ipxg_pkt_desc dl = b.desc[last];
    const uint32_t cdf = p.split_biflow ? 0u : first_dir(h.first_n);
    const uint32_t I = p.inactive_s, A = p.active_s;
    uint8_t bsplit = 0;
    const uint32_t creator = (live && !p.split_biflow && rw64(rec, RW_HASH) != h.key) ? 1u : 0u;
    if (live) {
        const bool dsrc = p.split_biflow || cdf == creator;
        const uint32_t flw = dsrc ? rw_sflags(rec) : rw_dflags(rec);
        if (first_syn(h.first_n) && (flw & 0x05)) {
            bsplit = IPXG_FLOW_END_EOF;
        } else {
            if (!have_df && ((int64_t)tmax - (int64_t)rec.w[RW_TLS] >= (int64_t)I ||
                             (int64_t)tmax - (int64_t)rec.w[RW_TFS] >= (int64_t)A)) {
                df = b.desc[first];
                have_df = true;
            }
            if (have_df) {
                if ((int64_t)df.ts_sec - (int64_t)rec.w[RW_TLS] >= (int64_t)I) bsplit = export_reason_w(rec);
                else if ((int64_t)df.ts_sec - (int64_t)rec.w[RW_TFS] >= (int64_t)A) bsplit = IPXG_FLOW_END_ACTIVE;
            }
        }
    }
    const bool cont = live && !bsplit;
    if (!cont && !have_df) {  // (a SYN-after-FIN split: the new record starts at the first packet)
        df = b.desc[first];
        have_df = true;
    }
    bool cx = force_cx || (h.state & SLOT_HOST) || p.plug_all;  // a process plugin's flow: the host walks it
    const uint32_t tb = h.tbits;
    if (tb >> 31) cx = true;
    else if (tb) {
        uint32_t x = tb >> __builtin_ctz(tb);
        if (x & (x + 1)) cx = true;  // an empty bucket between two busy ones
    }
    const uint32_t tfirst = cont ? rec.w[RW_TFS] : df.ts_sec;
    if ((int64_t)dl.ts_sec - (int64_t)tfirst >= (int64_t)A) cx = true;
    for (int dd = 0; dd < 2; ++dd) {
        if (!h.syn1[dd]) continue;
        const uint32_t sidx = h.syn1[dd] - 1;
        if (cont) {
            const uint32_t cf = (uint32_t)dd == creator ? rw_sflags(rec) : rw_dflags(rec);
            if (cf & 0x05) cx = true;
        }
        if (h.fin_n[dd] && sidx > ~h.fin_n[dd]) cx = true;
    }
    if (cx) {
        if (s != FIN_NO_SLOT) {
            HotSlot c = h;
            c.state = h.state | SLOT_COMPLEX | (p.plug_all ? SLOT_PLUGIN : 0u);
            c.pad = 0;
            t.hot(s) = c;
        }
        res.status = FIN_COMPLEX;
        return res;
    }
    if (bsplit) {
        tbl_load_tail(t, s, rec);
        res.do_export = true;
        res.reason = bsplit;
        er = rec;
    }
    if (!cont) {  // a record starts at the first packet: its fields from a re-parse
        DevPkt fp;
        ipxg_pkt_desc d2;
        if (LDSW) reparse_lds<true>(b, p, f, first, col, fp, d2);
        else reparse<true>(b, p, f, first, fp, d2);
        uint64_t lo, hf;
        uint32_t c2;
        canon(fp, p, lo, c2, hf);
        rec_create_w(rec, fp, df, hf, cdf);
    }
    const uint32_t sd = cont ? creator : rw_creator(rec);
    const uint64_t as = sd ? h.acc[1] : h.acc[0], ad = sd ? h.acc[0] : h.acc[1];  // (selects: no indexed copy)
    rec.w[RW_SPK] += (uint32_t)(as >> 40);
    rw64_set(rec, RW_SBYTES, rw64(rec, RW_SBYTES) + (as & ACC_BYTES_MASK));
    rec.w[RW_DPK] += (uint32_t)(ad >> 40);
    rw64_set(rec, RW_DBYTES, rw64(rec, RW_DBYTES) + (ad & ACC_BYTES_MASK));
    rec.w[RW_FLAGS] |= ((h.tflags >> (8 * sd)) & 0xFF) | (((h.tflags >> (8 * (sd ^ 1))) & 0xFF) << 8);
    rec.w[RW_TLS] = dl.ts_sec;
    rec.w[RW_TLU] = dl.ts_usec;
    res.created = !live;
    count_flow_ports_w(t, rec, (uint32_t)(as >> 40) + (uint32_t)(ad >> 40));
    if (fuse && !res.do_export) {
        if (cont) tbl_load_tail(t, s, rec);  // (fused finishes follow an empty table: none)
        er = rec;
        res.fin_export = true;
        if (s != FIN_NO_SLOT) clear_slot(&t.hot(s), 0, 0);  // empty (every slot empties at the finish)
        return res;
    }
    if (cont) {
        tbl_store_head(t, s, rec);
        if (!(slot_clean && h.state == SLOT_LIVE)) clear_slot(&t.hot(s), h.key, SLOT_LIVE);
        return res;
    }
    tbl_store_rec(t, s, rec);
    clear_slot(&t.hot(s), h.key, SLOT_LIVE);
    return res;
}

// ---- process-plugin pre-classifier rules (ipxg_plugin: TCP/UDP ports, payload prefixes) ------
// Does the parsed packet match rule r?  pay(k): byte k of its payload (k < 16, within payload_len).
template <class B>
__device__ __forceinline__ bool rule_match(const DevRule& r, const DevPkt& pk, const B& pay) {
    const bool tcp = pk.l4 == 6, udp = pk.l4 == 17;
    if (!((tcp && (r.proto_mask & 1)) || (udp && (r.proto_mask & 2)))) return false;
    for (uint32_t k = 0; k < r.n_ports; ++k)
        if (pk.src_port == r.ports[k] || pk.dst_port == r.ports[k]) return true;
    for (uint32_t q = 0; q < r.n_prefixes; ++q) {
        const uint32_t n = r.prefix_len[q];
        if (n == 0 || n > pk.payload_len) continue;
        const bool msk = (r.masked >> q) & 1u;
        bool eq = true;
        for (uint32_t k = 0; k < n && eq; ++k)
            eq = ((pay(k) ^ r.prefix[q][k]) & (msk ? r.prefix_mask[q][k] : 0xFFu)) == 0;
        if (eq) return true;
    }
    return false;
}

}  // namespace ipxg
