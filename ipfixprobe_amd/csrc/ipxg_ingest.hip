// ipxg_ingest.hip -- the per-batch ingest of the packet -> biflow engine (the binned
// pipeline), with no per-packet device-scope atomics (those execute at the memory side on
// CDNA4, ~20 G/s chip-wide for lane-scattered addresses: MI355X_MICROARCH.md "Global float
// atomics").
//
//   k_bin     persistent workgroups over tiles of BIN_K x 256 packets (one per lane per
//             step), buffer loads software-pipelined across the tiles: parse_fast reads
//             Eth/IPv4/UDP|TCP headers from registers (parse_packet, parser.cpp:673-805, for
//             that shape), key + inverse key and 2x XXH64 (create_hash_key + XXH64,
//             cache.cpp:525-574, xxhash.h:2885-2901) give the canonical hash, and a 16-byte
//             record {canonical hash, packet index, contribution} is ranked in its partition
//             (bits 32.. of the hash) with an LDS atomic.  At the tile's end the records are
//             sorted by partition in LDS and each run is written coalesced into the
//             workgroup's own segment of the partition.  Other frame shapes go to the
//             workgroup's slow list.                                        (HBM-bound)
//   k_bin_slow  the slow lists through the general LDS-staged parser (parse_frame), ranked
//             and emitted the same way into segment columns of their own.
//   k_reduce  one 1024-thread workgroup per partition: aggregates the partition's records
//             per flow in an LDS hash table (LDS atomics), then merges each flow into its
//             slot of the device table with plain stores (the workgroup owns its keys) and,
//             when nothing else of the batch can touch the flow, lists the slot for
//             k_fin_list.
//   k_fin_list  applies the reference's split rules to the listed slots (finalize_slot), so
//             the table is not scanned per batch.
//
// Records that do not fit (segment full, LDS table full) fall back to direct atomic
// accumulation (merge_packet_atomic); the engine then runs the k_finalize scan for the
// batch (ctl->pending).  Both paths are order-independent reductions keyed by packet index,
// so the result does not depend on which lane or workgroup runs first.
#include <atomic>

#include "ipxg_table.hpp"

namespace ipxg {

#ifndef IPXG_BIN_WAVES
#define IPXG_BIN_WAVES 2  // = the LDS limit (2 workgroups of 76 KiB per CU)
#endif
#ifndef IPXG_RED_U
#define IPXG_RED_U 4
#endif
// IPXG_PROBE builds accumulate per-phase shader clocks into ctl->probe (read with
// ipxg_probe_counters): k_bin [0] tile start, [1] packet loop, [2] emit, [3] slow-list flush;
// k_reduce [4] prefix + zero, [5] aggregate, [6] merge + list; k_bin_slow [8] entry + window
// loads (issue to arrival), [9] stage + parse + rank, [10] aggregate + emit, [11] packets.
#ifdef IPXG_PROBE
#define PROBE_T(v) const uint64_t v = __builtin_readcyclecounter()
#define PROBE_ADD(k, a, b) probe_acc[k] += (b) - (a)
#else
#define PROBE_T(v)
#define PROBE_ADD(k, a, b)
#endif
constexpr int BIN_K = IPXG_BIN_K;                 // packets per lane per tile
constexpr uint32_t BIN_TILE = BIN_TILE_PKTS;       // 2048 packets
static_assert(BIN_TILE == BIN_K * IPXG_BLOCK, "k_bin tile = one packet per lane per step");
constexpr uint32_t NO_REC = 0xFFFFFFFFu;
constexpr uint32_t RED_U = IPXG_RED_U;            // records in flight per thread
#ifndef IPXG_FIN_PROBE
#define IPXG_FIN_PROBE 1  // k_fin_list probes the table for the flows k_reduce lists (see k_reduce)
#endif
constexpr uint32_t RED_MAX_PROBE = 256;
constexpr uint32_t RED_FAILED = 0x80000000u;      // FlowAgg::tflags bit: table probe failed

__device__ __forceinline__ void defer_packet(BatchCtl* ctl, uint32_t* list, uint32_t idx, bool from_bin) {
    const uint32_t pos = atomicAdd(&ctl->deferred, 1u);
    list[pos] = idx;
    if (from_bin) atomicAdd(&ctl->a_deferred, 1u);
}

// ---- per-tile flow aggregation (LDS) --------------------------------------------------------
// Skewed traffic (Zipf popularity: the top flow of the configs[2] mix carries 12 % of all
// packets) would put most of a tile's records into one partition: its segments overflow and
// the overflow lands on one table slot with device atomics, and k_reduce's workgroup for that
// partition serialises on one LDS entry.  So every tile first counts its packets per flow in an
// LDS hash (keys in the stage area, which is free until the records are staged), and a flow
// with >= TAGG_MIN packets in the tile is folded into an LDS aggregate and emitted as one
// 3-slot aggregate record (ipxg_table.hpp) in place of its packet records: in the configs[2]
// mix a tile then emits ~1200 slots instead of 2048, and the most loaded partition carries
// 2.4x the mean instead of 32x.  With uniform traffic nearly every flow has one packet per
// tile and the records are exactly the packet records as before.
constexpr uint32_t TAGG_HASH = 4096;  // tile hash entries (2 per packet of the tile)
constexpr uint32_t TAGG_CAP = 128;    // aggregates per tile (a flow past the cap stays packets)

struct TileAgg {  // 64 B, LDS
    unsigned long long key;
    unsigned long long acc[2];
    uint32_t first_n, last1, tbits, tflags;
    uint32_t syn1[2], fin_n[2];
    uint32_t part, rank;
};

// The LDS arrays of a k_bin / k_bin_slow workgroup that the tile phases share.
struct BinLds {
    uint32_t* hist;     // per partition: rank counter, then the run start in the tile
    uint32_t* fill;     // per partition: slots in the workgroup's segment so far
    uint4* stage;       // BIN_TILE slots: the tile hash's keys, then the staged records
    uint32_t* cnt;      // TAGG_HASH: packets per tile-hash entry | (aggregate + 1) << 16
    TileAgg* agg;       // TAGG_CAP
    uint16_t* part_of;  // BIN_TILE: the partition of each staged slot
    uint32_t* scan_s;
    uint32_t* nagg;
};

// ---- phase A ------------------------------------------------------------------------------
// k_bin's loads are buffer loads through two wave-uniform resource descriptors (the
// descriptor array and the frame arena; 64-bit addresses with 16-byte unit offsets): each is
// one 16-byte (or 8-byte) load instruction, where a plain load was narrowed by the compiler
// to the bytes used (4 instructions for a 48-byte head); a lane with nothing to load gives an
// offset past the buffer's end and gets zeros, with no memory traffic.  The loads are unconditional, so the number in flight is
// the same on every path and s_waitcnt waits for exactly the one it needs.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t BUF_OOB = 0xFFFFFF00u;  // an offset past every buffer (arena_lim <= BUF_OOB)

// The first NC 16-byte chunks of a frame: 3 (bytes 0..47, parse_fast's shape) or, in the wide
// walk, 5 (bytes 0..79, parse_medium's: up to QinQ + IPv6 + TCP, or IPv6 + TCP timestamps;
// ~240 VGPRs, 2 waves per SIMD).
template <int NC>
struct Head {
    uint4 c[NC];
};

__device__ __forceinline__ uint4 u4(const u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

// Cache policy of the frame and descriptor loads: non-temporal (aux bit 1, `nt`).  Every
// frame and descriptor is read exactly once, so streaming them keeps L2 and the Infinity
// Cache for the 160 MB of partition records that k_reduce reads back right after: measured
// A/B on one box, k_bin -3 % and k_reduce -12 % against default-policy loads (sc0 alone:
// no change; sc0|nt: as nt).  Not so for the frame heads of the variable-length mixes (the
// wide walk and k_bin_slow): there a head is 5-8 chunk loads into one or two lines of a large
// frame, and with `nt` the lines were fetched again between the chunks -- default-policy
// loads: k_bin's HBM fetch -23 % (imix) / -27 % (quic), imix 8.5 -> 9.3, quic 4.8 -> 5.2 Gpkt/s.
#ifndef IPXG_LOAD_AUX
#define IPXG_LOAD_AUX 2
#endif
#ifndef IPXG_WIDE_LOAD_AUX
#define IPXG_WIDE_LOAD_AUX 0
#endif
// ok: load the frame's chunks (caplen >= 48: the first 3 always; in the wide walk the later
// ones only below caplen -- a chunk past it reads as zeros with no memory traffic)
// AUX >= 0: that policy instead (line mode's k_bin)
// (rs: the arena or the wave's window of it, o: the frame's byte offset there)
template <int NC, int AUX = -1>
__device__ __forceinline__ Head<NC> load_head(__amdgpu_buffer_rsrc_t rs, uint32_t o, uint32_t caplen, bool ok) {
    o = ok ? o : BUF_OOB;
    Head<NC> h;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const uint32_t ok_k = k < 3 || (uint32_t)(16 * k) < caplen;
        h.c[k] = u4(__builtin_amdgcn_raw_buffer_load_b128(rs, ok_k ? o + 16 * k : BUF_OOB, 0,
                                                          AUX >= 0 ? AUX : NC > 3 ? IPXG_WIDE_LOAD_AUX : IPXG_LOAD_AUX));
    }
    return h;
}
// The same through the frame's 64-bit address (16-byte unit offsets); a lane with nothing to
// load reads zeros from g_zero_head (one line for the wave, no arena traffic)
__device__ uint4 g_zero_head[8];
template <int NC>
__device__ __forceinline__ Head<NC> load_head_g(const uint8_t* frame, uint32_t caplen, bool ok) {
    const uint4* f = reinterpret_cast<const uint4*>(frame);
    Head<NC> h;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const bool ok_k = ok && (k < 3 || (uint32_t)(16 * k) < caplen);
        h.c[k] = *(ok_k ? f + k : g_zero_head + k);
    }
    return h;
}
// One aligned frame's head outside a pipelined walk: buffer loads with byte offsets; with
// 16-byte units plain loads through the frame's address (the chunks below caplen)
template <int NC>
__device__ __forceinline__ Head<NC> load_head_at(const BatchView& b, __amdgpu_buffer_rsrc_t rs_all, const ipxg_pkt_desc& d) {
    if (!b.oshift) return load_head<NC>(rs_all, d.offset, d.caplen, true);
    const uint4* f = reinterpret_cast<const uint4*>(frame_ptr(b, d));
    Head<NC> h;
#pragma unroll
    for (int k = 0; k < NC; ++k) h.c[k] = (k < 3 || (uint32_t)(16 * k) < d.caplen) ? f[k] : make_uint4(0, 0, 0, 0);
    return h;
}


// The narrow walk's heads, transposed (IPXG_BIN_XPOSE): when a wave's 64 frames sit back to back
// at a 64-byte pitch (a ballot over the descriptors' offsets -- the 64 B mixes), the wave reads
// its 4 KB as four contiguous 1 KB loads (lane = 16 bytes: 8 lines per instruction instead of 32
// per strided 16-byte load) and hands each lane its frame's first 48 bytes through the wave's
// LDS (80-byte frame pitch: conflict-free 16-byte reads); otherwise the 3 strided loads.  Always
// 4 loads, branch-free addresses: the same count in flight on every path.
#ifndef IPXG_BIN_XPOSE
#define IPXG_BIN_XPOSE 0
#endif
__device__ __forceinline__ Head<4> load_head_x(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool ok, bool& seq) {
    const uint32_t lane = lane_id();
    const uint32_t o0 = __builtin_amdgcn_readfirstlane(off);
    seq = __ballot(ok && off == o0 + 64u * lane) == ~0ull;  // wave-uniform
    const uint32_t o = ok ? off : BUF_OOB;
    Head<4> h;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t a = seq ? o0 + 1024u * k + 16u * lane : (k < 3 ? o + 16u * k : BUF_OOB);
        h.c[k] = u4(__builtin_amdgcn_raw_buffer_load_b128(rs, a, 0, IPXG_LOAD_AUX));
    }
    return h;
}
// chunk (lane & 3) of frame 16k + lane / 4 (load k) -> lane f's chunks 0..2, via xs (320 uint4)
__device__ __forceinline__ void xpose_head(uint4* xs, Head<4>& h) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k) xs[(16u * k + (lane >> 2)) * 5u + (lane & 3u)] = h.c[k];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the wave's own LDS stores, in order)
#pragma unroll
    for (int k = 0; k < 3; ++k) h.c[k] = xs[lane * 5u + k];
}

// descriptor i (zeros past the batch's end)
#ifndef IPXG_DESC_AUX
#define IPXG_DESC_AUX IPXG_LOAD_AUX
#endif
template <int AUX = -1>
__device__ __forceinline__ ipxg_pkt_desc load_desc(__amdgpu_buffer_rsrc_t desc, uint32_t i) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(desc, i * 16u, 0, AUX >= 0 ? AUX : IPXG_DESC_AUX);
    ipxg_pkt_desc d;
    d.offset = v.x;
    d.caplen = (uint16_t)v.y;
    d.wirelen = (uint16_t)(v.y >> 16);
    d.ts_sec = v.z;
    d.ts_usec = v.w;
    return d;
}

// the target of stores that carry no record (tile_emit; k_bin's prologue)
__device__ uint4 g_dummy_rec[32 * 64];

// The control-block counts of k_bin / k_bin_slow, summed per workgroup in LDS (bc: BLK_N words,
// zeroed) and added to the control block by one lane: every lane with a time bucket other than 0
// once did its own atomicOr on ctl->tb_any -- ~200k atomics on one address per configs[4] launch,
// half of k_bin_slow's time.
enum BlkCount { BLK_SPILLED, BLK_FOLDED, BLK_WALKED, BLK_TB, BLK_N };
__device__ __forceinline__ void block_ctl_counts(uint32_t* bc, uint32_t spilled, uint32_t folded, uint32_t walked,
                                                 uint32_t tb_or) {
    if (spilled) atomicAdd(&bc[BLK_SPILLED], spilled);
    if (folded) atomicAdd(&bc[BLK_FOLDED], folded);
    if (walked) atomicAdd(&bc[BLK_WALKED], walked);
    if (tb_or) atomicOr(&bc[BLK_TB], tb_or);
}
// after a barrier
__device__ __forceinline__ void flush_block_ctl(const uint32_t* bc, BatchCtl* ctl) {
    if (threadIdx.x != 0) return;
    if (bc[BLK_SPILLED]) {
        atomicAdd(&ctl->spilled, bc[BLK_SPILLED]);
        ctl->pending = 1;
    }
    if (bc[BLK_FOLDED]) atomicAdd(&ctl->agg_packets, bc[BLK_FOLDED]);
    if (bc[BLK_WALKED]) atomicAdd(&ctl->walked, bc[BLK_WALKED]);
    // no atomic while one bucket holds the batch, nor once the bits are set (a stale read: one more)
    const uint32_t tb = bc[BLK_TB];
    if (tb && (*(volatile uint32_t*)&ctl->tb_any & tb) != tb) atomicOr(&ctl->tb_any, tb);
}

// one device atomic per wave for a per-lane count (convergent: every lane calls it)
__device__ __forceinline__ void add_wave_sum(uint32_t* counter, uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane_id() == 0 && v) atomicAdd(counter, v);
}

// Without tile aggregation: rank every packet record in its partition.
template <int K>
__device__ __forceinline__ void tile_rank_all(uint32_t* hist, uint32_t pmask, const uint32_t (&r1)[K], uint32_t (&rk)[K]) {
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (rk[q] != NO_REC) rk[q] = atomicAdd(&hist[r1[q] & pmask], 1u);
}

// After tile_aggregate ranked the tile's packet records and aggregates in hist[part]: each
// partition's slots of the tile follow the ones of the block's earlier tiles in the block's own
// segment of that partition (fill[part] = slots so far), so no workgroup shares a write
// position with another and no device atomic is needed (a shared counter per partition, hit
// once per tile by every workgroup, saturated at the memory-side atomic rate).  The slots are
// first grouped by partition in LDS (stage) and then written with consecutive lanes on
// consecutive slots of a run: written straight from the lanes, 64 lanes stored to 64 different
// lines per instruction and the stores cost a third of k_bin's time.
// A full segment spills to direct accumulation (an aggregate spills whole: its slots that
// would fit become NO_REC fillers, so k_reduce never reads half an aggregate).
// LISTED: packet indices come from ix[] (k_bin_slow); else record q of the lane is packet
// tile + q * 256 + lane (k_bin).
// defer_spill (Params::defer_spill: this batch's k_bin runs while the previous batch's host walk
// still owns the table): what does not fit is deferred (the deferral lists, applied after k_reduce)
// instead of accumulated into the table.
// ---- write-through record stores; the streamed reduce's progress words ----------------------------
// The record area as a buffer resource (BinView::prog_mode & PROG_SC1: the host set it only for an
// area under 4 GiB): sc1 stores, whose lines pass the writer's L2 straight on to the Infinity Cache.
// Round 6: k_bin's records as write-through stores (the default) -- udp64 k_bin 214 -> 208 us, step
// 0.305 -> 0.300 ms, alternating on one box (profiles/r06/sc1_ab.txt): the records leave no dirty
// lines in L2 for the frames to evict and for the kernel's end to write back.  The streamed reduce
// (k_reduce_stream on another XCD) reads them with sc1 loads (MI355X_MICROARCH.md, hand-off table:
// sc1 stores, the writers' vmcnt(0), then an sc1 flag; sc1 polls and sc1 loads).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(const BinView& bv) {
    const uint64_t bytes = ((uint64_t)bv.cols << bv.part_bits) * bv.seg_cap * 16u;
    return __builtin_amdgcn_make_buffer_rsrc(bv.rec, 0, (int)(uint32_t)min<uint64_t>(bytes, BUF_OOB), 0x00020000);
}
constexpr int AUX_SC1 = 16;  // buffer-op cache policy: sc1
__device__ __forceinline__ void store_rec_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off, const uint4& r) {
    u32x4 v = {r.x, r.y, r.z, r.w};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX_SC1);
}
// partition q's progress word of column col: the whole lines stored (records fill, at most the
// segment's), the batch's tag, done
__device__ __forceinline__ void publish_prog(const BinView& bv, uint32_t col, uint32_t q, uint32_t fill, uint32_t done) {
    const uint32_t lines = min(fill, bv.seg_cap) >> 3;
    __hip_atomic_store(&bv.prog[(size_t)q * RS_MAX_COLS + col], bv.prog_tag | done | lines, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

template <bool LISTED, bool AGG, uint32_t PMAX = (1u << BIN_MAX_PART_BITS)>
__device__ __forceinline__ void tile_emit(const BinLds& L, uint32_t P, uint32_t pmask, const BinView& bv, uint32_t col,
                                          const TableView& t, BatchCtl* ctl, uint32_t* deferred_list,
                                          uint4* agg_list, const uint32_t (&r0)[BIN_K], const uint32_t (&r1)[BIN_K],
                                          const uint32_t (&r2)[BIN_K], const uint32_t (&rk)[BIN_K],
                                          const uint32_t (&ix)[BIN_K], uint32_t tile, uint32_t& spilled,
                                          bool defer_spill) {
    constexpr uint32_t PT = PMAX > IPXG_BLOCK ? PMAX / IPXG_BLOCK : 1;  // partitions per thread
    uint32_t* const hist = L.hist;
    uint32_t* const fill = L.fill;
    uint4* const stage = L.stage;
    __syncthreads();
    // tile-local exclusive prefix over the partitions: hist[q] <- start of q's run in stage
    const uint32_t q0 = threadIdx.x * PT;
    uint32_t cnt[PT], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
        cnt[k] = q0 + k < P ? hist[q0 + k] : 0;
        sum += cnt[k];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan<IPXG_BLOCK>(sum, L.scan_s, &total);
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
        if (q0 + k < P) hist[q0 + k] = run;
        run += cnt[k];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BIN_K; ++q) {
        if (rk[q] == NO_REC) continue;
        const uint32_t idx = LISTED ? ix[q] : tile + (uint32_t)q * IPXG_BLOCK + threadIdx.x;
        const uint32_t part = r1[q] & pmask;
        const uint32_t k = hist[part] + rk[q];
        stage[k] = make_uint4(r0[q], r1[q], idx, r2[q]);
        if (AGG) L.part_of[k] = (uint16_t)part;
    }
    const uint32_t na = AGG ? min(*L.nagg, TAGG_CAP) : 0;
    for (uint32_t a = threadIdx.x; a < na; a += IPXG_BLOCK) {
        const TileAgg& g = L.agg[a];
        FlowAgg f;
        f.key = g.key;
        f.acc[0] = g.acc[0];
        f.acc[1] = g.acc[1];
        f.first_n = g.first_n;
        f.last1 = g.last1;
        f.tbits = g.tbits;
        f.tflags = g.tflags;
        f.syn1[0] = g.syn1[0];
        f.syn1[1] = g.syn1[1];
        f.fin_n[0] = g.fin_n[0];
        f.fin_n[1] = g.fin_n[1];
        const uint32_t k = hist[g.part] + g.rank;
        agg_encode(f, stage[k], stage[k + 1], stage[k + 2]);
        L.part_of[k] = L.part_of[k + 1] = L.part_of[k + 2] = (uint16_t)g.part;
    }
    __syncthreads();
    // Fixed trip count and one store per iteration, always issued (a slot that does not go to
    // a segment is stored to a dummy line instead): on gfx950 stores count in vmcnt, and with a
    // variable number of them the compiler's waits for the next tile's prefetched loads had to
    // assume none were issued -- every later wait then also waited for the stores.  (A loop
    // here made it drain every load in flight before it.)
#pragma unroll
    for (uint32_t kk = 0; kk < BIN_TILE / IPXG_BLOCK; ++kk) {
        const uint32_t k = kk * IPXG_BLOCK + threadIdx.x;
        const bool valid = k < total;
        uint4 r = stage[valid ? k : 0];
        const uint32_t part = AGG ? L.part_of[valid ? k : 0] : (r.y & pmask);
        const uint32_t pos = fill[part] + (k - hist[part]);
        const bool agg = AGG && rec_is_agg(r);
        const uint32_t ai = agg ? rec_agg_slot(r) : 0;
        const bool fits = valid && (pos - ai + (agg ? 3 : 1) <= bv.seg_cap);
        const bool filler = valid && !fits && pos < bv.seg_cap;  // part of an aggregate that spills
        if (filler) r = make_uint4(0, 0, NO_REC, 0);
#ifdef IPXG_EXP_NOEMIT  // timing experiment: records dropped
        uint4* dst = &g_dummy_rec[threadIdx.x & 63];
#else
        uint4* dst = (fits || filler) ? &bv.rec[((size_t)part * bv.cols + col) * bv.seg_cap + pos]
                                      : &g_dummy_rec[threadIdx.x & 63];
#endif
        if (bv.prog_mode & PROG_SC1) {  // (uniform) write-through (rec_rsrc)
            store_rec_sc1(rec_rsrc(bv), (fits || filler) ? (uint32_t)(((size_t)part * bv.cols + col) * bv.seg_cap + pos) * 16u
                                                         : BUF_OOB, r);
        } else {
#ifdef IPXG_NT_REC_STORE  // tuning knob: streaming (non-temporal) record stores
        __builtin_nontemporal_store(r.x, &dst->x);
        __builtin_nontemporal_store(r.y, &dst->y);
        __builtin_nontemporal_store(r.z, &dst->z);
        __builtin_nontemporal_store(r.w, &dst->w);
#else
        *dst = r;
#endif
        }
        if (valid && !fits && ai == 0) {  // segment full: accumulate straight into the table
            spilled++;
            if (defer_spill) atomicAdd(&ctl->spill_deferred, 1u);
            if (!agg) {
                if (defer_spill || !merge_packet_atomic(t, ((uint64_t)r.y << 32) | r.x, r.z, r.w, &ctl->new_keys))
                    defer_packet(ctl, deferred_list, r.z, true);
            } else {
                const uint4 s0 = stage[k], s1 = stage[k + 1], s2 = stage[k + 2];
                if (defer_spill || !merge_agg_probe(t, agg_decode(s0, s1, s2), &ctl->new_keys)) {
                    defer_agg(&ctl->agg_deferred, agg_list, s0, s1, s2);
                    atomicAdd(&ctl->a_deferred, 1u);
                }
            }
        }
    }
    __syncthreads();  // hist is reset by the next tile
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k)
        if (q0 + k < P) fill[q0 + k] += cnt[k];
}

// the block's record counts per partition (its column of bv.count)
__device__ __forceinline__ void seg_counts(const uint32_t* fill, uint32_t P, const BinView& bv, uint32_t col) {
#ifdef IPXG_EXP_NOEMIT
    for (uint32_t q = threadIdx.x; q < P; q += IPXG_BLOCK) bv.count[seg_count_idx(bv, q, col)] = 0;
#else
    for (uint32_t q = threadIdx.x; q < P; q += IPXG_BLOCK) bv.count[seg_count_idx(bv, q, col)] = min(fill[q], bv.seg_cap);
#endif
}

// ---- line mode: whole-line record stores -------------------------------------------------
// A tile's run of one partition is a few records (udp64: 2048 packets over 256 partitions, 8 on
// average) at whatever offset the partition's segment has reached, so tile_emit writes most
// 128-byte lines in two or three pieces, tiles apart.  With the frames streaming through L2 the
// partial lines are written back partially, and a partial line costs the memory a
// read-modify-write: tools/membench's k_bin load pattern plus k_bin's 160 MB of records takes
// 195 us with whole-line stores and 264 us with the same runs shifted off the line boundaries
// (default-policy frame loads; with `nt` loads 250 / 263 us).  Line mode (the non-aggregating
// k_bin with at most LINE_P partitions) keeps each partition's last partial line in LDS (the
// carry) and stores only whole lines: a tile completes the lines its records and the carry fill,
// the rest stays for the next tile, and the last tile pads each carry to a whole line with
// NO_REC fillers (k_reduce skips them).  The carry's 28 KiB is paid for with 1024-packet tiles
// (LINE_K steps): the workgroup stays within the LDS of 3 per CU.
constexpr uint32_t LINE_P = BIN_LINE_P;  // partitions (at most)
#ifndef IPXG_LINE_K
#define IPXG_LINE_K 4
#endif
constexpr int LINE_K = IPXG_LINE_K;   // packets per lane per tile
constexpr uint32_t LINE_C = 7;        // carried records per partition (less than a line)
constexpr uint32_t LINE_MAXL = (LINE_K * IPXG_BLOCK + LINE_C * LINE_P) / 8;  // lines one tile completes, at most
constexpr uint32_t LINE_ITERS = (LINE_MAXL * 8 + IPXG_BLOCK - 1) / IPXG_BLOCK;   // store rounds per tile
#ifndef IPXG_LINE_AUX
#define IPXG_LINE_AUX 0  // cache policy of line mode's frame and descriptor loads (membench: default policy)
#endif

struct LineLds {
    uint32_t* hist;   // LINE_P: the tile's records per partition (rank counters)
    uint32_t* fill;   // LINE_P: records stored in the workgroup's segment (a multiple of 8)
    uint32_t* pos;    // LINE_P: the partition's run in stage | its first completed line << 16
    uint8_t* ccnt;    // LINE_P: carried records
    uint8_t* lpart;   // LINE_MAXL: the partition of each line the tile completes
    uint4* stage;     // LINE_K * 256: the tile's records, then grouped by partition
    uint4* carry;     // LINE_P * LINE_C
    uint32_t* scan_s;
};

// a record that found its segment full: accumulated into the table (or deferred), as tile_emit
__device__ __forceinline__ void line_spill(const TableView& t, BatchCtl* ctl, uint32_t* deferred_list, const uint4& r,
                                           uint32_t& spilled, bool defer_spill) {
    spilled++;
    if (defer_spill) atomicAdd(&ctl->spill_deferred, 1u);
    if (defer_spill || !merge_packet_atomic(t, ((uint64_t)r.y << 32) | r.x, r.z, r.w, &ctl->new_keys))
        defer_packet(ctl, deferred_list, r.z, true);
}

// After tile_rank_all (rk[q] = the record's rank in its partition, hist[] = the counts): the
// tile's records grouped by partition in stage, then every line that the carry and the tile's run
// complete stored whole (8 consecutive lanes per line, a wave stores 8 lines), then the rest
// carried.  Fixed store rounds (LINE_ITERS; a round past the tile's lines stores to a dummy line)
// for the reason tile_emit gives.
template <int K>
__device__ __forceinline__ void tile_emit_lines(const LineLds& L, uint32_t P, uint32_t pmask, const BinView& bv,
                                                uint32_t col, const TableView& t, BatchCtl* ctl,
                                                uint32_t* deferred_list, const uint32_t (&r0)[K],
                                                const uint32_t (&r1)[K], const uint32_t (&r2)[K],
                                                const uint32_t (&rk)[K], uint32_t tile, uint32_t& spilled,
                                                bool defer_spill, bool pub) {
    const uint32_t tid = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs_rec = rec_rsrc(bv);  // (streamed reduce: write-through record stores)
    __syncthreads();  // the counts are complete; every lane has its records back from stage
    uint32_t n = 0, cc = 0, W = 0;
    if (tid < P) {
        n = L.hist[tid];
        cc = L.ccnt[tid];
        W = (cc + n) & ~7u;  // records of the lines this tile completes
    }
    uint32_t tot;  // (run starts in the high half, first lines in the low: no carry across, 1024 + 352)
    const uint32_t sc = block_exclusive_scan<IPXG_BLOCK>((n << 16) | (W >> 3), L.scan_s, &tot);
    const uint32_t nrec = (tot & 0xFFFFu) * 8;
    if (tid < P) {
        L.pos[tid] = (sc >> 16) | ((sc & 0xFFFFu) << 16);
        for (uint32_t l = 0; l < (W >> 3); ++l) L.lpart[(sc & 0xFFFFu) + l] = (uint8_t)tid;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (rk[q] != NO_REC)
            L.stage[(L.pos[r1[q] & pmask] & 0xFFFFu) + rk[q]] =
                make_uint4(r0[q], r1[q], tile + (uint32_t)q * IPXG_BLOCK + tid, r2[q]);
    __syncthreads();
#pragma unroll
    for (uint32_t it = 0; it < LINE_ITERS; ++it) {
        const uint32_t k = it * IPXG_BLOCK + tid;
        const bool valid = k < nrec;
        const uint32_t part = valid ? L.lpart[k >> 3] : 0u;
        const uint32_t ps = L.pos[part], c = L.ccnt[part];
        const uint32_t j = valid ? ((k >> 3) - (ps >> 16)) * 8 + (k & 7) : 0u;  // record j of the partition's lines
        const uint4 r = j < c ? L.carry[part * LINE_C + j] : L.stage[(ps & 0xFFFFu) + j - c];
        const uint32_t at = L.fill[part] + j;
        const bool fits = valid && at < bv.seg_cap;  // (seg_cap and fill are multiples of 8: whole lines)
        uint4* dst = fits ? &bv.rec[((size_t)part * bv.cols + col) * bv.seg_cap + at] : &g_dummy_rec[tid & 63];
        if (bv.prog_mode & PROG_SC1) {  // (uniform) write-through: see rec_rsrc
            store_rec_sc1(rs_rec, fits ? (uint32_t)(((size_t)part * bv.cols + col) * bv.seg_cap + at) * 16u : BUF_OOB, r);
        } else {
#ifdef IPXG_NT_REC_STORE  // tuning knob: streaming (non-temporal) record stores
        __builtin_nontemporal_store(r.x, &dst->x);
        __builtin_nontemporal_store(r.y, &dst->y);
        __builtin_nontemporal_store(r.z, &dst->z);
        __builtin_nontemporal_store(r.w, &dst->w);
#else
        *dst = r;
#endif
        }
        if (valid && !fits) line_spill(t, ctl, deferred_list, r, spilled, defer_spill);
    }
    __syncthreads();  // the carry and the stage have been read
    if (tid < P) {
        const uint32_t st = L.pos[tid] & 0xFFFFu;
        if (W == 0) {
            for (uint32_t m = 0; m < n; ++m) L.carry[tid * LINE_C + cc + m] = L.stage[st + m];
            L.ccnt[tid] = (uint8_t)(cc + n);
        } else {
            const uint32_t nc = cc + n - W;
            for (uint32_t m = 0; m < nc; ++m) L.carry[tid * LINE_C + m] = L.stage[st + (W - cc) + m];
            L.ccnt[tid] = (uint8_t)nc;
            L.fill[tid] += W;
        }
    }
    // streamed reduce: every wave's record stores of the tile complete (write-through), then the
    // whole lines of each partition's segment published (one word per partition and column)
    if (pub) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (hist is reset by the next tile, whose packet loop rewrites the stage)
    if (pub && tid < P) publish_prog(bv, col, tid, L.fill[tid], 0u);
}

// The workgroup's carries after its last tile: one line per partition, padded with NO_REC.
__device__ __forceinline__ void line_flush(const LineLds& L, uint32_t P, const BinView& bv, uint32_t col,
                                           const TableView& t, BatchCtl* ctl, uint32_t* deferred_list,
                                           uint32_t& spilled, bool defer_spill) {
    for (uint32_t k = threadIdx.x; k < P * 8; k += IPXG_BLOCK) {
        const uint32_t part = k >> 3, j = k & 7, c = L.ccnt[part];
        if (c == 0) continue;
        const uint32_t at = L.fill[part] + j;
        const uint4 r = j < c ? L.carry[part * LINE_C + j] : make_uint4(0, 0, NO_REC, 0);
        const size_t k_at = ((size_t)part * bv.cols + col) * bv.seg_cap + at;
        if (at < bv.seg_cap) {
            if (bv.prog_mode & PROG_SC1) store_rec_sc1(rec_rsrc(bv), (uint32_t)k_at * 16u, r);
            else bv.rec[k_at] = r;
        } else if (j < c) {
            line_spill(t, ctl, deferred_list, r, spilled, defer_spill);
        }
    }
    __syncthreads();
    if (threadIdx.x < P && L.ccnt[threadIdx.x]) L.fill[threadIdx.x] += 8;
    __syncthreads();
}

// keep one keyed, unfragmented packet's record in slot j (ranked in tile_aggregate)
template <bool LISTED>
__device__ __forceinline__ void tile_rank(const Params& p, const BatchView& b, const DevPkt& pk,
                                          const ipxg_pkt_desc& d, uint32_t i, int j, uint32_t (&r0)[BIN_K],
                                          uint32_t (&r1)[BIN_K], uint32_t (&r2)[BIN_K], uint32_t (&rk)[BIN_K],
                                          uint32_t (&ix)[BIN_K], uint32_t& tb_or) {
    uint64_t lo, hf;
    uint32_t cdir;
#ifdef IPXG_EXP_NOHASH  // timing experiment only: one cheap mixer instead of 2x XXH64
    lo = (((uint64_t)(pk.sip[0] ^ pk.dip[0]) << 32) | (uint32_t)(pk.src_port ^ pk.dst_port)) * 0x9E3779B97F4A7C15ull;
    lo ^= lo >> 29;
    cdir = 0;
    hf = lo;
#else
    canon<false>(pk, p, lo, cdir, hf);
#endif
    const uint32_t m = pack_misc(pk, cdir, time_bucket(d.ts_sec, b.base_sec, p.bucket_w));
    tb_or |= misc_tb(m);
#pragma unroll
    for (int q = 0; q < BIN_K; ++q) {  // registers indexed by compile-time q only
        if (q == j) {
            r0[q] = (uint32_t)lo;
            r1[q] = (uint32_t)(lo >> 32);
            r2[q] = m;
            rk[q] = 0;
            if (LISTED) ix[q] = i;
        }
    }
}

// The same record as one 16-byte word {hash lo, hash hi, 0, misc} (k_bin without tile aggregation
// stages it in LDS during the packet loop: the tile's records then hold no registers there)
__device__ __forceinline__ uint4 make_record(const Params& p, const BatchView& b, const DevPkt& pk,
                                             const ipxg_pkt_desc& d, uint32_t& tb_or) {
    uint64_t lo, hf;
    uint32_t cdir;
#ifdef IPXG_EXP_NOHASH  // timing experiment only: one cheap mixer instead of XXH64
    lo = (((uint64_t)(pk.sip[0] ^ pk.dip[0]) << 32) | (uint32_t)(pk.src_port ^ pk.dst_port)) * 0x9E3779B97F4A7C15ull;
    lo ^= lo >> 29;
    cdir = 0;
    hf = lo;
#else
    canon<false>(pk, p, lo, cdir, hf);
#endif
    const uint32_t m = pack_misc(pk, cdir, time_bucket(d.ts_sec, b.base_sec, p.bucket_w));
    tb_or |= misc_tb(m);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), 0u, m);
}

// After the tile's packet loop (rk[q] != NO_REC: record q of this lane holds a packet):
// count the packets per flow in the LDS hash, fold the flows with >= TAGG_MIN packets into
// LDS aggregates, and rank the remaining packet records (rk[q] <- rank in its partition) and
// the aggregates (3 slots each) in the tile's partition histogram.
template <bool LISTED>
__device__ __forceinline__ void tile_aggregate(const BinLds& L, uint32_t pmask, uint32_t (&r0)[BIN_K],
                                               uint32_t (&r1)[BIN_K], uint32_t (&r2)[BIN_K], uint32_t (&rk)[BIN_K],
                                               const uint32_t (&ix)[BIN_K], uint32_t tile, uint32_t& folded) {
    const uint32_t tid = threadIdx.x;
    unsigned long long* hk = reinterpret_cast<unsigned long long*>(L.stage);
    static_assert(TAGG_HASH * 8 <= BIN_TILE * 16, "tile hash keys live in the stage area");
    __syncthreads();  // the stage area is free (the previous tile's emit, k_bin_slow's headers)
    for (uint32_t k = tid; k < TAGG_HASH; k += IPXG_BLOCK) {
        hk[k] = 0ull;
        L.cnt[k] = 0;
    }
    if (tid == 0) *L.nagg = 0;
    __syncthreads();
    uint32_t ent[BIN_K], lead = 0;
#pragma unroll
    for (int q = 0; q < BIN_K; ++q) {
        ent[q] = 0;
        if (rk[q] == NO_REC) continue;
        const unsigned long long lo = ((unsigned long long)r1[q] << 32) | r0[q];
        uint32_t e = r0[q] & (TAGG_HASH - 1);
        while (true) {  // <= 2048 keys in 4096 entries: terminates
            unsigned long long k = hk[e];
            if (k == 0ull) {
                k = atomicCAS(&hk[e], 0ull, lo);
                if (k == 0ull) break;
            }
            if (k == lo) break;
            e = (e + 1) & (TAGG_HASH - 1);
        }
        ent[q] = e;
        if (atomicAdd(&L.cnt[e], 1u) == 0) lead |= 1u << q;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BIN_K; ++q) {  // one leader per flow: an aggregate for a frequent flow
        if (!((lead >> q) & 1) || L.cnt[ent[q]] < TAGG_MIN) continue;
        const uint32_t a = atomicAdd(L.nagg, 1u);
        if (a >= TAGG_CAP) continue;
        TileAgg& g = L.agg[a];
        g.key = ((unsigned long long)r1[q] << 32) | r0[q];
        g.acc[0] = g.acc[1] = 0ull;
        g.first_n = g.last1 = g.tbits = g.tflags = 0;
        g.syn1[0] = g.syn1[1] = g.fin_n[0] = g.fin_n[1] = 0;
        g.part = r1[q] & pmask;
        L.cnt[ent[q]] |= (a + 1) << 16;  // only the leader writes its entry in this phase
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BIN_K; ++q) {
        if (rk[q] == NO_REC) continue;
        const uint32_t v = L.cnt[ent[q]];
        if (v >> 16) {  // fold into the flow's aggregate (lds_fold's reductions)
            TileAgg& g = L.agg[(v >> 16) - 1];
            const uint32_t idx = LISTED ? ix[q] : tile + (uint32_t)q * IPXG_BLOCK + tid, m = r2[q];
            const uint32_t cdir = misc_dir(m);
            atomicAdd(&g.acc[cdir], (1ull << 40) | (unsigned long long)misc_len(m));
            atomicMax(&g.last1, idx + 1);
            atomicMax(&g.first_n, first_key(idx, m));
            atomicOr(&g.tbits, 1u << misc_tb(m));
            const uint32_t fl = misc_flags(m);
            if (misc_tcp(m) && fl) {
                atomicOr(&g.tflags, fl << (8 * cdir));
                if (fl & 0x02) atomicMax(&g.syn1[cdir], idx + 1);
                if (fl & 0x05) atomicMax(&g.fin_n[cdir], ~idx);
            }
            rk[q] = NO_REC;
            folded++;
        } else {
            rk[q] = atomicAdd(&L.hist[r1[q] & pmask], 1u);
        }
    }
    __syncthreads();
    const uint32_t na = min(*L.nagg, TAGG_CAP);
    for (uint32_t a = tid; a < na; a += IPXG_BLOCK) L.agg[a].rank = atomicAdd(&L.hist[L.agg[a].part], 3u);
}

// ---- shape classes of the slow list ------------------------------------------------------
// k_bin_slow's general parser is a state machine (Ethernet -> VLAN -> MPLS / PPPoE / IPv4 ->
// GRE -> ... -> L4): a wave whose lanes walk different header chains executes every state's
// code on every step.  So k_bin tags each slow entry with the shape class of its first 48 bytes
// (a guess from fixed offsets -- it only orders the work, the parser decides everything) and
// k_bin_slow parses each tile's packets grouped by class.
constexpr uint32_t SLOW_NCLS = 16;
constexpr uint32_t SLOW_IDX_MASK = 0xFFFFFFu;  // entry.x: packet index (< 2^24) | class << 24
__device__ __forceinline__ uint32_t be16_lo(uint32_t w) { return ((w & 0xFF) << 8) | ((w >> 8) & 0xFF); }
__device__ __forceinline__ uint32_t slow_class(const uint4 c0, const uint4 c1, const uint4 c2) {
    const uint32_t et0 = be16_lo(c0.w);                        // bytes 12-13
    const bool t1 = et0 == 0x8100 || et0 == 0x88A8;
    const uint32_t et1 = be16_lo(c1.x);                        // bytes 16-17
    const bool t2 = t1 && (et1 == 0x8100 || et1 == 0x88A8);
    const uint32_t et = t2 ? be16_lo(c1.y) : (t1 ? et1 : et0);  // bytes 20-21
    // the L3 header at 14, 18 or 22: IPv4 protocol (+9), IPv6 next header (+6)
    const uint32_t v4p = t2 ? (c1.w >> 24) : (t1 ? (c1.z >> 24) : (c1.y >> 24));
    const uint32_t v6n = t2 ? (c1.w & 0xFF) : (t1 ? (c1.z & 0xFF) : (c1.y & 0xFF));
    uint32_t cls = 15;  // other link layers / ethertypes
    if (et == 0x0800) cls = v4p == 47 ? 1 : (v4p == 6 ? 2 : 0);
    else if (et == 0x86DD) cls = (v6n == 6 || v6n == 17) ? 3 : (v6n == 44 ? 4 : 5);
    else if (et == 0x8847 || et == 0x8848) {  // labels from byte 14 (untagged): bottom-of-stack bits
        const uint32_t n = (c1.x & 1) ? 1 : ((c1.y & 1) ? 2 : 3);  // S bit: byte 2 of a label
        cls = 5 + n;
    } else if (et == 0x8864) cls = 9;
    else if (et == 0x22F3) cls = 10;  // TRILL
    return cls;
}

// The plugins' rules (Params::plug, flattened) on a packet the wide walk parsed from registers:
// MARK_HIT when a port or payload-prefix rule matches (k_classify's rule_match), MARK_LATER when a
// prefix rule could only be decided past the register window (k_plugin_marks tests the frame),
// else 0.  The payload's first 4 bytes come from the window; bytes at or past caplen read as 0.
template <int WD>
__device__ __forceinline__ uint32_t plug_check(const Params& p, const uint32_t (&w)[WD], uint32_t caplen,
                                               const DevPkt& pk) {
    const uint32_t pm = pk.l4 == 6 ? 1u : 2u;  // (pk.l4 is TCP or UDP here)
    for (uint32_t k = 0; k < p.plug_nport; ++k) {
        const uint32_t e = p.plug_tab[PLUG_PORT + k];
        if (((e >> 16) & pm) && (pk.src_port == (e & 0xFFFF) || pk.dst_port == (e & 0xFFFF))) return MARK_HIT;
    }
    if (!p.plug_npref) return 0;
    const uint32_t off = pk.payload_off;
    const bool inwin = off + PLUG_PREFIX <= 4u * WD;
    uint32_t pay = 0;
    if (inwin) {
        const uint32_t q = off >> 2;
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int k = 0; k < WD; ++k) {  // (selects: no dynamic register index)
            a = (uint32_t)k == q ? w[k] : a;
            b = (uint32_t)k == q + 1 ? w[k] : b;
        }
        pay = __builtin_amdgcn_alignbyte(b, a, off & 3);
        const int valid = (int)caplen - (int)off;
        pay &= valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
    }
    uint32_t res = 0;
    for (uint32_t k = 0; k < p.plug_npref; ++k) {
        const uint32_t info = p.plug_tab[PLUG_PINFO + k], n = info & 0xFF;
        if (!((info >> 8) & pm) || n == 0 || n > pk.payload_len) continue;
        if (!inwin) {
            res = MARK_LATER;
            continue;
        }
        if (((pay ^ p.plug_tab[PLUG_PREF + k]) & p.plug_tab[PLUG_PMASK + k]) == 0) return MARK_HIT;
    }
    return res;
}

// Every packet of the batch, in tiles of BIN_K x 256, parsed in registers by parse_fast
// from buffer loads software-pipelined across the tiles (below).  Frames the register parser
// does not take go to the slow list for k_bin_slow.  No LDS header staging here: LDS holds
// the partition histogram, the block's segment fill counts, the tile's record stage and its
// slow list.
// AGG: with the per-tile flow aggregation (76 KiB of LDS, 2 workgroups per CU); without it
// 51 KiB (3 per CU).
// WIDE (the wide walk, for mixes of variable-length header chains): 80 bytes of each frame are
// loaded (5 chunks, same pipeline) and parse_medium takes VLAN/QinQ, IPv6 and TCP-timestamp
// frames from registers as well; the remaining shapes (MPLS, PPPoE, GRE, IPv6 extension
// headers, other TCP options, ...) still go to the slow list.
// The host picks the variants per batch (ipxg_engine.cpp: tile_agg, wide).
constexpr uint32_t KBIN_PMAX = 1u << IPXG_KBIN_PMAX_BITS;  // (the host picks at most IPXG_KBIN_PMAX_BITS)
#ifndef IPXG_BIN_NARROW_WPE
#define IPXG_BIN_NARROW_WPE 3  // waves per SIMD of the narrow, non-aggregating k_bin (its register budget)
#endif
// PLUG (with WIDE only): the process plugins' pre-classification in the same walk (Params::plug;
// the hits' keys and the undecided packets listed for k_plugin_marks) -- no k_classify pass.
// LINE (without AGG and PLUG): line mode (tile_emit_lines), 1024-packet tiles.
// G64 (the batch's offsets count 16-byte units, BatchView::oshift): heads through 64-bit addresses.
template <bool AGG, bool WIDE, bool PLUG = false, bool LINE = false, bool G64 = false>
__global__ __launch_bounds__(IPXG_BLOCK) __attribute__((amdgpu_waves_per_eu(AGG || WIDE ? 2 : IPXG_BIN_NARROW_WPE)))
void k_bin(BatchView b, Params p, TableView t, FragView f, BinView bv, BatchCtl* ctl, uint4* slow_list,
           uint32_t* deferred_list, uint4* agg_list, unsigned long long* stats) {
    static_assert(!PLUG || WIDE, "the plugin check reads the wide walk's window");
    static_assert(!LINE || (!AGG && !PLUG), "line mode: the plain record walk");
    static_assert(!LINE || !G64, "line mode: byte offsets");
    constexpr int K = LINE ? LINE_K : BIN_K;  // packets per lane per tile
    constexpr uint32_t TILE = (uint32_t)K * IPXG_BLOCK;
    constexpr uint32_t PM = LINE ? LINE_P : KBIN_PMAX;  // partitions (at most)
    constexpr int LAUX = LINE ? IPXG_LINE_AUX : -1;     // load policy (-1: the walk's default)
    if (p.pub_seq && blockIdx.x == 0) {  // the pending batch's control block to the host (k_publish's layout)
        const uint32_t* src = reinterpret_cast<const uint32_t*>(p.prev_ctl);
        for (uint32_t w = threadIdx.x; w < p.pub_words; w += IPXG_BLOCK) p.pub_dst[w] = src[w];
        if (threadIdx.x < 4) p.pub_dst[p.pub_words + threadIdx.x] = p.pub_ex[threadIdx.x];
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(&p.pub_dst[p.pub_words + 4], p.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (gated(p)) return;  // launched ahead of the host's reading of the previous batch, which needs it
    __shared__ uint32_t hist[PM];  // 8 KiB: per-partition rank / run start
    __shared__ uint32_t fill[PM];  // 8 KiB: slots in the block's segments
    __shared__ uint4 stage[TILE];                       // 32 KiB: tile hash keys, then the slots by partition
    __shared__ uint32_t lpos[LINE ? LINE_P : 1];        // line mode (LineLds)
    __shared__ uint8_t lccnt[LINE ? LINE_P : 1];
    __shared__ uint8_t llpart[LINE ? LINE_MAXL : 1];
    __shared__ uint4 lcarry[LINE ? LINE_P * LINE_C : 1];  // 28 KiB
    __shared__ uint32_t tcnt[AGG ? TAGG_HASH : 1];      // 16 KiB: tile hash counts / aggregate ids
    __shared__ TileAgg tagg[AGG ? TAGG_CAP : 1];        // 8 KiB
    __shared__ uint16_t part_of[AGG ? BIN_TILE : 1];    // 4 KiB
    __shared__ uint32_t scan_s[IPXG_BLOCK / 64 + 1];
    __shared__ uint32_t nagg;
    const BinLds L = {hist, fill, stage, tcnt, tagg, part_of, scan_s, &nagg};
    const LineLds LL = {hist, fill, lpos, lccnt, llpart, stage, lcarry, scan_s};
    uint32_t folded = 0;
    __shared__ uint32_t nslow[2];  // slow packets of the tile (by tile parity)
    __shared__ uint32_t nmark;     // PLUG: marks listed so far
    // timestamps (sec << 32 | usec) of each step's first and last packet per wave: the order
    // check across wave boundaries, done once per tile (within a wave it is a DPP shift)
    __shared__ uint64_t bnd_first[K][IPXG_BLOCK / 64], bnd_last[K][IPXG_BLOCK / 64];
    const uint32_t tid = threadIdx.x;
    for (uint32_t q = tid; q < (1u << bv.part_bits); q += IPXG_BLOCK) fill[q] = 0;
    if (LINE)
        for (uint32_t q = tid; q < LINE_P; q += IPXG_BLOCK) lccnt[q] = 0;
    if (tid < 2) nslow[tid] = 0;
    if (tid == 0) nmark = 0;
    uint4* const my_marks = PLUG ? bv.marks + (size_t)blockIdx.x * bv.slow_stride : nullptr;
    // the block's slow list: every packet of its tiles fits, so a slow packet is stored at
    // its rank without any device atomic (a returning one inside the pipelined loop made the
    // compiler drain every load in flight)
    uint4* const my_slow = slow_list + (size_t)blockIdx.x * bv.slow_stride;
    uint32_t slow_fill = 0, par = 0;
    if (b.n == 0) {
        if (LINE && bv.prog && tid < (1u << bv.part_bits)) publish_prog(bv, blockIdx.x, tid, 0u, PROG_DONE);
        return;
    }
    const uint32_t last = b.n - 1;
    const uint32_t base_sec = b.base_sec == BASE_FROM_DESC0 ? b.desc[0].ts_sec : b.base_sec;
    b.base_sec = base_sec;
    const uint32_t P = 1u << bv.part_bits, pmask = P - 1;
    const bool fast_ok = p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB;
    const uint64_t ts_before = p.prev_dev ? ((uint64_t)p.prev_ctl->last_sec << 32) | p.prev_ctl->last_usec
                                          : ((uint64_t)p.prev_sec << 32) | p.prev_usec;
    ParseCounts c = {};
    uint32_t spilled = 0, walked = 0, tb_or = 0;
    constexpr bool XP = IPXG_BIN_XPOSE && !WIDE && AGG && !G64;
    // Without tile aggregation the tile's records are staged in LDS as they are made (the stage
    // array, free during the packet loop: the aggregation's tile hash and XP's transposes use it):
    // the 32 record registers (8 steps x 4 words) are live only in the emit phase, not through the
    // parse and hash of every step -- k_bin's register peak.
    constexpr bool LR = !AGG;
    // the wide walk's window: 96 bytes (WIDE2_DW) without tile aggregation, 80 with it (its
    // registers: 245 VGPRs at 80 bytes)
    constexpr int WD = AGG ? WIDE_DW : WIDE2_DW;
    constexpr int NC = WIDE ? WD / 4 : (XP ? 4 : 3);
    // the wave's transpose area (XP): the stage array is free during the packet loop
    uint4* const xs = reinterpret_cast<uint4*>(stage) + (tid >> 6) * 320u;
    static_assert(!XP || IPXG_BLOCK / 64 * 320 <= TILE, "transpose areas fit the stage array");
    // (unit offsets: the heads are plain loads through 64-bit addresses, which no buffer range
    // clamps -- a descriptor past the arena reads as zeros here, as the byte-offset buffer loads
    // give it, instead of faulting the GPU)
    auto want = [&](const ipxg_pkt_desc& d) {
        return fast_ok && fast_shape(b, d) && (!G64 || ((uint64_t)d.offset << 4) + d.caplen <= b.arena_len);
    };
    bool nonmono = false;
    const __amdgpu_buffer_rsrc_t rs_desc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<ipxg_pkt_desc*>(b.desc), 0, (int)(b.n * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    const uint32_t lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x == 0 && tid == 0 && p.prev_valid) {
        const ipxg_pkt_desc d0 = b.desc[0];
        if ((((uint64_t)d0.ts_sec << 32) | d0.ts_usec) < ts_before) nonmono = true;
    }
#ifdef IPXG_PROBE
    uint64_t probe_acc[4] = {0, 0, 0, 0};
#endif
    // The block's tiles: F full rounds of interleaved tiles (tile k of block w is tile k * grid + w of
    // BIN_K 256-packet steps, so the grid streams through one region of the batch at a time), then
    // its even share of the remaining steps as one partial tile (round 5: the remainder went to the
    // first blocks as whole tiles -- 4883 udp64 tiles over 768 blocks left a seventh round on 275
    // of them; one contiguous range per block instead cost udp64 2 %, DRAM locality).  Step g of
    // the block is step g % BIN_K of its tile g / BIN_K (one packet per lane).  Software pipeline across the tiles: step g
    // issues the descriptor of step g + DA and the head of step g + HA (whose descriptor
    // arrived during the DA - HA steps since it was issued), so the loads stay in flight
    // through the tile's emit phase and its barriers.  The tile's steps are unrolled and
    // BIN_K is a multiple of DA and HA: every ring slot is a fixed register set.
#ifndef IPXG_BIN_DA
#define IPXG_BIN_DA 4
#endif
// (head distance 1 without tile aggregation: udp64 step -0.9 %, quic -0.7 % against 2; the
// aggregating walk keeps 2: imix +0.7 % at 1 -- gpurun_out/var5, var6)
#ifndef IPXG_BIN_HA
#define IPXG_BIN_HA 1
#endif
#ifndef IPXG_BIN_HA_AGG
#define IPXG_BIN_HA_AGG 2
#endif
    constexpr int DA = IPXG_BIN_DA, HA = AGG ? IPXG_BIN_HA_AGG : IPXG_BIN_HA;
    static_assert(K % DA == 0 && K % HA == 0 && HA < DA && DA <= K, "pipeline distances");
    const uint32_t nsteps = (b.n + IPXG_BLOCK - 1) / IPXG_BLOCK;
    const uint32_t G = gridDim.x;
#ifndef IPXG_BIN_BALANCE  // A/B knob: 0 = whole tiles only (the round-4 assignment) for every variant
#define IPXG_BIN_BALANCE 1
#endif
    // The remainder spread evenly pays with the tiling aggregation (imix k_bin -5 %); the plain
    // walk is bandwidth-bound -- a block alone on its CU in the last round runs faster -- and one
    // more (partial) tile's emit per block cost it 1.4 % (udp64, gpurun_out/v5b): whole tiles there.
    constexpr bool BAL = IPXG_BIN_BALANCE && AGG;
    const uint32_t tiles = (nsteps + K - 1) / K;
    const uint32_t F = BAL ? nsteps / (K * G) : (blockIdx.x < tiles ? (tiles - blockIdx.x + G - 1) / G : 0u);
    const uint32_t rb = BAL ? F * K * G : 0u;  // the remainder's first step
    const uint32_t rs = BAL ? nsteps - rb : 0u;     // ... and its steps (< K * G)
    const uint32_t r_lo = rb + (uint32_t)((uint64_t)rs * blockIdx.x / G);
    const uint32_t r_hi = rb + (uint32_t)((uint64_t)rs * (blockIdx.x + 1) / G);
    const uint32_t ntile = F + (r_hi > r_lo ? 1u : 0u);
    auto tile_lo = [&](uint32_t k) { return k < F ? (k * G + blockIdx.x) * K : r_lo; };  // first step
    auto tile_lim = [&](uint32_t k) {  // packet limit (exclusive) of tile k; an empty range past the last
        const uint32_t hi = k < F ? (k * G + blockIdx.x) * K + K : (k == F ? r_hi : r_lo);
        return min(b.n, hi * IPXG_BLOCK);
    };
    // a prefetch past a tile's range reads nothing (an index past every descriptor)
    auto clamp = [](uint32_t i, uint32_t lim) { return i < lim ? i : (BUF_OOB >> 4); };
    ipxg_pkt_desc Dr[DA];
    Head<NC> Hr[HA];
    bool Xr[HA];  // XP: ring slot h holds a transposed (contiguous) head load
    // The prologue issues its loads in the order the last DA steps of a tile do, with dummy
    // stores where a tile issues heads of its own steps and its record stores: the loop's
    // first waits are shared by the first tile and all later ones, and the compiler sizes
    // them for the path with the fewest memory operations after each load.
#pragma unroll
    for (int k = 0; k < DA; ++k) {
        const uint32_t i = clamp((tile_lo(0) + k) * IPXG_BLOCK + tid, ntile ? tile_lim(0) : 0u);
        Dr[k] = load_desc<LAUX>(rs_desc, i);
        if (k >= DA - HA) {
            const int h = k - (DA - HA);
            if constexpr (XP) Hr[h] = load_head_x(rs_arena, Dr[h].offset, want(Dr[h]), Xr[h]);  // (byte offsets)
            else if constexpr (G64) Hr[h] = load_head_g<NC>(b.arena + ((uint64_t)Dr[h].offset << 4), Dr[h].caplen, want(Dr[h]));
            else Hr[h] = load_head<NC, LAUX>(rs_arena, Dr[h].offset, Dr[h].caplen, want(Dr[h]));
        } else {
#pragma unroll
            for (int q = 0; q < 3; ++q) g_dummy_rec[(k * 3 + q) * 64 + (tid & 63)] = make_uint4(0, 0, 0, 0);
        }
    }
    constexpr uint32_t EMIT_ST = LINE ? LINE_ITERS : TILE / IPXG_BLOCK;  // a tile's record stores per lane
    static_assert((DA * 3 + EMIT_ST) * 64 <= 32 * 64, "g_dummy_rec");
#pragma unroll
    for (int q = 0; q < (int)EMIT_ST; ++q) g_dummy_rec[(DA * 3 + q) * 64 + (tid & 63)] = make_uint4(0, 0, 0, 0);
    for (uint32_t tk = 0; tk < ntile; ++tk) {
        const uint32_t tile = tile_lo(tk) * IPXG_BLOCK;
        const uint32_t lim = tile_lim(tk);
        const uint32_t next = tile_lo(tk + 1) * IPXG_BLOCK;  // the block's next tile
        const uint32_t next_lim = tk + 1 < ntile ? tile_lim(tk + 1) : 0u;  // (none: loads give zeros)
        // the timestamp of the packet before the tile (another workgroup's tile), for the
        // tile's first packet; consumed after the tile (zeros for the batch's first tile)
        const u32x2 tpred = __builtin_amdgcn_raw_buffer_load_b64(rs_desc, tile ? tile * 16u - 8u : BUF_OOB, 0, 0);
        PROBE_T(t0);
#pragma unroll
        for (uint32_t k = 0; k < (PM + IPXG_BLOCK - 1) / IPXG_BLOCK; ++k)
            if (k * IPXG_BLOCK + tid < P) hist[k * IPXG_BLOCK + tid] = 0;
        __syncthreads();
        if (tid == 0) nslow[par ^ 1] = 0;  // the next tile's (last read before this barrier)
        PROBE_T(t1);
        PROBE_ADD(0, t0, t1);
        uint32_t r0[K], r1[K], r2[K], rk[K], ix[K];
        if constexpr (!LR) {
#pragma unroll
            for (int q = 0; q < K; ++q) {
                r0[q] = r1[q] = r2[q] = ix[q] = 0;
                rk[q] = NO_REC;
            }
        }
        // The wide walk's steps are unrolled DA at a time (the register rings' period), not all
        // BIN_K: eight inlined copies of parse_medium made the kernel larger than the
        // instruction cache.  (Record slot j is then a runtime index: tile_rank selects.)
        constexpr int SU = WIDE ? DA : K;
#pragma unroll 1
        for (int g = 0; g < K; g += SU) {
#pragma unroll
        for (int jj = 0; jj < SU; ++jj) {
            const int j = g + jj;
            const uint32_t i = tile + j * IPXG_BLOCK + tid;
            // this step's packet, loaded HA (head) and DA (descriptor) steps ago
            const ipxg_pkt_desc dc = Dr[jj % DA];
            Head<NC> hc = Hr[jj % HA];
            if constexpr (XP) {
                if (Xr[jj % HA]) xpose_head(xs, hc);  // wave-uniform
            }
            // bytes 40-43 are not parsed: keep their register live until here, or the compiler
            // reuses it while the load is in flight and must drain every load to do so
            asm volatile("" ::"v"(hc.c[2].z));
            // issue: the descriptor DA steps ahead, the head HA steps ahead
            const uint32_t ia = j + DA < K ? tile + (j + DA) * IPXG_BLOCK + tid : next + (j + DA - K) * IPXG_BLOCK + tid;
            Dr[jj % DA] = load_desc<LAUX>(rs_desc, j + DA < K ? clamp(ia, lim) : clamp(ia, next_lim));
            const ipxg_pkt_desc dh = Dr[(jj + HA) % DA];
            if constexpr (XP) Hr[jj % HA] = load_head_x(rs_arena, dh.offset, want(dh), Xr[jj % HA]);
            else if constexpr (G64) Hr[jj % HA] = load_head_g<NC>(b.arena + ((uint64_t)dh.offset << 4), dh.caplen, want(dh));
            else Hr[jj % HA] = load_head<NC, LAUX>(rs_arena, dh.offset, dh.caplen, want(dh));
            const bool act = i < lim;
            // order check: the predecessor's timestamp is the lane below's (DPP; lane 0 compares
            // with itself here and with the previous wave's last packet after the tile)
            const uint32_t ps = (uint32_t)__builtin_amdgcn_update_dpp((int)dc.ts_sec, (int)dc.ts_sec, 0x138, 0xF, 0xF, false);
            const uint32_t pu = (uint32_t)__builtin_amdgcn_update_dpp((int)dc.ts_usec, (int)dc.ts_usec, 0x138, 0xF, 0xF, false);
            if (act && (dc.ts_sec < ps || (dc.ts_sec == ps && dc.ts_usec < pu))) nonmono = true;
            const uint64_t ts = ((uint64_t)dc.ts_sec << 32) | dc.ts_usec;
            if (lane == 0) bnd_first[j][wave] = ts;
            if (lane == 63) bnd_last[j][wave] = ts;
            DevPkt pk;
            bool have = false, slow = false;
#ifdef IPXG_EXP_LOADONLY  // timing experiment only: the loads, no parse/rank
            if (act) c.seen += hc.c[0].x ^ hc.c[1].y ^ hc.c[2].z ^ hc.c[0].w ^ hc.c[1].x ^ hc.c[2].y;
            if (false) {
#else
            if (act) {
#endif
                if constexpr (WIDE) {
                    uint32_t w[WD];
#pragma unroll
                    for (int k = 0; k < NC; ++k) {
                        w[4 * k] = hc.c[k].x;
                        w[4 * k + 1] = hc.c[k].y;
                        w[4 * k + 2] = hc.c[k].z;
                        w[4 * k + 3] = hc.c[k].w;
                    }
                    bool ext = false;
                    if (fast_ok && fast_shape(b, dc) && parse_medium<PLUG, WD>(w, dc.caplen, p.frag_enable, pk, c, ext)) {
                        have = true;
                        walked += ext ? 1 : 0;
                        if constexpr (PLUG) {
                            if (pk.l4 == 6 || pk.l4 == 17) {
                                const uint32_t kind = plug_check<WD>(p, w, dc.caplen, pk);
                                if (kind) {
                                    uint64_t lo = 0, hf;
                                    uint32_t cd;
                                    if (kind == MARK_HIT) canon<false>(pk, p, lo, cd, hf);
                                    my_marks[atomicAdd(&nmark, 1u)] =
                                        make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), i | (kind << 30), 0);
                                }
                            }
                        }
                    } else {
                        slow = true;
                    }
                } else {
                    if (fast_ok && fast_shape(b, dc) && parse_fast(hc.c[0], hc.c[1], hc.c[2], dc.caplen, p.frag_enable, pk, c))
                        have = true;
                    else
                        slow = true;
                }
            }
            if (slow)
                my_slow[slow_fill + atomicAdd(&nslow[par], 1u)] =
                    make_uint4(i | (slow_class(hc.c[0], hc.c[1], hc.c[2]) << 24), dc.offset,
                               (uint32_t)dc.caplen | ((uint32_t)dc.wirelen << 16), dc.ts_sec);
            if constexpr (LR)
                stage[j * IPXG_BLOCK + tid] = have ? make_record(p, b, pk, dc, tb_or) : make_uint4(0, 0, NO_REC, 0);
            else if (have)
                tile_rank<false>(p, b, pk, dc, i, j, r0, r1, r2, rk, ix, tb_or);
        }
        }
        if constexpr (LR) {  // the lane's own records back (tile_emit's first barrier precedes any other lane's writes)
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const uint4 r = stage[q * IPXG_BLOCK + tid];
                r0[q] = r.x;
                r1[q] = r.y;
                rk[q] = r.z;
                r2[q] = r.w;
                ix[q] = 0;
            }
        }
        PROBE_T(t2);
        PROBE_ADD(1, t1, t2);
#ifndef IPXG_EXP_NOSKEL  // timing experiment (with IPXG_EXP_LOADONLY only): no rank / emit phase at all
        if constexpr (AGG) tile_aggregate<false>(L, pmask, r0, r1, r2, rk, ix, tile, folded);
        else tile_rank_all<K>(hist, pmask, r1, rk);
        if constexpr (LINE)
            tile_emit_lines<K>(LL, P, pmask, bv, blockIdx.x, t, ctl, deferred_list, r0, r1, r2, rk, tile, spilled,
                               p.defer_spill != 0,
                               bv.prog && (bv.prog_mode & PROG_TILE) && (tk + 1) % bv.pub_every == 0);
        else
            tile_emit<false, AGG, KBIN_PMAX>(L, P, pmask, bv, blockIdx.x, t, ctl, deferred_list, agg_list, r0, r1, r2,
                                             rk, ix, tile, spilled, p.defer_spill != 0);
#endif
        PROBE_T(t3);
        PROBE_ADD(2, t2, t3);
        slow_fill += nslow[par];  // final: read after the tile's barriers
        par ^= 1;
        if (tid < K * (IPXG_BLOCK / 64)) {  // the wave boundaries of the tile
            const uint32_t j = tid / (IPXG_BLOCK / 64), w = tid % (IPXG_BLOCK / 64);
            const uint32_t i0 = tile + j * IPXG_BLOCK + w * 64;
            const uint64_t pred = w ? bnd_last[j][w - 1]
                                    : (j ? bnd_last[j - 1][IPXG_BLOCK / 64 - 1] : ((uint64_t)tpred.x << 32) | tpred.y);
            if (i0 != 0 && i0 < lim && bnd_first[j][w] < pred) nonmono = true;
        }
        PROBE_T(t4);
        PROBE_ADD(3, t3, t4);
    }
#ifdef IPXG_PROBE
    if (lane_id() == 0)
        for (int k = 0; k < 4; ++k) atomicAdd((unsigned long long*)&ctl->probe[k], (unsigned long long)probe_acc[k]);
#endif
    if (tid == 0 && blockIdx.x == gridDim.x - 1) {  // (its range ends with the batch)
        const ipxg_pkt_desc d = b.desc[last];  // the batch's last timestamp (next batch's order check)
        ctl->last_sec = d.ts_sec;
        ctl->last_usec = d.ts_usec;
    }
    if (nonmono) ctl->nonmono = 1;
    if (tid == 0) {
        bv.slow_cnt[blockIdx.x] = slow_fill;
        if (slow_fill) atomicAdd(&ctl->slow_count, slow_fill);
        if (slow_fill && p.slow_skip) ctl->slow_redo = 1;  // (no k_bin_slow behind this launch)
    }
    __syncthreads();  // the last tile's fill updates (tile_emit's tail) are other threads'
    if constexpr (LINE) line_flush(LL, P, bv, blockIdx.x, t, ctl, deferred_list, spilled, p.defer_spill != 0);
    seg_counts(fill, P, bv, blockIdx.x);
    if (PLUG && tid == 0) bv.mark_cnt[blockIdx.x] = nmark;
    // block statistics, hist reused as the counter block
    if (tid < ST_COUNT) hist[tid] = 0;
    if (tid < BLK_N) hist[ST_STRIDE + tid] = 0;
    __syncthreads();
    flush_counts(c, 0, 0, hist);
    block_ctl_counts(hist + ST_STRIDE, spilled, AGG ? folded : 0u, WIDE ? walked : 0u, tb_or);
    flush_block_stats(hist, stats);  // (its barrier completes the block's counters)
    flush_block_ctl(hist + ST_STRIDE, ctl);
    if (LINE && bv.prog) {  // streamed reduce: the column is complete -- its plain stores (segment counts,
                            // control block) released to agent scope first, then the words marked done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (tid < P) publish_prog(bv, blockIdx.x, tid, fill[tid], PROG_DONE);
    }
}

// A slow-list entry (k_bin -> k_bin_slow): {packet index, offset, caplen | wirelen << 16,
// ts_sec} -- the descriptor fields the slow pass reads, so one 16-byte load replaces the
// index load and the dependent descriptor load.
__device__ __forceinline__ ipxg_pkt_desc slow_desc(const uint4 e) {
    ipxg_pkt_desc d;
    d.offset = e.y;
    d.caplen = (uint16_t)e.z;
    d.wirelen = (uint16_t)(e.z >> 16);
    d.ts_sec = e.w;
    d.ts_usec = 0;  // not read by the slow pass
    return d;
}

// The first IPXG_WIN bytes of an aligned frame as 16-byte buffer loads (a chunk at or past
// caplen, and every chunk of an unaligned frame, reads as zeros with no memory traffic).
// e.y: the descriptor's offset field (16-byte units with IPXG_BATCH_OFFSET16, whose frames are
// all aligned).
constexpr int SLOW_NCH = IPXG_WIN / 16;
struct SlowWin {
    uint4 c[SLOW_NCH];
};

__device__ __forceinline__ bool slow_aligned(const BatchView& b, const uint4 e) { return b.oshift || !(e.y & 15); }
// (G64, 16-byte units: through the frame's 64-bit address, a chunk past caplen from g_zero_head)
template <bool G64>
__device__ __forceinline__ SlowWin load_win(__amdgpu_buffer_rsrc_t rs_all, const BatchView& b, const uint4 e) {
    const uint32_t cap = e.z & 0xFFFFu;
    SlowWin w;
    if constexpr (G64) {  // (a frame past the arena reads as zeros: as want() in k_bin)
        const uint4* f = reinterpret_cast<const uint4*>(b.arena + ((uint64_t)e.y << 4));
        const bool in = ((uint64_t)e.y << 4) + cap <= b.arena_len;
#pragma unroll
        for (int k = 0; k < SLOW_NCH; ++k) w.c[k] = *(in && (uint32_t)(16 * k) < cap ? f + k : g_zero_head + (k & 7));
        return w;
    }
    const uint32_t o = slow_aligned(b, e) ? e.y : BUF_OOB;
#pragma unroll
    for (int k = 0; k < SLOW_NCH; ++k)
        w.c[k] = u4(__builtin_amdgcn_raw_buffer_load_b128(rs_all, (uint32_t)(16 * k) < cap ? o + 16 * k : BUF_OOB, 0,
                                                          IPXG_WIDE_LOAD_AUX));
    return w;
}

// The window into the lane's LDS column, zero-masked past caplen, plus one zero chunk so
// straddling reads see zeros (stage_frame's layout); unaligned frames: stage_frame's byte loads.
__device__ __forceinline__ void put_window(uint32_t* col, const BatchView& b, const uint4 e, const SlowWin& w) {
    const uint32_t cap = e.z & 0xFFFFu;
    if (!slow_aligned(b, e)) {  // (byte offsets only)
        stage_frame(col, b.arena + e.y, cap);
        return;
    }
    const uint32_t nch = ((cap < IPXG_WIN ? cap : IPXG_WIN) + 15) >> 4;
#pragma unroll
    for (int ch = 0; ch < SLOW_NCH; ++ch) {
        if ((uint32_t)ch > nch) break;
        const uint32_t v[4] = {w.c[ch].x, w.c[ch].y, w.c[ch].z, w.c[ch].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int valid = (int)cap - (16 * ch + 4 * k);
            const uint32_t m = valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
            col[(4 * ch + k) * IPXG_BLOCK] = v[k] & m;
        }
    }
}

// One slow packet: staged, parsed by parse_frame, then keyless / fragment / record slot j.
template <bool AGG>
__device__ __forceinline__ void slow_packet(const Params& p, const BatchView& b, const FragView& f, BatchCtl* ctl,
                                            uint32_t* col, const uint4 e, const SlowWin& w, int j, ParseCounts& c,
                                            uint32_t& keyless, uint32_t& frags, uint32_t (&r0)[BIN_K],
                                            uint32_t (&r1)[BIN_K], uint32_t (&r2)[BIN_K], uint32_t (&rk)[BIN_K],
                                            uint32_t (&ix)[BIN_K], uint32_t& tb_or, uint4* marks, uint32_t* nmark) {
    const ipxg_pkt_desc d = slow_desc(e);
    const uint32_t i = e.x & SLOW_IDX_MASK;
    put_window(col, b, e, w);
    LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
    DevPkt pk;
    if (!parse_frame<false>(S, d.caplen, p.dlt, pk, c)) return;
    if (pk.ip_version != 4 && pk.ip_version != 6) {  // create_hash_key false
        keyless++;
        return;
    }
    // Params::plug: a TCP/UDP packet with its L4 header -- a first fragment too, as k_classify
    // tests them -- is classified from its frame by k_plugin_marks
    if (p.plug && !pk.frag_off && (pk.l4 == 6 || pk.l4 == 17))
        marks[atomicAdd(nmark, 1u)] = make_uint4(0, 0, i | (MARK_LATER << 30), 0);
    if (p.frag_enable && (pk.frag_off || pk.more_fragments)) {
        frags++;
        divert_fragment(pk, p, f, ctl, i);
        return;
    }
    tile_rank<true>(p, b, pk, d, i, j, r0, r1, r2, rk, ix, tb_or);
}

// The frames k_bin left for the general parser (VLAN/QinQ, MPLS, PPPoE, GRE, TRILL, IPv6
// and its extension headers, IPv4 options, TCP options, SLL/SLL2/raw link types, truncated
// or unaligned frames): staged in the lane's LDS column, parsed by parse_frame, ranked and
// emitted exactly like k_bin's records.  The list length is read on the device.
// Up to 256 VGPRs (2 waves/SIMD): the packet pairs' windows take 64; two pairs in flight per
// SIMD hide more latency than three single packets did.
template <bool AGG, bool G64 = false>
__global__ __launch_bounds__(IPXG_BLOCK) __attribute__((amdgpu_waves_per_eu(2)))
void k_bin_slow(BatchView b, Params p, TableView t, FragView f, BinView bv, BatchCtl* ctl,
                const uint4* slow_list, uint32_t* deferred_list, uint4* agg_list, unsigned long long* stats) {
    if (gated(p)) return;  // (k_bin returned too)
    // the header columns (parse), the tile hash and the tile's slots (emit) are never live
    // together: one 32 KiB area; 76 KiB in all with aggregation (2 workgroups per CU), 48 KiB
    // without (3 per CU)
    __shared__ uint4 stage[BIN_TILE];                   // 32 KiB: header columns / tile hash / slots
    __shared__ uint32_t hist[1u << BIN_MAX_PART_BITS];  // 8 KiB
    __shared__ uint32_t fill[1u << BIN_MAX_PART_BITS];  // 8 KiB
    __shared__ uint32_t tcnt[AGG ? TAGG_HASH : 1];      // 16 KiB
    __shared__ TileAgg tagg[AGG ? TAGG_CAP : 1];        // 8 KiB
    __shared__ uint16_t part_of[AGG ? BIN_TILE : 1];    // 4 KiB
    __shared__ uint32_t scan_s[IPXG_BLOCK / 64 + 1];
    __shared__ uint32_t nagg;
    const BinLds L = {hist, fill, stage, tcnt, tagg, part_of, scan_s, &nagg};
    uint32_t folded = 0;
    static_assert(sizeof(stage) >= IPXG_WIN_DW * IPXG_BLOCK * 4, "header columns exceed the stage");
    uint32_t* win = reinterpret_cast<uint32_t*>(stage);
    // the slow packets of k_bin workgroups blockIdx.x * G ... + G - 1 (BinView::slow_group), one list
    // after the other, into segment column bin_grid + blockIdx.x; spre: the lists' starts
    __shared__ uint32_t spre[SLOW_GROUP_MAX + 1];
    const uint32_t G = bv.slow_group ? bv.slow_group : 1u;
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t g = 0; g < G; ++g) {
            spre[g] = s;
            const uint32_t lb = blockIdx.x * G + g;
            s += lb < bv.bin_grid ? bv.slow_cnt[lb] : 0u;  // final: k_bin has completed
        }
        spre[G] = s;
    }
    __syncthreads();
    const uint32_t ns = spre[G];
    const uint4* const list = slow_list + (size_t)blockIdx.x * G * bv.slow_stride;
    // entry x of the merged lists (x < ns)
    auto slow_at = [&](uint32_t x) -> uint4 {
        if (G == 1) return list[x];
        uint32_t g = 0;
#pragma unroll
        for (uint32_t q = 1; q < SLOW_GROUP_MAX; ++q) g += (q < G && spre[q] <= x) ? 1u : 0u;
        return list[(size_t)g * bv.slow_stride + (x - spre[g])];
    };
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    const uint32_t bcol = bv.bin_grid + blockIdx.x;  // this block's segment column
    if (ns == 0) return;  // no work: k_reduce does not read the column (uniform)
#if defined(IPXG_EXP_SLOW) && IPXG_EXP_SLOW == 1  // timing experiment: the launch alone
    if (ns) return;
#endif
    // Params::plug: the slow packets' plugin checks listed after k_bin's marks of this workgroup
    __shared__ uint32_t nmark;
    uint4* const my_marks = p.plug ? bv.marks + (size_t)blockIdx.x * bv.slow_stride : nullptr;
    if (threadIdx.x == 0) nmark = p.plug ? bv.mark_cnt[blockIdx.x] : 0;
    for (uint32_t q = threadIdx.x; q < (1u << bv.part_bits); q += IPXG_BLOCK) fill[q] = 0;
    const uint32_t tid = threadIdx.x;
    if (b.base_sec == BASE_FROM_DESC0) b.base_sec = b.n ? b.desc[0].ts_sec : 0;
    const uint32_t P = 1u << bv.part_bits, pmask = P - 1;
    ParseCounts c = {};
    uint32_t keyless = 0, frags = 0, spilled = 0, tb_or = 0;
    uint32_t* col = &win[tid];
#ifdef IPXG_PROBE
    uint64_t probe_acc[4] = {0, 0, 0, 0};  // [0] loads, [1] parse + rank, [2] emit, [3] packets (lane 0)
#endif
    __shared__ uint32_t ccnt[SLOW_NCLS];  // the tile's packets per shape class, then the class's start
    uint16_t* const ord = reinterpret_cast<uint16_t*>(hist);  // sorted position -> entry (hist is free until the ranking)
    static_assert(sizeof(hist) >= BIN_TILE * sizeof(uint16_t), "tile order in the histogram area");
    for (uint32_t tile = 0; tile < ns; tile += BIN_TILE) {
        // group the tile's entries by shape class: counting sort of their positions into ord
        const uint32_t nt = min(ns - tile, BIN_TILE);
        if (tid < SLOW_NCLS) ccnt[tid] = 0;
        __syncthreads();
        uint32_t crk[BIN_K];  // class << 16 | rank in class
#pragma unroll
        for (int j = 0; j < BIN_K; ++j) {
            const uint32_t k = (uint32_t)j * IPXG_BLOCK + tid;
            crk[j] = 0xFFFFFFFFu;
            if (k < nt) {
                const uint32_t c = slow_at(tile + k).x >> 24;
                crk[j] = (c << 16) | atomicAdd(&ccnt[c], 1u);
            }
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t run = 0;
            for (uint32_t c = 0; c < SLOW_NCLS; ++c) {
                const uint32_t v = ccnt[c];
                ccnt[c] = run;
                run += v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < BIN_K; ++j)
            if (crk[j] != 0xFFFFFFFFu) ord[ccnt[crk[j] >> 16] + (crk[j] & 0xFFFF)] = (uint16_t)(j * IPXG_BLOCK + tid);
        __syncthreads();
        uint32_t r0[BIN_K], r1[BIN_K], r2[BIN_K], rk[BIN_K], ix[BIN_K];
#pragma unroll
        for (int q = 0; q < BIN_K; ++q) {
            r0[q] = r1[q] = r2[q] = ix[q] = 0;
            rk[q] = NO_REC;
        }
        // One packet per step with a rolling prefetch -- the entry two steps ahead and the window
        // one step ahead are in flight while this step's packet is parsed -- and ONE call site of
        // the general parser: two inlined copies (a pair per step) made the kernel's hot code
        // larger than the instruction cache.
        auto entry = [&](int j) {
            const uint32_t k = tile + (uint32_t)j * IPXG_BLOCK + tid;
            return j < BIN_K && k < ns ? slow_at(tile + ord[k - tile]) : make_uint4(0, BUF_OOB, 0, 0);
        };
        uint4 e0 = entry(0), e1 = entry(1);
        SlowWin w0 = load_win<G64>(rs_arena, b, e0);
#pragma unroll 1
        for (int j = 0; j < BIN_K; ++j) {
            const uint32_t k0 = tile + (uint32_t)j * IPXG_BLOCK + tid;
            if (k0 >= ns) break;
            PROBE_T(s0);
            const uint4 e2 = entry(j + 2);
            const SlowWin w1 = load_win<G64>(rs_arena, b, e1);
#ifdef IPXG_PROBE
            asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // w0 (the entry and window ahead stay in flight)
            const uint64_t s1 = __builtin_readcyclecounter();
            PROBE_ADD(0, s0, s1);
            probe_acc[3] += 1;
#endif
#if defined(IPXG_EXP_SLOW) && IPXG_EXP_SLOW == 2  // timing experiment: no parse
            if (e0.z == 0xFFFFFFFFu)
#endif
            slow_packet<AGG>(p, b, f, ctl, col, e0, w0, j, c, keyless, frags, r0, r1, r2, rk, ix, tb_or, my_marks, &nmark);
#ifdef IPXG_PROBE
            PROBE_T(s2);
            PROBE_ADD(1, s1, s2);
#endif
            e0 = e1;
            e1 = e2;
            w0 = w1;
        }
        PROBE_T(s3);
        __syncthreads();  // ord (in hist) is read by the loop above
        for (uint32_t q = tid; q < P; q += IPXG_BLOCK) hist[q] = 0;
        if (!AGG) __syncthreads();  // (tile_aggregate starts with a barrier)
        if (AGG) tile_aggregate<true>(L, pmask, r0, r1, r2, rk, ix, tile, folded);
        else tile_rank_all(hist, pmask, r1, rk);
        tile_emit<true, AGG>(L, P, pmask, bv, bcol, t, ctl, deferred_list, agg_list, r0, r1, r2, rk, ix, tile,
                             spilled, p.defer_spill != 0);
        PROBE_T(s4);
        PROBE_ADD(2, s3, s4);
    }
#ifdef IPXG_PROBE
    if (lane_id() == 0) {
        atomicAdd((unsigned long long*)&ctl->probe[8], (unsigned long long)probe_acc[0]);
        atomicAdd((unsigned long long*)&ctl->probe[9], (unsigned long long)probe_acc[1]);
        atomicAdd((unsigned long long*)&ctl->probe[10], (unsigned long long)probe_acc[2]);
        atomicAdd((unsigned long long*)&ctl->probe[11], (unsigned long long)probe_acc[3]);
    }
#endif
    __syncthreads();  // the last tile's fill updates (tile_emit's tail) are other threads'
    seg_counts(fill, P, bv, bcol);
    if (p.plug && tid == 0) bv.mark_cnt[blockIdx.x] = nmark;
#if defined(IPXG_EXP_SLOW) && IPXG_EXP_SLOW == 3  // timing experiment: no statistics atomics
    return;
#endif
    if (tid < ST_COUNT) hist[tid] = 0;
    if (tid < BLK_N) hist[ST_STRIDE + tid] = 0;
    __syncthreads();
    flush_counts(c, keyless, frags, hist);
    block_ctl_counts(hist + ST_STRIDE, spilled, AGG ? folded : 0u, 0u, tb_or);
#if defined(IPXG_EXP_SLOW) && IPXG_EXP_SLOW == 4  // timing experiment: no statistics atomics
    __syncthreads();
#else
    flush_block_stats(hist, stats);  // (its barrier completes the block's counters)
#endif
#if defined(IPXG_EXP_SLOW) && IPXG_EXP_SLOW == 5  // timing experiment: no control-block atomics
    return;
#endif
    flush_block_ctl(hist + ST_STRIDE, ctl);
}

typedef void (*BinKernel)(BatchView, Params, TableView, FragView, BinView, BatchCtl*, uint4*, uint32_t*, uint4*,
                          unsigned long long*);
template <bool G64>
static BinKernel bin_kernel_g(bool agg, bool wide, bool plug) {
    if (plug) return agg ? k_bin<true, true, true, false, G64> : k_bin<false, true, true, false, G64>;  // (plug: the wide walk)
    return agg ? (wide ? k_bin<true, true, false, false, G64> : k_bin<true, false, false, false, G64>)
               : (wide ? k_bin<false, true, false, false, G64> : k_bin<false, false, false, false, G64>);
}
static BinKernel bin_kernel(bool agg, bool wide, bool plug, bool line, bool g64) {
    if (g64) return bin_kernel_g<true>(agg, wide, plug);  // (no line mode: setup_bins)
    if (line && !agg && !plug) return wide ? k_bin<false, true, false, true> : k_bin<false, false, false, true>;
    return bin_kernel_g<false>(agg, wide, plug);
}

uint32_t bin_resident_blocks(int device, bool agg, bool wide, bool plug, bool line, bool g64) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bin_kernel(agg, wide, plug, line, g64), IPXG_BLOCK, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    return (uint32_t)std::max(1, std::min(cus * per_cu, (int)BIN_MAX_GRID));
}

void launch_bin(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, BinView bv,
                BatchCtl* ctl, uint4* slow_list, uint32_t* deferred_list, uint4* agg_list,
                unsigned long long* stats) {
    hipLaunchKernelGGL(bin_kernel(p.tile_agg != 0, p.wide != 0, p.plug != 0, bv.line != 0, b.oshift != 0), dim3(bv.bin_grid), dim3(IPXG_BLOCK), 0, st, b, p,
                       t, f, bv, ctl, slow_list, deferred_list, agg_list, stats);
}

void launch_bin_slow(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, BinView bv,
                     BatchCtl* ctl, const uint4* slow_list, uint32_t* deferred_list, uint4* agg_list,
                     unsigned long long* stats) {
    typedef void (*SlowKernel)(BatchView, Params, TableView, FragView, BinView, BatchCtl*, const uint4*, uint32_t*,
                               uint4*, unsigned long long*);
    const SlowKernel k = b.oshift ? (p.tile_agg ? k_bin_slow<true, true> : k_bin_slow<false, true>)
                                  : (p.tile_agg ? k_bin_slow<true> : k_bin_slow<false>);
    const uint32_t g = bv.slow_group ? bv.slow_group : 1u;
    bv.slow_group = g;
    hipLaunchKernelGGL(k, dim3((bv.bin_grid + g - 1) / g), dim3(IPXG_BLOCK), 0, st, b, p, t, f, bv, ctl, slow_list,
                       deferred_list, agg_list, stats);
}

// ---- phase B ------------------------------------------------------------------------------
// LDS flow table of k_reduce: linear probing on the low bits of the canonical hash
template <uint32_t NE = RED_ENTRIES>
__device__ __forceinline__ int lds_slot(FlowAgg* ht, uint64_t lo, bool insert) {
    uint32_t e = (uint32_t)lo & (NE - 1);
    for (uint32_t probe = 0; probe < RED_MAX_PROBE; ++probe) {
        unsigned long long k = ht[e].key;
        if (k == 0) {
            if (!insert) return -1;
            k = atomicCAS(&ht[e].key, 0ull, (unsigned long long)lo);
            if (k == 0) return (int)e;
        }
        if (k == lo) return (int)e;
        e = (e + 1) & (NE - 1);
    }
    return -1;
}

// one_tb: every record of the batch is in time bucket 0 (ctl->tb_any == 0), so the occupancy
// map of every flow is bit 0 -- set once per flow after the fold, not once per record
__device__ __forceinline__ void lds_fold(FlowAgg& a, uint32_t idx, uint32_t m, bool one_tb) {
    const uint32_t cdir = misc_dir(m);
    atomicAdd(&a.acc[cdir], (1ull << 40) | (unsigned long long)misc_len(m));
    atomicMax(&a.last1, idx + 1);
    atomicMax(&a.first_n, first_key(idx, m));
    if (!one_tb) atomicOr(&a.tbits, 1u << misc_tb(m));
    const uint32_t fl = misc_flags(m);
    if (misc_tcp(m) && fl) {
        atomicOr(&a.tflags, fl << (8 * cdir));
        if (fl & 0x02) atomicMax(&a.syn1[cdir], idx + 1);
        if (fl & 0x05) atomicMax(&a.fin_n[cdir], ~idx);
    }
}

enum RedCount { C_KEYS, C_TOUCH, C_SPILL, C_FAIL, C_N };
constexpr uint32_t RED_MAX_COLS = 2 * BIN_MAX_GRID;

// record k (0 <= k < total) of the partition: in the segment s with pre[s] <= k < pre[s+1]
__device__ __forceinline__ const uint4* seg_ptr(const uint4* segs, const uint32_t* pre, uint32_t cols,
                                                uint32_t seg_cap, uint32_t k) {
    uint32_t lo = 0;  // the last s with pre[s] <= k: a fixed number of steps, no branches
#pragma unroll
    for (uint32_t step = RED_MAX_COLS / 2; step; step >>= 1) {
        const uint32_t m = lo + step;
        lo = (m < cols && pre[m] <= k) ? m : lo;
    }
    return segs + (size_t)lo * seg_cap + (k - pre[lo]);
}
__device__ __forceinline__ uint4 seg_record(const uint4* segs, const uint32_t* pre, uint32_t cols,
                                            uint32_t seg_cap, uint32_t k) {
    return *seg_ptr(segs, pre, cols, seg_cap, k);
}

__device__ __forceinline__ void lds_fold_agg(FlowAgg& e, const FlowAgg& a) {
    if (a.acc[0]) atomicAdd(&e.acc[0], a.acc[0]);
    if (a.acc[1]) atomicAdd(&e.acc[1], a.acc[1]);
    atomicMax(&e.last1, a.last1);
    atomicMax(&e.first_n, a.first_n);
    atomicOr(&e.tbits, a.tbits);
    if (a.tflags) atomicOr(&e.tflags, a.tflags);
    for (int d = 0; d < 2; ++d) {
        if (a.syn1[d]) atomicMax(&e.syn1[d], a.syn1[d]);
        if (a.fin_n[d]) atomicMax(&e.fin_n[d], a.fin_n[d]);
    }
}

// Fold one record slot into the workgroup's LDS flow table (or straight into the device table
// when the LDS table is full).  rp = the slot's address (an aggregate's head reads its two
// payload slots after it; the payload slots themselves are skipped).
// ok: the slot exists (tested here, not by overwriting the loaded value: a write into the
// load's destination made the compiler wait for each load as soon as it was issued)
// The rare cases of red_record out of line -- an aggregate (3 slots), a record whose flow found
// no LDS entry -- so the RED_U-unrolled fold loop inlines only the common path (probe + fold):
// with every case inlined in every unrolled copy k_reduce's code was 117 KB.
__device__ __noinline__ void red_agg(FlowAgg* ht, const TableView& t, BatchCtl* ctl, uint4* agg_list, uint32_t* cnt,
                                     const uint4 r, const uint4* rp) {
    if (rec_agg_slot(r) != 0) return;
    const uint4 s1 = rp[1], s2 = rp[2];
    const FlowAgg a = agg_decode(r, s1, s2);
    const int e = lds_slot(ht, a.key, true);
    if (e >= 0) {
        lds_fold_agg(ht[e], a);
    } else {
        atomicAdd(&cnt[C_SPILL], 1u);
        if (!merge_agg_probe(t, a, &ctl->new_keys)) defer_agg(&ctl->agg_deferred, agg_list, r, s1, s2);
    }
}
__device__ __noinline__ void red_spill(const TableView& t, BatchCtl* ctl, uint32_t* deferred_list, uint32_t* cnt,
                                       const uint4 r) {
    atomicAdd(&cnt[C_SPILL], 1u);
    if (!merge_packet_atomic(t, ((uint64_t)r.y << 32) | r.x, r.z, r.w, &ctl->new_keys))
        defer_packet(ctl, deferred_list, r.z, false);
}

// lds_slot's continuation after a first read k of entry e that was not the key: insert into an
// empty entry, or probe on.  Inline: at the udp64 partitions' ~0.2 load of the LDS table one
// record in five finds another flow in its home entry, so nearly every wave-group has a lane
// here, and as a call (scratch saves of the caller's registers, a full vmcnt drain) it stalled
// the group's prefetched record loads.
template <uint32_t NE = RED_ENTRIES>
__device__ __forceinline__ int red_probe(FlowAgg* ht, uint64_t lo, uint32_t e, unsigned long long k) {
    for (uint32_t probe = 0; probe < RED_MAX_PROBE; ++probe) {
        if (k == 0) {
            k = atomicCAS(&ht[e].key, 0ull, (unsigned long long)lo);
            if (k == 0) return (int)e;
        }
        if (k == lo) return (int)e;
        e = (e + 1) & (NE - 1);
        k = ht[e].key;
    }
    return -1;
}

__device__ __forceinline__ void red_record(FlowAgg* ht, const TableView& t, BatchCtl* ctl, uint32_t* deferred_list,
                                           uint4* agg_list, uint32_t* cnt, const uint4& r, const uint4* rp, bool ok,
                                           bool one_tb) {
    if (!ok || r.z == NO_REC) return;
    if (rec_is_agg(r)) {
        red_agg(ht, t, ctl, agg_list, cnt, r, rp);
        return;
    }
    const int e = lds_slot(ht, ((uint64_t)r.y << 32) | r.x, true);
    if (e >= 0) lds_fold(ht[e], r.z, r.w, one_tb);
    else red_spill(t, ctl, deferred_list, cnt, r);
}

// The end of a partition's reduce (k_reduce, k_reduce_stream), after the fold: each LDS aggregate of
// the NE-entry table (NT threads) merged into its table slot or listed for k_fin_list, the flows
// whose slot probe failed deferred with their records (rec_at(k): the partition's record k of
// total), the workgroup's counts added to the control block.
// fuse: nothing else of this batch can touch these flows (no packet went to the fragment or
// deferred paths; spilled packets were accumulated by k_bin, before the merge): then the merged
// slot is complete and goes on the finalise list (k_fin_list).
template <uint32_t NE, uint32_t NT, typename RecAt>
__device__ __forceinline__ void red_tail(FlowAgg* ht, const TableView& t, BatchCtl* ctl, HotSlot* fin_list,
                                         uint32_t* deferred_list, uint4* agg_list, uint32_t* cnt, uint32_t* scan_s,
                                         uint32_t* fin_base, bool one_tb, bool fuse, uint32_t total, RecAt rec_at) {
    const uint32_t tid = threadIdx.x;
    // (IPXG_FIN_PROBE=0: the slots probed here as before, the resolved images listed -- A/B knob)
    const bool unresolved = fuse && IPXG_FIN_PROBE;
    uint32_t n_keys = 0, n_touch = 0, n_list = 0;
    constexpr uint32_t EPT = NE / NT;  // LDS entries per thread
    HotSlot img[EPT];
    bool listed[EPT];
    bool failed = false;
    // fuse: the flows go on the finalise list as they are, unresolved -- k_fin_list probes the
    // table for them, one lane per flow at its occupancy, so the random slot reads of a 1M-flow
    // batch overlap there instead of stalling this LDS-bound workgroup (one per CU).  Otherwise
    // the thread's entries' home slots are read, and the empty ones claimed, together (one
    // memory round trip for all of them, not one chain per entry); a home slot held by another
    // key continues with the general probe.
    uint64_t hkey[EPT];
    unsigned long long old[EPT];
#pragma unroll
    for (uint32_t q = 0; q < EPT; ++q) {
        hkey[q] = ht[tid + q * NT].key;
        if (hkey[q] && !unresolved) img[q] = t.hot((uint32_t)hkey[q] & t.mask);
    }
#pragma unroll
    for (uint32_t q = 0; q < EPT; ++q) {
        old[q] = ~0ull;
        if (hkey[q] && !unresolved && img[q].key == 0)
            old[q] = atomicCAS((unsigned long long*)&t.hot((uint32_t)hkey[q] & t.mask).key, 0ull,
                               (unsigned long long)hkey[q]);
    }
#pragma unroll
    for (uint32_t q = 0; q < EPT; ++q) {
        const uint32_t e = tid + q * NT;
        FlowAgg a = ht[e];
        if (one_tb) a.tbits |= 1u;  // bucket 0 (lds_fold skipped the per-record OR)
        listed[q] = false;
        if (a.key && unresolved) {  // the aggregate as a slot image, its slot probed by k_fin_list
            n_touch++;
            HotSlot u = {};
            u.key = a.key;
            agg_fold(u, a);
            u.pad = FIN_UNRESOLVED;
            img[q] = u;
            listed[q] = true;
            n_list++;
        } else if (a.key) {
            n_touch++;
            bool claimed = false;
            HotSlot* hp = &t.hot((uint32_t)a.key & t.mask);  // this workgroup is the slot's only writer here
            if (img[q].key == a.key) {
                // found at home
            } else if (img[q].key == 0 && old[q] == 0) {
                img[q] = HotSlot{};
                img[q].key = a.key;
                claimed = true;
            } else if (img[q].key == 0 && old[q] == a.key) {
                img[q] = *hp;  // inserted meanwhile by another path
            } else {
                hp = probe_insert_full(t, a.key, img[q], claimed);
            }
            if (claimed) n_keys++;
            if (!hp) {
                ht[e].tflags = a.tflags | RED_FAILED;
                failed = true;
            } else {
                agg_fold(img[q], a);
                if (fuse) {  // the merged image goes to k_fin_list, which writes the slot back
                    img[q].pad = t.slot_index(hp);
                    listed[q] = true;
                    n_list++;
                } else {
                    *hp = img[q];
                }
            }
        }
    }
    // one reservation on the finalise list per workgroup (a single counter saturates at ~88
    // returning atomics per us: MI355X_MICROARCH.md "dequeue")
    uint32_t listed_n;
    uint32_t pos = block_exclusive_scan<NT>(n_list, scan_s, &listed_n);
    if (tid == 0) *fin_base = listed_n ? atomicAdd(&ctl->fin_count, listed_n) : 0;
    __syncthreads();
    pos += *fin_base;
#pragma unroll
    for (uint32_t q = 0; q < EPT; ++q)
        if (listed[q]) fin_list[pos++] = img[q];
    if (__any(failed) && (tid & 63) == 0) atomicOr(&cnt[C_FAIL], 1u);
    wave_add_lds(&cnt[C_KEYS], n_keys);
    wave_add_lds(&cnt[C_TOUCH], n_touch);
    __syncthreads();
    if (cnt[C_FAIL]) {  // defer the packets (and aggregates) of the flows that found no slot
        for (uint32_t k = tid; k < total; k += NT) {
            const uint4 r = rec_at(k);
            if (r.z == NO_REC || (rec_is_agg(r) && rec_agg_slot(r) != 0)) continue;
            const int e = lds_slot<NE>(ht, ((uint64_t)r.y << 32) | r.x, false);
            if (e < 0 || !(ht[e].tflags & RED_FAILED)) continue;
            if (rec_is_agg(r))  // its payload slots follow it in the same segment
                defer_agg(&ctl->agg_deferred, agg_list, r, rec_at(k + 1), rec_at(k + 2));
            else
                defer_packet(ctl, deferred_list, r.z, false);
        }
    }
    if (tid == 0) {
        if (cnt[C_KEYS]) atomicAdd(&ctl->new_keys, cnt[C_KEYS]);
        if (cnt[C_TOUCH]) atomicAdd(&ctl->touched, cnt[C_TOUCH]);
        if (cnt[C_SPILL]) atomicAdd(&ctl->spilled, cnt[C_SPILL]);
        if (!fuse || cnt[C_SPILL] || cnt[C_FAIL]) ctl->pending = 1;
    }
}

// One workgroup per partition: the partition's records sit in one segment per k_bin /
// k_bin_slow workgroup (bv.count gives their lengths); a prefix sum over the segment lengths
// in LDS maps the partition's record k to its segment.
__global__ __launch_bounds__(RED_THREADS) void k_reduce(TableView t, BinView bv, BatchCtl* ctl, HotSlot* fin_list,
                                                        uint32_t* deferred_list, uint4* agg_list, BatchCtl* zero_ctl,
                                                        uint32_t* zero_ex) {
    __shared__ FlowAgg ht[RED_ENTRIES];  // 112 KiB
    __shared__ uint32_t pre[RED_MAX_COLS + 1];
    __shared__ uint32_t ne[RED_MAX_COLS];  // non-empty segments
    __shared__ uint32_t cnt[C_N];
    __shared__ uint32_t scan_s[RED_THREADS / 64 + 1];
    __shared__ uint32_t fin_base;
    const uint32_t part = red_part(blockIdx.x, 1u << bv.part_bits);
    const uint32_t tid = threadIdx.x;
    if (blockIdx.x == 0) {  // the other control block for the next batch, the cleared export counters
        if (zero_ctl)
            for (uint32_t w = tid; w < sizeof(BatchCtl) / 4; w += RED_THREADS) reinterpret_cast<uint32_t*>(zero_ctl)[w] = 0;
        if (zero_ex && tid < 3) zero_ex[tid] = 0;
    }
    if (bv.slow_skip && ctl->slow_redo) return;  // slow packets without a slow pass: the host runs both again
    // the columns written: every k_bin workgroup's, and those of the k_bin_slow workgroups
    // that had slow packets (the others return without writing theirs)
    const uint32_t cols = bv.cols;

    PROBE_T(q0t);
    // segment lengths -> exclusive prefix (cols <= RED_MAX_COLS = 4 per thread)
    uint32_t v[RED_MAX_COLS / RED_THREADS], my = 0;
#pragma unroll
    for (uint32_t q = 0; q < RED_MAX_COLS / RED_THREADS; ++q) {
        const uint32_t c = tid * (RED_MAX_COLS / RED_THREADS) + q;
        v[q] = c < bv.bin_grid || (c < cols && slow_col_written(bv, c - bv.bin_grid)) ? bv.count[seg_count_idx(bv, part, c)] : 0;
        my += v[q];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan<RED_THREADS>(my, scan_s, &total);
    if (total == 0) return;  // uniform over the workgroup
    if (tid == 0) {  // the partition's load (segment sizing of the next batch)
        atomicMax(&ctl->max_part, total);
        atomicAdd(&ctl->total_slots, total);
    }
    uint32_t ne_n = 0;
#pragma unroll
    for (uint32_t q = 0; q < RED_MAX_COLS / RED_THREADS; ++q) {
        const uint32_t c = tid * (RED_MAX_COLS / RED_THREADS) + q;
        if (c < cols) pre[c] = run;
        run += v[q];
        ne_n += v[q] ? 1 : 0;
    }
    if (tid == 0) pre[cols] = total;
    // the non-empty segments, listed in column order
    uint32_t nseg;
    uint32_t at = block_exclusive_scan<RED_THREADS>(ne_n, scan_s, &nseg);
#pragma unroll
    for (uint32_t q = 0; q < RED_MAX_COLS / RED_THREADS; ++q)
        if (v[q]) ne[at++] = tid * (RED_MAX_COLS / RED_THREADS) + q;
    {
        uint4* z = reinterpret_cast<uint4*>(ht);
        for (uint32_t q = tid; q < sizeof(ht) / 16; q += RED_THREADS) z[q] = make_uint4(0, 0, 0, 0);
    }
    if (tid < C_N) cnt[tid] = 0;
    __syncthreads();
    PROBE_T(q1t);
    const uint4* segs = bv.rec + (size_t)part * bv.cols * bv.seg_cap;
    const bool one_tb = ctl->tb_any == 0;  // final: k_bin and k_bin_slow have completed
    const uint32_t lane = tid & 63, wave = tid >> 6;
    constexpr uint32_t NW = RED_THREADS / 64;
    if (total < nseg * 16) {
        // Short segments (many partitions and workgroups for the batch: ~2-5 records per
        // segment with 1M flows): a wave per segment would leave most lanes idle, so each
        // thread takes record k of the partition, found by a binary search over the segment
        // prefix in LDS (consecutive threads, consecutive records within a segment).
        for (uint32_t k0 = 0; k0 < total; k0 += RED_THREADS * RED_U) {
            uint4 r[RED_U];
            const uint4* rp[RED_U];
#pragma unroll
            for (uint32_t u = 0; u < RED_U; ++u) {
                const uint32_t k = k0 + u * RED_THREADS + tid;
                rp[u] = k < total ? seg_ptr(segs, pre, cols, bv.seg_cap, k) : segs;
                r[u] = *rp[u];
            }
#pragma unroll
            for (uint32_t u = 0; u < RED_U; ++u)
                red_record(ht, t, ctl, deferred_list, agg_list, cnt, r[u], rp[u], k0 + u * RED_THREADS + tid < total, one_tb);
        }
    } else {
        // Chunks of 64 records: a non-empty segment of len records gives ceil(len / 64) chunks,
        // listed in LDS as {column << 20 | chunk << 6 | records - 1} (ne[], in windows of
        // RED_MAX_COLS entries).  Waves take chunks wv, wv + NW, ... (lane = record of the chunk:
        // coalesced loads, no search).  A wave reads the descriptors of its next 64 chunks with
        // ONE LDS read (lane j: its j-th chunk) and walks them by v_readlane into SGPRs, so no
        // LDS round trip stands between a chunk and its loads; RED_U chunks per group, two groups
        // in flight (A/B) while the previous one is folded.  (Round 3 took whole segments: a
        // segment's records past the first 64 were loaded synchronously inside the fold, and the
        // segment's position came from two dependent LDS reads per group behind the other waves'
        // atomics -- with the udp64 partitions' ~76-record segments k_reduce waited on memory once
        // per segment.)
        const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);
        uint32_t nch = 0;
#pragma unroll
        for (uint32_t q = 0; q < RED_MAX_COLS / RED_THREADS; ++q) nch += (v[q] + 63) >> 6;
        uint32_t total_ch;
        const uint32_t cb0 = block_exclusive_scan<RED_THREADS>(nch, scan_s, &total_ch);
        for (uint32_t w0 = 0; w0 < total_ch; w0 += RED_MAX_COLS) {  // uniform
            __syncthreads();  // ne[] is free (the non-empty list above / the previous window)
            uint32_t at = cb0;
#pragma unroll
            for (uint32_t q = 0; q < RED_MAX_COLS / RED_THREADS; ++q) {
                const uint32_t c = tid * (RED_MAX_COLS / RED_THREADS) + q;
                for (uint32_t j = 0; j * 64 < v[q]; ++j, ++at)
                    if (at - w0 < RED_MAX_COLS) ne[at - w0] = (c << 20) | (j << 6) | (min(64u, v[q] - j * 64) - 1);
            }
            __syncthreads();
            const uint32_t nw = min(RED_MAX_COLS, total_ch - w0);
            for (uint32_t g = wv; g < nw; g += 64 * NW) {  // uniform over the wave
                const uint32_t mine = g + lane * NW;
                const uint32_t cd = mine < nw ? ne[mine] : 0u;
                const uint32_t left = (nw - g + NW - 1) / NW;
                const uint32_t ng = left < 64 ? left : 64;  // the wave's chunks in this group
                uint4 ra[RED_U], rb[RED_U];
                uint32_t ca[RED_U], cbk[RED_U];
                auto issue = [&](uint32_t j0, uint4(&r)[RED_U], uint32_t(&cs)[RED_U]) {
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u) {
                        const uint32_t j = j0 + u < ng ? j0 + u : 0;
                        cs[u] = __builtin_amdgcn_readlane(cd, j);
                    }
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u) {
                        const uint32_t n = (cs[u] & 63) + 1;
#ifndef IPXG_RED_NT  // streaming (non-temporal) record loads: each is read once (udp64 step -0.5 %, gpurun_out/r5rnt2)
#define IPXG_RED_NT 1
#endif
#if IPXG_RED_NT
                        {
                            typedef uint32_t rv4 __attribute__((ext_vector_type(4)));
                            const rv4 v = __builtin_nontemporal_load(reinterpret_cast<const rv4*>(
                                &segs[(size_t)(cs[u] >> 20) * bv.seg_cap + ((cs[u] >> 6) & 0x3FFF) * 64 +
                                      (lane < n ? lane : 0)]));
                            r[u] = make_uint4(v.x, v.y, v.z, v.w);
                        }
#else
                        r[u] = segs[(size_t)(cs[u] >> 20) * bv.seg_cap + ((cs[u] >> 6) & 0x3FFF) * 64 +
                                    (lane < n ? lane : 0)];  // unconditional load
#endif
                    }
                };
                auto fold = [&](const uint4(&r)[RED_U], const uint32_t(&cs)[RED_U], uint32_t j0) {
                    bool ok[RED_U];
                    uint32_t e[RED_U];
                    unsigned long long k[RED_U];
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u) {
                        ok[u] = j0 + u < ng && lane <= (cs[u] & 63) && r[u].z != NO_REC;
                        e[u] = r[u].x & (RED_ENTRIES - 1);
                    }
#ifdef IPXG_EXP_RED_NOFOLD  // timing experiment: the record loads without the fold
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u)
                        if (ok[u] && r[u].x == 0x9E3779B9u && r[u].y == 0x7F4A7C15u) atomicAdd(&cnt[C_FAIL], 1u);
                    return;
#endif
                    // the probes' first reads, issued together (no atomic of this group before them)
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u) k[u] = ok[u] && !rec_is_agg(r[u]) ? ht[e[u]].key : 0ull;
#pragma unroll
                    for (uint32_t u = 0; u < RED_U; ++u) {
                        if (!ok[u]) continue;
                        const uint4* rp = segs + (size_t)(cs[u] >> 20) * bv.seg_cap + ((cs[u] >> 6) & 0x3FFF) * 64 + lane;
                        if (rec_is_agg(r[u])) {
                            red_agg(ht, t, ctl, agg_list, cnt, r[u], rp);
                            continue;
                        }
                        const uint64_t lo = ((uint64_t)r[u].y << 32) | r[u].x;
                        const int slot = k[u] == lo ? (int)e[u] : red_probe(ht, lo, e[u], k[u]);
                        if (slot >= 0) lds_fold(ht[slot], r[u].z, r[u].w, one_tb);
                        else red_spill(t, ctl, deferred_list, cnt, r[u]);
                    }
                };
                issue(0, ra, ca);
                for (uint32_t j0 = 0; j0 < ng; j0 += 2 * RED_U) {  // uniform
                    issue(j0 + RED_U, rb, cbk);
                    fold(ra, ca, j0);
                    if (j0 + RED_U >= ng) break;
                    issue(j0 + 2 * RED_U, ra, ca);
                    fold(rb, cbk, j0 + RED_U);
                }
            }
        }
    }
    __syncthreads();
    PROBE_T(q2t);
    // Nothing else of this batch can touch these flows when no packet went to the fragment or
    // deferred paths (spilled packets were accumulated by k_bin, before this kernel): then the
    // merged slot is complete and goes on the finalise list (k_fin_list).
    const bool fuse = ctl->frag_count == 0 && ctl->a_deferred == 0;
    red_tail<RED_ENTRIES, RED_THREADS>(ht, t, ctl, fin_list, deferred_list, agg_list, cnt, scan_s, &fin_base, one_tb,
                                       fuse, total, [&](uint32_t k) { return seg_record(segs, pre, cols, bv.seg_cap, k); });
    PROBE_T(q3t);
#ifdef IPXG_PROBE
    if (tid == 0) {
        atomicAdd((unsigned long long*)&ctl->probe[4], (unsigned long long)(q1t - q0t));
        atomicAdd((unsigned long long*)&ctl->probe[5], (unsigned long long)(q2t - q1t));
        atomicAdd((unsigned long long*)&ctl->probe[6], (unsigned long long)(q3t - q2t));
    }
#endif
}

void launch_reduce(hipStream_t st, TableView t, BinView bv, BatchCtl* ctl, HotSlot* fin_list,
                   uint32_t* deferred_list, uint4* agg_list, BatchCtl* zero_ctl, uint32_t* zero_ex) {
    hipLaunchKernelGGL(k_reduce, dim3(1u << bv.part_bits), dim3(RED_THREADS), 0, st, t, bv, ctl, fin_list,
                       deferred_list, agg_list, zero_ctl, zero_ex);
}

// ---- the streamed reduce (line mode, round 6) --------------------------------------------------
// k_reduce's fold, run while k_bin produces the records: one workgroup per partition, launched
// beside k_bin on a stream of its own (k_bin then runs two workgroups per CU, this one the third
// resident workgroup of its CU).  Each round it polls the partition's progress word of every k_bin
// column (sc1 loads), folds the lines published since the previous round (sc1 loads of lines k_bin
// stored write-through moments before: Infinity-Cache hits, not a second HBM pass of the 160 MB of
// udp64 records), and sleeps when nothing is new.  Once every column is marked done -- k_bin
// released its control-block words before marking it -- the partition's flows are merged and listed
// exactly as k_reduce does (red_tail).  A slow pass flagged by k_bin (slow_redo) leaves everything to
// the host's rerun of k_bin_slow and k_reduce: nothing is written to the table before that check, and
// flows that found no LDS entry are only applied after it (a second pass over their records).
constexpr uint32_t RS_THREADS = 512;  // 2 waves per SIMD: beside two k_bin workgroups' (147 VGPRs each)
constexpr uint32_t RS_LIST = 1024;    // lines folded per poll, at most
constexpr uint32_t RS_U = 2;          // wave loads (8 lines each) in flight per lane
constexpr uint64_t RS_STALL_TICKS = 300000000ull;  // 3 s of the 100 MHz real-time clock without progress

__device__ __forceinline__ uint32_t rs_col(const uint32_t* pre, uint32_t G, uint32_t k) {  // the last c with pre[c] <= k
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = RS_MAX_COLS / 2; step; step >>= 1) {
        const uint32_t m = lo + step;
        lo = (m < G && pre[m] <= k) ? m : lo;
    }
    return lo;
}

__global__ __launch_bounds__(RS_THREADS) void k_reduce_stream(Params p, TableView t, BinView bv, BatchCtl* ctl,
                                                              HotSlot* fin_list, uint32_t* deferred_list,
                                                              uint4* agg_list) {
    if (gated(p)) return;  // (k_bin returned at once too: it publishes nothing)
    __shared__ FlowAgg ht[RS_ENTRIES];       // 56 KiB
    __shared__ uint32_t used[RS_MAX_COLS];   // lines of each column's segment folded
    __shared__ uint32_t list[RS_LIST + 1];   // this poll's lines (column << 20 | line); at the end the prefix
                                             // of the columns' records (G + 1 words)
    __shared__ uint32_t cnt[C_N];
    __shared__ uint32_t scan_s[RS_THREADS / 64 + 1];
    __shared__ uint32_t fin_base;
    __shared__ uint32_t flag[2];             // [0] the LDS table was full for some flow, [1] stalled
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t P = 1u << bv.part_bits, part = red_part(blockIdx.x, P);
    const uint32_t G = bv.bin_grid;  // (<= RS_MAX_COLS = RS_THREADS: the host)
    {
        uint4* z = reinterpret_cast<uint4*>(ht);
        for (uint32_t q = tid; q < sizeof(ht) / 16; q += RS_THREADS) z[q] = make_uint4(0, 0, 0, 0);
    }
    if (tid < G) used[tid] = 0;
    if (tid < C_N) cnt[tid] = 0;
    if (tid < 2) flag[tid] = 0;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(bv);
    const size_t seg0 = (size_t)part * bv.cols;  // segment of column c: seg0 + c
    const uint32_t* words = bv.prog + (size_t)part * RS_MAX_COLS;
    uint64_t t_prog = __builtin_amdgcn_s_memrealtime();
    constexpr uint32_t NW = RS_THREADS / 64;
    for (;;) {
        uint32_t avail = 0;
        bool done = true;
        if (tid < G) {
            const uint32_t v = __hip_atomic_load(&words[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool cur = (v & PROG_EPOCH_MASK) == bv.prog_tag;
            const uint32_t lines = cur ? (v & PROG_LINES) : 0u;
            avail = lines > used[tid] ? lines - used[tid] : 0u;
            done = cur && (v & PROG_DONE) != 0;
        }
        uint32_t tot;
        const uint32_t x = block_exclusive_scan<RS_THREADS>(avail, scan_s, &tot);
        const uint32_t take = x >= RS_LIST ? 0u : min(avail, RS_LIST - x);
        for (uint32_t j = 0; j < take; ++j) list[x + j] = (tid << 20) | (used[tid] + j);
        // (every column done and all of its lines listed: this poll's fold is the last)
        const bool all_done = __syncthreads_and(done && take == avail);
        const uint32_t nl = min(tot, RS_LIST);
        const uint32_t rs_exp = bv.rs_sleep >> 16;  // timing experiments (IPXG_RS_EXP): 1 no fold, 2 no loads
        for (uint32_t g0 = (tid >> 6) * 8; g0 < (rs_exp == 2 ? 0u : nl); g0 += NW * 8 * RS_U) {  // uniform over the wave
            uint4 r[RS_U];
#pragma unroll
            for (uint32_t u = 0; u < RS_U; ++u) {
                const uint32_t li = g0 + u * NW * 8 + (lane >> 3);
                uint32_t off = BUF_OOB;
                if (li < nl) {
                    const uint32_t e = list[li];
                    off = (uint32_t)(((seg0 + (e >> 20)) * bv.seg_cap + (e & 0xFFFFFu) * 8u + (lane & 7)) * 16u);
                }
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX_SC1);
                r[u] = make_uint4(v.x, v.y, li < nl ? v.z : NO_REC, v.w);
            }
#pragma unroll
            for (uint32_t u = 0; u < RS_U; ++u) {
                if (r[u].z == NO_REC) continue;
                if (rs_exp == 1) {
                    if (r[u].x == 0x12345678u) flag[0] = 1;
                    continue;
                }
                const int e = lds_slot<RS_ENTRIES>(ht, ((uint64_t)r[u].y << 32) | r[u].x, true);
                if (e >= 0) lds_fold(ht[e], r[u].z, r[u].w, false);
                else flag[0] = 1;  // (applied after the slow_redo check, below)
            }
        }
        __syncthreads();
        if (tid < G) used[tid] += take;
        if (all_done) break;
        if (nl == 0) {
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (tid == 0 && now - t_prog > RS_STALL_TICKS) flag[1] = 1;
            for (uint32_t k = 0; k < (bv.rs_sleep & 0xFFFFu); ++k) __builtin_amdgcn_s_sleep(64);
        } else {
            t_prog = __builtin_amdgcn_s_memrealtime();
        }
        __syncthreads();
        if (flag[1]) {  // k_bin stopped publishing (a fault would end the kernel): reported, nothing merged
            if (tid == 0) atomicOr(&ctl->guard, GUARD_STREAM_STALL);
            return;
        }
    }
    // every column done: k_bin's control-block words are final
    if (bv.slow_skip && __hip_atomic_load(&ctl->slow_redo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    uint32_t total;
    {
        const uint32_t mine = tid < G ? used[tid] * 8u : 0u;
        const uint32_t x = block_exclusive_scan<RS_THREADS>(mine, scan_s, &total);
        if (tid < G) list[tid] = x;
        __syncthreads();
    }
    if (total == 0) return;  // (uniform)
    if (tid == 0) {  // the partition's load (segment sizing of the next batch)
        atomicMax(&ctl->max_part, total);
        atomicAdd(&ctl->total_slots, total);
    }
    auto rec_at = [&](uint32_t k) {
        const uint32_t c = rs_col(list, G, k);
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
            rs, (uint32_t)(((seg0 + c) * bv.seg_cap + (k - list[c])) * 16u), 0, AUX_SC1);
        return make_uint4(v.x, v.y, v.z, v.w);
    };
    if (flag[0]) {  // flows that found no LDS entry: their records straight into the table
        for (uint32_t k = tid; k < total; k += RS_THREADS) {
            const uint4 r = rec_at(k);
            if (r.z == NO_REC || lds_slot<RS_ENTRIES>(ht, ((uint64_t)r.y << 32) | r.x, false) >= 0) continue;
            red_spill(t, ctl, deferred_list, cnt, r);
        }
        __syncthreads();
    }
    const bool fuse = __hip_atomic_load(&ctl->frag_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                      __hip_atomic_load(&ctl->a_deferred, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    red_tail<RS_ENTRIES, RS_THREADS>(ht, t, ctl, fin_list, deferred_list, agg_list, cnt, scan_s, &fin_base, false, fuse,
                                     total, rec_at);
}

void launch_reduce_stream(hipStream_t st, const Params& p, TableView t, BinView bv, BatchCtl* ctl, HotSlot* fin_list,
                          uint32_t* deferred_list, uint4* agg_list) {
    hipLaunchKernelGGL(k_reduce_stream, dim3(1u << bv.part_bits), dim3(RS_THREADS), 0, st, p, t, bv, ctl, fin_list,
                       deferred_list, agg_list);
}

// ---- finalisation of the flows k_reduce completed -----------------------------------------
// One lane per listed slot: finalize_slot with the creator's headers staged in the lane's
// LDS column (256-thread blocks keep the register budget of the general parser).
// finishing (ipxg_finish right behind an asynchronous submit into an empty table): when
// nothing of the batch needs the host (no fragments, deferrals or scan), every flow this
// kernel completes is exported as FORCED and its slot emptied here -- the finish's export
// folded into the finalise pass, so no table scan (k_finish) follows.  Flows it marks complex
// stay; the host then runs the sequential path and a k_finish for them (ctl->fused tells it).
// An unresolved entry (k_reduce's fuse mode) is probed here: its slot found or claimed
// (probe_insert_full), the aggregate folded into the slot's image; a probe that fails (a table
// full near the slot) marks the entry FIN_DEFERRED and counts it in ctl->fin_deferred -- the host
// grows the table and runs this kernel again over those entries only (deferred_only), not
// finishing.
// Workgroups of FIN_THREADS (a multiple of 256: each lane's LDS column lies in the window of its
// 256-lane group, stage_frame's column stride).  Round 6: a timing build without the export-slot
// reservation (a returning atomic per workgroup and pass) and the control-block counts took udp64's
// k_fin_list from 26 to 20.5 us; 768-thread workgroups (one per CU at 168 VGPRs), a third of the
// reservations, moved nothing on udp64 and cost quic +9 %, imix +8 % (more passes per workgroup) --
// the reservation's cost is its round trip in every pass, not the count (profiles/r06/fin_ab.txt).
#ifndef IPXG_FIN_THREADS
#define IPXG_FIN_THREADS 256
#endif
constexpr uint32_t FIN_THREADS = IPXG_FIN_THREADS;
static_assert(FIN_THREADS % IPXG_BLOCK == 0 && FIN_THREADS <= 1024, "k_fin_list workgroup");
#ifndef IPXG_FIN_WAVES  // tuning knob: k_fin_list's waves per SIMD (register budget)
#define IPXG_FIN_WAVES (FIN_THREADS >= 1024 ? 4 : FIN_THREADS >= 512 ? FIN_THREADS / 256 : 3)
#endif
__global__ __launch_bounds__(FIN_THREADS) __attribute__((amdgpu_waves_per_eu(IPXG_FIN_WAVES))) void k_fin_list(BatchView b, Params p, TableView t, FragView f,
                                                         ExportView ex, BatchCtl* ctl, HotSlot* fin_list,
                                                         unsigned long long* stats, uint32_t finishing,
                                                         uint32_t deferred_only, uint32_t ex_start) {
    __shared__ uint32_t win[IPXG_WIN_DW * FIN_THREADS];
    __shared__ uint32_t sc[ST_COUNT];
    __shared__ uint32_t cnt[7];  // new live, complex, exported, IPv6 exports, new keys, deferred, export holes
    __shared__ uint32_t scan_s[FIN_THREADS / 64 + 1];
    __shared__ uint32_t ex_base;
    if (p.slow_skip && ctl->slow_redo) return;  // (k_reduce returned too; `fused` stays 0)
    const uint32_t nf = ctl->fin_count;  // final: k_reduce has completed
    const bool fused = finishing && !(ctl->frag_count || ctl->deferred || ctl->agg_deferred || ctl->pending);
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl->fused = fused ? 1u : 0u;
    if (blockIdx.x * FIN_THREADS >= nf) return;
    const uint32_t tid = threadIdx.x;
    if (tid < ST_COUNT) sc[tid] = 0;
    if (tid < 7) cnt[tid] = 0;
    __syncthreads();
    const bool force_cx = p.force_complex || ctl->nonmono;
    const bool slot_clean = ctl->spilled == 0;  // no packet was folded into a slot directly (k_bin / k_reduce)
    // In list order (a fused finish with ex_start != EX_START_NONE): each listed flow exports at most
    // one record, so list entry k's export goes to record ex_start + k -- no reservation, which cost a
    // returning atomic on the one counter per workgroup and pass, waited for before the stores (udp64
    // k_fin_list 26 -> 20.5 us without it, profiles/r06/fin_ab.txt).  ex_start is the export count the
    // host knows when nothing else appends before this kernel; workgroup 0 checks it against the
    // counter (GUARD_EX_START) and sets the counter to ex_start + nf at its end (no other workgroup
    // reads it).  Entries that do not export -- flows that turn complex or find no slot -- leave their
    // records as holes (zeroed: end reason 0) counted in ctl->ex_holes; those flows send the batch to
    // the host, which closes the holes (k_ex_compact) before it reads the exports.
    const bool lorder = fused && !deferred_only && ex_start != EX_START_NONE;
    uint32_t n_holes = 0;
    if (lorder && blockIdx.x == 0 && tid == 0 && *ex.count != ex_start) atomicOr(&ctl->guard, GUARD_EX_START);
    // the batch's latest second: its last packet's, when no timestamp went backwards (else every
    // flow is complex anyway, force_cx)
    const uint32_t tmax = force_cx || b.n == 0 ? TMAX_UNKNOWN : b.desc[b.n - 1].ts_sec;
    uint32_t n_live = 0, n_cx = 0, n_ex = 0, n_v6 = 0, n_keys = 0, n_def = 0;
#ifdef IPXG_PROBE  // k_fin_list [12] list image + slot probe, [13] finalize_slot, [14] export reservation + stores,
                   // [15] statistics and control-block counts (workgroup 0's thread 0 ... each workgroup's)
    uint64_t probe_acc[4] = {0, 0, 0, 0};
#endif
    uint32_t* const col = &win[(tid / IPXG_BLOCK) * (IPXG_WIN_DW * IPXG_BLOCK) + tid % IPXG_BLOCK];  // (the lane's LDS column)
    for (uint32_t base = blockIdx.x * FIN_THREADS; base < nf; base += gridDim.x * FIN_THREADS) {  // block-uniform
        PROBE_T(f0);
        const uint32_t k = base + tid;
        bool do_export = false;  // er is exported with `reason` (a boundary split, or the fused finish)
        uint8_t reason = 0;
        RecW er;
        HotSlot h;
        bool go = k < nf;
        if (go) {
            h = fin_list[k];  // the slot's merged image and its index in pad, or an unresolved aggregate
            if (deferred_only) go = h.pad == FIN_DEFERRED;
            else if (h.pad == FIN_DEFERRED) go = false;  // (not from this batch's k_reduce)
        }
        // fused finish into a table that was empty before the batch: a new flow is created and
        // exported here, so it needs no slot -- no probe, no claim (two dependent round trips
        // per flow), unless it turns out complex (claimed below)
        const bool no_slot = go && fused && !deferred_only && !p.classify && h.pad >= FIN_DEFERRED;
        if (no_slot) h.pad = FIN_NO_SLOT;
        if (go && !no_slot && h.pad >= FIN_DEFERRED) {
            FlowAgg a;
            a.key = h.key;
            a.acc[0] = h.acc[0];
            a.acc[1] = h.acc[1];
            a.first_n = h.first_n;
            a.last1 = h.last1;
            a.tbits = h.tbits;
            a.tflags = h.tflags;
            a.fin_n[0] = h.fin_n[0];
            a.fin_n[1] = h.fin_n[1];
            a.syn1[0] = h.syn1[0];
            a.syn1[1] = h.syn1[1];
            HotSlot img;
            bool claimed;
            HotSlot* hp = probe_insert_full(t, a.key, img, claimed);
            if (!hp) {  // the table is full near its slot: after a rehash, again
                fin_list[k].pad = FIN_DEFERRED;
                n_def++;
                go = false;
            } else {
                n_keys += claimed ? 1u : 0u;
                agg_fold(img, a);
                img.pad = t.slot_index(hp);
                h = img;
                if (deferred_only) fin_list[k].pad = FIN_UNRESOLVED;  // done: later re-runs skip it
            }
        }
        PROBE_T(f1);
        PROBE_ADD(0, f0, f1);
        if (go) {
            const FinResult fr = finalize_slot<true>(b, p, t, f, h.pad, h, force_cx, col, er, fused, slot_clean, tmax);
            if (fr.status == FIN_COMPLEX && no_slot) {  // a complex flow: its slot now, for the sequential path
                HotSlot img;
                bool claimed;
                HotSlot* hp = probe_insert_full(t, h.key, img, claimed);
                if (!hp) {  // (the host grows the table and runs the list again: deferred_only)
                    fin_list[k].pad = FIN_DEFERRED;
                    n_def++;
                } else {
                    n_keys += claimed ? 1u : 0u;
                    HotSlot c = h;  // (a slot empty before the batch: the image is the whole slot)
                    c.state = h.state | SLOT_COMPLEX;
                    c.pad = 0;
                    *hp = c;
                    n_cx++;
                }
            } else if (fr.status == FIN_COMPLEX) n_cx++;
            else if (!fused && fr.created) n_live++;
            do_export = fr.do_export || fr.fin_export;
            reason = fr.fin_export ? (uint8_t)IPXG_FLOW_END_FORCED : fr.reason;
        }
        PROBE_T(f2);
        PROBE_ADD(1, f1, f2);
        // one reservation in the export buffer per workgroup and pass (a returning atomic per
        // wave on the one counter serialised ~1600 waves at ~12 ns each: MI355X_MICROARCH.md
        // "fanin" / "dequeue")
        if (lorder) {  // uniform
            if (k < nf) {
                if (do_export) {
                    store_export_w(ex, ex_start + k, er, reason);
                    n_ex++;
                    n_v6 += rw_ipver(er) == 6 ? 1 : 0;
                } else {
                    store_export_hole(ex, ex_start + k);
                    n_holes++;
                }
            }
            count_exports_wave(sc, do_export, er, reason);
            PROBE_T(f3x);
            PROBE_ADD(2, f2, f3x);
            continue;
        }
        uint32_t btot;
        const uint32_t pos = block_exclusive_scan<FIN_THREADS>(do_export ? 1u : 0u, scan_s, &btot);
        if (btot == 0) continue;  // uniform
#if defined(IPXG_EXP_FIN) && IPXG_EXP_FIN == 2  // timing experiment only: no export reservation (positions wrong)
        if (tid == 0) ex_base = base;
#else
        if (tid == 0) ex_base = atomicAdd(ex.count, btot);
#endif
        __syncthreads();
        if (do_export) {
            store_export_w(ex, ex_base + pos, er, reason);
            n_ex++;
            n_v6 += rw_ipver(er) == 6 ? 1 : 0;
        }
        count_exports_wave(sc, do_export, er, reason);
        __syncthreads();  // ex_base is rewritten by the next pass
        PROBE_T(f3);
        PROBE_ADD(2, f2, f3);
    }
    PROBE_T(f4);
    wave_add_lds(&cnt[0], n_live);
    wave_add_lds(&cnt[1], n_cx);
    wave_add_lds(&cnt[2], n_ex);
    wave_add_lds(&cnt[3], n_v6);
    wave_add_lds(&cnt[4], n_keys);
    wave_add_lds(&cnt[5], n_def);
    wave_add_lds(&cnt[6], n_holes);
#if defined(IPXG_EXP_FIN) && IPXG_EXP_FIN >= 1  // timing experiment only: no statistics / control-block counts
    return;
#endif
    flush_block_stats(sc, stats);
    if (tid == 0) {
        if (cnt[3] && ex.count6) atomicAdd(ex.count + 2, cnt[3]);  // count_v6_exports' counter
        if (cnt[0]) atomicAdd(&ctl->new_live, cnt[0]);
        if (cnt[1]) atomicAdd(&ctl->complex_count, cnt[1]);
        // (a fused finish's exports are counted by nothing but the export counter: no guarded
        // k_finish / k_expire follows it -- the one contended control-block word per workgroup saved)
        if (cnt[2] && !lorder) atomicAdd(&ctl->exported, cnt[2]);
        if (cnt[4]) atomicAdd(&ctl->new_keys, cnt[4]);
        if (cnt[6]) atomicAdd(&ctl->ex_holes, cnt[6]);
        if (lorder && blockIdx.x == 0) *ex.count = ex_start + nf;  // (workgroup 0 has list entries: nf > 0)
        if (cnt[5]) atomicAdd(&ctl->fin_deferred, cnt[5]);
    }
#ifdef IPXG_PROBE
    PROBE_T(f5);
    PROBE_ADD(3, f4, f5);
    if (tid == 0)
        for (int k = 0; k < 4; ++k) atomicAdd((unsigned long long*)&ctl->probe[12 + k], (unsigned long long)probe_acc[k]);
#endif
}

void launch_fin_list(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, ExportView ex,
                     BatchCtl* ctl, HotSlot* fin_list, unsigned long long* stats, uint32_t max_n,
                     bool finishing, bool deferred_only, uint32_t ex_start) {
    // at most one wave of resident workgroups (3 per CU): a grid past it ran its last blocks'
    // several passes over the list in a second wave on a third of the chip
    // (per device, computed once; engines on several devices or threads share the cache: relaxed
    // atomics, every writer stores the same value for its device)
    static std::atomic<uint32_t> resident_of[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::atomic<uint32_t>& slot = resident_of[dev & 63];
    uint32_t resident = slot.load(std::memory_order_relaxed);
    if (!resident) {
        int cus = 0, per_cu = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_fin_list, FIN_THREADS, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        resident = (uint32_t)std::max(1, cus * per_cu);
        slot.store(resident, std::memory_order_relaxed);
    }
    uint32_t grid = (max_n + FIN_THREADS - 1) / FIN_THREADS;
    if (grid > resident) grid = resident;
    hipLaunchKernelGGL(k_fin_list, dim3(grid ? grid : 1), dim3(FIN_THREADS), 0, st, b, p, t, f, ex, ctl, fin_list,
                       stats, finishing ? 1u : 0u, deferred_only ? 1u : 0u, ex_start);
}

// ---- complex flows: their packets ----------------------------------------------------------
// Every packet of the batch is parsed again to find the complex flows' packets (k_complex_rank
// has put their keys in cx.keys) and listed in its flow's segment.  Frames of the shapes k_bin's
// wide walk takes go through the same register parser (80-byte head by buffer loads); the rest
// through the general parser -- the gather used to parse every frame with the general LDS
// parser, twice k_bin's time per batch on the configs[2] mix with its plugins registered.
// Packet i parsed as the gather needs it (the wide register walk, else the general parser in the
// lane's LDS column), its canonical key in lo; false: no IP flow key.
__device__ __forceinline__ bool gather_key(const BatchView& b, const Params& p, const FragView& f,
                                           __amdgpu_buffer_rsrc_t rs_desc, __amdgpu_buffer_rsrc_t rs_arena,
                                           uint32_t* col, uint32_t i, uint64_t& lo) {
    const bool eth = p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB;
    const ipxg_pkt_desc d = load_desc(rs_desc, i);
    DevPkt pk;
    ParseCounts c = {};
    bool ok = false;
    const bool reg = eth && fast_shape(b, d) && frame_off(b, d) + 80u <= b.arena_len;
    if (reg) {
        const Head<5> h = load_head_at<5>(b, rs_arena, d);
        uint32_t w[WIDE_DW];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            w[4 * k] = h.c[k].x;
            w[4 * k + 1] = h.c[k].y;
            w[4 * k + 2] = h.c[k].z;
            w[4 * k + 3] = h.c[k].w;
        }
        bool ext = false;
        ok = parse_medium(w, d.caplen, p.frag_enable, pk, c, ext);
    }
    if (!ok) {
        DevPkt q;
        stage_frame(col, frame_ptr(b, d), d.caplen);
        LdsFrame S{{col, {frame_ptr(b, d), d.caplen}}};
        if (!parse_frame<false>(S, d.caplen, p.dlt, q, c)) return false;
        pk = q;
    }
    if (pk.ip_version != 4 && pk.ip_version != 6) return false;
    if (p.frag_enable && (pk.frag_off || pk.more_fragments)) apply_frag_ports(p, f, i, pk);
    uint64_t hf;
    uint32_t cdir;
    canon<false>(pk, p, lo, cdir, hf);
    return true;
}

__device__ __forceinline__ void gather_append(const ComplexView& cx, BatchCtl* ctl, uint32_t r, uint32_t i) {
    const uint32_t pos = atomicAdd(&cx.cursor[r], 1u);
    if (pos < cx.len[r]) cx.list[cx.seg[r] + pos] = ((uint64_t)r << 24) | i;
    else atomicOr(&ctl->guard, 2u);  // more packets than the flow's slot counted (guard)
}

__global__ __launch_bounds__(IPXG_BLOCK) void k_complex_gather(BatchView b, Params p, FragView f, ComplexView cx,
                                                               BatchCtl* ctl) {
    __shared__ uint32_t win[IPXG_WIN_DW * IPXG_BLOCK];
    uint32_t* col = &win[threadIdx.x];
    const __amdgpu_buffer_rsrc_t rs_desc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<ipxg_pkt_desc*>(b.desc), 0, (int)(b.n * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    for (uint32_t i = blockIdx.x * IPXG_BLOCK + threadIdx.x; i < b.n; i += gridDim.x * IPXG_BLOCK) {
        uint64_t lo;
        if (!gather_key(b, p, f, rs_desc, rs_arena, col, i, lo)) continue;
        const int64_t rr = complex_rank_of(cx, lo);
        if (rr >= 0) gather_append(cx, ctl, (uint32_t)rr, i);
    }
}

// Would k_bin's walk for this batch (p.wide, p.tile_agg: the variant it ran) have taken packet d
// in registers?  pk: the parse when it would.  (A frame it left to k_bin_slow was never in one of
// its tile aggregates.)
__device__ __forceinline__ bool kbin_takes(const BatchView& b, const Params& p, __amdgpu_buffer_rsrc_t rs_arena,
                                           const ipxg_pkt_desc& d, DevPkt& pk) {
    const bool fast_ok = p.dlt == 0 || p.dlt == IPXG_DLT_EN10MB;
    if (!(fast_ok && fast_shape(b, d))) return false;
    ParseCounts c = {};
    bool ext = false;
    if (!p.wide) {
        const Head<3> h = load_head_at<3>(b, rs_arena, d);
        return parse_fast(h.c[0], h.c[1], h.c[2], d.caplen, p.frag_enable, pk, c);
    }
    if (p.tile_agg) {
        const Head<WIDE_DW / 4> h = load_head_at<WIDE_DW / 4>(b, rs_arena, d);
        uint32_t w[WIDE_DW];
#pragma unroll
        for (int k = 0; k < WIDE_DW / 4; ++k) {
            w[4 * k] = h.c[k].x;
            w[4 * k + 1] = h.c[k].y;
            w[4 * k + 2] = h.c[k].z;
            w[4 * k + 3] = h.c[k].w;
        }
        return parse_medium<false, WIDE_DW>(w, d.caplen, p.frag_enable, pk, c, ext);
    }
    const Head<WIDE2_DW / 4> h = load_head_at<WIDE2_DW / 4>(b, rs_arena, d);
    uint32_t w[WIDE2_DW];
#pragma unroll
    for (int k = 0; k < WIDE2_DW / 4; ++k) {
        w[4 * k] = h.c[k].x;
        w[4 * k + 1] = h.c[k].y;
        w[4 * k + 2] = h.c[k].z;
        w[4 * k + 3] = h.c[k].w;
    }
    return parse_medium<false, WIDE2_DW>(w, d.caplen, p.frag_enable, pk, c, ext);
}

// The packets k_bin folded into tile aggregates of complex flows (k_complex_gather_rec lists each
// such aggregate's flow key and index range, which lies inside one k_bin tile): only those ranges
// are parsed again, a workgroup per range, and a packet is taken when k_bin's walk took it and it
// is the aggregate's flow's -- inside its tile a flow's register-walk packets are either all in
// its aggregate or all plain records (and its slow-path packets are k_bin_slow's records), so none
// is gathered twice.
__global__ __launch_bounds__(IPXG_BLOCK) void k_complex_gather_ranges(BatchView b, Params p, FragView f,
                                                                      ComplexView cx, BatchCtl* ctl,
                                                                      const uint4* ranges, uint32_t nr) {
    (void)f;
    const __amdgpu_buffer_rsrc_t rs_desc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<ipxg_pkt_desc*>(b.desc), 0, (int)(b.n * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_arena = arena_rsrc(b);
    for (uint32_t q = blockIdx.x; q < nr; q += gridDim.x) {  // (block-uniform)
        const uint4 rg = ranges[q];
        const uint64_t key = ((uint64_t)rg.y << 32) | rg.x;
        const int64_t rr = complex_rank_of(cx, key);
        if (rr < 0) continue;
        const uint32_t last = min(rg.w, b.n - 1);
        for (uint32_t i = rg.z + threadIdx.x; i <= last; i += IPXG_BLOCK) {
            DevPkt pk;
            if (!kbin_takes(b, p, rs_arena, load_desc(rs_desc, i), pk)) continue;
            if (pk.ip_version != 4 && pk.ip_version != 6) continue;
            uint64_t lo, hf;
            uint32_t cdir;
            canon<false>(pk, p, lo, cdir, hf);
            if (lo == key) gather_append(cx, ctl, (uint32_t)rr, i);
        }
    }
}

void launch_complex_gather_ranges(hipStream_t st, const BatchView& b, const Params& p, FragView f, ComplexView cx,
                                  BatchCtl* ctl, const uint4* ranges, uint32_t nr) {
    uint32_t g = nr < 4096 ? nr : 4096;
    hipLaunchKernelGGL(k_complex_gather_ranges, dim3(g ? g : 1), dim3(IPXG_BLOCK), 0, st, b, p, f, cx, ctl, ranges, nr);
}

void launch_complex_gather(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                           ComplexView cx, BatchCtl* ctl) {
    (void)t;
    uint32_t g = (b.n + IPXG_BLOCK - 1) / IPXG_BLOCK;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_complex_gather, dim3(g ? g : 1), dim3(IPXG_BLOCK), 0, st, b, p, f, cx, ctl);
}

// The complex flows' packets from the batch's partition records instead of the frames: 16 bytes
// per packet read, no parse (the re-parse gather reads every frame head and parses it).  A
// workgroup per 256 segments (a k_bin / k_bin_slow workgroup's records of one partition: a few
// records each on the 1M-flow mixes): their lengths scanned in LDS, then a thread per record,
// found by a binary search over the prefix -- consecutive threads read consecutive records.
// (Round 4 first ran a thread per segment: a lane walked its segment alone, every load of a wave
// touched 64 lines -- 0.37 ms per 10M-packet configs[2] batch.)  A complex flow with packets
// folded into a tile aggregate (no per-packet index left) lists the aggregate's range or flags
// the batch for the re-parse gather.
__global__ __launch_bounds__(256) void k_complex_gather_rec(BinView bv, ComplexView cx, BatchCtl* ctl, uint32_t nseg,
                                                           uint4* ranges, uint32_t range_cap) {
    __shared__ uint32_t pre[257];
    __shared__ uint32_t scan_s[256 / 64 + 1];
    for (uint32_t s0 = blockIdx.x * 256; s0 < nseg; s0 += gridDim.x * 256) {  // block-uniform
        const uint32_t s = s0 + threadIdx.x;
        uint32_t n = 0;
        if (s < nseg) {
            const uint32_t c = s % bv.cols;
            if (c < bv.bin_grid || slow_col_written(bv, c - bv.bin_grid)) n = bv.count[seg_count_idx(bv, s / bv.cols, c)];  // (else a k_bin_slow column left unwritten)
        }
        uint32_t tot;
        const uint32_t at = block_exclusive_scan<256>(n, scan_s, &tot);
        pre[threadIdx.x] = at;
        if (threadIdx.x == 0) pre[256] = tot;
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < tot; k += 256) {
            uint32_t lo = 0, hi = 256;  // pre[lo] <= k < pre[hi]: lo = the segment holding record k
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (pre[mid] <= k) lo = mid;
                else hi = mid;
            }
            const uint32_t ss = s0 + lo, j = k - pre[lo], sn = pre[lo + 1] - pre[lo];
            const uint32_t c = ss % bv.cols;
            const uint4* seg = bv.rec + (size_t)ss * bv.seg_cap;
            const uint4 r = seg[j];
            if (r.z == NO_REC) continue;
            if (rec_is_agg(r)) {
                if (rec_agg_slot(r) == 0 && complex_rank_of(cx, ((uint64_t)r.y << 32) | r.x) >= 0) {
                    // a k_bin aggregate (its packets inside one tile): its range is parsed again
                    // (k_complex_gather_ranges); k_bin_slow's span tiles: the whole batch then
                    uint32_t q = c < bv.bin_grid && j + 2 < sn ? atomicAdd(&ctl->cx_ranges, 1u) : range_cap;
                    if (q < range_cap) {
                        const FlowAgg a = agg_decode(r, seg[j + 1], seg[j + 2]);
                        ranges[q] = make_uint4(r.x, r.y, first_idx(a.first_n), a.last1 - 1);
                    } else {
                        atomicOr(&ctl->cx_agg, 1u);
                    }
                }
                continue;
            }
            const int64_t rr = complex_rank_of(cx, ((uint64_t)r.y << 32) | r.x);
            if (rr < 0) continue;
            const uint32_t rk = (uint32_t)rr;
            const uint32_t pos = atomicAdd(&cx.cursor[rk], 1u);
            if (pos < cx.len[rk]) cx.list[cx.seg[rk] + pos] = ((uint64_t)rk << 24) | (r.z & 0xFFFFFFu);
            else atomicOr(&ctl->guard, 2u);
        }
        __syncthreads();  // (pre is rewritten by the next group)
    }
}

void launch_complex_gather_rec(hipStream_t st, const BinView& bv, ComplexView cx, BatchCtl* ctl, uint4* ranges,
                               uint32_t range_cap) {
    const uint32_t nseg = (1u << bv.part_bits) * bv.cols;
    uint32_t g = (nseg + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_complex_gather_rec, dim3(g ? g : 1), dim3(256), 0, st, bv, cx, ctl, nseg, ranges, range_cap);
}

}  // namespace ipxg
