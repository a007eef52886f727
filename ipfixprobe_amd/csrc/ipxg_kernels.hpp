// ipxg_kernels.hpp -- device data layout shared by the kernels and the host engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ipxg.h"

namespace ipxg {

// One flow-table slot's hot half: the 64-byte line every packet of the flow touches.
// All-zero == empty and "no packets this batch", so the table is cleared by a memset.
// Per-batch accumulators are folded into the cold record by k_finalize and re-zeroed.
struct alignas(64) HotSlot {
    uint64_t key;      // 0  canonical flow hash: min(XXH64(key), XXH64(key_inv)); 0 = empty
    uint32_t first_n;  // 8  the batch's first packet of the flow, max-reduced: first_key(); 0 = none
    uint32_t tbits;    // 12 occupancy of (inactive/2)-second buckets since the batch start,
                       //    bit 31 = beyond bucket 30
    uint64_t acc[2];   // 16 per canonical direction: packets << 40 | IP bytes
    uint32_t last1;    // 32 last packet index in this batch + 1, max-reduced; 0 = untouched
    uint32_t tflags;   // 36 OR of TCP flags, canonical dir 0 in bits 0-7, dir 1 in bits 8-15
    uint32_t fin_n[2]; // 40 ~(first FIN|RST packet index) per direction, max-reduced
    uint32_t syn1[2];  // 48 last SYN packet index + 1 per direction, max-reduced
    uint32_t state;    // 56 SLOT_LIVE | SLOT_COMPLEX
    uint32_t pad;      // 60 (a finalise-list image: the slot's index)
};
static_assert(sizeof(HotSlot) == 64, "hot slot must be one 64-byte line");

constexpr uint32_t SLOT_LIVE = 1u, SLOT_COMPLEX = 2u;
constexpr uint32_t SLOT_PLUGIN = 4u;  // a process plugin's packet in this batch: replayed on the host
constexpr uint32_t SLOT_FOLLOW = 8u;  // a plugin follows every packet of the flow (ipxg_plugin.follow_packets):
                                      // replayed on the host in every batch until the host walk drops it
constexpr uint32_t SLOT_HOST = SLOT_PLUGIN | SLOT_FOLLOW;
constexpr uint64_t ACC_BYTES_MASK = (1ull << 40) - 1;
constexpr uint32_t MAX_PROBE = 64;

// Per-batch control block, zeroed before every batch.
struct BatchCtl {
    uint32_t nonmono;        // a packet's timestamp went backwards
    uint32_t frag_count;     // fragments routed to the fragmentation-cache path
    uint32_t deferred;       // packets whose table probe exceeded MAX_PROBE (list length)
    uint32_t a_deferred;     //   of which deferred by k_bin (read by k_reduce)
    uint64_t cx_alloc;       // (rank << 32) | packets, complex-flow segment allocator
    uint32_t complex_count;  // flows handed to the sequential path
    uint32_t pending;        // touched slots left for the k_finalize scan
    uint32_t keys;           // non-empty slots (k_finalize / k_count scans)
    uint32_t live;           // live records (k_finalize / k_count scans)
    uint32_t new_keys;       // slots claimed during this batch
    uint32_t new_live;       // records created on a non-live slot by k_reduce
    uint32_t cx_new_live;    // ... by k_complex_walk
    uint32_t last_sec, last_usec;  // timestamp of the batch's last packet
    uint32_t exported;       // records exported while applying this batch
    uint32_t touched;        // flow aggregates built by k_reduce (partition sizing)
    uint32_t spilled;        // packets that fell back to direct atomic accumulation
    uint32_t slow_count;     // packets k_bin left for k_bin_slow (statistics)
    uint32_t fin_count;      // slots k_reduce listed for k_fin_list
    uint32_t hold;           // set by a guarded k_finish that did not run (see k_finish)
    uint32_t agg_deferred;   // tile aggregates whose table probe failed (3-slot list length)
    uint32_t max_part;       // most record slots in one partition (segment sizing, k_reduce)
    uint32_t total_slots;    // record slots over all partitions (k_reduce)
    uint32_t agg_packets;    // packets folded into tile aggregates (k_bin / k_bin_slow)
    uint32_t walked;         // wide walk: packets of its extra shapes (variant choice)
    uint32_t fused;          // k_fin_list exported and emptied the flows it finalised (finish fused)
    uint32_t plugin_fail;    // k_classify found no slot for a plugin flow (table too full)
    int32_t strict_live;     // strict mode: records created - records exported
    uint32_t strict_fail;    // strict mode: a replay lane gave up waiting (IPXG_EDEVICE)
    uint32_t tb_any;         // OR of the time buckets of k_bin / k_bin_slow's records (0: all in bucket 0)
    uint32_t fin_deferred;   // finalise-list aggregates whose table probe failed (k_fin_list: table full)
    uint32_t cx_agg;         // k_complex_gather_rec: a complex flow's packets were folded into a k_bin_slow
                             // tile aggregate (or more k_bin aggregates than the range list holds)
    uint32_t cx_ranges;      // k_complex_gather_rec: k_bin tile aggregates of complex flows listed
    uint32_t guard;          // bounds checks that failed (reported as IPXG_EDEVICE): 1 more complex
                             // slots than counted, 2 a complex flow's segment overran, 4 a plugin slot index
                             // past the table, 8 (GUARD_STREAM_STALL) k_reduce_stream waited seconds for k_bin,
                             // 16 (GUARD_EX_START) k_fin_list found the export counter not at the host's count
    uint32_t spill_deferred; // of `deferred`: spills k_bin / k_bin_slow deferred (Params::defer_spill)
    uint32_t expired;        // records k_expire exported (the host's live count follows it, no table recount)
    uint32_t slow_redo;      // k_bin listed slow packets in a batch launched without k_bin_slow (Params::slow_skip):
                             // k_reduce and k_fin_list returned at once, the host runs all three again
    uint32_t tls_inv;        // k_expire's scan: ~(the least time_last_sec of the records it left live), 1 with
                             // none left, 0 when it did not scan (the engine's idle floor, ipxg_engine.cpp)
    uint32_t ex_holes;       // export records a fused k_fin_list reserved but did not fill (end reason 0:
                             // flows that turned complex or found no slot); the host closes them (k_ex_compact)
    uint64_t probe[16];       // IPXG_PROBE builds: per-phase shader clocks (ipxg_probe_counters)
};

// Fragmentation-cache ring entry (fragmentationKeyData.hpp:49-112), 4 per bucket.
struct FragEntry {
    uint64_t kw[5];  // the 40-byte FragmentationKey as little-endian words
    uint16_t sport, dport;
    uint32_t sec, usec;
    uint32_t pad[3];
};
static_assert(sizeof(FragEntry) == 64, "");

// Device statistics, sharded to spread the per-block atomics: workgroup b adds to row b % STAT_SHARDS
// (256-byte rows, two lines of their own).  A kernel's workgroups mostly end together and each
// adds its ~15 non-zero counters: with 16 rows the atomics of k_bin_slow's 768 workgroups queued
// on 32 lines for ~33 us per launch (configs[4]: 63 -> 30 us without them); at 1024 rows about
// one workgroup per row.
constexpr int STAT_SHARDS = 1024;
constexpr int ST_STRIDE = 32;  // counters per row (>= ST_COUNT)
enum StatIdx {
    ST_SEEN, ST_PARSED, ST_UNKNOWN, ST_IPV4, ST_IPV6, ST_TCP, ST_UDP, ST_MPLS, ST_PPPOE, ST_TRILL,
    ST_VLAN, ST_IPV4_BYTES, ST_IPV6_BYTES, ST_KEYLESS, ST_FRAGMENTED, ST_FRAG_FILLED,
    ST_END_INACTIVE, ST_END_ACTIVE, ST_END_EOF, ST_END_FORCED, ST_END_NO_RES,
    ST_PKTS_1, ST_PKTS_2_5, ST_PKTS_6_10, ST_PKTS_11_20, ST_PKTS_21_50, ST_PKTS_51, ST_COUNT
};
static_assert(ST_COUNT <= ST_STRIDE, "statistics row");
#ifdef __HIPCC__
// the calling workgroup's row of the sharded statistics
__device__ __forceinline__ unsigned long long* stat_row(unsigned long long* stats) {
    return stats + (size_t)(blockIdx.x % STAT_SHARDS) * ST_STRIDE;
}
#endif

// FlowRecordStats bucket of a record of n = src_packets + dst_packets packets
// (update_flow_record_stats, cache.cpp:601-616: 0 falls to the last bucket, as there)
__host__ __device__ inline uint32_t pkts_bucket(uint64_t n) {
    return n == 1 ? 0 : (n >= 2 && n <= 5) ? 1 : (n >= 6 && n <= 10) ? 2 : (n >= 11 && n <= 20) ? 3
         : (n >= 21 && n <= 50) ? 4 : 5;
}

// Everything a kernel needs about the engine, passed by value.
// A slot's 128-byte line: its hot half and the first half of its flow record (the words a
// continuing flow's batch reads and updates: times, counters, TCP flags), so the finalise of a
// continuing flow touches one line; the record's second half (addresses, MACs, VLAN, extension),
// written at creation and read at export, lives in a table of its own (`tail`).
struct alignas(128) SlotLine {
    HotSlot hot;
    uint32_t head[16];  // ipxg_flow_record bytes 0-63
};
static_assert(sizeof(SlotLine) == 128, "slot line");
constexpr uint32_t REC_TAIL_WORDS = 16;  // ipxg_flow_record bytes 64-127 per slot

struct TableView {
    SlotLine* line;
    uint32_t* tail;  // REC_TAIL_WORDS per slot
    uint32_t* slot_rank;
    uint32_t mask;  // capacity - 1
    unsigned long long* port_cnt;  // ps=true: TopPorts' TCP then UDP frequencies (2 x 65536), else null
    __host__ __device__ HotSlot& hot(uint32_t s) const { return line[s].hot; }
    __host__ __device__ uint32_t slot_index(const HotSlot* h) const {
        return (uint32_t)(reinterpret_cast<const SlotLine*>(h) - line);
    }
};

struct ExportView {
    ipxg_flow_record* buf;
    uint32_t* count;  // [0] records appended, [1] overflow flag (never set when sized right),
                      // [2] of them IPv6-template records (ip_version 6), when count6
    uint32_t cap;
    uint32_t count6;  // keep [2] (the engine's IPFIX message layer has been used)
};

struct Params {
    uint32_t dlt;
    uint32_t active_s, inactive_s;
    uint32_t bucket_w;       // seconds per tbits bucket = inactive/2
    uint32_t split_biflow;
    uint32_t frag_enable;
    uint32_t frag_size, frag_timeout_s;
    uint32_t force_complex;  // route every touched flow to the sequential path
    uint32_t prev_valid;     // prev_sec/prev_usec hold the previous batch's last timestamp
    uint32_t prev_sec, prev_usec;
    uint32_t tile_agg;       // k_bin / k_bin_slow aggregate frequent flows per tile (skewed traffic)
    uint32_t wide;           // k_bin's wide walk (96-byte loads, parse_medium)
    uint32_t spin_max;       // strict replay: polling rounds without progress before giving up
    uint32_t classify;       // k_classify ran for the batch (process plugins): slots were claimed and
                             // marked before k_reduce, so every listed flow must find its slot
    // plug: the plugins' rules checked inside k_bin (the wide walk) instead of by k_classify --
    // flattened here so the check reads kernel arguments only: ports (port | proto_mask << 16) and
    // payload prefixes of at most PLUG_PREFIX bytes (bytes little-endian in pref, compare mask in
    // pmask, len | proto_mask << 8 in pinfo)
    uint32_t plug;
    uint32_t defer_spill;    // k_bin / k_bin_slow defer what does not fit its segment (tile_emit): the
                             // batch was launched during the previous batch's host walk
    uint32_t plug_nport, plug_npref;
    // 4 x 16 words on the device (ipxg_add_plugin uploads them): ports, prefixes, prefix masks,
    // prefix infos -- a pointer, not 256 bytes of kernel arguments on every launch (a kernel's
    // dispatch reads its arguments: +1 us per launch at 512 bytes, tools/gapbench)
    const uint32_t* plug_tab;
    // A front launched before the host has read the previous batch's control block (ipxg_submit
    // right behind an asynchronous batch or ipxg_finish, ipxg_engine.cpp `pend`): k_bin, k_bin_slow
    // and k_pstats first test that block (complete on the device: stream order) and return at once,
    // writing nothing, when the host has work left for that batch (gate_closed); prev_dev: the order
    // check's previous timestamp is that block's last_sec / last_usec, not prev_sec / prev_usec.
    const BatchCtl* prev_ctl;
    uint32_t gate_mode;  // GATE_NONE: no gate
    uint32_t prev_dev;
    // pub_seq != 0: k_bin's workgroup 0 first publishes prev_ctl (pub_words words) and the export
    // counters into the host mirror with this sequence number (k_publish's layout), so the host reads
    // the pending batch without a publish kernel (and its kernel boundary) between the batches
    uint32_t* pub_dst;
    const uint32_t* pub_ex;
    uint32_t pub_words, pub_seq;
    // a registered process plugin acts on every packet (ipxg_plugin.all_packets): every flow the
    // batch touches goes to the host walk (finalize_slot marks it SLOT_PLUGIN with SLOT_COMPLEX)
    uint32_t plug_all;
    // k_bin_slow not launched: the previous batch had no slow packet (the empty launch and its
    // kernel boundary cost ~7 us per batch); k_bin flags slow packets it lists (BatchCtl::slow_redo)
    uint32_t slow_skip;
};

// What the host still has to do for a batch after its last kernel, from its control block:
// fragments, deferred packets or aggregates, the table scan, complex flows, a finalise-list
// retry, a plugin slot failure or a fired guard -- and for a finish, the flows it left (GATE_FIN_*).
// The host (consume_pend) and the gated kernels evaluate the same function on the same block.
enum GateMode : uint32_t { GATE_NONE = 0, GATE_BATCH = 1, GATE_FIN_FUSED = 2, GATE_FIN_GUARDED = 3, GATE_EXPIRE = 4 };
__host__ __device__ inline bool gate_closed(const BatchCtl& c, uint32_t mode) {
    const bool work = c.frag_count || c.deferred || c.agg_deferred || c.pending || c.complex_count ||
                      c.fin_deferred || c.plugin_fail || c.guard || c.slow_redo;
    if (mode == GATE_FIN_FUSED) return work || !c.fused;
    if (mode == GATE_FIN_GUARDED || mode == GATE_EXPIRE) return work || c.hold;
    return work;
}
__device__ __forceinline__ bool gated(const Params& p) {
    return p.gate_mode != GATE_NONE && gate_closed(*p.prev_ctl, p.gate_mode);
}
constexpr uint32_t PLUG_PREFIX = 4;
enum PlugTab : uint32_t { PLUG_PORT = 0, PLUG_PREF = 16, PLUG_PMASK = 32, PLUG_PINFO = 48, PLUG_TAB_WORDS = 64 };

// ---- strict mode (ipxg_strict.hip): the reference's line table -------------------------------
struct StrictView {
    ipxg_flow_record* rec;  // 2^s records, [line << line_bits | slot]
    uint64_t* hash;         // their FlowRecord::m_hash (0 = empty)
    uint64_t* perm;         // per line: position j -> record slot, bits 4j..4j+3
    uint32_t* tlast;        // per slot: the record's time_last_sec, 0xFFFFFFFF while empty (the sweep's test)
    uint32_t* lb;           // per line: a lower bound of every time_last it holds during the batch; [lines]:
                            // ~(the batch's first second) (k_strict_prep2's atomicMax)
    uint32_t line_bits;     // l= (line size 2^l, at most 16)
    uint32_t lines;         // 2^s >> l
    uint32_t slot_mask;     // 2^s - 1
};
struct StrictPkt {          // what put_pkt_recursive reads of a keyed packet (h_fwd 0: not keyed)
    uint64_t h_fwd, h_inv;
    uint32_t ts_sec, ts_usec;
    uint16_t ip_len;
    uint8_t tcp_flags, ip_proto;
    uint32_t sweep;  // 1: its sweep step may export (k_strict_events); 0: provably exports nothing
};
static_assert(sizeof(StrictPkt) == 32, "");
constexpr uint32_t STRICT_LANES = 768;           // the replay's one workgroup (3 waves per SIMD; the DAG is ~260 packets wide at the reference default)
constexpr uint32_t STRICT_NONE = 0xFFFFFFFFu;
#ifndef IPXG_STRICT_SPIN_MAX
#define IPXG_STRICT_SPIN_MAX (1u << 24)
#endif
constexpr uint32_t STRICT_SPIN_MAX = IPXG_STRICT_SPIN_MAX;  // polling rounds without any packet finishing

struct BatchView {
    const uint8_t* arena;
    const ipxg_pkt_desc* desc;
    uint32_t n;
    uint32_t base_sec;   // tbits bucket origin (first packet's seconds), or BASE_FROM_DESC0
    uint32_t arena_lim;  // min(arena bytes, 0xFFFFFF00): the range of the byte-offset buffer loads
    uint32_t oshift;     // 4: descriptor offsets count 16-byte units (IPXG_BATCH_OFFSET16), else 0
    uint64_t arena_len;  // bytes valid in the arena
};
constexpr uint32_t BASE_FROM_DESC0 = 0xFFFFFFFFu;
#ifdef __HIPCC__
// frame d's byte offset in the arena, and its address
__device__ __forceinline__ uint64_t frame_off(const BatchView& b, const ipxg_pkt_desc& d) {
    return (uint64_t)d.offset << b.oshift;
}
__device__ __forceinline__ const uint8_t* frame_ptr(const BatchView& b, const ipxg_pkt_desc& d) {
    return b.arena + frame_off(b, d);
}
__device__ __forceinline__ bool frame_aligned(const BatchView& b, const ipxg_pkt_desc& d) {
    return b.oshift != 0 || (d.offset & 15) == 0;
}
// The register parsers' buffer loads take 32-bit byte offsets: they address an arena of up to
// 4 GiB through one resource.  With 16-byte units (arenas up to 64 GiB) the frames are read
// through their 64-bit addresses instead (a structured resource, record index x 16, wraps at
// 4 GiB on gfx950 too: tools/sbtest; a per-wave 4 GiB window of the arena sent the frames of
// two receive pools far apart -- the configs[2] placement -- to the slow path).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t arena_rsrc(const BatchView& b) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(b.arena), 0, (int)b.arena_lim, 0x00020000);
}
#endif

struct FragView {
    FragEntry* ent;      // frag_size * 4
    uint32_t* cnt;       // frag_size
    uint64_t* list;      // (bucket << 24) | packet index, frag_count entries
    uint64_t* sorted;
    uint32_t* ports;     // per packet index: resolved (sport << 16) | dport
};

// Phase-A output of the ingest (k_bin / k_bin_slow -> k_reduce): per partition of the
// canonical flow hash (bits 32.. of lo), one segment per k_bin and per k_bin_slow workgroup
// ("column"), so every workgroup appends to its own segments without device atomics.
// Record = {lo, hi, packet index, pack_misc()}.  Segment (part, col) starts at record
// (part * cols + col) * seg_cap; count[seg_count_idx(part, col)] = its length.
struct BinView {
    uint4* rec;          // parts * cols * seg_cap records
    uint32_t* count;     // parts * cols segment lengths (seg_count_idx; every column written per batch)
    uint32_t seg_cap;    // records per segment (a full segment spills to device atomics)
    uint32_t cols;       // 2 * bin_grid: k_bin's columns, then k_bin_slow's
    uint32_t bin_grid;   // workgroups of k_bin (and of k_bin_slow)
    uint32_t part_bits;  // parts = 1 << part_bits
    uint32_t slow_stride;  // k_bin workgroup b lists its slow packets (16-B entries) at slow_list[b * slow_stride ...]
    uint32_t* slow_cnt;    // bin_grid: slow packets listed by each k_bin workgroup
    uint4* marks;          // Params::plug: workgroup b's plugin marks at marks[b * slow_stride ...] (k_bin's,
    uint32_t* mark_cnt;    //   then k_bin_slow's), mark_cnt[b] of them: {key lo, key hi, index | kind << 30, 0}
    uint32_t slow_skip;    // Params::slow_skip (k_reduce returns when k_bin flagged slow_redo)
    uint32_t line;         // k_bin's line mode (ipxg_ingest.hip: whole-line record stores; seg_cap % 8 == 0)
    // streamed reduce (line mode, round 6): k_bin workgroup col publishes after every tile, for each
    // partition q, prog[col << part_bits | q] = prog_tag | the whole lines of its segment stored so far
    // (| PROG_DONE after its last tile), and k_reduce_stream folds them while k_bin runs; null: no
    // streaming (k_reduce after k_bin)
    uint32_t* prog;
    uint32_t prog_tag;     // the batch's epoch << PROG_EPOCH_SHIFT (never 0): a word of an older batch reads as 0 lines
    uint32_t prog_mode;    // PROG_SC1: write-through record stores; PROG_TILE: a publish every pub_every tiles (else: at the end)
    uint32_t pub_every;    // tiles between k_bin's publishes
    uint32_t rs_sleep;     // k_reduce_stream: s_sleep(64) calls between polls that found nothing new
    // k_bin_slow workgroup j takes the slow lists of k_bin workgroups j * slow_group ... + slow_group - 1
    // in turn (ceil(bin_grid / slow_group) workgroups, columns bin_grid + j): with a sparse slow path
    // (configs[4]: ~260 packets per list) whole tiles, and record segments holding several records
    // instead of a fraction of one -- measured slower (ipxg_engine.cpp setup_bins), so 1 by default
    uint32_t slow_group;
};
constexpr uint32_t SLOW_GROUP_MAX = 8;
#ifdef __HIPCC__
// k_bin_slow column j (of bin_grid) holds records: one of its lists had packets (else the workgroup
// returned without writing the column's counts)
__device__ __forceinline__ bool slow_col_written(const BinView& bv, uint32_t j) {
    bool w = false;
    const uint32_t G = bv.slow_group ? bv.slow_group : 1u;  // (a view never set up: one list each)
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t b = j * G + g;
        w = w || (b < bv.bin_grid && bv.slow_cnt[b] != 0);
    }
    return w;
}
#endif
constexpr uint32_t PROG_SC1 = 1u, PROG_TILE = 2u;
constexpr uint32_t BIN_LINE_P = 256;  // line mode's partitions, at most (ipxg_ingest.hip LINE_P)
// The streamed reduce (k_reduce_stream): one 1024-thread workgroup per partition beside two k_bin
// workgroups per CU (2 x 48 KiB of LDS + its 64 KiB), a 1024-entry LDS flow table, at most
// RS_MAX_COLS k_bin columns.  Progress words prog[partition * RS_MAX_COLS + column] (a partition's
// words contiguous: its reducer polls 16 lines): lines in bits 0-19, the batch's epoch in 20-29, done in 31.
constexpr uint32_t RS_ENTRIES = 1024;
constexpr uint32_t RS_MAX_COLS = 512;
constexpr uint32_t RS_TARGET_FLOWS = 600;  // flows per partition the host sizes the streamed reduce for
constexpr uint32_t PROG_LINES = 0xFFFFFu, PROG_EPOCH_SHIFT = 20, PROG_EPOCH_MASK = 0x3FFu << 20,
                   PROG_DONE = 0x80000000u;
constexpr uint32_t GUARD_STREAM_STALL = 8u;  // BatchCtl::guard: k_reduce_stream saw no progress for seconds
constexpr uint32_t GUARD_EX_START = 16u;     // ... k_fin_list's list-order exports: the export counter was not ex_start
// The segment counts, column-major: workgroup col's counts of all partitions are contiguous, so
// each k_bin / k_bin_slow workgroup writes whole lines of them (partition-major, every count was
// a 4-byte piece of a line the other columns' workgroups, on other XCDs, wrote the rest of).
// k_reduce's workgroup for a partition reads one count per column; its partition is chosen so
// that the 32 partitions sharing a line of counts run on one XCD (red_part).
#ifndef IPXG_COUNTS_T
#define IPXG_COUNTS_T 1
#endif
__host__ __device__ inline size_t seg_count_idx(const BinView& bv, uint32_t part, uint32_t col) {
    return IPXG_COUNTS_T ? ((size_t)col << bv.part_bits) | part : (size_t)part * bv.cols + col;
}
// k_reduce workgroup b's partition (of P): workgroups go to the 8 XCDs round-robin (b % 8)
__host__ __device__ inline uint32_t red_part(uint32_t b, uint32_t P) {
    if (!IPXG_COUNTS_T || P < 256) return b;
    const uint32_t x = b & 7u, i = b >> 3;
    return (i >> 5) * 256u + x * 32u + (i & 31u);
}
#ifndef IPXG_BIN_K
#define IPXG_BIN_K 8  // packets per lane per k_bin tile
#endif
constexpr uint32_t BIN_TILE_PKTS = IPXG_BIN_K * 256u;  // packets per k_bin tile (256-lane workgroups)
#ifndef IPXG_BIN_MAX_PART_BITS
#define IPXG_BIN_MAX_PART_BITS 11
#endif
constexpr uint32_t BIN_MAX_PART_BITS = IPXG_BIN_MAX_PART_BITS;  // <= 2048 partitions (LDS histograms of k_bin)
#ifndef IPXG_KBIN_PMAX_BITS  // tuning knob: k_bin's LDS partition histograms (the host caps the partitions to it)
#define IPXG_KBIN_PMAX_BITS IPXG_BIN_MAX_PART_BITS
#endif
static_assert(IPXG_KBIN_PMAX_BITS <= IPXG_BIN_MAX_PART_BITS, "k_bin's histograms");
constexpr uint32_t BIN_MAX_GRID = 2048;     // k_bin workgroups (persistent over the tiles)
constexpr uint32_t RED_THREADS = 1024;      // k_reduce workgroup
#ifndef IPXG_RED_ENTRIES
#define IPXG_RED_ENTRIES 2048
#endif
constexpr uint32_t RED_ENTRIES = IPXG_RED_ENTRIES;  // k_reduce LDS flow table (56 B entries)
// flows per partition the host sizes for: <= 0.6 of the LDS table's entries (linear probing).
// (600 until round 3: on the 1M-flow mixes twice the k_reduce workgroups, each zeroing and
// scanning its LDS table for half the flows -- k_reduce -30 % quic, -50 % imix at 1200)
constexpr uint32_t RED_TARGET_FLOWS = 1200;
constexpr uint32_t RED_MIN_FLOWS = 256;  // below 256 partitions (one per CU), flows per partition at least

struct ComplexView {
    uint64_t* list;      // (rank << 24) | packet index
    uint64_t* sorted;
    uint32_t* cursor;    // per rank
    uint32_t* slot_of;   // per rank
    uint32_t* seg;       // per rank: segment start
    uint32_t* len;       // per rank: packets
    unsigned long long* keys;  // open-addressing set of the complex flows' keys (kmask + 1
    uint32_t* key_rank;        // entries, zeroed) -> rank: k_complex_gather finds a packet's flow
    uint32_t kmask;            // here, not by probing the flow table (whose chains a fused
                               // finish may have cut: k_fin_list empties slots)
    // a bitmap of the keys' low words (bmask + 1 words, zeroed; null: none), set by k_complex_rank:
    // a key whose bit is clear is no complex flow's -- one read of an L2-resident bitmap instead of
    // a probe into the key set for the ~97 % of a gather's packets that belong to no complex flow
    uint32_t* bloom;
    uint32_t bmask;
};

// Parser side statistics (ps=true): TopPorts frequencies [tcp 65536][udp 65536], then
// VlanStats per VLAN id, VS_N u64 counters each in ipxg_vlan_stats order.
constexpr uint32_t VS_N = 8 + 2 * IPXG_SIZE_BUCKETS;
constexpr size_t PSTAT_PORTS = 2 * 65536;
constexpr size_t PSTAT_WORDS = PSTAT_PORTS + (size_t)IPXG_VLAN_IDS * VS_N;

// A registered plugin's pre-classifier rule (ipxg_plugin's rule fields), on the device.
struct DevRule {
    uint32_t proto_mask, n_ports;
    uint16_t ports[IPXG_PLUGIN_MAX_PORTS];
    uint32_t n_prefixes;
    uint8_t prefix_len[IPXG_PLUGIN_MAX_PREFIXES];
    uint8_t prefix[IPXG_PLUGIN_MAX_PREFIXES][IPXG_PLUGIN_PREFIX_LEN];
    uint32_t masked;  // bit q: prefix q compares under prefix_mask[q]
    uint8_t prefix_mask[IPXG_PLUGIN_MAX_PREFIXES][IPXG_PLUGIN_PREFIX_LEN];
};

// A plugin flow between the device and the host walk: its slot, packets (segment of the complex
// path's sorted list), slot state and key, and its record (k_plugin_pack -> host -> k_plugin_apply).
struct PluginFlow {
    uint32_t slot, seg, len, state;
    uint64_t key;
    uint64_t pad;
    ipxg_flow_record rec;
};
static_assert(sizeof(PluginFlow) == 160, "plugin flow image");

// ---- launchers (ipxg_kernels.hip / ipxg_sort.hip) ---------------------------------------
// k_bin workgroups resident on the whole device at once (its persistent grid); agg: the
// tile-aggregating variant (more LDS)
uint32_t bin_resident_blocks(int device, bool agg, bool wide, bool plug, bool line, bool g64);
// deferred_list: packet indices (counter ctl->deferred); agg_list: deferred tile aggregates,
// 3 record slots each (counter ctl->agg_deferred)
void launch_bin(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, BinView bv,
                BatchCtl* ctl, uint4* slow_list, uint32_t* deferred_list, uint4* agg_list,
                unsigned long long* stats);
void launch_bin_slow(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, BinView bv,
                     BatchCtl* ctl, const uint4* slow_list, uint32_t* deferred_list, uint4* agg_list,
                     unsigned long long* stats);
// fin_list: the merged images of the slots k_reduce completed (HotSlot::pad = slot index).
// zero_ctl (or null): the other control block, zeroed by workgroup 0 for the next batch's front
// (the host has read it); zero_ex (or null): the export counters, zeroed (ipxg_clear_exports) --
// both ride on this kernel instead of a fill command of their own.
void launch_reduce(hipStream_t st, TableView t, BinView bv, BatchCtl* ctl, HotSlot* fin_list,
                   uint32_t* deferred_list, uint4* agg_list, BatchCtl* zero_ctl = nullptr,
                   uint32_t* zero_ex = nullptr);
// The streamed form (bv.prog set): launched beside k_bin on a stream of its own (gated as k_bin on
// Params::gate_mode); it folds each partition's records as k_bin publishes them and ends with
// k_reduce's merge and finalise list once every k_bin workgroup is done.
void launch_reduce_stream(hipStream_t st, const Params& p, TableView t, BinView bv, BatchCtl* ctl, HotSlot* fin_list,
                          uint32_t* deferred_list, uint4* agg_list);
constexpr uint32_t FIN_UNRESOLVED = 0xFFFFFFFFu;  // a finalise-list entry's pad: the flow's slot not probed yet
constexpr uint32_t FIN_DEFERRED = 0xFFFFFFFEu;    // ... its probe failed (table full): again after a rehash
// ex_start: a fused finish's exports in list order from this export count (the device counter's value,
// known to the host: nothing appends before the kernel), or EX_START_NONE (reserved per workgroup pass)
constexpr uint32_t EX_START_NONE = 0xFFFFFFFFu;
void launch_fin_list(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f, ExportView ex,
                     BatchCtl* ctl, HotSlot* fin_list, unsigned long long* stats, uint32_t max_n,
                     bool finishing, bool deferred_only = false, uint32_t ex_start = EX_START_NONE);
// Params::plug: the marks k_bin and k_bin_slow listed -- plugin flows found in registers (slot
// claimed and marked SLOT_PLUGIN here) and packets to classify from their frames (k_classify's
// test) -- before k_reduce
constexpr uint32_t MARK_HIT = 1u, MARK_LATER = 2u;
void launch_plugin_marks(hipStream_t st, const BatchView& b, const Params& p, TableView t, const DevRule* rules,
                         uint32_t nrules, BatchCtl* ctl, const BinView& bv);
void launch_classify(hipStream_t st, const BatchView& b, const Params& p, TableView t, const DevRule* rules,
                     uint32_t nrules, BatchCtl* ctl);
// The host walk's inputs on the device, flows in order of their first packet (ipxg_bridge.hip):
// keys / skeys [ncx], flows [ncx], flen / first [ncx + 1], idx [npk], clen / off [npk + 1],
// hstate [ncx] (slot states), lflag / lpos [ncx + 1] (live flags, their exclusive prefix),
// recs [ncx] (the live flows' records, compacted), count (zeroed by the caller),
// tot [4] = {flows, packets, bytes, live flows}
// A walked packet as the host walk reads it: its parsed fields, descriptor and batch index in one
// record, so a chunk of the walk's input crosses to the host in one copy (k_plugin_pkts)
struct WalkPkt {
    ipxg_parsed_pkt pk;
    ipxg_pkt_desc d;
    uint32_t idx;
};
// wpk [npk]: the walked packets (k_plugin_pkts, inside launch_plugin_order); budget > 0: a walked
// packet that no plugin's rule matches crosses with its headers and `budget` payload bytes only
// (ipxg_plugin.follow_bytes), the rest with the whole frame
struct PluginOrder {
    uint64_t *keys, *skeys;
    PluginFlow* flows;
    uint32_t *flen, *first, *idx, *count, *hstate, *lflag, *lpos;
    ipxg_flow_record* recs;
    uint64_t *clen, *off, *tot;
    void* temp;
    size_t temp_bytes;
    WalkPkt* wpk;
    const DevRule* rules;
    uint32_t nrules, budget;
};
void launch_plugin_order(hipStream_t st, const BatchView& b, const Params& p, FragView f, TableView t, ComplexView cx,
                         uint32_t ncx, uint32_t npk, const PluginOrder& o);
size_t plugin_order_temp(uint32_t ncx, uint32_t npk);
void launch_plugin_bytes(hipStream_t st, const BatchView& b, const uint32_t* idx, const uint64_t* off, uint32_t m,
                         uint8_t* out);
// The host walk's results, read by one kernel straight from page-locked host memory (one launch
// instead of a copy command per walk thread and array): chunk c = n[c] records at src[c] (a
// device-visible address) to dst + at[c].
constexpr int HOST_CHUNKS = 64;
struct HostChunks {
    const uint4* src[HOST_CHUNKS];
    uint32_t n[HOST_CHUNKS];
    uint32_t at[HOST_CHUNKS];
    uint32_t count, max_n;
};
void launch_host_gather(hipStream_t st, const HostChunks& c, ipxg_flow_record* dst);
// the write-back: slot states of the nf flows, then the records recs[0..nrec) of the flows live
// after the walk (each carrying its flow's index in reserved2)
void launch_plugin_apply(hipStream_t st, TableView t, const PluginFlow* flows, const uint32_t* state, uint32_t nf,
                         const ipxg_flow_record* recs, uint32_t nrec, BatchCtl* ctl);
void launch_pstats(hipStream_t st, const BatchView& b, const Params& p, unsigned long long* pstat);
void launch_ingest(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                   BatchCtl* ctl, uint32_t* deferred_list, unsigned long long* stats);
void launch_frag_walk(hipStream_t st, const BatchView& b, const Params& p, FragView f, uint32_t nfrag,
                      unsigned long long* stats);
void launch_frag_accumulate(hipStream_t st, const BatchView& b, const Params& p, TableView t,
                            FragView f, uint32_t nfrag, BatchCtl* ctl, uint32_t* deferred_list);
void launch_deferred(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                     const uint32_t* in_list, uint32_t n_in, BatchCtl* ctl, uint32_t* out_list);
void launch_deferred_agg(hipStream_t st, TableView t, const uint4* in_list, uint32_t n_in, BatchCtl* ctl,
                         uint4* out_list);
void launch_finalize(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                     ExportView ex, BatchCtl* ctl, unsigned long long* stats);
void launch_complex_rank(hipStream_t st, TableView t, ComplexView cx, BatchCtl* ctl, uint32_t cap, uint32_t ncx);
void launch_complex_gather(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                           ComplexView cx, BatchCtl* ctl);
// the same from the batch's partition records (k_bin / k_bin_slow), when every packet of the batch
// left one (no spills, deferrals or fragments); ctl->cx_agg set: redo with the re-parse above
void launch_complex_gather_rec(hipStream_t st, const BinView& bv, ComplexView cx, BatchCtl* ctl, uint4* ranges,
                               uint32_t range_cap);
void launch_complex_gather_ranges(hipStream_t st, const BatchView& b, const Params& p, FragView f, ComplexView cx,
                                  BatchCtl* ctl, const uint4* ranges, uint32_t nr);
void launch_complex_walk(hipStream_t st, const BatchView& b, const Params& p, TableView t, FragView f,
                         ComplexView cx, uint32_t nranks, ExportView ex, BatchCtl* ctl,
                         unsigned long long* stats);
// guard != nullptr: an expire enqueued right behind a batch (ipxg_expire with an asynchronous batch
// in flight), held back exactly as k_finish's guard; expired: += the records it exports.
// floor: every live record's time_last_sec is at least this (IDLE_FLOOR_NONE: not known); when no
// record can be idle at `now` the kernel returns without scanning (a guarded one only behind a
// batch whose order check held); tls_inv: BatchCtl::tls_inv of the scan.
constexpr int64_t IDLE_FLOOR_NONE = INT64_MIN;
void launch_expire(hipStream_t st, const Params& p, TableView t, uint32_t cap, int64_t now,
                   ExportView ex, unsigned long long* stats, BatchCtl* guard, uint32_t* expired,
                   uint32_t ex_before = 0, uint32_t live_before = 0, int64_t floor = IDLE_FLOOR_NONE,
                   uint32_t* tls_inv = nullptr);
void launch_finish(hipStream_t st, TableView t, uint32_t cap, ExportView ex, unsigned long long* stats,
                   BatchCtl* guard = nullptr, uint32_t ex_before = 0, uint32_t live_before = 0);
void launch_publish(hipStream_t st, const uint32_t* ctl, const uint32_t* ex, uint32_t* dst, uint32_t ctl_words,
                    uint32_t seq);
// The export records [lo, hi) with their holes (end reason 0, BatchCtl::ex_holes) dropped, in order;
// the export count set to what remains.
void launch_ex_compact(hipStream_t st, ExportView ex, uint32_t lo, uint32_t hi);
void launch_ipfix_basic(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint32_t dir, uint64_t* block_tot,
                        uint8_t* out, uint64_t* offsets);
// IPFIX message plan (host, ipxg_engine.cpp): data sets in rank order per class (class 0 = the
// IPv4 template's records, then class 1 = IPv6), and the messages.
struct IpfixSet {
    uint32_t cls, count;
    uint64_t ord0;  // rank (in its class) of the set's first record
    uint64_t off;   // byte offset of the set header in the output
};
struct IpfixMsg {
    uint64_t off;
    uint32_t len, seq;
};
// block_tot[nb + 1] <- exclusive prefix of the IPv6-template records per 256-record block (+ total)
void launch_ipfix_count6(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint64_t* block_tot);
void launch_ipfix_messages(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint32_t dir,
                           const uint64_t* block_pre6, const IpfixSet* sets, uint32_t nsets4, uint32_t nsets6,
                           const IpfixMsg* msgs, uint32_t nmsgs, uint32_t odid, uint32_t export_time, uint8_t* out);
void launch_rehash(hipStream_t st, TableView from, uint32_t from_cap, TableView to, uint32_t* fail);
void launch_parse_batch(hipStream_t st, const BatchView& b, uint32_t dlt, ipxg_parsed_pkt* out);
void launch_xxh64(hipStream_t st, const uint8_t* keys, uint32_t keylen, uint32_t n, uint64_t seed,
                  uint64_t* out);

// rocPRIM radix sort of 64-bit keys (slow paths only).  temp may be null to query size.
hipError_t sort_pairs_u32(void* temp, size_t& temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                          uint32_t* vout, uint32_t n, int end_bit, hipStream_t st);
hipError_t exclusive_scan_u64(void* temp, size_t& temp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                              hipStream_t st);
hipError_t exclusive_scan_u32(void* temp, size_t& temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                              hipStream_t st);
void launch_strict_prep1(hipStream_t st, const BatchView& b, const Params& p, FragView f, BatchCtl* ctl,
                         unsigned long long* stats);
void launch_strict_prep2(hipStream_t st, const BatchView& b, const Params& p, FragView f, StrictPkt* sp,
                         ipxg_flow_record* crec, uint32_t* keyed, uint32_t* ts_acc);
void launch_strict_lb(hipStream_t st, StrictView v);
void launch_strict_events(hipStream_t st, StrictView v, StrictPkt* sp, const uint32_t* keyed, const uint32_t* qx,
                          uint32_t n, uint64_t q_base, uint32_t split, uint32_t inactive, uint32_t* keys,
                          uint32_t* vals);
void launch_strict_dag(hipStream_t st, const uint32_t* keys_sorted, const uint32_t* vals_sorted, uint32_t m,
                       const uint32_t* keys, const uint32_t* keyed, uint32_t n, uint32_t lines, uint32_t* succ,
                       uint8_t* pred, uint32_t* indeg, uint32_t* queue, uint32_t* q_count);
// sched: one workgroup (wgs_per_xcd 0) -- the ready count k_strict_ready left; several
// (8 x wgs_per_xcd launched, one XCD's take part) -- a zeroed STRICT_SCHED_BYTES block whose word
// STRICT_SCHED_TAIL_WORD holds that count
constexpr uint32_t STRICT_SCHED_BYTES = 512;
constexpr uint32_t STRICT_WGS_DEFAULT = 12;  // replay workgroups per XCD (of 256 lanes): 114 Mpkt/s at s=17
constexpr uint32_t STRICT_SCHED_TAIL_WORD = 32;  // the ready count / queue tail (its own 128-byte line)
void launch_strict_walk(hipStream_t st, StrictView v, const Params& p, const StrictPkt* sp,
                        const ipxg_flow_record* crec, const uint32_t* keyed, const uint32_t* qx, const uint32_t* succ,
                        uint32_t* indeg, uint32_t* queue, uint32_t* sched, uint32_t n, uint64_t q_base,
                        ExportView ex, BatchCtl* ctl, unsigned long long* stats, uint32_t wgs_per_xcd);
void launch_strict_expire(hipStream_t st, StrictView v, const Params& p, uint64_t q, int64_t now, ExportView ex,
                          BatchCtl* ctl, unsigned long long* stats);
void launch_strict_finish(hipStream_t st, StrictView v, ExportView ex, BatchCtl* ctl, unsigned long long* stats);
void launch_strict_clear(hipStream_t st, StrictView v);
hipError_t sort_keys_u64(void* temp, size_t& temp_bytes, const uint64_t* in, uint64_t* out,
                         uint32_t n, int end_bit, hipStream_t st);

}  // namespace ipxg
