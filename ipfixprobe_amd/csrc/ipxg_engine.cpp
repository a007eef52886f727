// ipxg_engine.cpp -- host side of the C-ABI (include/ipxg.h): device memory, the per-batch
// kernel sequence, table growth, the export buffer, and statistics.
//
// Per ipxg_submit (one batch, arrival order):
//   stage (H2D if host batch) -> k_bin (register parser) -> k_bin_slow (general parser, the
//   frames k_bin left) -> k_reduce (per-flow merge) -> k_fin_list (split rules)
//   -> [sync: control block]
//   -> fragments? sort + k_frag_walk + k_frag_accumulate
//   -> deferred probes? grow table (k_rehash) + k_deferred, until none
//   -> anything k_reduce could not finalise (ctl->pending)? k_finalize scan -> [sync]
//   -> complex flows? k_complex_rank -> gather -> sort -> k_complex_walk
//   -> grow the table if its load passed 1/2.
// In the common case (no fragments, no overflow) that is four kernels and one host sync.
#include <hip/hip_runtime.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ipxg.h"
#include "ipxg_kernels.hpp"
#include "ipxg_walkpool.hpp"

using namespace ipxg;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Host memory for the walk's copies and for the write-back kernel: pinned allocations from the
// HIP runtime (hipHostMalloc, mapped: a device-visible address in `dev`), growth only -- each
// engine allocates a few and frees them at destroy.  (Earlier: malloc memory registered with
// hipHostRegister and unregistered on growth; full GPU test runs then failed intermittently with
// faults surfacing at later pageable copies -- the runtime-managed pinned path replaced it.)
// IPXG_WALK_PAGEABLE=1: plain malloc memory, copies through the runtime's staging (A/B).
static std::atomic<uint64_t> g_hostvec_allocs{0}, g_hostvec_unpinned{0};  // (IPXG_WALK_TRACE)
template <class T>
struct HostVec {
    T* p = nullptr;
    T* dev = nullptr;  // its device-visible address when page-locked (kernels read it over PCIe)
    size_t n = 0, cap = 0;
    bool reg = false;
    HostVec() = default;
    HostVec(const HostVec&) = delete;
    HostVec& operator=(const HostVec&) = delete;
    ~HostVec() { release(); }
    void release() {
        if (p) {
            if (reg) (void)hipHostFree(p);
            else std::free(p);
        }
        p = dev = nullptr;
        n = cap = 0;
        reg = false;
    }
    // capacity for k elements; keep: the first n survive a reallocation
    bool reserve(size_t k, bool pin, bool keep = false) {
        if (k <= cap) return true;
        const size_t want = std::max(k, cap + cap / 2 + 1024);
        const size_t bytes = (want * sizeof(T) + 4095) & ~(size_t)4095;
        void* q = nullptr;
        bool pinned = pin && hipHostMalloc(&q, bytes, hipHostMallocMapped) == hipSuccess;
        if (!pinned && posix_memalign(&q, 4096, bytes)) return false;
        const size_t kept = keep ? n : 0;
        if (kept) std::memcpy(q, p, kept * sizeof(T));
        release();
        p = static_cast<T*>(q);
        cap = bytes / sizeof(T);
        n = kept;
        reg = pinned;
        if (reg && hipHostGetDevicePointer((void**)&dev, p, 0) != hipSuccess) dev = nullptr;
        g_hostvec_allocs++;
        if (pin && !reg) g_hostvec_unpinned++;
        return true;
    }
    bool resize(size_t k, bool pin) {
        if (!reserve(k, pin)) return false;
        n = k;
        return true;
    }
    void push_back(const T& v) {  // (grows page-locked; std::bad_alloc when the host is out of memory)
        if (n == cap && !reserve(n + 1, reg || !p, true)) throw std::bad_alloc();
        p[n++] = v;
    }
    void clear() { n = 0; }
    bool empty() const { return n == 0; }
    T* data() { return p; }
    const T* data() const { return p; }
    size_t size() const { return n; }
};

// The host walk's input crosses PCIe in WALK_CHUNKS chunks of flows (in walk order); the hooks
// start on a chunk as soon as its copies land, while the next chunks are still copying.
constexpr unsigned WALK_CHUNKS = 4;
// A work unit's exports, on a cache line of its own (the threads append concurrently).
struct alignas(128) ExportVec {
    HostVec<ipxg_flow_record> v;              // page-locked, sized by the engine's thread before the walk
    std::vector<ipxg_flow_record> spill;      // what did not fit (the walk threads make no HIP call)
    HostVec<ipxg_flow_record> orec;           // the records of its range's flows live after the walk
                                              // (one per flow at most; the flow's index in reserved2)
};

struct ipxg_engine {
    ipxg_config cfg;
    hipStream_t st = nullptr;
    std::string err;
    // flow table
    uint32_t cap = 0;
    SlotLine* line = nullptr;  // hot slot + record head per slot (TableView)
    uint32_t* tail = nullptr;  // record tails
    uint32_t* slot_rank = nullptr;
    uint32_t keys = 0, live = 0;
    // export buffer: records [ex_head, ex_count) are pending
    ipxg_flow_record* ex = nullptr;
    uint32_t ex_cap = 0;
    uint32_t* ex_count_d = nullptr;  // [0] count, [1] overflow flag, [2] IPv6 records (after the ctl blocks)
    // ipxg_clear_exports' zeroing of ex_count_d, deferred to the next device work on exports (the
    // next submit folds it into its control-block memset: one fill command per step, not two)
    bool ex_zero_pending = false;
    uint32_t ex_count = 0, ex_head = 0;
    uint32_t ex_count6 = 0;          // [2] at the last readback
    bool ex6_valid = false;          // [2] counts exactly the records [0, ex_count) (ex_head == 0)
    bool count6_on = false;          // kernels keep [2]: switched on by the first IPFIX message call
    // control / stats
    // Control blocks, double-buffered: consecutive batches alternate (launch_front), so a batch's
    // block stays intact until the host has read it while the next batch's front already runs
    // (`pend`); one allocation [block 0][block 1][export counters].  A block is zeroed for its next
    // batch by k_reduce of the batch on the other block (launch_rest), or by a fill when not.
    BatchCtl* ctl_blk[2] = {nullptr, nullptr};
    int cur = 0;                         // the block (and event set) of the batch being launched
    bool blk_zero[2] = {false, false};   // zeroed on the stream since its last use
    BatchCtl* ctl_d = nullptr;  // = ctl_blk[cur] (swapped while a pending batch is completed)
    BatchCtl* ctl_h = nullptr;  // host-mapped mirror: BatchCtl, export counters, publish sequence word
    uint32_t* ctl_hd = nullptr;  // its device address
    uint32_t pub_seq = 0;        // the last sequence number published
    bool no_grow = false;        // ensure() refuses to reallocate (a front launched ahead: IPXG_EGROW)
    // A/B knobs (environment, read at ipxg_create): IPXG_SYNC_FINISH=1 -- ipxg_finish waits for its
    // batch as before round 5; IPXG_NO_AHEAD=1 -- ipxg_submit launches no front ahead
    bool sync_finish = false, no_ahead = false;
    bool no_line = false;  // IPXG_NO_LINE=1: k_bin without line mode (A/B knob)
    // The streamed reduce (round 6, line mode): k_reduce_stream on a stream of its own (rst) beside
    // k_bin, forked right before k_bin (rs_fork) and joined before k_fin_list (rs_join); k_bin's
    // progress words in `prog`, tagged with the batch's epoch (1..1023; the words are cleared when
    // it wraps or their layout changes).  Off by default: measured slower than k_reduce after
    // k_bin; IPXG_STREAM=1 switches it on (A/B knob).
    bool no_stream = true;
    hipStream_t rst = nullptr;
    hipEvent_t rs_fork = nullptr, rs_join = nullptr;
    DevBuf prog;
    uint32_t prog_epoch = 0, prog_g = 0, prog_p = 0;
    uint32_t stream_grid = 0;  // k_bin's workgroups when streamed: two per CU (<= RS_MAX_COLS)
    uint32_t prog_mode = PROG_SC1 | PROG_TILE;  // IPXG_PROG_MODE (timing experiments)
    uint32_t pub_every = 4, rs_sleep = 4;       // IPXG_PUB_EVERY, IPXG_RS_SLEEP (tuning knobs)
    // every live record's time_last_sec is at least this (k_expire's last scan; packets since then kept
    // the order, so none is older), or IDLE_FLOOR_NONE: ipxg_expire at a time when none can be idle
    // scans nothing (the streaming step's expire every batch)
    int64_t idle_floor = IDLE_FLOOR_NONE;
    bool no_idle_floor = false;                 // IPXG_NO_IDLE_FLOOR=1: every ipxg_expire scans (A/B)
    bool fin_lorder = true;                     // IPXG_FIN_LORDER=0: a fused finish reserves its exports per pass (A/B)
    uint32_t rec_sc1 = 1;                       // IPXG_REC_SC1: 0 plain record stores, 1 write-through in line mode, 2 always
    // A batch (or finish) whose last kernels and control-block publish are enqueued but whose block
    // the host has not read: completed by the next entry point (consume_pend) -- ipxg_submit of a
    // device batch first launches its own front behind it, gated on that block (Params::gate_mode),
    // so the device does not wait for the host between batches.
    struct {
        bool on = false;
        uint32_t mode = GATE_NONE;   // GATE_BATCH, GATE_FIN_FUSED, GATE_FIN_GUARDED
        bool clear_after = false;    // ipxg_clear_exports since: the batch's exports are dropped
        int blk = 0;
        uint32_t seq = 0;
        BatchView bv;
        Params p;
        uint32_t n = 0;
        BinView bins;                // its partition records (k_complex_gather_rec), bins_valid, part_bits_last
        bool bins_valid = false;
        uint32_t part_bits = 0;
        bool spec_closed = false;    // (consume_pend's result) the front launched ahead returned at once
        int64_t now = 0;             // GATE_EXPIRE: ipxg_expire's clock
        // its block reaches the host mirror by the next front's k_bin (Params::pub_*: no publish
        // kernel of its own between batches), else consume_pend publishes it
        bool published = false;
    } pend;
    uint32_t* misc_d = nullptr;  // [0] rehash failures
    unsigned long long* stats_d = nullptr;
    unsigned long long* pstat_d = nullptr;  // ps=true: TopPorts + VlanStats (PSTAT_WORDS)
    // process-plugin bridge: the registered plugins, their rules on the device, and what the
    // host walks add to the device-side counters (exports by reason, TopPorts)
    std::vector<ipxg_plugin> plugins;
    uint64_t follow_max = 0;  // the largest follow_packets of the registered plugins
    uint32_t walk_budget = 0;  // payload bytes of a walked packet outside every rule (0: whole frames)
    bool walk_full = false;    // IPXG_WALK_FULL=1: whole frames always (A/B knob)
    bool plug_all = false;    // a registered plugin acts on every packet (ipxg_plugin.all_packets)
    double walk_phase_ms[7] = {0, 0, 0, 0, 0, 0, 0};  // plugin_walk's phases (IPXG_WALK_TRACE)
    long walk_faults[7] = {0, 0, 0, 0, 0, 0, 0};        // ... and the minor page faults in each
    bool walk_trace = false;                             // IPXG_WALK_TRACE set at ipxg_create
    bool strict_prune = true;                            // strict: idle-free sweep steps left out of the DAG
    uint32_t strict_wgs = STRICT_WGS_DEFAULT;            // strict: replay workgroups per XCD (0: one workgroup)
    uint32_t* st_sched = nullptr;                        // strict: the multi-workgroup scheduler block
    DevBuf rules_d, pf_d, pf_idx, pf_wpk, pf_off, pf_bytes, pf_keys, pf_flen, pf_tmp, pf_live, pf_recs;
    // their host copies, kept across batches (HostVec: page-locked malloc memory)
    HostVec<uint32_t> hw_state, hw_lpos;  // the flows' slot states (then their new ones); live record positions
    HostVec<ipxg_flow_record> hw_recs;    // the live flows' records
    HostVec<uint32_t> hw_first;
    HostVec<uint64_t> hw_off;
    HostVec<WalkPkt> hw_wpk;  // the walked packets: parsed fields, descriptor, batch index
    HostVec<uint8_t> hw_bytes;
    bool walk_pin = true;  // HostVec page-locked (IPXG_WALK_PAGEABLE unset)
    uint64_t host_end[5] = {0, 0, 0, 0, 0};
    uint64_t host_pkts[6] = {0, 0, 0, 0, 0, 0};
    uint64_t host_unreasoned = 0;  // counted exports without an end reason (total_exported only)
    // the walk's threads (ipxg_set_walk_threads; 0 = default) and what each keeps across
    // batches: its exports of the current batch, its TopPorts counts (2 x 65536 when ps=true;
    // summed when read) and, for t >= 1, its copies of the plugins (ipxg_plugin.copy_ctx)
    uint32_t walk_threads = 0;
    bool walked = false;  // a plugin walk has called hooks (plugin instances no longer pristine)
    // a process plugin failed (IPXG_EPLUGIN): only ipxg_reset / ipxg_destroy until reset; its message
    bool failed = false;
    std::string fail_msg;
    WalkPool* pool = nullptr;
    std::vector<std::unique_ptr<ExportVec>> hw_ex;       // [u]: the walk's work units' outputs
    hipEvent_t walk_ev[WALK_CHUNKS] = {};                // the copies of each chunk of the walk's input
    std::vector<std::vector<uint64_t>> host_ports;      // [t]
    std::vector<std::vector<ipxg_plugin>> walk_pl;      // [t - 1]: thread t's plugin instances
    // staging for host batches
    DevBuf arena, desc;
    // scratch
    DevBuf defer_a, defer_b, frag_list, frag_sorted, frag_ports, sort_tmp;
    DevBuf adefer_a, adefer_b;           // deferred tile aggregates (3 x 16 B each)
    DevBuf cx_list, cx_sorted, cx_rank;  // cx_rank: 4 u32 arrays of nranks, then the key set
    DevBuf bin_rec, bin_count;           // k_bin -> k_reduce partitions
    uint32_t bin_slots[2][2][2][2][2] = {};  // k_bin workgroups resident at once (its grid), [agg][wide][plug][line][g64]
    // the plugins' rules flattened for k_bin's own check (Params::plug); plug_ok: they fit
    bool plug_ok = false;
    uint32_t plug_nport = 0, plug_npref = 0;
    uint32_t plug_port[16] = {}, plug_pref[16] = {}, plug_pmask[16] = {}, plug_pinfo[16] = {};
    DevBuf marks, mark_cnt;
    DevBuf plug_d;  // the flattened rules on the device (Params::plug_tab)
    bool wide = false;                   // the next batch's k_bin walks every header chain (WIDE)
    bool tile_agg = true;                // the next batch aggregates frequent flows per tile
    // an IPXG_BATCH_ASYNC batch whose kernels are enqueued but whose control block the host
    // has not read yet (completed by the next call on the engine)
    struct {
        bool on = false;
        bool tail = false;  // k_fin_list not launched yet (the next call picks its mode)
        BatchView bv;
        Params p;
        uint32_t n = 0;
    } inflight;
    // The next batch's front (control-block clear, k_bin, k_bin_slow) launched from inside the host
    // walk of the batch in flight, right after the walk's input copies: the device bins batch k+1
    // while the hooks run on batch k.  ipxg_submit of a device batch sets `want` around completing
    // the batch in flight; the walk launches it (`launched`) when the plugins' check rides in k_bin
    // (a k_classify pass would write the table the walk still owns).  k_bin then defers what does
    // not fit its segments (Params::defer_spill) instead of accumulating into the table.
    struct {
        bool want = false, launched = false;
        BatchView bv;
        uint32_t n = 0;
        Params p;
        BinView bins;
        BatchCtl snap;  // the walked batch's control block, as the walk found it
    } early;
    BatchCtl* aux_ctl_d = nullptr;  // k_plugin_apply's guard word while ctl_d holds the next batch's
    hipStream_t wst = nullptr;      // the host walk's input copies (beside the next batch's front)
    DevBuf slow_list, slow_cnt, fin_list;  // k_bin -> k_bin_slow, k_reduce -> k_fin_list
    // asynchronous host batches: two staging slots, filled on a copy stream while the other
    // slot's batch is in the kernels (the double-buffered ingest ring)
    DevBuf stage_arena[2], stage_desc[2];
    hipStream_t cst = nullptr;
    hipEvent_t copied[2] = {nullptr, nullptr};
    // k_classify runs beside k_bin / k_bin_slow on its own stream; k_reduce waits for it.  Both
    // sides may touch the same slots -- k_classify claims slots and ORs SLOT_PLUGIN, k_bin's spills
    // (a full segment: tile_emit) claim and accumulate into slots -- which is safe only because every
    // slot write on either side is an atomic CAS or RMW: a plain slot store added to either path
    // would race
    hipStream_t cls_st = nullptr;
    hipEvent_t cls_fork = nullptr, cls_join = nullptr;
    int stage_next = 0;
    DevBuf ipf_rec, ipf_out, ipf_tot, ipf_off;  // IPFIX formatting scratch
    DevBuf ipf_msg, ipf_plan;                   // IPFIX messages: output, plan (sets + messages)
    DevBuf ipf_dmsg[2];                         // ipxg_device_ipfix_messages' output, alternating
    uint32_t ipf_dnext = 0;
    // ipxg_device_ipfix_messages formats on a side stream (fst), forked from the engine's stream;
    // the engine's stream joins it (fmt_done) before the next kernel that appends exports
    hipStream_t fst = nullptr;
    hipEvent_t fmt_fork = nullptr, fmt_done = nullptr;
    bool fmt_pending = false;
    // recorded by ipxg_submit before its first kernel: every export of the batches completed
    // before it is in place (an asynchronous batch's formatting forks from here, beside its kernels)
    hipEvent_t ex_ev = nullptr;
    bool ex_ev_valid = false;  // recorded for the batch in flight (only while fst exists)
    uint8_t* plan_h = nullptr;                  // pinned staging of the plan (asynchronous upload)
    const uint64_t* ipf_counts = nullptr;       // device: {bytes, records} of the last message call
    size_t plan_h_bytes = 0;
    hipEvent_t plan_ev = nullptr;               // the last plan upload
    uint32_t last_touched = 0;           // flow aggregates of the previous batch
    uint32_t last_slow = 0xFFFFFFFFu;    // its slow-list packets (0: the next batch skips k_bin_slow; unknown at first)
    bool no_slow_skip = false;           // A/B knob IPXG_NO_SLOW_SKIP=1: k_bin_slow always launched
    uint32_t last_n = 0;                 // its packets
    double skew = 1.0;                   // previous batch: most loaded partition / mean partition
    uint32_t part_bits_last = 0;         // partitions of the last binned batch (log2)
    FragEntry* frag_ent = nullptr;
    uint32_t* frag_cnt = nullptr;
    // strict mode (strict=true): the reference's line table, replayed in packet order
    bool strict = false;
    StrictView sv = {};
    uint64_t strict_q = 0;  // sweep steps taken (keyed packets + expire calls): the cursor
    DevBuf st_pkt, st_crec, st_keyed, st_qx, st_keys, st_vals, st_keys2, st_vals2, st_succ, st_pred, st_indeg, st_queue;
    // host-side counters
    BinView bins_last = {};   // the last binned batch's partition records (k_complex_gather_rec)
    bool bins_valid = false;
    uint64_t gather_fallbacks = 0;  // complex gathers redone by re-parse (a complex flow in a tile aggregate)
    uint64_t gather_ranges = 0;     // tile aggregates of complex flows parsed again by range
    uint64_t complex_total = 0, rehashes = 0, batches = 0, spilled = 0, slow_pkts = 0, agg_pkts = 0, walked_pkts = 0;
    bool prev_valid = false;
    uint32_t prev_sec = 0, prev_usec = 0;
    // stage timing
    bool prof = false;
    int prof_level = 0;  // 1: every stage, 2: k_bin only, 3: k_bin and k_bin_slow
    // events on one batch of every prof_every (ipxg_profile's period): each event record is a
    // packet of its own on the stream (~4-5 us of GPU time, tools/gapbench), so the bench samples
    uint32_t prof_every = 1;
    uint64_t prof_seq = 0;
    bool prof_set[2] = {false, false};  // the batch of event set k (= its control block) is sampled
    hipEvent_t evs[2][12] = {};  // one set per control block (a pending batch keeps its events)
    hipEvent_t* ev = evs[0];
    bool early_timed = false;  // the batch in flight had an early front: its k_reduce is timed from ev[11]
    ipxg_timing tm = {};
};

static void free_walk_copies(ipxg_engine* e);

// events: 0 | k_bin | 1 | k_bin_slow | 2 | k_reduce | 3 | k_fin_list | 4;
//         [5,6] slow paths, [7,8] k_finalize, [9,10] finish; 11: k_reduce's start after an early
//         front (2 was recorded during the previous batch's host walk)
static bool prof_on(const ipxg_engine* e) { return e->prof && e->prof_set[e->ev == e->evs[1] ? 1 : 0]; }
// a batch starts (its front, or a strict batch): sampled or not
static void prof_begin_batch(ipxg_engine* e) {
    e->prof_set[e->cur] = e->prof && (e->prof_seq++ % e->prof_every) == 0;
}
static void ev_rec(ipxg_engine* e, int i) {
    // level 2: only the events around k_bin / k_ingest (0, 1), level 3 also k_bin_slow (2):
    // the others cost host time
    if (prof_on(e) && (e->prof_level == 1 || i <= 1 || (e->prof_level == 3 && i == 2)))
        if (hipEventRecord(e->ev[i], e->st) != hipSuccess) (void)hipGetLastError();
}
// (an event this batch did not record -- a path it did not take -- gives 0; its error is taken
// off HIP's last-error slot, which the next HIPCHK(hipGetLastError()) would otherwise report as
// the failure of whatever launch came next: "invalid resource handle" in a plugin batch's walk)
static double ev_ms(ipxg_engine* e, int a, int b = -1) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e->ev[a], e->ev[b < 0 ? a + 1 : b]) != hipSuccess) {
        (void)hipGetLastError();
        return 0.0;
    }
    return ms;
}

#define HIPCHK(e, call)                                                                  \
    do {                                                                                 \
        hipError_t _r = (call);                                                          \
        if (_r != hipSuccess) {                                                          \
            (e)->err = std::string(#call) + ": " + hipGetErrorString(_r);                \
            return IPXG_EDEVICE;                                                         \
        }                                                                                \
    } while (0)

static int set_err(ipxg_engine* e, int code, const std::string& msg) {
    if (e) e->err = msg;
    return code;
}

// (internal) a buffer would have to grow while ipxg_engine::no_grow is set
constexpr int IPXG_EGROW = 100;

static int ensure(ipxg_engine* e, DevBuf& b, size_t need) {
    if (b.bytes >= need && b.p) return IPXG_OK;
    if (e->no_grow) return IPXG_EGROW;  // (a front launched ahead: the pending batch may still read it)
    size_t nb = std::max<size_t>(need, b.bytes + b.bytes / 2);
    if (nb < 256) nb = 256;
    if (b.p) HIPCHK(e, hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, nb) != hipSuccess) return set_err(e, IPXG_ENOMEM, "hipMalloc failed");
    b.bytes = nb;
    return IPXG_OK;
}

static TableView table_view(ipxg_engine* e) {
    return TableView{e->line, e->tail, e->slot_rank, e->cap - 1, e->pstat_d};  // pstat_d starts with the ports
}

static ExportView export_view(ipxg_engine* e) {
    if (e->ex_zero_pending) {  // every kernel that appends exports gets its view here
        e->ex_zero_pending = false;
        (void)hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st);
    }
    return ExportView{e->ex, e->ex_count_d, e->ex_cap, e->count6_on ? 1u : 0u};
}

// Partitions for k_bin/k_reduce: enough that a partition's flows fit k_reduce's LDS table
// (RED_TARGET_FLOWS each), estimated from the previous batch's touched flows, never more
// than the batch's packets.  k_bin runs bin_grid persistent workgroups over tiles of
// BIN_TILE_PKTS packets; each owns one segment per partition, sized for its mean share of the
// packets times max(3 when aggregating else 1.5, 1.25 x the previous batch's most loaded
// partition / mean), plus 4 standard deviations (binomial) and a margin; what does not fit
// spills to atomics.  Memory is plentiful (288 GB of HBM) and only the slots written are
// read, so the margin is generous: skewed traffic (tile aggregation leaves the configs[2] Zipf
// mix at ~2.4x) does not spill after its first batch.
static bool wide_walk(const ipxg_engine* e) {
    if (e->cfg.flags & IPXG_CFG_WALK_WIDE) return true;
    if (e->cfg.flags & IPXG_CFG_WALK_NARROW) return false;
    return e->wide || e->plug_ok;  // (the plugins' check rides on the wide walk)
}

// k_bin checks the plugins' rules itself (no k_classify pass): rules that fit Params::plug, and
// the wide walk
static bool plug_fold(const ipxg_engine* e) {
    return e->plug_ok && !e->plugins.empty() && wide_walk(e) && !(e->cfg.flags & IPXG_CFG_ATOMIC_INGEST) &&
           !std::getenv("IPXG_CLASSIFY_PASS");  // (A/B knob: the separate k_classify pass)
}

// stream_ok: the batch may take the streamed reduce (line mode, no k_bin_slow launched behind k_bin,
// no process plugins, not an early front); it does when its flows fit the streamed reducer's LDS
// tables (RS_TARGET_FLOWS per partition) and the record area a 32-bit buffer range.
static int setup_bins(ipxg_engine* e, uint32_t n, bool g64, BinView& bv, bool stream_ok = false) {
    // the flows this batch touches: the previous batch's (scaled up to a larger batch), else the
    // live table's, else one per packet
    uint64_t est = e->last_touched ? e->last_touched : e->live;
    if (e->last_touched && e->last_n && n > e->last_n) est = est * n / e->last_n;
    if (est == 0 || est > n) est = n;
    uint32_t bits = 0;
    while (bits < BIN_MAX_PART_BITS && ((uint64_t)RED_TARGET_FLOWS << bits) < est) bits++;
    // at least a workgroup per CU (256) while partitions keep >= RED_MIN_FLOWS flows each
    while (bits < 8 && ((uint64_t)RED_MIN_FLOWS << bits) < est) bits++;
    if (const char* pb = std::getenv("IPXG_PART_BITS"))  // tuning knob (experiments only)
        bits = std::min<uint32_t>((uint32_t)std::atoi(pb), BIN_MAX_PART_BITS);
    bits = std::min<uint32_t>(bits, IPXG_KBIN_PMAX_BITS);  // (k_bin's histograms)
    const uint32_t P = 1u << bits;
    const uint64_t tiles = ((uint64_t)n + BIN_TILE_PKTS - 1) / BIN_TILE_PKTS;
    const int ag = e->tile_agg ? 1 : 0, wd = wide_walk(e) ? 1 : 0, pl = plug_fold(e) ? 1 : 0;
    // line mode (whole-line record stores) for the plain walk over at most BIN_LINE_P partitions
    // (g64: 16-byte unit offsets, the heads read through 64-bit addresses -- k_bin's G64 variants;
    // line mode has none)
    const int ln = !ag && !pl && !g64 && P <= BIN_LINE_P && !(e->cfg.flags & IPXG_CFG_ATOMIC_INGEST) && !e->no_line ? 1 : 0;
    uint32_t& slots = e->bin_slots[ag][wd][pl][ln][g64 ? 1 : 0];
    if (!slots) {
        slots = bin_resident_blocks(e->cfg.device_id, ag != 0, wd != 0, pl != 0, ln != 0, g64);
        if (const char* g = std::getenv("IPXG_BIN_GRID"))  // tuning knob (experiments only)
            slots = std::max(1u, std::min<uint32_t>((uint32_t)std::atoi(g), BIN_MAX_GRID));
    }
    if (!e->stream_grid) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->cfg.device_id) != hipSuccess || cus < 1)
            cus = 256;
        e->stream_grid = std::min<uint32_t>(2u * (uint32_t)cus, RS_MAX_COLS);
        if (const char* g = std::getenv("IPXG_STREAM_GRID"))  // tuning knob (experiments only)
            e->stream_grid = std::max(1u, std::min<uint32_t>((uint32_t)std::atoi(g), RS_MAX_COLS));
    }
    auto seg_for = [&](uint32_t grid) {
        const uint64_t per_block = std::min<uint64_t>((tiles + grid - 1) / grid * BIN_TILE_PKTS, n);
        const double mean = (double)per_block / P;
        // aggregating batches follow a skewed one (the most loaded partition ~2.4x the mean with
        // the configs[2] Zipf mix); the others spill only if the skew changed since the last batch
        const double factor = std::max(e->tile_agg ? 3.0 : 1.5, 1.25 * e->skew);
        uint64_t seg = ((uint64_t)(mean * factor + 4.0 * std::sqrt(mean) + 16.0) + 3) & ~3ull;
        if (ln) seg = (seg + 8 + 7) & ~7ull;  // whole lines, and the carry's padded last line
        return seg;
    };
    bool sm = ln && stream_ok && !e->no_stream && est <= (uint64_t)RS_TARGET_FLOWS << bits;
    uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, sm ? e->stream_grid : slots);
    uint64_t seg = seg_for(grid);
    if (sm && (uint64_t)P * 2 * grid * seg * 16 >= 0xFFFFFF00ull) {  // (the record area's buffer range)
        sm = false;
        grid = (uint32_t)std::min<uint64_t>(tiles, slots);
        seg = seg_for(grid);
    }
    const uint32_t cols = 2 * grid;
    int rc;
    if ((rc = ensure(e, e->bin_rec, (size_t)P * cols * seg * sizeof(uint4)))) return rc;
    if ((rc = ensure(e, e->bin_count, (size_t)P * cols * sizeof(uint32_t)))) return rc;
    // each k_bin workgroup's slow list holds every packet of its tiles
    const uint64_t slow_stride = (tiles + grid - 1) / grid * BIN_TILE_PKTS;
    if ((rc = ensure(e, e->slow_list, (size_t)grid * slow_stride * sizeof(uint4)))) return rc;
    if ((rc = ensure(e, e->slow_cnt, (size_t)grid * sizeof(uint32_t)))) return rc;
    bv.slow_stride = (uint32_t)slow_stride;
    bv.slow_cnt = (uint32_t*)e->slow_cnt.p;  // written by every k_bin workgroup
    bv.marks = nullptr;
    bv.mark_cnt = nullptr;
    if (pl) {  // (as the slow lists: room for every packet of a workgroup's tiles)
        if ((rc = ensure(e, e->marks, (size_t)grid * slow_stride * sizeof(uint4)))) return rc;
        if ((rc = ensure(e, e->mark_cnt, (size_t)grid * sizeof(uint32_t)))) return rc;
        bv.marks = (uint4*)e->marks.p;
        bv.mark_cnt = (uint32_t*)e->mark_cnt.p;  // written by every k_bin workgroup
    }
    // no clearing: every k_bin / k_bin_slow workgroup writes its whole column of counts
    bv.rec = (uint4*)e->bin_rec.p;
    bv.count = (uint32_t*)e->bin_count.p;
    bv.seg_cap = (uint32_t)seg;
    bv.line = (uint32_t)ln;
    bv.cols = cols;
    bv.bin_grid = grid;
    bv.part_bits = bits;
    bv.prog = nullptr;
    bv.prog_tag = 0;
    // line mode's record stores write-through (rec_rsrc, ipxg_ingest.hip) where the record area fits
    // the 32-bit buffer range: udp64 step -1.8 %; the partial-line stores of tile_emit (the 1M-flow
    // mixes) lose with it (quic +1.7 %, imix +-0, profiles/r06/sc1_ab.txt).  IPXG_REC_SC1=0: plain
    // stores (A/B knob); 2: write-through in every mode
    bv.prog_mode = e->rec_sc1 && (ln || e->rec_sc1 == 2) && (uint64_t)P * cols * seg * 16 < 0xFFFFFF00ull ? PROG_SC1 : 0u;
    bv.pub_every = 1;
    bv.rs_sleep = 0;
    // IPXG_SLOW_GROUP=n (A/B knob): each k_bin_slow workgroup takes n k_bin workgroups' slow lists --
    // denser record segments, a quarter of the count columns, but configs[4]'s slow pass went from 44
    // to 82 us per batch at n = 4 and k_reduce from 200 to 230 (fewer, longer workgroups: the slow
    // parser is latency-bound), so one list each.  Not with process plugins (a workgroup appends the
    // marks of its own k_bin workgroup's list).
    bv.slow_group = 1;
    if (const char* sg = std::getenv("IPXG_SLOW_GROUP"))
        bv.slow_group = e->plugins.empty() ? std::max(1u, std::min<uint32_t>((uint32_t)std::atoi(sg), SLOW_GROUP_MAX)) : 1u;
    if (sm) {
        if ((rc = ensure(e, e->prog, (size_t)RS_MAX_COLS * P * sizeof(uint32_t)))) return rc;
        if (++e->prog_epoch > (PROG_EPOCH_MASK >> PROG_EPOCH_SHIFT) || grid != e->prog_g || P != e->prog_p) {
            HIPCHK(e, hipMemsetAsync(e->prog.p, 0, (size_t)RS_MAX_COLS * P * sizeof(uint32_t), e->st));  // (epoch 0: none)
            e->prog_epoch = 1;
            e->prog_g = grid;
            e->prog_p = P;
        }
        bv.prog = (uint32_t*)e->prog.p;
        bv.prog_tag = e->prog_epoch << PROG_EPOCH_SHIFT;
        bv.prog_mode = (e->prog_mode & PROG_TILE) | ((e->prog_mode & PROG_SC1) ? PROG_SC1 : 0u);
        bv.pub_every = e->pub_every;
        bv.rs_sleep = e->rs_sleep;
    }
    e->part_bits_last = bits;
    return IPXG_OK;
}

static FragView frag_view(ipxg_engine* e) {
    return FragView{e->frag_ent, e->frag_cnt, (uint64_t*)e->frag_list.p, (uint64_t*)e->frag_sorted.p,
                    (uint32_t*)e->frag_ports.p};
}

static Params params(ipxg_engine* e) {
    Params p = {};
    p.dlt = e->cfg.datalink;
    p.active_s = e->cfg.active_s;
    p.inactive_s = e->cfg.inactive_s;
    p.bucket_w = std::max<uint32_t>(1, e->cfg.inactive_s / 2);
    p.split_biflow = e->cfg.split_biflow;
    p.frag_enable = e->cfg.frag_enable;
    p.frag_size = e->cfg.frag_size ? e->cfg.frag_size : 10007;
    p.frag_timeout_s = e->cfg.frag_timeout_s;
    p.force_complex = e->cfg.inactive_s < 2 ? 1 : 0;
    p.prev_valid = e->prev_valid;
    p.prev_sec = e->prev_sec;
    p.prev_usec = e->prev_usec;
    p.tile_agg = e->tile_agg ? 1 : 0;
    p.wide = wide_walk(e) ? 1 : 0;
    p.plug = plug_fold(e) ? 1 : 0;
    if (p.plug) {
        p.plug_nport = e->plug_nport;
        p.plug_npref = e->plug_npref;
        p.plug_tab = (const uint32_t*)e->plug_d.p;
    }
    p.plug_all = e->plug_all ? 1u : 0u;
    p.spin_max = STRICT_SPIN_MAX;
    if (const char* sm = std::getenv("IPXG_STRICT_SPIN_MAX"))  // test knob: a short watchdog
        p.spin_max = std::max<uint32_t>(16, (uint32_t)std::strtoul(sm, nullptr, 0));
    return p;
}

static int alloc_table(ipxg_engine* e, uint32_t cap, SlotLine** line, uint32_t** tail, uint32_t** rank) {
    if (hipMalloc((void**)line, sizeof(SlotLine) * (size_t)cap) != hipSuccess) return IPXG_ENOMEM;
    if (hipMalloc((void**)tail, sizeof(uint32_t) * REC_TAIL_WORDS * (size_t)cap) != hipSuccess) {
        hipFree(*line);
        return IPXG_ENOMEM;
    }
    if (hipMalloc((void**)rank, sizeof(uint32_t) * (size_t)cap) != hipSuccess) {
        hipFree(*line);
        hipFree(*tail);
        return IPXG_ENOMEM;
    }
    HIPCHK(e, hipMemsetAsync(*line, 0, sizeof(SlotLine) * (size_t)cap, e->st));
    return IPXG_OK;
}

constexpr size_t CTL_EX_OFF = (sizeof(BatchCtl) + 15) & ~(size_t)15;  // a block's stride; the export words in the mirror
constexpr size_t CTL_BYTES = CTL_EX_OFF + 32;  // the host mirror: block, export words, sequence word

static const uint32_t* ex_host(const ipxg_engine* e) {
    return reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(e->ctl_h) + CTL_EX_OFF);
}
static volatile uint32_t* seq_host(const ipxg_engine* e) {
    return reinterpret_cast<volatile uint32_t*>(reinterpret_cast<char*>(e->ctl_h) + CTL_EX_OFF + 16);
}

// Wait for the stream by polling: the blocking wait (interrupt) added tens of microseconds of
// idle GPU per batch; the engine's syncs are short.
static hipError_t stream_wait(hipStream_t st) {
    hipError_t r;
    while ((r = hipStreamQuery(st)) == hipErrorNotReady) {
    }
    return r;
}

static int check_ex(ipxg_engine* e) {
    if (e->ex_zero_pending) return IPXG_OK;  // the device counters are stale until zeroed; the host's are 0
    e->ex_count = ex_host(e)[0];
    e->ex_count6 = ex_host(e)[2];
    if (ex_host(e)[1]) return set_err(e, IPXG_EDEVICE, "a kernel counted more exports than the export buffer holds (its capacity is sized before the launch from the live and batch counts)");
    return IPXG_OK;
}

// A fused k_fin_list left holes in its export reservation (flows that turned complex or found no
// slot; their batch goes to the sequential path anyway): closed on the device before anything reads
// the exports, and the published count lowered to match.  The records below the host's count were
// there before the batch; if the counters were reset meanwhile (ipxg_clear_exports), from 0.
static int close_export_holes(ipxg_engine* e) {
    if (e->ex_zero_pending) return IPXG_OK;  // (the exports are dropped anyway)
    uint32_t* pub = const_cast<uint32_t*>(ex_host(e));
    const uint32_t hi = std::min(pub[0], e->ex_cap), holes = e->ctl_h->ex_holes;
    const uint32_t lo = e->ex_count <= hi ? e->ex_count : 0u;
    if (holes > hi - lo) return set_err(e, IPXG_EDEVICE, "more export holes than reserved records");
    launch_ex_compact(e->st, export_view(e), lo, hi);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipStreamSynchronize(e->st));
    pub[0] = hi - holes;
    e->tm.ex_compactions++;
    return IPXG_OK;
}

// the control block and the export counter into host-mapped memory (a one-block kernel on
// the stream: cheaper than a D2H copy command); seq: with a sequence number the host polls
static int publish_ctl(ipxg_engine* e, bool with_seq = false) {
    uint32_t seq = 0;
    if (with_seq) {
        if (++e->pub_seq == 0) e->pub_seq = 1;  // (0: no sequence word)
        seq = e->pub_seq;
    }
    launch_publish(e->st, reinterpret_cast<const uint32_t*>(e->ctl_d), e->ex_count_d, e->ctl_hd,
                   (uint32_t)(CTL_EX_OFF / 4), seq);
    HIPCHK(e, hipGetLastError());
    return IPXG_OK;
}

// Wait for the publish with sequence number `seq` (publish_ctl(e, true)) by polling its word in
// host memory: the stream may hold more work behind it (a front launched ahead).  A device error
// or a stream that drained without the word is reported, never waited on forever.
static int wait_seq(ipxg_engine* e, uint32_t seq) {
    volatile uint32_t* w = seq_host(e);
    for (uint64_t k = 1;; ++k) {
        if (*w == seq) break;
        if ((k & 1023) == 0) {
            const hipError_t r = hipStreamQuery(e->st);
            if (r != hipSuccess && r != hipErrorNotReady) HIPCHK(e, r);
            if (r == hipSuccess && *w != seq) return set_err(e, IPXG_EDEVICE, "control block publish never arrived");
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return IPXG_OK;
}

static int sync_ctl(ipxg_engine* e) {
    int rc;
    if ((rc = publish_ctl(e))) return rc;
    HIPCHK(e, stream_wait(e->st));
    return check_ex(e);
}

// Rebuild the table at new_cap, dropping dead slots (no live record, untouched).
static int rehash(ipxg_engine* e, uint32_t new_cap) {
    SlotLine* nh;
    uint32_t* nc;
    uint32_t* nr;
    int rc = alloc_table(e, new_cap, &nh, &nc, &nr);
    if (rc) return set_err(e, rc, "table allocation failed (capacity " + std::to_string(new_cap) + ")");
    HIPCHK(e, hipMemsetAsync(e->misc_d, 0, sizeof(uint32_t), e->st));
    TableView to{nh, nc, nr, new_cap - 1, e->pstat_d};
    launch_rehash(e->st, table_view(e), e->cap, to, e->misc_d);
    HIPCHK(e, hipGetLastError());
    uint32_t fail = 0;
    HIPCHK(e, hipMemcpyAsync(&fail, e->misc_d, sizeof(uint32_t), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    HIPCHK(e, hipFree(e->line));
    HIPCHK(e, hipFree(e->tail));
    HIPCHK(e, hipFree(e->slot_rank));
    e->line = nh;
    e->tail = nc;
    e->slot_rank = nr;
    e->cap = new_cap;
    e->rehashes++;
    if (fail) return set_err(e, IPXG_ENOMEM, "rehash could not place every flow");
    return IPXG_OK;
}

// The engine's stream waits for the device IPFIX formatting in flight (ipxg_device_ipfix_messages
// on fst: it reads the exports and the IPFIX scratch buffers) before anything that appends or
// moves exports or reuses those buffers.  Stream order only: no host wait.
static int join_fmt(ipxg_engine* e) {
    if (!e->fmt_pending) return IPXG_OK;
    e->fmt_pending = false;
    HIPCHK(e, hipStreamWaitEvent(e->st, e->fmt_done, 0));
    return IPXG_OK;
}

static int ensure_export(ipxg_engine* e, size_t extra) {
    size_t pending = e->ex_count - e->ex_head;
    if (e->ex_count + extra <= e->ex_cap) return IPXG_OK;
    {
        const int rc0 = join_fmt(e);  // (the records move)
        if (rc0) return rc0;
    }
    size_t need = pending + extra;
    if (need > 0xFFFFFFF0ull) return set_err(e, IPXG_ENOMEM, "export buffer would exceed 2^32 records");
    if (need <= e->ex_cap && e->ex_head >= pending) {  // compact in place (no overlap)
        if (pending)
            HIPCHK(e, hipMemcpyAsync(e->ex, e->ex + e->ex_head, pending * sizeof(ipxg_flow_record),
                                     hipMemcpyDeviceToDevice, e->st));
    } else {
        size_t ncap = std::max<size_t>(need, (size_t)e->ex_cap * 2);
        ipxg_flow_record* nb;
        if (hipMalloc((void**)&nb, ncap * sizeof(ipxg_flow_record)) != hipSuccess)
            return set_err(e, IPXG_ENOMEM, "export buffer allocation failed");
        if (pending)
            HIPCHK(e, hipMemcpyAsync(nb, e->ex + e->ex_head, pending * sizeof(ipxg_flow_record),
                                     hipMemcpyDeviceToDevice, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
        HIPCHK(e, hipFree(e->ex));
        e->ex = nb;
        e->ex_cap = (uint32_t)ncap;
    }
    e->ex_head = 0;
    e->ex_count = (uint32_t)pending;
    e->ex6_valid = false;  // [2] counted records that are gone now
    HIPCHK(e, hipMemcpyAsync(e->ex_count_d, &e->ex_count, sizeof(uint32_t), hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return IPXG_OK;
}

static uint32_t pow2_at_least(uint64_t v) {
    uint32_t c = 16;
    while (c < v && c < (1u << 30)) c <<= 1;
    return c;
}

extern "C" {

void ipxg_config_default(ipxg_config* cfg) {
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->cache_exp = 17;  // cache.hpp:54
    cfg->line_exp = 4;    // cache.hpp:60
    cfg->active_s = 300;  // cache.hpp:63-64
    cfg->inactive_s = 30;
    cfg->split_biflow = 0;
    cfg->frag_enable = 1;  // cache.hpp:99-102
    cfg->frag_size = 10007;
    cfg->frag_timeout_s = 3;
    cfg->device_id = 0;
    cfg->batch_pkts = 1u << 20;
    cfg->datalink = IPXG_DLT_EN10MB;
}

// Timing-experiment builds drop or fake work (-DIPXG_EXP_NOEMIT/NOHASH/LOADONLY) or add clock
// probes (-DIPXG_PROBE); one such variant in round 2 (an atomic skipped in k_reduce) left slots
// half-claimed and ipxg_finish then read past the table (an illegal memory access).  Their
// engines only start for a tuning run that asks for them (IPXG_TUNING=1).
#if defined(IPXG_TUNING_BUILD) || defined(IPXG_EXP_NOEMIT) || defined(IPXG_EXP_NOHASH) || \
    defined(IPXG_EXP_LOADONLY) || defined(IPXG_PROBE)
static constexpr bool kTuningBuild = true;
#else
static constexpr bool kTuningBuild = false;
#endif

int ipxg_create(const ipxg_config* cfg, ipxg_engine** out) {
    if (!cfg || !out) return IPXG_EINVAL;
    *out = nullptr;
    if (kTuningBuild) {
        const char* t = std::getenv("IPXG_TUNING");
        if (!t || std::strcmp(t, "1") != 0) {
            std::fprintf(stderr, "ipxg: timing-experiment build of libipxg refused (set IPXG_TUNING=1)\n");
            return IPXG_ESTATE;
        }
    }
    if (cfg->cache_exp < 4 || cfg->cache_exp > 30) return IPXG_EINVAL;
    if (cfg->frag_enable && cfg->frag_size == 0) return IPXG_EINVAL;
    ipxg_engine* e = new ipxg_engine();
    e->cfg = *cfg;
    e->walk_trace = std::getenv("IPXG_WALK_TRACE") != nullptr;
    e->walk_pin = std::getenv("IPXG_WALK_PAGEABLE") == nullptr;
    e->sync_finish = std::getenv("IPXG_SYNC_FINISH") != nullptr && std::atoi(std::getenv("IPXG_SYNC_FINISH")) != 0;
    e->no_ahead = std::getenv("IPXG_NO_AHEAD") != nullptr && std::atoi(std::getenv("IPXG_NO_AHEAD")) != 0;
    e->no_line = std::getenv("IPXG_NO_LINE") != nullptr && std::atoi(std::getenv("IPXG_NO_LINE")) != 0;
    e->no_stream = !(std::getenv("IPXG_STREAM") != nullptr && std::atoi(std::getenv("IPXG_STREAM")) != 0);
    if (const char* pm = std::getenv("IPXG_PROG_MODE")) e->prog_mode = (uint32_t)std::atoi(pm) & 3u;
    if (const char* fl = std::getenv("IPXG_FIN_LORDER")) e->fin_lorder = std::atoi(fl) != 0;
    e->no_idle_floor = std::getenv("IPXG_NO_IDLE_FLOOR") != nullptr && std::atoi(std::getenv("IPXG_NO_IDLE_FLOOR")) != 0;
    if (const char* rs = std::getenv("IPXG_REC_SC1")) e->rec_sc1 = (uint32_t)std::max(0, std::atoi(rs));
    if (const char* pe = std::getenv("IPXG_PUB_EVERY")) e->pub_every = std::max(1, std::atoi(pe));
    if (const char* rsl = std::getenv("IPXG_RS_SLEEP")) e->rs_sleep = (uint32_t)std::max(0, std::atoi(rsl));
    if (const char* rx = std::getenv("IPXG_RS_EXP")) e->rs_sleep |= (uint32_t)std::atoi(rx) << 16;  // (timing only)
    e->walk_full = std::getenv("IPXG_WALK_FULL") != nullptr && std::atoi(std::getenv("IPXG_WALK_FULL")) != 0;
    e->no_slow_skip = std::getenv("IPXG_NO_SLOW_SKIP") != nullptr && std::atoi(std::getenv("IPXG_NO_SLOW_SKIP")) != 0;
    if (const char* sp_env = std::getenv("IPXG_STRICT_PRUNE")) e->strict_prune = std::atoi(sp_env) != 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        delete e;
        return IPXG_EDEVICE;
    }
    if (cfg->device_id < 0 || cfg->device_id >= ndev || hipSetDevice(cfg->device_id) != hipSuccess) {
        delete e;
        return IPXG_EINVAL;
    }
    int rc = IPXG_OK;
    auto fail = [&](int code) {
        ipxg_destroy(e);
        return code;
    };
    if (hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) != hipSuccess) return fail(IPXG_EDEVICE);
    // the reference sizes its table 2^s with 16-way lines; ours is open-addressed and grows,
    // so start at 2^s but never below 2^16
    uint32_t cap = 1u << std::max<uint32_t>(cfg->cache_exp, 16);
    if ((rc = alloc_table(e, cap, &e->line, &e->tail, &e->slot_rank))) return fail(rc);
    if (const char* a = std::getenv("IPXG_TILE_AGG")) e->tile_agg = std::atoi(a) != 0;  // tests / experiments
    e->cap = cap;
    e->ex_cap = 1u << 16;
    if (hipMalloc((void**)&e->ex, (size_t)e->ex_cap * sizeof(ipxg_flow_record)) != hipSuccess) return fail(IPXG_ENOMEM);
    {
        char* blk;
        if (hipMalloc((void**)&blk, 2 * CTL_EX_OFF + 16) != hipSuccess) return fail(IPXG_ENOMEM);
        e->ctl_blk[0] = reinterpret_cast<BatchCtl*>(blk);
        e->ctl_blk[1] = reinterpret_cast<BatchCtl*>(blk + CTL_EX_OFF);
        e->ex_count_d = reinterpret_cast<uint32_t*>(blk + 2 * CTL_EX_OFF);
        e->ctl_d = e->ctl_blk[0];
        if (hipMemsetAsync(blk, 0, 2 * CTL_EX_OFF + 16, e->st) != hipSuccess) return fail(IPXG_EDEVICE);
        e->blk_zero[1] = true;  // (block 0 is the current one: never marked zero)
    }
    if (hipHostMalloc((void**)&e->ctl_h, CTL_BYTES, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return fail(IPXG_ENOMEM);
    std::memset(e->ctl_h, 0, CTL_BYTES);
    if (hipHostGetDevicePointer((void**)&e->ctl_hd, e->ctl_h, 0) != hipSuccess) return fail(IPXG_EDEVICE);
    if (hipMalloc((void**)&e->misc_d, 16 * sizeof(uint32_t)) != hipSuccess) return fail(IPXG_ENOMEM);
    if (hipMalloc((void**)&e->stats_d, STAT_SHARDS * ST_STRIDE * sizeof(unsigned long long)) != hipSuccess)
        return fail(IPXG_ENOMEM);
    const uint32_t fs = cfg->frag_size ? cfg->frag_size : 10007;
    if (hipMalloc((void**)&e->frag_ent, (size_t)fs * 4 * sizeof(FragEntry)) != hipSuccess) return fail(IPXG_ENOMEM);
    if (hipMalloc((void**)&e->frag_cnt, (size_t)fs * sizeof(uint32_t)) != hipSuccess) return fail(IPXG_ENOMEM);
    if (hipMemsetAsync(e->frag_cnt, 0, (size_t)fs * sizeof(uint32_t), e->st) != hipSuccess) return fail(IPXG_EDEVICE);
    if (hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st) != hipSuccess) return fail(IPXG_EDEVICE);
    if (hipMemsetAsync(e->stats_d, 0, STAT_SHARDS * ST_STRIDE * sizeof(unsigned long long), e->st) != hipSuccess)
        return fail(IPXG_EDEVICE);
    if (e->cfg.flags & IPXG_CFG_STRICT) {
        if (cfg->line_exp > 4 || cfg->line_exp > cfg->cache_exp || cfg->cache_exp - cfg->line_exp > 24 ||
            (cfg->flags & (IPXG_CFG_ATOMIC_INGEST | IPXG_CFG_PARSER_STATS)))
            return fail(IPXG_EINVAL);
        e->strict = true;
        const uint32_t S = 1u << cfg->cache_exp;
        e->sv.line_bits = cfg->line_exp;
        e->sv.lines = S >> cfg->line_exp;
        e->sv.slot_mask = S - 1;
        if (hipMalloc((void**)&e->sv.rec, (size_t)S * sizeof(ipxg_flow_record)) != hipSuccess) return fail(IPXG_ENOMEM);
        // (hash and time_last padded by 64 bytes: the multi-workgroup replay reads lines as 16-byte loads)
        if (hipMalloc((void**)&e->sv.hash, (size_t)S * 8 + 64) != hipSuccess) return fail(IPXG_ENOMEM);
        if (hipMalloc((void**)&e->sv.perm, (size_t)e->sv.lines * 8) != hipSuccess) return fail(IPXG_ENOMEM);
        if (hipMalloc((void**)&e->sv.tlast, (size_t)S * 4 + 64) != hipSuccess) return fail(IPXG_ENOMEM);
        if (hipMalloc((void**)&e->st_sched, STRICT_SCHED_BYTES) != hipSuccess) return fail(IPXG_ENOMEM);
        // the replay on several workgroups of one XCD (IPXG_STRICT_WGS: workgroups per XCD, 0 = one
        // workgroup); its buffer loads address the record array with 32-bit offsets
        if (const char* w_env = std::getenv("IPXG_STRICT_WGS")) e->strict_wgs = (uint32_t)std::atoi(w_env);
        if (e->strict_wgs > 32 || (size_t)S * sizeof(ipxg_flow_record) > 0x7FFFFFFFull) e->strict_wgs = 0;
        if (hipMalloc((void**)&e->sv.lb, ((size_t)e->sv.lines + 1) * 4) != hipSuccess) return fail(IPXG_ENOMEM);
        launch_strict_clear(e->st, e->sv);
        if (hipGetLastError() != hipSuccess) return fail(IPXG_EDEVICE);
    }
    if (e->cfg.flags & IPXG_CFG_PARSER_STATS) {
        if (hipMalloc((void**)&e->pstat_d, PSTAT_WORDS * 8) != hipSuccess) return fail(IPXG_ENOMEM);
        if (hipMemsetAsync(e->pstat_d, 0, PSTAT_WORDS * 8, e->st) != hipSuccess) return fail(IPXG_EDEVICE);
    }
    if (hipStreamSynchronize(e->st) != hipSuccess) return fail(IPXG_EDEVICE);
    *out = e;
    return IPXG_OK;
}

int ipxg_destroy(ipxg_engine* e) {
    if (e && e->walk_trace && e->tm.plugin_flows)
        std::fprintf(stderr,
                     "ipxg plugin walk ms: order %.1f copies %.1f walk %.1f back %.1f"
                     " | minor faults: %ld %ld %ld %ld | host buffers allocated %lu, not page-locked %lu"
                     " | complex gathers re-parsed %lu, aggregate ranges %lu\n",
                     e->walk_phase_ms[0], e->walk_phase_ms[1], e->walk_phase_ms[5], e->walk_phase_ms[6],
                     e->walk_faults[0], e->walk_faults[1], e->walk_faults[5], e->walk_faults[6],
                     (unsigned long)g_hostvec_allocs.load(), (unsigned long)g_hostvec_unpinned.load(),
                     (unsigned long)e->gather_fallbacks, (unsigned long)e->gather_ranges);
    if (!e) return IPXG_OK;
    if (e->st) hipStreamSynchronize(e->st);
    if (e->fst) hipStreamSynchronize(e->fst);
    if (e->wst) hipStreamSynchronize(e->wst);
    delete e->pool;
    free_walk_copies(e);
    hipFree(e->line);
    hipFree(e->tail);
    hipFree(e->slot_rank);
    hipFree(e->ex);
    hipFree(e->ctl_blk[0]);
    hipFree(e->aux_ctl_d);
    if (e->wst) (void)hipStreamDestroy(e->wst);
    if (e->ctl_h) hipHostFree(e->ctl_h);
    hipFree(e->misc_d);
    hipFree(e->stats_d);
    if (e->cst) (void)hipStreamDestroy(e->cst);
    for (hipEvent_t ev : e->copied)
        if (ev) (void)hipEventDestroy(ev);
    if (e->cls_st) (void)hipStreamDestroy(e->cls_st);
    for (hipEvent_t ev : {e->cls_fork, e->cls_join})
        if (ev) (void)hipEventDestroy(ev);
    if (e->rst) {
        (void)hipStreamSynchronize(e->rst);
        (void)hipStreamDestroy(e->rst);
    }
    for (hipEvent_t ev : {e->rs_fork, e->rs_join})
        if (ev) (void)hipEventDestroy(ev);
    if (e->pstat_d) hipFree(e->pstat_d);
    hipFree(e->sv.rec);
    hipFree(e->sv.hash);
    hipFree(e->sv.perm);
    hipFree(e->sv.tlast);
    hipFree(e->sv.lb);
    hipFree(e->st_sched);
    hipFree(e->frag_ent);
    hipFree(e->frag_cnt);
    if (e->plan_h) hipHostFree(e->plan_h);
    if (e->plan_ev) (void)hipEventDestroy(e->plan_ev);
    if (e->fst) (void)hipStreamDestroy(e->fst);
    for (hipEvent_t ev : {e->fmt_fork, e->fmt_done, e->ex_ev})
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : e->walk_ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& set : e->evs)
        for (hipEvent_t ev : set)
            if (ev) (void)hipEventDestroy(ev);
    for (DevBuf* b : {&e->stage_arena[0], &e->stage_arena[1], &e->stage_desc[0], &e->stage_desc[1], &e->rules_d, &e->pf_d, &e->pf_idx, &e->pf_wpk, &e->pf_off, &e->pf_bytes,
                      &e->pf_keys, &e->pf_flen, &e->pf_tmp, &e->pf_live, &e->pf_recs,
                      &e->arena, &e->desc, &e->defer_a, &e->defer_b, &e->adefer_a, &e->adefer_b, &e->frag_list,
                      &e->frag_sorted,
                      &e->frag_ports, &e->sort_tmp, &e->cx_list, &e->cx_sorted, &e->cx_rank, &e->bin_rec,
                      &e->bin_count, &e->slow_list, &e->slow_cnt, &e->fin_list, &e->ipf_rec, &e->ipf_out,
                      &e->ipf_tot, &e->ipf_off, &e->ipf_msg, &e->ipf_dmsg[0], &e->ipf_dmsg[1], &e->ipf_plan, &e->st_pkt, &e->st_crec, &e->st_keyed,
                      &e->st_qx, &e->st_keys, &e->st_vals, &e->st_keys2, &e->st_vals2, &e->st_succ, &e->st_pred, &e->st_indeg,
                      &e->st_queue, &e->marks, &e->mark_cnt, &e->plug_d, &e->prog})
        hipFree(b->p);
    if (e->st) (void)hipStreamDestroy(e->st);
    delete e;
    return IPXG_OK;
}

const char* ipxg_last_error(const ipxg_engine* e) { return e ? e->err.c_str() : "null engine"; }

void* ipxg_stream(ipxg_engine* e) { return e ? (void*)e->st : nullptr; }

void* ipxg_ipfix_stream(ipxg_engine* e) {
    if (!e) return nullptr;
    return e->fst ? (void*)e->fst : (void*)e->st;
}

static int post_batch(ipxg_engine* e, BatchView bv, Params p, uint32_t n, bool binned, bool finishing);

// The in-flight asynchronous batch, if any: wait for its kernels and run post_batch.  Every
// entry point that reads or changes engine state calls this first.
// The asynchronous batch's last kernel, launched by the next call: k_fin_list, with the
// finish folded in when that call is ipxg_finish on a table that was empty before the batch.
static int launch_tail(ipxg_engine* e, bool finishing) {
    if (!e->inflight.tail) return IPXG_OK;
    e->inflight.tail = false;
    {
        const int rc0 = join_fmt(e);  // (k_fin_list appends exports)
        if (rc0) return rc0;
    }
    ev_rec(e, 3);
    // a finish fused into the pass writes its exports in list order from the export count, which the
    // host knows exactly when no batch is pending (its exports counted) -- 0 after ipxg_clear_exports
    const uint32_t ex_start = !finishing || e->pend.on || !e->fin_lorder ? EX_START_NONE : e->ex_zero_pending ? 0u : e->ex_count;
    launch_fin_list(e->st, e->inflight.bv, e->inflight.p, table_view(e), frag_view(e), export_view(e), e->ctl_d,
                    (HotSlot*)e->fin_list.p, e->stats_d, e->inflight.n, finishing, false, ex_start);
    ev_rec(e, 4);
    HIPCHK(e, hipGetLastError());
    return IPXG_OK;
}

static int complete_batch_impl(ipxg_engine* e, bool spec);
// (every entry point completes the batch in flight and the pending batch first: no C++ exception
// leaves it, and a failed engine completes nothing).  spec: ipxg_submit launched its front ahead.
static int complete_batch(ipxg_engine* e, bool spec = false) {
    if (e->failed)
        return set_err(e, IPXG_ESTATE, "engine stopped by a process plugin error (ipxg_reset or ipxg_destroy): " +
                                           e->fail_msg);
    if (!e->inflight.on && !e->pend.on) return IPXG_OK;
    try {
        return complete_batch_impl(e, spec);
    } catch (const std::bad_alloc&) {
        return set_err(e, IPXG_ENOMEM, "host allocation failed");
    } catch (...) {
        return set_err(e, IPXG_EDEVICE, "internal error: exception while completing a batch");
    }
}

// The pending state of a batch whose last kernels are enqueued: its control block published with
// a sequence number, completed later by consume_pend.
static void set_pend(ipxg_engine* e, uint32_t mode, const BatchView& bv, const Params& p, uint32_t n) {
    auto& q = e->pend;
    q.on = true;
    q.mode = mode;
    q.clear_after = false;
    q.blk = e->cur;
    q.seq = 0;
    q.published = false;
    q.bv = bv;
    q.p = p;
    q.n = n;
    q.bins = e->bins_last;
    q.bins_valid = e->bins_valid;
    q.part_bits = e->part_bits_last;
    q.spec_closed = false;
}

// The in-flight asynchronous batch's end: its tail (k_fin_list) and its control block's publish
// are enqueued, the host does not wait (the batch is pending until consume_pend).
static int enqueue_batch_end(ipxg_engine* e) {
    int rc;
    if ((rc = launch_tail(e, false))) return rc;
    e->inflight.on = false;
    set_pend(e, GATE_BATCH, e->inflight.bv, e->inflight.p, e->inflight.n);
    return IPXG_OK;
}

static int consume_pend(ipxg_engine* e, bool spec);
static int expire_table(ipxg_engine* e, int64_t now_sec);

static int complete_batch_impl(ipxg_engine* e, bool spec) {
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    int rc;
    if (e->inflight.on && (rc = enqueue_batch_end(e))) return rc;
    return consume_pend(e, spec);
}

// The fragmentation cache over the batch's nf listed fragments (fragmentationCache.cpp):
// ordered by (bucket, arrival), each bucket's ring replayed; the ports land in frag_ports.
static int frag_replay(ipxg_engine* e, const BatchView& bv, const Params& p, uint32_t nf) {
    int rc;
    if ((rc = ensure(e, e->frag_sorted, (size_t)nf * 8))) return rc;
    size_t tb = 0;
    HIPCHK(e, sort_keys_u64(nullptr, tb, nullptr, nullptr, nf, 64, e->st));
    if ((rc = ensure(e, e->sort_tmp, tb))) return rc;
    FragView fv = frag_view(e);
    tb = e->sort_tmp.bytes;
    HIPCHK(e, sort_keys_u64(e->sort_tmp.p, tb, fv.list, fv.sorted, nf, 64, e->st));
    launch_frag_walk(e->st, bv, p, fv, nf, e->stats_d);
    HIPCHK(e, hipGetLastError());
    return IPXG_OK;
}

// Strict mode: one batch through the reference's line table (ipxg_strict.hip), synchronously.
static int strict_submit(ipxg_engine* e, const BatchView& bv, uint32_t n) {
    int rc;
    const Params p = params(e);
    const uint64_t m = 3ull * n;  // events: forward, inverse and sweep line per packet
    if (e->cfg.frag_enable) {
        if ((rc = ensure(e, e->frag_list, (size_t)n * 8))) return rc;
        if ((rc = ensure(e, e->frag_ports, (size_t)n * 4))) return rc;
    }
    if ((rc = ensure(e, e->st_pkt, (size_t)n * sizeof(StrictPkt)))) return rc;
    if ((rc = ensure(e, e->st_crec, (size_t)n * sizeof(ipxg_flow_record)))) return rc;
    if ((rc = ensure(e, e->st_keyed, (size_t)n * 4))) return rc;
    if ((rc = ensure(e, e->st_qx, (size_t)n * 4))) return rc;
    for (DevBuf* b : {&e->st_keys, &e->st_vals, &e->st_keys2, &e->st_vals2})
        if ((rc = ensure(e, *b, m * 4))) return rc;
    if ((rc = ensure(e, e->st_succ, (size_t)n * 16))) return rc;   // per event slot: the line's next packet
    if ((rc = ensure(e, e->st_pred, (size_t)n * 4))) return rc;    // per event slot: has a predecessor
    if ((rc = ensure(e, e->st_indeg, (size_t)n * 4))) return rc;
    if ((rc = ensure(e, e->st_queue, (size_t)n * 4 + 16))) return rc;  // ready queue + its initial count
    // every record alive now plus every record this batch creates may leave during it
    if ((rc = ensure_export(e, (size_t)e->sv.slot_mask + 1 + n))) return rc;
    HIPCHK(e, hipMemsetAsync(e->ctl_d, 0, sizeof(BatchCtl), e->st));
    prof_begin_batch(e);
    ev_rec(e, 0);
    launch_strict_prep1(e->st, bv, p, frag_view(e), e->ctl_d, e->stats_d);
    HIPCHK(e, hipGetLastError());
    if (e->cfg.frag_enable) {
        if ((rc = sync_ctl(e))) return rc;
        const uint32_t nf = e->ctl_h->frag_count;
        if (nf && (rc = frag_replay(e, bv, p, nf))) return rc;
    }
    StrictPkt* sp = (StrictPkt*)e->st_pkt.p;
    ipxg_flow_record* crec = (ipxg_flow_record*)e->st_crec.p;
    uint32_t* keyed = (uint32_t*)e->st_keyed.p;
    uint32_t* qx = (uint32_t*)e->st_qx.p;
    uint32_t* ts_acc = e->sv.lb + e->sv.lines;
    HIPCHK(e, hipMemsetAsync(ts_acc, 0, 4, e->st));
    launch_strict_prep2(e->st, bv, p, frag_view(e), sp, crec, keyed, ts_acc);
    HIPCHK(e, hipGetLastError());
    launch_strict_lb(e->st, e->sv);
    HIPCHK(e, hipGetLastError());
    size_t tb = 0, tb2 = 0;
    int bits = 1;
    while ((1ull << bits) <= e->sv.lines) bits++;  // line numbers and the no-event key (lines)
    HIPCHK(e, exclusive_scan_u32(nullptr, tb, keyed, qx, n, e->st));
    HIPCHK(e, sort_pairs_u32(nullptr, tb2, nullptr, nullptr, nullptr, nullptr, (uint32_t)m, bits, e->st));
    if ((rc = ensure(e, e->sort_tmp, std::max(tb, tb2)))) return rc;
    tb = e->sort_tmp.bytes;
    HIPCHK(e, exclusive_scan_u32(e->sort_tmp.p, tb, keyed, qx, n, e->st));
    uint32_t *ks = (uint32_t*)e->st_keys.p, *vs = (uint32_t*)e->st_vals.p;
    uint32_t *ks2 = (uint32_t*)e->st_keys2.p, *vs2 = (uint32_t*)e->st_vals2.p;
    // (IPXG_STRICT_PRUNE=0: every sweep step kept as a DAG event -- a bound of 0 keeps them all)
    launch_strict_events(e->st, e->sv, sp, keyed, qx, n, e->strict_q, p.split_biflow, e->strict_prune ? p.inactive_s : 0u,
                         ks, vs);
    HIPCHK(e, hipGetLastError());
    tb = e->sort_tmp.bytes;
    HIPCHK(e, sort_pairs_u32(e->sort_tmp.p, tb, ks, ks2, vs, vs2, (uint32_t)m, bits, e->st));
    uint32_t* queue = (uint32_t*)e->st_queue.p;
    // the ready count: the single workgroup's initial tail, or the scheduler block's tail word
    uint32_t* sched = e->strict_wgs ? e->st_sched : queue + n;
    uint32_t* q_count = e->strict_wgs ? e->st_sched + STRICT_SCHED_TAIL_WORD : queue + n;
    HIPCHK(e, hipMemsetAsync(queue, 0xFF, (size_t)n * 4, e->st));  // STRICT_NONE: not filled yet
    HIPCHK(e, hipMemsetAsync(q_count, 0, 4, e->st));
    if (e->strict_wgs) HIPCHK(e, hipMemsetAsync(e->st_sched, 0, STRICT_SCHED_BYTES, e->st));
    launch_strict_dag(e->st, ks2, vs2, (uint32_t)m, ks, keyed, n, e->sv.lines, (uint32_t*)e->st_succ.p,
                      (uint8_t*)e->st_pred.p, (uint32_t*)e->st_indeg.p, queue, q_count);
    launch_strict_walk(e->st, e->sv, p, sp, crec, keyed, qx, (const uint32_t*)e->st_succ.p, (uint32_t*)e->st_indeg.p,
                       queue, sched, n, e->strict_q, export_view(e), e->ctl_d, e->stats_d, e->strict_wgs);
    HIPCHK(e, hipGetLastError());
    ev_rec(e, 1);
    uint32_t tail[2] = {0, 0};  // the last packet's keyed rank and mark: keyed packets in the batch
    HIPCHK(e, hipMemcpyAsync(&tail[0], qx + n - 1, 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(&tail[1], keyed + n - 1, 4, hipMemcpyDeviceToHost, e->st));
    if ((rc = sync_ctl(e))) return rc;
    if (e->ctl_h->strict_fail) return set_err(e, IPXG_EDEVICE, "strict replay: a lane waited STRICT_SPIN_MAX rounds without any packet of the batch finishing");
    if (prof_on(e)) {
        e->tm.ingest_ms += ev_ms(e, 0);
        e->tm.ingest_launches++;
        e->tm.ingest_packets += n;
    }
    e->strict_q += (uint64_t)tail[0] + tail[1];
    e->live = (uint32_t)((int64_t)e->live + e->ctl_h->strict_live);
    e->keys = e->live;
    e->batches++;
    return IPXG_OK;
}

// The batch's front: per-batch scratch, its control block (the other of the two, cleared),
// partitions sized, then k_bin and k_bin_slow (binned) -- from ipxg_submit, or from the previous
// batch's host walk (early: its spills deferred, Params::defer_spill).  The export counters are
// left alone (a pending clear rides on k_reduce, launch_rest).
// ahead: launched before the host has read the pending batch's control block (ipxg_engine::pend):
// the front's kernels test that block and return at once when the host has work left for it;
// nothing is reallocated (IPXG_EGROW before anything is enqueued).  reuse_blk: the front again,
// on the block of a front launched ahead that returned (consume_pend's spec_closed).
struct Ahead {
    uint32_t mode;         // pend.mode
    const BatchCtl* prev;  // the pending batch's control block
    uint32_t seq;          // k_bin publishes it with this sequence number
};
static int launch_front(ipxg_engine* e, const BatchView& bv, uint32_t n, bool binned, bool async, bool early, Params& p,
                        BinView& bins, const Ahead* ahead = nullptr, bool reuse_blk = false) {
    int rc;
    // every allocation first (a front launched ahead enqueues nothing before it knows they fit)
    // per-batch scratch sized for the worst case (every packet deferred / a fragment)
    if ((rc = ensure(e, e->defer_a, (size_t)n * 4))) return rc;
    if ((rc = ensure(e, e->defer_b, (size_t)n * 4))) return rc;
    // deferred aggregates: each covers >= TAGG_MIN (3) packets, 48 bytes
    if ((rc = ensure(e, e->adefer_a, ((size_t)n / 3 + 1) * 48))) return rc;
    if ((rc = ensure(e, e->adefer_b, ((size_t)n / 3 + 1) * 48))) return rc;
    if (e->cfg.frag_enable) {
        if ((rc = ensure(e, e->frag_list, (size_t)n * 8))) return rc;
        if ((rc = ensure(e, e->frag_ports, (size_t)n * 4))) return rc;
    }
    BinView nb = {};
    // (p.slow_skip below: the streamed reduce needs k_bin's records to be the batch's only ones)
    const bool skip_slow = binned && e->last_slow == 0 && e->plugins.empty() && !e->no_slow_skip;
    if (binned) {
        const uint32_t bits_before = e->part_bits_last;
        if ((rc = setup_bins(e, n, bv.oshift != 0, nb, skip_slow && !early))) return rc;
        if ((rc = ensure(e, e->fin_list, (size_t)n * sizeof(HotSlot)))) {
            e->part_bits_last = bits_before;
            return rc;
        }
    }
    // the batch's control block (and event set): the other one, which k_reduce of the batch on this
    // one zeroed (blk_zero), else a fill; the current block is never marked zero
    if (!reuse_blk) {
        e->cur ^= 1;
        e->ctl_d = e->ctl_blk[e->cur];
        e->ev = e->evs[e->cur];
    }
    if (!e->blk_zero[e->cur]) HIPCHK(e, hipMemsetAsync(e->ctl_d, 0, sizeof(BatchCtl), e->st));
    e->blk_zero[e->cur] = false;

    p = params(e);
    p.defer_spill = early ? 1u : 0u;
    if (ahead) {
        p.gate_mode = ahead->mode;
        p.prev_ctl = ahead->prev;
        // behind a batch, or an expire behind a batch (k_expire leaves the block's last_sec / last_usec
        // alone): the order check continues from its last packet (read on the device), as without a
        // front ahead; behind a finish: none, as after every finish
        p.prev_valid = p.prev_dev = ahead->mode == GATE_BATCH || ahead->mode == GATE_EXPIRE ? 1u : 0u;
        p.pub_dst = e->ctl_hd;
        p.pub_ex = e->ex_count_d;
        p.pub_words = (uint32_t)(CTL_EX_OFF / 4);
        p.pub_seq = ahead->seq;
    }
    // no k_bin_slow behind k_bin when the previous batch listed no slow packet (with process plugins
    // it also lists their checks: always launched); a batch that does list one is run again from
    // k_bin_slow by post_batch (BatchCtl::slow_redo)
    p.slow_skip = skip_slow ? 1u : 0u;
    nb.slow_skip = p.slow_skip;
    FragView fv = frag_view(e);
    bins = nb;
    e->bins_last = bins;
    e->bins_valid = binned;
    // (the point an asynchronous batch's neighbour formatting forks from: only once the engine
    // formats on its own stream -- an event record is a stream packet of its own, ~5 us of GPU time)
    e->ex_ev_valid = false;
    if (async && !early && e->fst) {
        if (!e->ex_ev) HIPCHK(e, hipEventCreateWithFlags(&e->ex_ev, hipEventDisableTiming));
        HIPCHK(e, hipEventRecord(e->ex_ev, e->st));
        e->ex_ev_valid = true;
    }
    prof_begin_batch(e);
    if (e->pstat_d) launch_pstats(e->st, bv, p, e->pstat_d);  // ahead of the timed stages
    // the process plugins' flows: SLOT_PLUGIN in the table before k_reduce folds the batch;
    // k_bin and k_bin_slow write partition records and, on a full segment, atomic slot updates
    // (tile_emit's spill); k_classify's slot updates are atomic too, so it runs beside them
    const bool classify = !e->plugins.empty() && binned;
    p.classify = classify ? 1u : 0u;
    if (classify && !p.plug) {
        if (!e->cls_st) {
            HIPCHK(e, hipStreamCreateWithFlags(&e->cls_st, hipStreamNonBlocking));
            HIPCHK(e, hipEventCreateWithFlags(&e->cls_fork, hipEventDisableTiming));
            HIPCHK(e, hipEventCreateWithFlags(&e->cls_join, hipEventDisableTiming));
        }
        HIPCHK(e, hipEventRecord(e->cls_fork, e->st));
        HIPCHK(e, hipStreamWaitEvent(e->cls_st, e->cls_fork, 0));
        launch_classify(e->cls_st, bv, p, table_view(e), (const DevRule*)e->rules_d.p, (uint32_t)e->plugins.size(),
                        e->ctl_d);
        HIPCHK(e, hipEventRecord(e->cls_join, e->cls_st));
    }
    ev_rec(e, 0);
    if (binned) {
        uint32_t* dl = (uint32_t*)e->defer_a.p;
        uint4* sl = (uint4*)e->slow_list.p;
        uint4* al = (uint4*)e->adefer_a.p;
        if (bins.prog) {  // the streamed reduce, forked beside k_bin (joined in launch_rest)
            if (!e->rst) {
                // (the highest priority: its workgroups are dispatched before k_bin's, one per CU,
                // and k_bin's fill the room they leave -- two per CU)
                int lo_pri = 0, hi_pri = 0;
                HIPCHK(e, hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
                if (std::getenv("IPXG_RS_LOWPRI")) hi_pri = lo_pri;  // (A/B knob)
                HIPCHK(e, hipStreamCreateWithPriority(&e->rst, hipStreamNonBlocking, hi_pri));
                HIPCHK(e, hipEventCreateWithFlags(&e->rs_fork, hipEventDisableTiming));
                HIPCHK(e, hipEventCreateWithFlags(&e->rs_join, hipEventDisableTiming));
            }
            HIPCHK(e, hipEventRecord(e->rs_fork, e->st));
            HIPCHK(e, hipStreamWaitEvent(e->rst, e->rs_fork, 0));
            launch_reduce_stream(e->rst, p, table_view(e), bins, e->ctl_d, (HotSlot*)e->fin_list.p, dl, al);
            HIPCHK(e, hipEventRecord(e->rs_join, e->rst));
        }
        launch_bin(e->st, bv, p, table_view(e), fv, bins, e->ctl_d, sl, dl, al, e->stats_d);
        ev_rec(e, 1);
        if (!p.slow_skip) {
            launch_bin_slow(e->st, bv, p, table_view(e), fv, bins, e->ctl_d, sl, dl, al, e->stats_d);
            ev_rec(e, 2);
        }
    }
    HIPCHK(e, hipGetLastError());
    return IPXG_OK;
}

// The rest of the batch after its front: the plugin marks, k_reduce (and k_fin_list for a
// synchronous batch), or the atomic ingest; an asynchronous batch is left in flight.
static int launch_rest(ipxg_engine* e, const BatchView& bv, Params p, const BinView& bins, uint32_t n, bool binned,
                       bool async) {
    int rc;
    // The front has run: nothing launched from here on tests the pending batch's block, which that
    // batch's completion re-zeroes -- a later k_bin_slow redo (post_batch) with the gate still in p
    // found it "closed" and returned without writing its records
    p.gate_mode = GATE_NONE;
    p.pub_seq = 0;
    FragView fv = frag_view(e);
    const bool classify = p.classify != 0;
    if (binned) {
        uint32_t* dl = (uint32_t*)e->defer_a.p;
        HotSlot* fl = (HotSlot*)e->fin_list.p;
        uint4* al = (uint4*)e->adefer_a.p;
        if (classify && p.plug)  // the flows k_bin / k_bin_slow found: claimed and marked before k_reduce
            launch_plugin_marks(e->st, bv, p, table_view(e), (const DevRule*)e->rules_d.p,
                                (uint32_t)e->plugins.size(), e->ctl_d, bins);
        else if (classify)
            HIPCHK(e, hipStreamWaitEvent(e->st, e->cls_join, 0));
        // the previous exports' IPFIX formatting ran beside k_bin; this batch's export writers
        // (k_fin_list and the host paths after it) follow it
        if ((rc = join_fmt(e))) return rc;
        // k_reduce also zeroes the other control block (its batch is complete: the host read it
        // before this launch) for the next front, and the export counters of a pending clear
        if (bins.prog) {  // the streamed reduce ran beside k_bin (launch_front): joined here
            HIPCHK(e, hipStreamWaitEvent(e->st, e->rs_join, 0));
        } else {
            uint32_t* zx = nullptr;
            if (e->ex_zero_pending) {
                zx = e->ex_count_d;
                e->ex_zero_pending = false;
            }
            launch_reduce(e->st, table_view(e), bins, e->ctl_d, fl, dl, al, e->ctl_blk[e->cur ^ 1], zx);
            e->blk_zero[e->cur ^ 1] = true;
        }
        if (!async) {
            ev_rec(e, 3);
            launch_fin_list(e->st, bv, p, table_view(e), fv, export_view(e), e->ctl_d, fl, e->stats_d, n, false);
            ev_rec(e, 4);
        }
    } else {
        if ((rc = join_fmt(e))) return rc;
        launch_ingest(e->st, bv, p, table_view(e), fv, e->ctl_d, (uint32_t*)e->defer_a.p, e->stats_d);
        ev_rec(e, 1);
    }
    HIPCHK(e, hipGetLastError());
    if (async) {
        e->inflight.on = true;  // the next call launches k_fin_list, publishes and reads the control block
        e->inflight.tail = true;
        e->inflight.bv = bv;
        e->inflight.p = p;
        e->inflight.n = n;
        return IPXG_OK;
    }
    if ((rc = sync_ctl(e))) return rc;
    return post_batch(e, bv, p, n, binned, false);
}

// The arena's size limit: 4 GiB with byte offsets, 2^32 16-byte units less a page with
// IPXG_BATCH_OFFSET16 (descriptor offsets are 32-bit either way)
static constexpr uint64_t ARENA16_MAX = (1ull << 36) - 4096;
static int check_arena(ipxg_engine* e, const ipxg_batch* batch) {
    if (batch->flags & IPXG_BATCH_OFFSET16) {
        if (batch->arena_len > ARENA16_MAX) return set_err(e, IPXG_ETOOBIG, "arena larger than 64 GiB - 4 KiB");
    } else if (batch->arena_len > (1ull << 32)) {
        return set_err(e, IPXG_ETOOBIG, "arena larger than 4 GiB (IPXG_BATCH_OFFSET16 takes up to 64 GiB)");
    }
    return IPXG_OK;
}
static void set_arena_view(BatchView& bv, const ipxg_batch* batch) {
    bv.arena_lim = (uint32_t)std::min<uint64_t>(batch->arena_len, 0xFFFFFF00ull);
    bv.arena_len = batch->arena_len;
    bv.oshift = (batch->flags & IPXG_BATCH_OFFSET16) ? 4u : 0u;
}

static int submit_impl(ipxg_engine* e, const ipxg_batch* batch) {
    if (!e || !batch) return IPXG_EINVAL;
    const uint32_t n = batch->n;
    if (n == 0) return IPXG_OK;
    if (n > IPXG_MAX_BATCH) return set_err(e, IPXG_ETOOBIG, "batch larger than IPXG_MAX_BATCH");
    int rc;
    if ((rc = check_arena(e, batch))) return rc;
    if (!batch->arena || !batch->desc) return set_err(e, IPXG_EINVAL, "null arena/desc");
    const bool binned = !(e->cfg.flags & IPXG_CFG_ATOMIC_INGEST);
    const bool dev_batch = (batch->flags & IPXG_BATCH_DEVICE) != 0;
    const bool async = (batch->flags & IPXG_BATCH_ASYNC) && binned && !e->strict;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    BatchView bv;
    bv.n = n;
    set_arena_view(bv, batch);
    int slot = -1;
    if (!dev_batch && async) {
        // Host batch, asynchronous: its H2D copy goes into the staging slot the batch in
        // flight does not use, on the copy stream, before that batch is completed -- the copy
        // overlaps the kernels of the previous batch (slot reuse is safe: the batch that used
        // this slot was completed by the previous call).
        slot = e->stage_next;
        e->stage_next ^= 1;
        if (!e->cst) {
            HIPCHK(e, hipStreamCreateWithFlags(&e->cst, hipStreamNonBlocking));
            HIPCHK(e, hipEventCreateWithFlags(&e->copied[0], hipEventDisableTiming));
            HIPCHK(e, hipEventCreateWithFlags(&e->copied[1], hipEventDisableTiming));
        }
        if ((rc = ensure(e, e->stage_arena[slot], batch->arena_len + 64))) return rc;
        if ((rc = ensure(e, e->stage_desc[slot], (size_t)n * sizeof(ipxg_pkt_desc)))) return rc;
        HIPCHK(e, hipMemcpyAsync(e->stage_arena[slot].p, batch->arena, batch->arena_len, hipMemcpyHostToDevice,
                                 e->cst));
        HIPCHK(e, hipMemcpyAsync(e->stage_desc[slot].p, batch->desc, (size_t)n * sizeof(ipxg_pkt_desc),
                                 hipMemcpyHostToDevice, e->cst));
        HIPCHK(e, hipEventRecord(e->copied[slot], e->cst));
    }
    // a device batch behind an asynchronous batch with plugins in flight: its front may run during
    // that batch's host walk (early_front)
    e->early.launched = false;
    e->early.want = dev_batch && async && e->inflight.on && !e->plugins.empty() && !e->ex_zero_pending;
    if (e->early.want) {
        e->early.bv = bv;
        e->early.bv.arena = batch->arena;
        e->early.bv.desc = batch->desc;
        e->early.bv.base_sec = BASE_FROM_DESC0;
        e->early.n = n;
    }
    // A device batch behind a batch or finish whose control block the host has not read: its front
    // (k_bin, k_bin_slow) is launched first, gated on that block, and the host completes the pending
    // batch while the front runs -- unless a buffer would have to grow (the pending batch may still
    // read it) or process plugins are registered (their walk has the early front instead).
    bool ahead = false;
    Params p;
    BinView bins = {};
    if (dev_batch && async && binned && !e->strict && e->plugins.empty() && !e->failed && !e->no_ahead &&
        (e->inflight.on || e->pend.on)) {
        if (e->inflight.on && (rc = enqueue_batch_end(e))) return rc;
        BatchView abv = bv;
        abv.arena = batch->arena;
        abv.desc = batch->desc;
        abv.base_sec = BASE_FROM_DESC0;
        uint32_t seq = e->pub_seq + 1;
        if (seq == 0) seq = 1;
        const Ahead ah{e->pend.mode, e->ctl_blk[e->pend.blk], seq};
        e->no_grow = true;
        rc = launch_front(e, abv, n, true, true, false, p, bins, &ah);
        e->no_grow = false;
        if (rc == IPXG_EGROW) {
            rc = IPXG_OK;  // (nothing enqueued: the front follows the completion)
        } else if (rc) {
            return rc;
        } else {
            ahead = true;
            e->pub_seq = seq;  // k_bin publishes the pending batch's block
            e->pend.seq = seq;
            e->pend.published = true;
        }
    }
    rc = complete_batch(e, ahead);
    e->early.want = false;
    if (rc) {
        // this batch's front already ran (launched ahead, or from the failed batch's host walk): its
        // packets are counted in the statistics and its block holds them, so a retry of this submit
        // would count them twice -- the engine stops until ipxg_reset
        if ((e->early.launched || ahead) && !e->failed) {
            e->failed = true;
            e->fail_msg = std::string("the batch before this one failed after this batch's front ran: ") + e->err;
        }
        e->early.launched = false;
        return rc;
    }
    if (dev_batch) {
        bv.arena = batch->arena;
        bv.desc = batch->desc;
    } else if (slot >= 0) {
        HIPCHK(e, hipStreamWaitEvent(e->st, e->copied[slot], 0));
        bv.arena = (const uint8_t*)e->stage_arena[slot].p;
        bv.desc = (const ipxg_pkt_desc*)e->stage_desc[slot].p;
    } else {
        if ((rc = ensure(e, e->arena, batch->arena_len + 64))) return rc;
        if ((rc = ensure(e, e->desc, (size_t)n * sizeof(ipxg_pkt_desc)))) return rc;
        HIPCHK(e, hipMemcpyAsync(e->arena.p, batch->arena, batch->arena_len, hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipMemcpyAsync(e->desc.p, batch->desc, (size_t)n * sizeof(ipxg_pkt_desc),
                                 hipMemcpyHostToDevice, e->st));
        bv.arena = (const uint8_t*)e->arena.p;
        bv.desc = (const ipxg_pkt_desc*)e->desc.p;
    }
    bv.base_sec = BASE_FROM_DESC0;  // kernels read desc[0] themselves (no host round trip)
    if (ahead) {
        e->early_timed = false;
        // the gate was closed (the pending batch needed the host): its kernels returned at once
        if (e->pend.spec_closed && (rc = launch_front(e, bv, n, true, true, false, p, bins, nullptr, true))) return rc;
        if ((rc = ensure_export(e, n))) return rc;
        return launch_rest(e, bv, p, bins, n, true, true);
    }
    if (e->strict) {
        if (e->ex_zero_pending) {
            e->ex_zero_pending = false;
            HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
        }
        if ((rc = join_fmt(e))) return rc;
        return strict_submit(e, bv, n);
    }
    if (e->early.launched) {
        // the front of this batch ran during the previous batch's host walk (early_front): the rest
        e->early.launched = false;
        e->early_timed = true;
        ev_rec(e, 11);
        p = e->early.p;
        bins = e->early.bins;
        if ((rc = ensure_export(e, n))) return rc;
        e->ex_ev_valid = false;
        if (e->fst) {
            if (!e->ex_ev) HIPCHK(e, hipEventCreateWithFlags(&e->ex_ev, hipEventDisableTiming));
            HIPCHK(e, hipEventRecord(e->ex_ev, e->st));  // (after the previous batch's walk exports)
            e->ex_ev_valid = true;
        }
        return launch_rest(e, bv, p, bins, n, true, true);
    }
    if ((rc = ensure_export(e, n))) return rc;
    e->early_timed = false;
    if ((rc = launch_front(e, bv, n, binned, async, false, p, bins))) return rc;
    return launch_rest(e, bv, p, bins, n, binned, async);
}

// Everything after the batch's main kernels, from the control block in e->ctl_h: timing,
// the fragment, deferral, table-scan and complex paths when the batch needs them, then the
// host's accounting.  `finishing`: a finish follows at once (no table growth needed).
// ---- process-plugin bridge: the host walk ----------------------------------------------------
// put_pkt_recursive (cache.cpp:330-491) for the plugin flows of a batch, one flow at a time,
// with every registered plugin's hooks at their call sites and flush() (cache.cpp:290-320);
// the same per-packet rules as the device's sequential walk (k_complex_walk) and the oracle.
// Not emulated here, as nowhere in the engine: the per-packet expiry sweep (only end reasons
// differ) and the 16-way line (no NO_RES evictions).
namespace {

struct alignas(128) WalkOut {  // one per walk thread, on cache lines of its own
    HostVec<ipxg_flow_record>& ex;  // exported records, in order (then spill)
    std::vector<ipxg_flow_record>& spill;
    uint64_t end[5] = {0, 0, 0, 0, 0};   // by end reason (export statistics)
    uint64_t pkts[6] = {0, 0, 0, 0, 0, 0};  // FlowRecordStats buckets
    uint64_t unreasoned = 0;  // export_flow with end_reason 0 (post_create FLUSH of a new record)
    uint64_t v6 = 0;          // IPv6 records among ex
};

// A hook returned IPXG_PLUGIN_ERROR (the reference plugin threw PluginError): raised inside the
// walk's own code and caught by the walk thread (walk_range), which stops its range -- as the
// reference's input worker leaves its loop at the first PluginError (workers.cpp:107-112).
struct HookFail {
    size_t plugin;
    const char* hook;
};

// canon_dir (ipxg_table.hpp) on the host walk's parsed packet: its address words are the
// device's little-endian words of the address bytes
static uint32_t host_canon_dir(const ipxg_parsed_pkt& k) {
    const int nw = k.ip_version == 6 ? 4 : 1;
    for (int w = 0; w < nw; ++w) {
        uint32_t a, b;
        std::memcpy(&a, k.src_ip + 4 * w, 4);
        std::memcpy(&b, k.dst_ip + 4 * w, 4);
        if (a != b) return a > b ? 1u : 0u;
    }
    return k.src_port > k.dst_port ? 1u : 0u;
}

struct FlowWalk {
    const std::vector<ipxg_plugin>& pl;
    const Params& p;
    WalkOut& out;
    ipxg_flow_record rec;
    bool live;

    static int ret(int r, size_t k, const char* hook) {
        if (r < 0) throw HookFail{k, hook};
        return r;
    }
    int pre_create(ipxg_packet_view* v) {
        int r = 0;
        for (size_t k = 0; k < pl.size(); ++k)
            if (pl[k].pre_create) r |= ret(pl[k].pre_create(pl[k].ctx, v), k, "pre_create");
        return r;
    }
    int post_create(const ipxg_packet_view* v) {
        int r = 0;
        for (size_t k = 0; k < pl.size(); ++k)
            if (pl[k].post_create) r |= ret(pl[k].post_create(pl[k].ctx, &rec, v), k, "post_create");
        return r;
    }
    int pre_update(ipxg_packet_view* v) {
        int r = 0;
        for (size_t k = 0; k < pl.size(); ++k)
            if (pl[k].pre_update) r |= ret(pl[k].pre_update(pl[k].ctx, &rec, v), k, "pre_update");
        return r;
    }
    int post_update(const ipxg_packet_view* v) {
        int r = 0;
        for (size_t k = 0; k < pl.size(); ++k)
            if (pl[k].post_update) r |= ret(pl[k].post_update(pl[k].ctx, &rec, v), k, "post_update");
        return r;
    }
    void pre_export() {
        for (const ipxg_plugin& q : pl)
            if (q.pre_export) q.pre_export(q.ctx, &rec);
    }
    // export_flow (cache.cpp:262-274): the record with its end reason, counted; slot erased
    void export_flow(uint8_t reason, bool counted = true) {
        ipxg_flow_record o = rec;
        o.end_reason = reason;
        o.reserved0 = IPXG_REC_PRE_EXPORTED;  // (a flush's too: the reference has no pre_export there)
        std::memset(o.reserved, 0, sizeof(o.reserved));
        if (out.ex.size() < out.ex.cap) out.ex.push_back(o);
        else out.spill.push_back(o);
        out.v6 += o.ip_version == 6 ? 1 : 0;
        // m_total_exported and update_flow_record_stats count every export_flow;
        // update_flow_end_reason_stats ignores a reason outside 1..5 (cache.cpp:264-267,618-638)
        if (!counted) return;
        if (reason >= 1 && reason <= 5) out.end[reason - 1]++;
        else out.unreasoned++;
        out.pkts[pkts_bucket((uint64_t)o.src_packets + o.dst_packets)]++;
    }
    // FlowRecord::create (cache.cpp:94-132), the engine's record layout (rec_create)
    void create(const ipxg_parsed_pkt& k, const ipxg_packet_view& v) {
        std::memset(&rec, 0, sizeof(rec));
        rec.flow_hash = k.hash_fwd;
        rec.time_first_sec = rec.time_last_sec = v.ts_sec;
        rec.time_first_usec = rec.time_last_usec = v.ts_usec;
        rec.ip_version = k.ip_version;
        rec.ip_proto = k.ip_proto;
        std::memcpy(rec.src_ip, k.src_ip, 16);
        std::memcpy(rec.dst_ip, k.dst_ip, 16);
        std::memcpy(rec.src_mac, k.src_mac, 6);
        std::memcpy(rec.dst_mac, k.dst_mac, 6);
        if (k.ip_proto == 6 || k.ip_proto == 17 || k.ip_proto == 1 || k.ip_proto == 58) {
            rec.src_port = k.src_port;
            rec.dst_port = k.dst_port;
        }
        rec.vlan_id = (uint16_t)k.vlan_id;
        rec.reserved[0] = p.split_biflow ? 0 : (uint8_t)host_canon_dir(k);  // creator's canonical dir
        rec.src_packets = 1;
        rec.src_bytes = k.ip_len;
        if (k.ip_proto == 6) rec.src_tcp_flags = k.tcp_flags;
        live = true;
    }
    // FlowRecord::update (cache.cpp:134-152)
    void update(const ipxg_parsed_pkt& k, const ipxg_packet_view& v, bool src) {
        rec.time_last_sec = v.ts_sec;
        rec.time_last_usec = v.ts_usec;
        if (src) {
            rec.src_packets++;
            rec.src_bytes += k.ip_len;
            if (k.ip_proto == 6) rec.src_tcp_flags |= k.tcp_flags;
        } else {
            rec.dst_packets++;
            rec.dst_bytes += k.ip_len;
            if (k.ip_proto == 6) rec.dst_tcp_flags |= k.tcp_flags;
        }
    }
    // flush (cache.cpp:290-320)
    void flush(int ret, const ipxg_parsed_pkt& k, ipxg_packet_view* v, bool src) {
        if (ret == IPXG_FLOW_FLUSH_WITH_REINSERT) {
            export_flow(IPXG_FLOW_END_FORCED, false);  // ipx_ring_push only: not counted
            rec.ext = 0;                                // remove_extensions
            rec.time_first_sec = rec.time_last_sec;     // reuse (cache.cpp:73-83)
            rec.time_first_usec = rec.time_last_usec;
            rec.src_packets = rec.dst_packets = 0;
            rec.src_bytes = rec.dst_bytes = 0;
            rec.src_tcp_flags = rec.dst_tcp_flags = 0;
            update(k, *v, src);
            const int r2 = post_create(v);
            if (r2 & IPXG_FLOW_FLUSH) flush(r2, k, v, src);
        } else {
            export_flow(IPXG_FLOW_END_FORCED);
            live = false;
        }
    }
    void put(const ipxg_parsed_pkt& k, ipxg_packet_view* v) {
        for (;;) {  // the recursion of put_pkt_recursive after an export
            pre_create(v);  // its return is not used (cache.cpp:332)
            const bool src = !live || p.split_biflow || k.hash_fwd == rec.flow_hash;
            v->source_pkt = src ? 1 : 0;  // cache.cpp:428
            if (live) {
                const uint8_t flw = src ? rec.src_tcp_flags : rec.dst_tcp_flags;
                if ((k.tcp_flags & 0x02) && (flw & 0x05)) {  // :431-438
                    export_flow(IPXG_FLOW_END_EOF);
                    live = false;
                    continue;
                }
                if ((int64_t)v->ts_sec - (int64_t)rec.time_last_sec >= (int64_t)p.inactive_s) {  // :453
                    const uint8_t reason = ((rec.src_tcp_flags | rec.dst_tcp_flags) & 0x05) ? IPXG_FLOW_END_EOF
                                                                                            : IPXG_FLOW_END_INACTIVE;
                    rec.end_reason = reason;
                    pre_export();
                    export_flow(reason);
                    live = false;
                    continue;
                }
                if ((int64_t)v->ts_sec - (int64_t)rec.time_first_sec >= (int64_t)p.active_s) {  // :464
                    rec.end_reason = IPXG_FLOW_END_ACTIVE;
                    pre_export();
                    export_flow(IPXG_FLOW_END_ACTIVE);
                    live = false;
                    continue;
                }
                int ret = pre_update(v);  // :474-486
                if (ret & IPXG_FLOW_FLUSH) {
                    flush(ret, k, v, src);
                    return;
                }
                update(k, *v, src);
                ret = post_update(v);
                if (ret & IPXG_FLOW_FLUSH) flush(ret, k, v, src);
                return;
            }
            create(k, *v);  // :441-449
            if (post_create(v) & IPXG_FLOW_FLUSH) {
                export_flow(rec.end_reason);  // end reason as the record holds it
                live = false;
            }
            return;
        }
    }
};

}  // namespace

// The walk threads' plugin copies (ipxg_plugin.copy_ctx), released.
static void free_walk_copies(ipxg_engine* e) {
    for (std::vector<ipxg_plugin>& v : e->walk_pl)
        for (ipxg_plugin& q : v)
            if (q.free_ctx && q.ctx) q.free_ctx(q.ctx);
    e->walk_pl.clear();
}

// Walk threads wanted: the configured count (default: the host's hardware threads, at most 16);
// one when a registered plugin cannot be copied.
static unsigned walk_want(const ipxg_engine* e) {
    for (const ipxg_plugin& q : e->plugins)
        if (!q.copy_ctx || !q.free_ctx) return 1;
    return std::min<unsigned>(HOST_CHUNKS, e->walk_threads ? e->walk_threads
                                                           : std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
}

// Every registered plugin copied for walk threads 1 .. want-1 (walk_pl[t-1][k]: thread t's copy
// of plugin k).  Copies are made from instances no walk has used yet, at registration: a
// ProcessPlugin's copy() copies its state, and the reference copies its prototypes before the
// pipelines start (ipfixprobe.cpp:430-436) -- TLSPlugin / HTTPPlugin keep a preallocated
// extension pointer (tls.cpp:412-425, http.cpp:592-598) that a copy of a used instance would
// share with it.
static int make_walk_copies(ipxg_engine* e) {
    const unsigned want = walk_want(e);
    if (want <= 1) return IPXG_OK;
    if (e->walk_pl.size() + 1 < want) e->walk_pl.resize(want - 1);
    for (unsigned t = 0; t + 1 < want; ++t) {
        std::vector<ipxg_plugin>& v = e->walk_pl[t];
        while (v.size() < e->plugins.size()) {
            ipxg_plugin q = e->plugins[v.size()];
            q.ctx = q.copy_ctx(q.ctx);
            if (!q.ctx) return set_err(e, IPXG_ENOMEM, "a process plugin's copy_ctx failed");
            v.push_back(q);
        }
    }
    return IPXG_OK;
}

// Threads for a walk of nf flows / m packets: the wanted count, fewer for a small walk (~2k
// packets per thread at least).  Starts the pool on first use.
static unsigned walk_pool(ipxg_engine* e, uint32_t nf, uint32_t m) {
    const unsigned want = walk_want(e);
    const unsigned by_size = std::max<uint32_t>(1, m / 2048);
    unsigned T = std::min<unsigned>({want, by_size, std::max<uint32_t>(nf, 1)});
    for (unsigned t = 1; t < T; ++t)
        if (t > e->walk_pl.size() || e->walk_pl[t - 1].size() != e->plugins.size()) T = t;
    if (T <= 1) return 1;
    if (!e->pool || e->pool->size() < T) {
        delete e->pool;
        e->pool = new WalkPool(want);
    }
    return T;
}

static int set_walk_threads_impl(ipxg_engine* e, uint32_t threads) {
    if (!e || threads > 256) return IPXG_EINVAL;
    const uint32_t old = e->walk_threads;
    e->walk_threads = threads;
    const unsigned want = walk_want(e);
    if (want > e->walk_pl.size() + 1 && e->walked) {  // the new copies would copy used instances
        e->walk_threads = old;
        return set_err(e, IPXG_ESTATE, "walk threads raised after the first plugin walk");
    }
    return make_walk_copies(e);
}

// After the batch's complex path (its packets gathered and sorted, the device walk done): walk
// the plugin flows on the host and write them back.  *live_delta: records created - closed.
static int early_front(ipxg_engine* e, const Params& p_walked, uint32_t n_walked);

static int plugin_walk(ipxg_engine* e, const BatchView& bv, const Params& p, const ComplexView& cx, uint32_t ncx,
                       uint32_t npk, int64_t* live_delta) {
    const auto t0 = std::chrono::steady_clock::now();
    auto tm = t0;
    // IPXG_WALK_TRACE: the walk's phases (0: the device ordering + the sizes' round trip, 1: the
    // copies to the host, 5: the host loop, 6: the write-back) summed, with their minor page
    // faults, printed when the engine closes
    const bool trace = e->walk_trace;
    long flt = 0;
    auto faults = []() {
        struct rusage u;
        getrusage(RUSAGE_THREAD, &u);
        return (long)u.ru_minflt;
    };
    if (trace) flt = faults();
#define WALK_MARK(k)                                                                                         \
    do {                                                                                                   \
        const auto t_ = std::chrono::steady_clock::now();                                                  \
        e->walk_phase_ms[k] += std::chrono::duration<double, std::milli>(t_ - tm).count();                 \
        tm = t_;                                                                                           \
        if (trace) {                                                                                       \
            const long f_ = faults();                                                                      \
            e->walk_faults[k] += f_ - flt;                                                                 \
            flt = f_;                                                                                      \
        }                                                                                                  \
    } while (0)
    struct Clock {  // the walk's wall time, however it returns
        ipxg_engine* e;
        std::chrono::steady_clock::time_point t0;
        ~Clock() { e->tm.plugin_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } clock{e, t0};
    int rc;
    *live_delta = 0;
    // on the device: the plugin flows in order of their first packet, their packets' list and
    // byte offsets (launch_plugin_order), then the parsed packets and the frame bytes in that
    // order; one round trip for the sizes
    const size_t tmp_b = plugin_order_temp(ncx, npk);
    if ((rc = ensure(e, e->pf_keys, (size_t)ncx * 16 + 16))) return rc;
    if ((rc = ensure(e, e->pf_d, (size_t)ncx * sizeof(PluginFlow) + 16))) return rc;
    if ((rc = ensure(e, e->pf_flen, ((size_t)ncx + 1) * 8 + 16))) return rc;
    if ((rc = ensure(e, e->pf_idx, (size_t)npk * 4 + 16))) return rc;
    if ((rc = ensure(e, e->pf_off, ((size_t)npk + 1) * 16 + 16))) return rc;
    if ((rc = ensure(e, e->pf_tmp, tmp_b + 64))) return rc;
    if ((rc = ensure(e, e->pf_live, (3 * (size_t)ncx + 2) * 4 + 16))) return rc;
    if ((rc = ensure(e, e->pf_recs, (size_t)ncx * sizeof(ipxg_flow_record) + 16))) return rc;
    PluginOrder o;
    o.keys = (uint64_t*)e->pf_keys.p;
    o.skeys = o.keys + ncx;
    o.flows = (PluginFlow*)e->pf_d.p;
    o.flen = (uint32_t*)e->pf_flen.p;
    o.first = o.flen + ncx + 1;
    o.idx = (uint32_t*)e->pf_idx.p;
    o.off = (uint64_t*)e->pf_off.p;
    o.clen = o.off + npk + 1;
    o.tot = (uint64_t*)e->pf_tmp.p;
    o.count = (uint32_t*)(o.tot + 4);
    o.hstate = (uint32_t*)e->pf_live.p;
    o.lflag = o.hstate + ncx;
    o.lpos = o.lflag + ncx + 1;
    o.recs = (ipxg_flow_record*)e->pf_recs.p;
    o.temp = (char*)e->pf_tmp.p + 64;
    o.temp_bytes = tmp_b;
    if ((rc = ensure(e, e->pf_wpk, (size_t)npk * sizeof(WalkPkt) + 16))) return rc;
    o.wpk = (WalkPkt*)e->pf_wpk.p;
    o.rules = (const DevRule*)e->rules_d.p;
    o.nrules = (uint32_t)e->plugins.size();
    o.budget = e->walk_budget;
    HIPCHK(e, hipMemsetAsync(o.count, 0, sizeof(uint32_t), e->st));
    HIPCHK(e, hipMemsetAsync(o.clen, 0, ((size_t)npk + 1) * 8, e->st));
    launch_plugin_order(e->st, bv, p, frag_view(e), table_view(e), cx, ncx, npk, o);
    HIPCHK(e, hipGetLastError());
    uint64_t tot[4] = {0, 0, 0, 0};
    HIPCHK(e, hipMemcpyAsync(tot, o.tot, sizeof(tot), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));  WALK_MARK(0);
    const uint32_t nf = (uint32_t)tot[0], m = (uint32_t)tot[1];
    const uint64_t nbytes = tot[2];
    const uint32_t nlive = (uint32_t)tot[3];
    if (!nf) return IPXG_OK;
    if ((rc = ensure(e, e->pf_bytes, nbytes + 16))) return rc;
    launch_plugin_bytes(e->st, bv, o.idx, o.off, m, (uint8_t*)e->pf_bytes.p);
    HIPCHK(e, hipGetLastError());
    const bool pin = e->walk_pin;
    if (!e->hw_state.resize(nf, pin) || !e->hw_recs.resize(nlive, pin) || !e->hw_first.resize(nf + 1, pin) ||
        !e->hw_wpk.resize(m, pin) ||
        !e->hw_off.resize((size_t)m + 1, pin) || !e->hw_bytes.resize(nbytes + 2048, pin) || !e->hw_lpos.resize(nf + 1, pin))
        return set_err(e, IPXG_ENOMEM, "host walk buffers");
    uint32_t* fstate = e->hw_state.data();
    const ipxg_flow_record* recs_in = e->hw_recs.data();
    uint32_t* lpos = e->hw_lpos.data();
    const uint32_t* first = e->hw_first.data();
    WalkPkt* wp = e->hw_wpk.data();
    const uint64_t* off = e->hw_off.data();
    const uint8_t* bytes = e->hw_bytes.data();
    // The walk's input in two steps (page-locked host buffers; the walk threads make no HIP call):
    // first the per-flow arrays and the live records, which the split into work units needs;
    // then the packets -- their WalkPkt records (parsed fields, descriptor, index), frame bytes -- in WALK_CHUNKS chunks
    // of whole work units, each chunk's copies behind an event.  The threads take units in walk
    // order and start a unit once its chunk has landed, so the hooks run while the later chunks
    // are still crossing PCIe (one round of copies took 18.5 of the configs[2] step's 37 ms host
    // walk, the hooks 15: VERDICT r3 item 8).  The calling thread waits for the chunk events.
    HIPCHK(e, hipMemcpyAsync(e->hw_first.data(), o.first, ((size_t)nf + 1) * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(e->hw_off.data(), o.off, ((size_t)m + 1) * 8, hipMemcpyDeviceToHost, e->st));
    // (the flows' slot states; the records of the live ones go with their chunk below -- the
    // 160-byte flow images stay on the device for the write-back)
    HIPCHK(e, hipMemcpyAsync(fstate, o.hstate, (size_t)nf * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->tm.plugin_flows += nf;
    e->tm.plugin_packets += m;
    // what crosses PCIe to the host for the walk: the frames (or their budgets), the packet and
    // flow records, the per-flow arrays
    e->tm.plugin_d2h_bytes += nbytes + (uint64_t)m * (sizeof(WalkPkt) + 8) + (uint64_t)nlive * sizeof(ipxg_flow_record) +
                              (uint64_t)nf * 8 + 8;

    lpos[0] = 0;  // flow f's record in recs_in, when it is live
    for (uint32_t f = 0; f < nf; ++f) lpos[f + 1] = lpos[f] + ((fstate[f] & SLOT_LIVE) ? 1u : 0u);
    if (lpos[nf] != nlive)  // (the chunks' record copies below are sized by these positions)
        return set_err(e, IPXG_EDEVICE, "plugin walk: the walked flows marked live differ in number from the records k_plugin_pack packed");
    // work units: contiguous flow ranges of about equal packet counts (flows in order of their
    // first packet), four per thread (at most HOST_CHUNKS), grouped into the copy chunks; each
    // unit's export buffer sized here for two exports per packet (more -- REINSERT chains -- go to
    // its overflow vector)
    const unsigned T = walk_pool(e, nf, m);
    e->walked = true;
    const unsigned U = std::min<unsigned>(HOST_CHUNKS, std::max<unsigned>(1, std::min<uint32_t>(4 * T, nf)));
    const unsigned C = std::min<unsigned>(WALK_CHUNKS, U);
    std::vector<uint32_t> fr(U + 1);
    for (unsigned u = 0; u <= U; ++u)
        fr[u] = u == 0 ? 0 : u == U ? nf
                       : (uint32_t)(std::lower_bound(first, first + nf, (uint32_t)((uint64_t)m * u / U)) - first);
    auto chunk_of = [&](unsigned u) { return (unsigned)((uint64_t)u * C / U); };
    // the chunks cross on a stream of their own; the engine's stream is idle here (synchronised
    // above) and runs the next batch's front beside them (early_front).  (Two copy streams
    // alternating by chunk: no faster, quic 409 -> 404 Mpkt/s.)
    if (!e->wst) HIPCHK(e, hipStreamCreateWithFlags(&e->wst, hipStreamNonBlocking));
    const hipStream_t cs = e->wst;
    auto sync_copies = [&]() { (void)hipStreamSynchronize(cs); };
    for (unsigned c = 0; c < C; ++c) {
        unsigned u0 = 0;
        while (chunk_of(u0) < c) u0++;
        unsigned u1 = u0;
        while (u1 < U && chunk_of(u1) == c) u1++;
        const uint32_t k0 = first[fr[u0]], k1 = first[fr[u1]];
        const uint32_t l0 = lpos[fr[u0]], l1 = lpos[fr[u1]];  // the chunk's live records
        if (l1 > l0)
            HIPCHK(e, hipMemcpyAsync(e->hw_recs.data() + l0, o.recs + l0, (size_t)(l1 - l0) * sizeof(ipxg_flow_record),
                                     hipMemcpyDeviceToHost, cs));
        if (k1 > k0) {
            HIPCHK(e, hipMemcpyAsync(wp + k0, (WalkPkt*)e->pf_wpk.p + k0, (size_t)(k1 - k0) * sizeof(WalkPkt),
                                     hipMemcpyDeviceToHost, cs));
            if (off[k1] > off[k0])
                HIPCHK(e, hipMemcpyAsync(e->hw_bytes.data() + off[k0], (uint8_t*)e->pf_bytes.p + off[k0], off[k1] - off[k0],
                                         hipMemcpyDeviceToHost, cs));
        }
        if (!e->walk_ev[c]) HIPCHK(e, hipEventCreateWithFlags(&e->walk_ev[c], hipEventDisableTiming));
        HIPCHK(e, hipEventRecord(e->walk_ev[c], cs));
    }
    // the next batch's front beside the copies and the hooks (its kernels on the engine's stream;
    // the write-back below follows them there)
    if ((rc = early_front(e, p, bv.n))) {
        sync_copies();
        return rc;
    }
    BatchCtl* const apply_ctl = e->early.launched ? e->aux_ctl_d : e->ctl_d;
    WALK_MARK(1);
    while (e->hw_ex.size() < U) e->hw_ex.emplace_back(new ExportVec);
    const bool ports = e->pstat_d != nullptr;
    if (ports && e->host_ports.size() < T) e->host_ports.resize(T);
    std::vector<WalkOut> wos;
    wos.reserve(U);
    for (unsigned u = 0; u < U; ++u) {
        ExportVec& xv = *e->hw_ex[u];
        xv.v.clear();
        xv.spill.clear();
        xv.orec.clear();
        const size_t nfu = fr[u + 1] - fr[u];
        if (!xv.v.reserve(2 * (size_t)(first[fr[u + 1]] - first[fr[u]]) + 16, e->walk_pin) ||
            !xv.orec.reserve(nfu + 1, e->walk_pin))
            return set_err(e, IPXG_ENOMEM, "host walk export buffers");
        wos.push_back(WalkOut{xv.v, xv.spill});
    }
    std::vector<int64_t> dlive(U, 0);
    std::vector<int> wfail(T, 0);  // a walk thread: 2 out of host memory, 3 a plugin failed
    std::vector<std::string> wmsg(T);
    std::unique_ptr<std::atomic<uint32_t>[]> ready(new std::atomic<uint32_t>[C]);
    for (unsigned c = 0; c < C; ++c) ready[c].store(0);
    std::atomic<uint32_t> next_unit{0};
    std::atomic<uint32_t> copy_fail{0};
    // the first failure stops every thread from taking more units: the reference stops at the first
    // PluginError, so no plugin instance advances past it
    std::atomic<bool> stop{false};
    auto walk_unit = [&](unsigned t, unsigned u) {
        const uint32_t f0 = fr[u], f1 = fr[u + 1];
        WalkOut& wo = wos[u];
        const std::vector<ipxg_plugin>& pl = t ? e->walk_pl[t - 1] : e->plugins;
        uint64_t* pa = nullptr;
        if (ports) {
            if (e->host_ports[t].empty()) e->host_ports[t].assign(2 * 65536, 0);
            pa = e->host_ports[t].data();
        }
        int64_t dl = 0;
        ExportVec& xv = *e->hw_ex[u];
        for (uint32_t f = f0; f < f1; ++f) {
            const bool live0 = (fstate[f] & SLOT_LIVE) != 0;
            ipxg_flow_record r0;
            if (live0) r0 = recs_in[lpos[f]];
            else std::memset(&r0, 0, sizeof(r0));
            FlowWalk w{pl, p, wo, r0, live0};
            const bool was_live = w.live;
            for (uint32_t k = first[f]; k < first[f + 1]; ++k) {
                ipxg_packet_view v;
                std::memset(&v, 0, sizeof(v));
                v.pkt = &wp[k].pk;
                v.data = bytes + off[k];
                v.caplen = wp[k].d.caplen;
                v.wirelen = wp[k].d.wirelen;
                v.ts_sec = wp[k].d.ts_sec;
                v.ts_usec = wp[k].d.ts_usec;
                v.index = wp[k].idx;
                w.put(wp[k].pk, &v);
            }
            // a plugin that follows every packet of a flow it claimed (ext set) keeps it on the
            // host walk until the flow holds follow_packets packets (ipxg_plugin.follow_packets)
            const bool follow =
                w.live && w.rec.ext && (uint64_t)w.rec.src_packets + w.rec.dst_packets < e->follow_max;
            fstate[f] = w.live ? (SLOT_LIVE | (follow ? SLOT_FOLLOW : 0u)) : 0u;
            if (w.live) {  // (capacity: one record per flow of the unit)
                ipxg_flow_record o2 = w.rec;
                std::memcpy(o2.reserved2, &f, 4);
                xv.orec.push_back(o2);
            }
            dl += (w.live ? 1 : 0) - (was_live ? 1 : 0);
            const uint32_t flen = first[f + 1] - first[f];
            // TopPorts from the flow's packets (count_flow_ports: every packet counts both ports)
            const ipxg_flow_record& r = w.rec;
            if (pa && (r.ip_proto == 6 || r.ip_proto == 17) && (r.src_port || r.dst_port)) {
                uint64_t* a = pa + (r.ip_proto == 17 ? 65536 : 0);
                a[r.src_port] += flen;
                a[r.dst_port] += flen;
            }
        }
        dlive[u] = dl;
    };
    auto walk_range = [&](unsigned t) {
        if (t == 0) {  // the chunks' arrival, in order (the caller's HIP calls; then it walks too)
            for (unsigned c = 0; c < C; ++c) {
                if (hipEventSynchronize(e->walk_ev[c]) != hipSuccess) copy_fail.store(1);
                ready[c].store(1, std::memory_order_release);
            }
        }
        try {
            for (;;) {
                if (stop.load(std::memory_order_acquire)) break;
                const unsigned u = next_unit.fetch_add(1);
                if (u >= U) break;
                const unsigned c = chunk_of(u);
                while (!ready[c].load(std::memory_order_acquire)) std::this_thread::yield();
                if (copy_fail.load()) break;
                walk_unit(t, u);
            }
        } catch (const HookFail& h) {
            stop.store(true, std::memory_order_release);
            wfail[t] = 3;
            const ipxg_plugin& q = (t ? e->walk_pl[t - 1] : e->plugins)[h.plugin];
            const char* m = q.error ? q.error(q.ctx) : nullptr;
            wmsg[t] = "process plugin " + std::to_string(h.plugin) + " " + h.hook + ": " +
                      (m ? m : "returned IPXG_PLUGIN_ERROR");
        } catch (const std::bad_alloc&) {
            stop.store(true, std::memory_order_release);
            wfail[t] = 2;
        } catch (const std::exception& x) {  // (a hook that threw past the C ABI)
            stop.store(true, std::memory_order_release);
            wfail[t] = 3;
            wmsg[t] = std::string("process plugin walk: ") + x.what();
        } catch (...) {
            stop.store(true, std::memory_order_release);
            wfail[t] = 3;
            wmsg[t] = "process plugin walk: a hook raised a non-standard exception";
        }
    };
    if (T > 1) e->pool->run(walk_range, T);  // (threads T.. of a larger pool sit this walk out)
    else walk_range(0);
    if (copy_fail.load()) {
        (void)hipStreamSynchronize(e->st);
        sync_copies();
        return set_err(e, IPXG_EDEVICE, "plugin walk: a copy of the walk's input failed");
    }
    if (T > 1 && e->pool->take_escaped()) {  // (walk_range catches everything: not expected)
        wfail[0] = 3;
        wmsg[0] = "process plugin walk: an exception left a walk thread";
    }
    // failures a hook could not return (pre_export returns nothing): each instance's error()
    for (unsigned t = 0; t < T; ++t) {
        if (wfail[t]) continue;
        const std::vector<ipxg_plugin>& pl = t ? e->walk_pl[t - 1] : e->plugins;
        for (size_t k = 0; k < pl.size() && !wfail[t]; ++k)
            if (const char* m = pl[k].error ? pl[k].error(pl[k].ctx) : nullptr) {
                wfail[t] = 3;
                wmsg[t] = "process plugin " + std::to_string(k) + ": " + m;
            }
    }
    for (unsigned t = 0; t < T; ++t)
        if (wfail[t] == 2) {
            (void)hipStreamSynchronize(e->st);
            return set_err(e, IPXG_ENOMEM, "plugin walk: host memory for the exports");
        }
    for (unsigned t = 0; t < T; ++t)
        if (wfail[t] == 3) {  // the batch is lost; the engine stops until ipxg_reset
            (void)hipStreamSynchronize(e->st);
            e->failed = true;
            e->fail_msg = wmsg[t];
            return set_err(e, IPXG_EPLUGIN, wmsg[t]);
        }
    // the units' exports follow each other in unit order (copied to the device below)
    size_t nx = 0;
    WalkOut& wo = wos[0];
    for (unsigned u = 0; u < U; ++u) nx += wos[u].ex.size() + wos[u].spill.size();
    for (unsigned u = 1; u < U; ++u) {
        for (int k = 0; k < 5; ++k) wo.end[k] += wos[u].end[k];
        for (int k = 0; k < 6; ++k) wo.pkts[k] += wos[u].pkts[k];
        wo.unreasoned += wos[u].unreasoned;
        wo.v6 += wos[u].v6;
    }
    for (unsigned u = 0; u < U; ++u) *live_delta += dlive[u];
    for (uint32_t k = 0; k < m; ++k) {  // (the frames' own lengths: off[] steps are rounded to 16 bytes)
        const uint64_t cl = wp[k].d.caplen;
        e->tm.plugin_bytes += cl;
        e->tm.plugin_extra_bytes += cl > 128 ? cl - 128 : 0;
    }
    WALK_MARK(5);
    // back to the device: the slot states, the live flows' records, then the exports after the
    // batch's own
    // (the threads' records and exports are read by one kernel straight from their page-locked
    // buffers -- one launch instead of a copy command per thread and array, ~10 us each)
    HIPCHK(e, hipMemcpyAsync(o.hstate, fstate, (size_t)nf * 4, hipMemcpyHostToDevice, e->st));
    auto gather = [&](auto pick, ipxg_flow_record* dst, uint32_t at0, uint32_t& moved) -> int {
        HostChunks c;
        c.count = c.max_n = 0;
        uint32_t at = at0;
        for (unsigned u = 0; u < U; ++u) {
            const HostVec<ipxg_flow_record>& x = pick(u);
            const uint32_t k = (uint32_t)x.size();
            if (!k) continue;
            if (x.dev) {
                c.src[c.count] = reinterpret_cast<const uint4*>(x.dev);
                c.n[c.count] = k;
                c.at[c.count] = at;
                c.max_n = std::max(c.max_n, k);
                c.count++;
            } else {  // (not page-locked: a copy command)
                HIPCHK(e, hipMemcpyAsync(dst + at, x.data(), (size_t)k * sizeof(ipxg_flow_record),
                                         hipMemcpyHostToDevice, e->st));
            }
            at += k;
        }
        launch_host_gather(e->st, c, dst);
        HIPCHK(e, hipGetLastError());
        moved = at - at0;
        return IPXG_OK;
    };
    uint32_t nout = 0;
    if ((rc = gather([&](unsigned u) -> const HostVec<ipxg_flow_record>& { return e->hw_ex[u]->orec; }, o.recs, 0,
                     nout)))
        return rc;
    launch_plugin_apply(e->st, table_view(e), o.flows, o.hstate, nf, o.recs, nout, apply_ctl);
    HIPCHK(e, hipGetLastError());
    if (nx) {
        if ((rc = ensure_export(e, nx))) return rc;
        uint32_t moved = 0;
        if ((rc = gather([&](unsigned u) -> const HostVec<ipxg_flow_record>& { return wos[u].ex; }, e->ex, e->ex_count,
                         moved)))
            return rc;
        size_t at = e->ex_count + moved;
        for (unsigned u = 0; u < U; ++u) {  // what overflowed the units' buffers (REINSERT chains)
            const std::vector<ipxg_flow_record>& y = wos[u].spill;
            if (!y.empty())
                HIPCHK(e, hipMemcpyAsync(e->ex + at, y.data(), y.size() * sizeof(ipxg_flow_record),
                                         hipMemcpyHostToDevice, e->st));
            at += y.size();
        }
        uint32_t c3[3] = {e->ex_count + (uint32_t)nx, 0, e->ex_count6 + (uint32_t)wo.v6};
        HIPCHK(e, hipMemcpyAsync(e->ex_count_d, c3, sizeof(c3), hipMemcpyHostToDevice, e->st));
        e->ex_zero_pending = false;  // all three counters written
        e->ex_count = c3[0];
        e->ex_count6 = c3[2];
    }
    HIPCHK(e, hipStreamSynchronize(e->st));
    if (e->early.launched) {  // k_plugin_apply's guard word (post_batch's check on ctl_d otherwise)
        uint32_t g = 0;
        HIPCHK(e, hipMemcpy(&g, &e->aux_ctl_d->guard, sizeof(g), hipMemcpyDeviceToHost));
        if (g) {
            HIPCHK(e, hipMemset(&e->aux_ctl_d->guard, 0, sizeof(g)));
            return set_err(e, IPXG_EDEVICE, "k_plugin_apply: a walked flow's index or table slot was out of range");
        }
    }
    for (int k = 0; k < 5; ++k) e->host_end[k] += wo.end[k];
    for (int k = 0; k < 6; ++k) e->host_pkts[k] += wo.pkts[k];
    e->host_unreasoned += wo.unreasoned;
    WALK_MARK(6);
#undef WALK_MARK
    return IPXG_OK;
}

static int add_plugin_impl(ipxg_engine* e, const ipxg_plugin* pl) {
    if (!e || !pl) return IPXG_EINVAL;
    if (pl->n_ports > IPXG_PLUGIN_MAX_PORTS || pl->n_prefixes > IPXG_PLUGIN_MAX_PREFIXES)
        return set_err(e, IPXG_EINVAL, "plugin rule: too many ports or prefixes");
    for (uint32_t q = 0; q < pl->n_prefixes; ++q)
        if (pl->prefix_len[q] > IPXG_PLUGIN_PREFIX_LEN) return set_err(e, IPXG_EINVAL, "plugin rule: prefix too long");
    if (e->cfg.flags & (IPXG_CFG_ATOMIC_INGEST | IPXG_CFG_STRICT))
        return set_err(e, IPXG_EINVAL, "process plugins need the binned ingest");
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    e->plugins.push_back(*pl);
    if (const int rc1 = make_walk_copies(e)) {  // the walk threads' copies of the new plugin
        e->plugins.pop_back();
        // a copy failed on some thread: the threads before it already hold a copy of the new
        // plugin -- free those, so every thread's instances line up with e->plugins again
        // (else a later registration would skip them and those threads would call the failed
        // plugin's copy in the next one's place)
        for (std::vector<ipxg_plugin>& v : e->walk_pl)
            while (v.size() > e->plugins.size()) {
                if (v.back().free_ctx && v.back().ctx) v.back().free_ctx(v.back().ctx);
                v.pop_back();
            }
        return rc1;
    }
    e->follow_max = std::max<uint64_t>(e->follow_max, pl->follow_packets);
    if (pl->all_packets) e->plug_all = true;  // (every touched flow walked: the rules do not matter)
    // the walk's byte budget: with every registered plugin declaring one (follow_bytes), a walked
    // packet no rule matches crosses to the host with its headers and the largest budget's payload
    // bytes; any plugin without one (or acting on every packet) keeps whole frames
    {
        uint32_t b = 0;
        bool all = !e->plug_all && !e->walk_full;
        for (const ipxg_plugin& q : e->plugins) {
            if (q.follow_bytes == 0) all = false;
            b = std::max(b, q.follow_bytes);
        }
        e->walk_budget = all ? b : 0u;
    }
    std::vector<DevRule> rules(e->plugins.size());
    for (size_t k = 0; k < rules.size(); ++k) {
        const ipxg_plugin& q = e->plugins[k];
        DevRule& r = rules[k];
        std::memset(&r, 0, sizeof(r));
        r.proto_mask = q.proto_mask;
        r.n_ports = q.n_ports;
        std::memcpy(r.ports, q.ports, sizeof(r.ports));
        r.n_prefixes = q.n_prefixes;
        std::memcpy(r.prefix_len, q.prefix_len, sizeof(r.prefix_len));
        std::memcpy(r.prefix, q.prefix, sizeof(r.prefix));
        r.masked = q.masked;
        std::memcpy(r.prefix_mask, q.prefix_mask, sizeof(r.prefix_mask));
    }
    // flattened for k_bin (Params::plug): every port and every prefix of at most PLUG_PREFIX bytes
    // with its protocols; a rule set that does not fit keeps the k_classify pass
    e->plug_ok = true;
    e->plug_nport = e->plug_npref = 0;
    for (const ipxg_plugin& q : e->plugins) {
        for (uint32_t k = 0; k < q.n_ports; ++k) {
            if (e->plug_nport == 16) {
                e->plug_ok = false;
                break;
            }
            e->plug_port[e->plug_nport++] = q.ports[k] | ((q.proto_mask & 3u) << 16);
        }
        for (uint32_t k = 0; k < q.n_prefixes; ++k) {
            const uint32_t n = q.prefix_len[k];
            if (n > PLUG_PREFIX || e->plug_npref == 16) {
                e->plug_ok = false;
                break;
            }
            uint32_t v = 0, m = 0;
            for (uint32_t j = 0; j < n; ++j) {
                v |= (uint32_t)q.prefix[k][j] << (8 * j);
                m |= (uint32_t)(((q.masked >> k) & 1u) ? q.prefix_mask[k][j] : 0xFFu) << (8 * j);
            }
            e->plug_pref[e->plug_npref] = v & m;
            e->plug_pmask[e->plug_npref] = m;
            e->plug_pinfo[e->plug_npref] = n | ((q.proto_mask & 3u) << 8);
            e->plug_npref++;
        }
    }
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if ((rc = ensure(e, e->rules_d, rules.size() * sizeof(DevRule)))) return rc;
    HIPCHK(e, hipMemcpyAsync(e->rules_d.p, rules.data(), rules.size() * sizeof(DevRule), hipMemcpyHostToDevice, e->st));
    uint32_t tab[PLUG_TAB_WORDS];
    std::memcpy(tab + PLUG_PORT, e->plug_port, sizeof(e->plug_port));
    std::memcpy(tab + PLUG_PREF, e->plug_pref, sizeof(e->plug_pref));
    std::memcpy(tab + PLUG_PMASK, e->plug_pmask, sizeof(e->plug_pmask));
    std::memcpy(tab + PLUG_PINFO, e->plug_pinfo, sizeof(e->plug_pinfo));
    if ((rc = ensure(e, e->plug_d, sizeof(tab)))) return rc;
    HIPCHK(e, hipMemcpyAsync(e->plug_d.p, tab, sizeof(tab), hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return IPXG_OK;
}

// What the next batch's launch takes from this batch's control block: the order check's
// timestamp, the partition sizing, the tile aggregation and header walk choices (post_batch; the
// early front, from the walked batch's block before its host walk ends).
static void take_batch_knobs(ipxg_engine* e, const BatchCtl& c2, const Params& p, uint32_t n, bool binned) {
    e->last_touched = c2.touched;
    e->last_slow = c2.slow_count;
    e->last_n = n;
    if (binned && c2.total_slots) {  // the next batch's segment sizing
        const uint32_t P = 1u << e->part_bits_last;
        e->skew = (double)c2.max_part * P / c2.total_slots;
    }
    // Tile aggregation for the next batch: kept while it folds >= 2 % of the packets, switched
    // on when the partitions' loads show skew (the most loaded > 2x the mean); the first batch
    // aggregates.  Uniform traffic folds nothing and skips the aggregation's LDS passes.
    if (binned) {
        if (p.tile_agg) e->tile_agg = (uint64_t)c2.agg_packets * 50 >= n;
        else e->tile_agg = e->skew > 2.0;
        if (const char* a = std::getenv("IPXG_TILE_AGG")) e->tile_agg = std::atoi(a) != 0;  // experiments
        // The wide walk for the next batch: switched on when >= 1/32 of the packets went to the
        // slow list (a mix of variable-length header chains: VLAN, IPv6, TCP options, tunnels),
        // kept while >= 1/32 are not the plain shape; plain traffic keeps the narrow 48-byte
        // loads.  walk=wide|narrow pins it.
        e->wide = (uint64_t)(c2.slow_count + (p.wide ? c2.walked : 0)) * 32 >= n;
    }
    // a batch not checked against the one before (the first after a finish or reset), or one whose
    // timestamps went backwards, may have left records older than the idle floor
    if (c2.nonmono || !(p.prev_valid || p.prev_dev)) e->idle_floor = IDLE_FLOOR_NONE;
    e->prev_valid = true;
    e->prev_sec = c2.last_sec;
    e->prev_usec = c2.last_usec;
}

// k_expire's scan result (BatchCtl::tls_inv) as the idle floor; 0: it did not scan (the floor stands).
// With no record left live the floor is the last packet's second: every later record is at least
// that recent (the order held), not "never idle" -- a floor above it skipped the expiry of flows
// created after the scan (tests/test_stdplugins.py test_expired_followed_flow_leaves_the_host_walk).
static void take_idle_floor(ipxg_engine* e, uint32_t tls_inv) {
    if (tls_inv == 1) e->idle_floor = e->prev_valid ? (int64_t)e->prev_sec : IDLE_FLOOR_NONE;
    else if (tls_inv) e->idle_floor = (int64_t)(uint32_t)~tls_inv;
}


// The next batch's front from inside this batch's host walk (ipxg_engine::early), once the walk's
// input has been copied out: the device state the walk still changes is the walked flows' slots
// and the exports, which k_bin / k_bin_slow do not touch with their spills deferred.  The walked
// batch's control block is kept in early.snap (ctl_d is the next batch's from here on).
static int early_front(ipxg_engine* e, const Params& p_walked, uint32_t n_walked) {
    if (!e->early.want || e->early.launched) return IPXG_OK;
    std::memcpy(&e->early.snap, e->ctl_h, sizeof(BatchCtl));
    take_batch_knobs(e, e->early.snap, p_walked, n_walked, true);
    if (!plug_fold(e)) return IPXG_OK;  // (a k_classify pass would claim slots the walk still owns)
    if (!e->aux_ctl_d) {
        if (hipMalloc((void**)&e->aux_ctl_d, sizeof(BatchCtl)) != hipSuccess)
            return set_err(e, IPXG_ENOMEM, "hipMalloc failed");
        HIPCHK(e, hipMemsetAsync(e->aux_ctl_d, 0, sizeof(BatchCtl), e->st));
    }
    int rc;
    if ((rc = launch_front(e, e->early.bv, e->early.n, true, true, true, e->early.p, e->early.bins))) return rc;
    e->early.launched = true;
    e->tm.plugin_overlapped++;
    return IPXG_OK;
}

static int post_batch(ipxg_engine* e, BatchView bv, Params p, uint32_t n, bool binned, bool finishing) {
    int rc;
    FragView fv = frag_view(e);
    BatchCtl c1 = *e->ctl_h;
    if (prof_on(e)) {
        e->tm.ingest_ms += ev_ms(e, 0);
        e->tm.ingest_launches++;
        e->tm.ingest_packets += n;
        if (binned && e->prof_level == 3 && !p.slow_skip) e->tm.ingest_slow_ms += ev_ms(e, 1);
        if (binned && e->prof_level == 1) {
            if (!p.slow_skip) e->tm.ingest_slow_ms += ev_ms(e, 1);
            e->tm.reduce_ms += e->early_timed ? ev_ms(e, 11, 3) : ev_ms(e, p.slow_skip ? 1 : 2, 3);
            e->tm.fin_ms += ev_ms(e, 3);
            e->tm.reduce_launches++;
        }
    }
    if (c1.guard & GUARD_STREAM_STALL)
        return set_err(e, IPXG_EDEVICE, "k_reduce_stream: no k_bin progress word changed for seconds");
    bool slow = false;
    if (c1.slow_redo) {
        // k_bin listed slow packets although the batch was launched without k_bin_slow (the previous
        // batch had none): k_reduce and k_fin_list returned at once -- the slow pass, k_reduce and
        // k_fin_list now, in order (not finishing: a finish's flows are then exported by k_finish)
        ev_rec(e, 5);
        slow = true;
        p.slow_skip = 0;
        p.gate_mode = GATE_NONE;  // (a front launched ahead: its gate was that of the batch before)
        p.pub_seq = 0;
        BinView bins = e->bins_last;
        bins.slow_skip = 0;
        HIPCHK(e, hipMemsetAsync(&e->ctl_d->slow_redo, 0, sizeof(uint32_t), e->st));
        launch_bin_slow(e->st, bv, p, table_view(e), fv, bins, e->ctl_d, (uint4*)e->slow_list.p, (uint32_t*)e->defer_a.p,
                        (uint4*)e->adefer_a.p, e->stats_d);
        launch_reduce(e->st, table_view(e), bins, e->ctl_d, (HotSlot*)e->fin_list.p, (uint32_t*)e->defer_a.p,
                      (uint4*)e->adefer_a.p);
        {
            const int rc0 = join_fmt(e);  // (k_fin_list appends exports)
            if (rc0) return rc0;
        }
        launch_fin_list(e->st, bv, p, table_view(e), fv, export_view(e), e->ctl_d, (HotSlot*)e->fin_list.p, e->stats_d,
                        n, false);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        c1 = *e->ctl_h;
        e->tm.slow_redos++;
    }

    // fragmentation cache: order fragments by (bucket, arrival) and replay the rings
    uint32_t ndef = c1.deferred, nadef = c1.agg_deferred;
    if (c1.frag_count) {
        if (!slow) ev_rec(e, 5);
        slow = true;
        const uint32_t nf = c1.frag_count;
        if ((rc = frag_replay(e, bv, p, nf))) return rc;
        fv = frag_view(e);
        launch_frag_accumulate(e->st, bv, p, table_view(e), fv, nf, e->ctl_d, (uint32_t*)e->defer_a.p);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        ndef = e->ctl_h->deferred;
        nadef = e->ctl_h->agg_deferred;
    }
    // table overflow: grow and re-apply the deferred packets and tile aggregates -- first without
    // growing when k_bin deferred its spills (Params::defer_spill: the table was not full)
    bool grow = c1.spill_deferred == 0;
    while (ndef || nadef) {
        if (!slow) ev_rec(e, 5);
        slow = true;
        if (grow && (rc = rehash(e, e->cap * 2))) return rc;
        grow = true;
        HIPCHK(e, hipMemsetAsync(&e->ctl_d->deferred, 0, sizeof(uint32_t), e->st));
        HIPCHK(e, hipMemsetAsync(&e->ctl_d->agg_deferred, 0, sizeof(uint32_t), e->st));
        if (ndef)
            launch_deferred(e->st, bv, p, table_view(e), frag_view(e), (const uint32_t*)e->defer_a.p, ndef,
                            e->ctl_d, (uint32_t*)e->defer_b.p);
        if (nadef)
            launch_deferred_agg(e->st, table_view(e), (const uint4*)e->adefer_a.p, nadef, e->ctl_d,
                                (uint4*)e->adefer_b.p);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        ndef = e->ctl_h->deferred;
        nadef = e->ctl_h->agg_deferred;
        std::swap(e->defer_a, e->defer_b);
        std::swap(e->adefer_a, e->adefer_b);
    }
    // finalise-list flows whose table probe failed in k_fin_list (a batch of many new flows into
    // a small table): grow the table and finalise just those, until none is left
    uint32_t nfd = c1.fin_deferred;
    while (nfd) {
        if (!slow) ev_rec(e, 5);
        slow = true;
        if ((rc = rehash(e, e->cap * 2))) return rc;
        HIPCHK(e, hipMemsetAsync(&e->ctl_d->fin_deferred, 0, sizeof(uint32_t), e->st));
        launch_fin_list(e->st, bv, p, table_view(e), frag_view(e), export_view(e), e->ctl_d, (HotSlot*)e->fin_list.p,
                        e->stats_d, c1.fin_count, false, true);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        nfd = e->ctl_h->fin_deferred;
    }
    if (slow) {
        ev_rec(e, 6);
        HIPCHK(e, hipStreamSynchronize(e->st));
        if (prof_on(e) && e->prof_level == 1) {
            e->tm.slow_ms += ev_ms(e, 5);
            e->tm.slow_launches++;
        }
    }
    // slots k_reduce could not finalise (fragments, deferrals, spills, multi-workgroup
    // partitions; every slot in the atomic ingest mode): the full-table scan
    const bool scan = !binned || c1.pending || c1.frag_count || c1.deferred || c1.agg_deferred;
    if (scan) {
        p.force_complex = p.force_complex || c1.nonmono;
        ev_rec(e, 7);
        launch_finalize(e->st, bv, p, table_view(e), frag_view(e), export_view(e), e->ctl_d, e->stats_d);
        ev_rec(e, 8);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        if (prof_on(e) && e->prof_level == 1) {
            e->tm.finalize_ms += ev_ms(e, 7);
            e->tm.finalize_launches++;
        }
    }
    if (c1.plugin_fail) return set_err(e, IPXG_EDEVICE, "flow table too full to mark a process plugin's flow");
    int64_t plugin_live = 0;
    const uint32_t ncx = e->ctl_h->complex_count;
    if (ncx) {
        ev_rec(e, 5);
        e->complex_total += ncx;
        const uint32_t kcap = pow2_at_least((uint64_t)ncx * 2 + 1);  // the complex flows' key set
        // its bitmap: >= 16 bits per complex flow (<= 1/16 false hits), 8 KB .. 2 MB
        const uint32_t bwords = std::min<uint32_t>(1u << 19, std::max<uint32_t>(2048, pow2_at_least((uint64_t)ncx) / 2));
        if ((rc = ensure(e, e->cx_rank, (size_t)ncx * 4 * 4 + (size_t)kcap * 12 + (size_t)bwords * 4))) return rc;
        uint32_t* cr = (uint32_t*)e->cx_rank.p;
        unsigned long long* ck = reinterpret_cast<unsigned long long*>(cr + 4 * (size_t)ncx);
        uint32_t* bloom = reinterpret_cast<uint32_t*>(ck + kcap) + kcap;
        HIPCHK(e, hipMemsetAsync(ck, 0, (size_t)kcap * 8, e->st));
        HIPCHK(e, hipMemsetAsync(bloom, 0, (size_t)bwords * 4, e->st));
        ComplexView cx = {nullptr, nullptr, cr, cr + ncx, cr + 2 * (size_t)ncx, cr + 3 * (size_t)ncx,
                          ck, reinterpret_cast<uint32_t*>(ck + kcap), kcap - 1, bloom, bwords - 1};
        launch_complex_rank(e->st, table_view(e), cx, e->ctl_d, e->cap, ncx);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        if ((uint32_t)(e->ctl_h->cx_alloc >> 32) != ncx || e->ctl_h->guard)
            return set_err(e, IPXG_EDEVICE, "k_complex_rank found a different number of complex slots than the finalisers counted");
        const uint32_t npk = (uint32_t)(e->ctl_h->cx_alloc & 0xFFFFFFFFu);
        if ((rc = ensure(e, e->cx_list, (size_t)npk * 8 + 8))) return rc;
        if ((rc = ensure(e, e->cx_sorted, (size_t)npk * 8 + 8))) return rc;
        cx.list = (uint64_t*)e->cx_list.p;
        cx.sorted = (uint64_t*)e->cx_sorted.p;
        // the complex flows' packets: from the batch's partition records when no packet was
        // spilled, deferred or fragmented -- the packets k_bin folded into tile aggregates of
        // complex flows by parsing again only those aggregates' index ranges (one tile each) --
        // else by re-parsing every frame.  (Round 3 took the records only with no tile aggregate at
        // all: the Zipf mix of configs[2] re-parsed the whole batch in 50 of 50 batches.)
        bool by_rec = binned && e->bins_valid && !c1.spilled && !c1.deferred && !c1.a_deferred &&
                      !c1.agg_deferred && !c1.frag_count && !std::getenv("IPXG_GATHER_PARSE");
        if (by_rec) {
            uint4* ranges = (uint4*)e->adefer_b.p;  // (free: no aggregate was deferred)
            const uint32_t range_cap = (uint32_t)(e->adefer_b.bytes / sizeof(uint4));
            HIPCHK(e, hipMemsetAsync(&e->ctl_d->cx_agg, 0, 2 * sizeof(uint32_t), e->st));  // cx_agg, cx_ranges
            launch_complex_gather_rec(e->st, e->bins_last, cx, e->ctl_d, ranges, range_cap);
            HIPCHK(e, hipGetLastError());
            if ((rc = sync_ctl(e))) return rc;
            if (e->ctl_h->cx_agg) {  // start over: cursors back to 0
                by_rec = false;
                e->gather_fallbacks++;
                HIPCHK(e, hipMemsetAsync(cx.cursor, 0, (size_t)ncx * sizeof(uint32_t), e->st));
            } else if (const uint32_t nr = e->ctl_h->cx_ranges) {
                launch_complex_gather_ranges(e->st, bv, p, frag_view(e), cx, e->ctl_d, ranges, nr);
                e->gather_ranges += nr;
            }
        }
        if (!by_rec) launch_complex_gather(e->st, bv, p, table_view(e), frag_view(e), cx, e->ctl_d);
        HIPCHK(e, hipGetLastError());
        int bits = 24;
        while ((1ull << (bits - 24)) < ncx) bits++;
        size_t tb = 0;
        HIPCHK(e, sort_keys_u64(nullptr, tb, nullptr, nullptr, npk, bits, e->st));
        if ((rc = ensure(e, e->sort_tmp, tb))) return rc;
        tb = e->sort_tmp.bytes;
        HIPCHK(e, sort_keys_u64(e->sort_tmp.p, tb, cx.list, cx.sorted, npk, bits, e->st));
        launch_complex_walk(e->st, bv, p, table_view(e), frag_view(e), cx, ncx, export_view(e), e->ctl_d,
                            e->stats_d);
        ev_rec(e, 6);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        if (e->ctl_h->guard) return set_err(e, IPXG_EDEVICE, "k_complex_gather: a complex flow had more packets in the batch than its slot counted (its segment's size)");
        if (!e->plugins.empty()) {  // the process plugins' flows: walked on the host
            int64_t dl = 0;
            if ((rc = plugin_walk(e, bv, p, cx, ncx, npk, &dl))) return rc;
            plugin_live += dl;
            if (e->early.launched) {  // (ctl_d is the next batch's now: this batch's block from the walk's start)
                std::memcpy(e->ctl_h, &e->early.snap, sizeof(BatchCtl));
            } else {
                if ((rc = sync_ctl(e))) return rc;
                if (e->ctl_h->guard) return set_err(e, IPXG_EDEVICE, "k_plugin_apply: a walked flow's index or table slot was out of range");
            }
        }
        if (prof_on(e) && e->prof_level == 1) {
            e->tm.slow_ms += ev_ms(e, 5);
            e->tm.slow_launches++;
        }
    }
    const BatchCtl& c2 = *e->ctl_h;
    if (scan) {  // the scan counted every slot
        e->keys = c2.keys;
        e->live = c2.live;
    } else {
        e->keys += c2.new_keys;
        e->live += c2.new_live;
    }
    e->live += c2.cx_new_live;
    e->live = (uint32_t)((int64_t)e->live + plugin_live);
    // (an early front took the knobs already, before the next batch's partitions replaced
    // part_bits_last)
    if (!e->early.launched) take_batch_knobs(e, c2, p, n, binned);
    e->agg_pkts += c2.agg_packets;
    e->spilled += c2.spilled;
    e->slow_pkts += c2.slow_count;
    e->walked_pkts += c2.walked;
    e->batches++;
    // keep the load factor <= 1/2 for the next batch (dead slots are dropped by the rebuild)
    if (!finishing && (uint64_t)e->keys * 2 > e->cap) {
        uint32_t ncap = pow2_at_least((uint64_t)e->live * 4 + 1);
        if (ncap < e->cap) ncap = e->cap;
        if ((rc = rehash(e, ncap))) return rc;
        e->keys = e->live;
    }
    return IPXG_OK;
}

// export_expired(now) (cache.cpp:508-523) over the whole table: k_expire exports every live record
// idle for inactive_s and counts them into the control block (BatchCtl::expired), which the host's
// live count follows -- no recount of the table (round 4 scanned it a second time with k_count and
// waited for the stream twice per call: the stream step's 0.155 ms).  With an
// asynchronous batch in flight the expire is enqueued right behind the batch's tail, guarded like
// the finish (k_expire returns when the batch needs the host), and the call returns at once: the
// next call completes both (consume_pend, GATE_EXPIRE) -- ipxg_submit after launching its front
// ahead, so the streaming step does not wait for the host either (workers.cpp:83-94: the
// reference's storage worker calls export_expired on the input's timeout, between blocks).
static int expire_impl(ipxg_engine* e, int64_t now_sec) {
    if (e) {
        const int rc0 = join_fmt(e);  // (k_expire appends exports)
        if (rc0) return rc0;
    }
    if (!e) return IPXG_EINVAL;
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if (e->inflight.on && !e->strict && !e->failed && e->inflight.tail) {
        if (e->pend.on && (rc = consume_pend(e, false))) return rc;  // (not expected: a batch is in flight)
        // room for the batch's exports and for every record it may leave live (the guard holds otherwise)
        if ((rc = ensure_export(e, (size_t)e->live + 2ull * e->inflight.n))) return rc;
        if ((rc = launch_tail(e, false))) return rc;
        e->inflight.on = false;
        const Params& ip = e->inflight.p;  // (the floor holds behind the batch if its order was checked)
        launch_expire(e->st, params(e), table_view(e), e->cap, now_sec, export_view(e), e->stats_d, e->ctl_d,
                      &e->ctl_d->expired, e->ex_count, e->live,
                      (ip.prev_valid || ip.prev_dev) && !e->no_idle_floor ? e->idle_floor : IDLE_FLOOR_NONE,
                      &e->ctl_d->tls_inv);
        HIPCHK(e, hipGetLastError());
        set_pend(e, GATE_EXPIRE, e->inflight.bv, e->inflight.p, e->inflight.n);
        e->pend.now = now_sec;
        if (e->sync_finish) return consume_pend(e, false);
        return IPXG_OK;
    }
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    if (e->strict) {  // the reference's export_expired(now): one sweep step (cache.cpp:508-523)
        if ((rc = ensure_export(e, 16))) return rc;
        HIPCHK(e, hipMemsetAsync(e->ctl_d, 0, sizeof(BatchCtl), e->st));
        if (e->sv.line_bits) launch_strict_expire(e->st, e->sv, params(e), e->strict_q, now_sec, export_view(e), e->ctl_d,
                                                  e->stats_d);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        e->strict_q++;
        e->live = (uint32_t)((int64_t)e->live + e->ctl_h->strict_live);
        e->keys = e->live;
        return IPXG_OK;
    }
    return expire_table(e, now_sec);
}

// One export_expired(now) over the table, unguarded, waited for: the live count follows the records
// k_expire exported (BatchCtl::expired of the current block).
static int expire_table(ipxg_engine* e, int64_t now_sec) {
    int rc;
    if (e->idle_floor != IDLE_FLOOR_NONE && now_sec - (int64_t)e->cfg.inactive_s < e->idle_floor && !e->no_idle_floor)
        return IPXG_OK;  // no live record can be idle yet: nothing to scan
    if ((rc = ensure_export(e, std::max(e->live, e->keys)))) return rc;
    HIPCHK(e, hipMemsetAsync(&e->ctl_d->expired, 0, sizeof(uint32_t), e->st));
    HIPCHK(e, hipMemsetAsync(&e->ctl_d->tls_inv, 0, sizeof(uint32_t), e->st));
    launch_expire(e->st, params(e), table_view(e), e->cap, now_sec, export_view(e), e->stats_d, nullptr,
                  &e->ctl_d->expired, 0, 0, IDLE_FLOOR_NONE, &e->ctl_d->tls_inv);
    HIPCHK(e, hipGetLastError());
    if ((rc = sync_ctl(e))) return rc;
    const uint32_t x = e->ctl_h->expired;
    e->live = x > e->live ? 0u : e->live - x;
    take_idle_floor(e, e->ctl_h->tls_inv);
    return IPXG_OK;
}

// The finish proper: every live record exported FORCED by a table scan (k_finish), which also
// empties the table (cache.cpp:276-288).
static int finish_table(ipxg_engine* e) {
    int rc;
    if ((rc = ensure_export(e, std::max(e->live, e->keys)))) return rc;
    ev_rec(e, 9);
    launch_finish(e->st, table_view(e), e->cap, export_view(e), e->stats_d);  // also empties the table
    HIPCHK(e, hipGetLastError());
    ev_rec(e, 10);
    if ((rc = sync_ctl(e))) return rc;
    if (prof_on(e) && e->prof_level == 1) {
        e->tm.finish_ms += ev_ms(e, 9);
        e->tm.finish_launches++;
    }
    e->keys = e->live = 0;
    e->prev_valid = false;
    e->idle_floor = IDLE_FLOOR_NONE;
    return IPXG_OK;
}

// Completes the pending batch (or finish): waits for its control block's publish (the sequence
// word, not the stream: a front launched ahead may be queued behind it), then does what the host
// does after the batch's kernels -- post_batch; for a finish, the flows its fused k_fin_list left or
// its guarded k_finish held back -- on the batch's own control block and event set.  spec: ipxg_submit
// launched the next batch's front ahead, gated on this block; pend.spec_closed then says that the
// gate was closed (that front returned at once and must be launched again).
static int consume_pend(ipxg_engine* e, bool spec) {
    auto& q = e->pend;
    if (!q.on) return IPXG_OK;
    q.on = false;
    int rc;
    const int now = e->cur;
    const BinView bins_now = e->bins_last;
    const bool valid_now = e->bins_valid;
    const uint32_t bits_now = e->part_bits_last;
    const bool swapped = now != q.blk;  // (a front launched ahead switched blocks)
    if (swapped) {
        e->cur = q.blk;
        e->ctl_d = e->ctl_blk[q.blk];
        e->ev = e->evs[q.blk];
    }
    e->bins_last = q.bins;
    e->bins_valid = q.bins_valid;
    e->part_bits_last = q.part_bits;
    rc = IPXG_OK;
    if (!q.published) {  // (no front ahead published it)
        rc = publish_ctl(e, true);
        q.seq = e->pub_seq;
    }
    if (!rc) rc = wait_seq(e, q.seq);
    q.spec_closed = !rc && spec && gate_closed(*e->ctl_h, q.mode);
    if (!rc && (e->ctl_h->guard & GUARD_EX_START))
        rc = set_err(e, IPXG_EDEVICE, "k_fin_list: the export counter was not at the host's count (list-order exports)");
    if (!rc && e->ctl_h->ex_holes) rc = close_export_holes(e);
    if (!rc) rc = check_ex(e);
    if (!rc) {
        if (q.mode == GATE_BATCH) {
            rc = post_batch(e, q.bv, q.p, q.n, true, false);
        } else if (q.mode == GATE_EXPIRE) {  // k_expire right behind the batch, unless its guard held it
            const bool held = e->ctl_h->hold != 0;
            const uint32_t x = held ? 0u : e->ctl_h->expired;
            const uint32_t ti = held ? 0u : e->ctl_h->tls_inv;
            rc = post_batch(e, q.bv, q.p, q.n, true, false);
            if (!rc && !held) {
                e->live = x > e->live ? 0u : e->live - x;
                take_idle_floor(e, ti);  // (it ran with no host work left by the batch: the scan is exact)
            } else if (!rc) {
                rc = expire_table(e, q.now);  // the batch is complete now: expire normally
            }
        } else if (q.mode == GATE_FIN_FUSED) {
            // k_fin_list exported what it finalised: complete unless it could not fuse (host work)
            // or left complex flows
            const bool done = e->ctl_h->fused && !e->ctl_h->complex_count && !e->ctl_h->fin_deferred;
            rc = post_batch(e, q.bv, q.p, q.n, true, true);
            if (!rc && done) {
                e->keys = e->live = 0;
                e->prev_valid = false;
                e->idle_floor = IDLE_FLOOR_NONE;
            } else if (!rc) {
                rc = finish_table(e);  // the remaining flows
            }
        } else {  // GATE_FIN_GUARDED: k_finish right behind the batch, unless its guard held it
            const bool held = e->ctl_h->hold != 0;
            rc = hipMemsetAsync(&e->ctl_d->hold, 0, sizeof(uint32_t), e->st) == hipSuccess ? IPXG_OK
                     : set_err(e, IPXG_EDEVICE, "hipMemsetAsync failed");
            if (!rc) rc = post_batch(e, q.bv, q.p, q.n, true, !held);
            if (!rc && !held) {
                if (prof_on(e) && e->prof_level == 1) {
                    e->tm.finish_ms += ev_ms(e, 9);
                    e->tm.finish_launches++;
                }
                e->keys = e->live = 0;
                e->prev_valid = false;
                e->idle_floor = IDLE_FLOOR_NONE;
            } else if (!rc) {
                rc = finish_table(e);  // the batch is complete now: finish normally
            }
        }
    }
    if (swapped) {
        e->cur = now;
        e->ctl_d = e->ctl_blk[now];
        e->ev = e->evs[now];
    }
    if (spec && !q.spec_closed) {  // (closed: the front is launched again and sets them)
        e->bins_last = bins_now;
        e->bins_valid = valid_now;
        e->part_bits_last = bits_now;
    }
    if (q.clear_after) {  // ipxg_clear_exports after this batch: its exports (and the follow-ups') dropped
        e->ex_count = e->ex_head = 0;
        e->ex6_valid = e->count6_on;
        e->ex_zero_pending = true;
    }
    return rc;
}

static int finish_impl(ipxg_engine* e) {
    if (!e) return IPXG_EINVAL;
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if (e->pend.on) {  // a batch or finish still pending
        if (e->failed) return complete_batch(e);  // (IPXG_ESTATE)
        if ((rc = consume_pend(e, false))) return rc;
    }
    if ((rc = join_fmt(e))) return rc;
    if (e->strict) {  // finish (cache.cpp:276-288): every record FORCED
        if ((rc = ensure_export(e, e->live))) return rc;
        HIPCHK(e, hipMemsetAsync(e->ctl_d, 0, sizeof(BatchCtl), e->st));
        launch_strict_finish(e->st, e->sv, export_view(e), e->ctl_d, e->stats_d);
        HIPCHK(e, hipGetLastError());
        if ((rc = sync_ctl(e))) return rc;
        e->live = (uint32_t)((int64_t)e->live + e->ctl_h->strict_live);
        if (e->live) return set_err(e, IPXG_EDEVICE, "strict finish: records still live after the whole table was exported");
        e->keys = 0;
        return IPXG_OK;
    }
    if (e->inflight.on) {
        // The batch's k_fin_list is still to be launched: into a table that was empty before
        // the batch, it exports what it finalises itself (fused finish, no table scan).
        // Otherwise the finish is enqueued right behind the batch, guarded on the device
        // (k_finish's guard).  Either way the host does not wait: the finish is pending (its
        // control block published with a sequence number) and the next call completes it --
        // ipxg_submit of a device batch after launching that batch's front behind it, so the
        // device runs step after step without waiting for the host (workers.cpp:66-122: the
        // reference's storage loop does not block between blocks either).
        const bool fuse = e->inflight.tail && e->live == 0 && e->keys == 0;
        if ((rc = launch_tail(e, fuse))) return rc;
        if (!fuse) {
            ev_rec(e, 9);
            launch_finish(e->st, table_view(e), e->cap, export_view(e), e->stats_d, e->ctl_d, e->ex_count, e->live);
            HIPCHK(e, hipGetLastError());
            ev_rec(e, 10);
        }
        // the batch is consumed here whatever happens next: an error below must not make the
        // next call run post_batch again on a table k_finish may already have emptied
        e->inflight.on = false;
        set_pend(e, fuse ? GATE_FIN_FUSED : GATE_FIN_GUARDED, e->inflight.bv, e->inflight.p, e->inflight.n);
        if (e->sync_finish) return consume_pend(e, false);
        return IPXG_OK;
    }
    return finish_table(e);
}

int ipxg_reset(ipxg_engine* e) {
    if (!e) return IPXG_EINVAL;
    if (e->fst) (void)hipStreamSynchronize(e->fst);  // (the formatting in flight reads what reset clears)
    e->fmt_pending = false;
    if (e->failed) {  // a process plugin's failure: the lost batch's host state is dropped too
        e->failed = false;
        e->fail_msg.clear();
        e->inflight.on = e->inflight.tail = false;
        e->pend.on = false;
    }
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    HIPCHK(e, hipMemsetAsync(e->line, 0, sizeof(SlotLine) * (size_t)e->cap, e->st));
    if (e->strict) {
        launch_strict_clear(e->st, e->sv);
        HIPCHK(e, hipGetLastError());
        e->strict_q = 0;
    }
    const uint32_t fs = e->cfg.frag_size ? e->cfg.frag_size : 10007;
    HIPCHK(e, hipMemsetAsync(e->frag_cnt, 0, (size_t)fs * sizeof(uint32_t), e->st));
    HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
    e->ex_zero_pending = false;
    if (e->pstat_d) HIPCHK(e, hipMemsetAsync(e->pstat_d, 0, PSTAT_WORDS * 8, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->ex_count = e->ex_head = 0;
    e->ex6_valid = e->count6_on;
    e->keys = e->live = 0;
    e->last_touched = 0;
    e->prev_valid = false;
    e->idle_floor = IDLE_FLOOR_NONE;
    return IPXG_OK;
}

static int pending_exports_impl(ipxg_engine* e, size_t* n) {
    if (!e || !n) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    *n = e->ex_count - e->ex_head;
    return IPXG_OK;
}

static int poll_exports_impl(ipxg_engine* e, ipxg_flow_record* out, size_t cap, size_t* n) {
    if (!e || !n || (cap && !out)) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    size_t k = std::min<size_t>(cap, e->ex_count - e->ex_head);
    if (k) {
        HIPCHK(e, hipSetDevice(e->cfg.device_id));
        HIPCHK(e, hipMemcpyAsync(out, e->ex + e->ex_head, k * sizeof(ipxg_flow_record), hipMemcpyDeviceToHost,
                                 e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
        // pre_export of the device's exports that carry plugin state (IPXG_REC_PRE_EXPORTED)
        if (!e->plugins.empty())
            for (size_t i = 0; i < k; ++i) {
                ipxg_flow_record& r = out[i];
                if (!r.ext || (r.reserved0 & IPXG_REC_PRE_EXPORTED)) continue;
                for (const ipxg_plugin& q : e->plugins)
                    if (q.pre_export) q.pre_export(q.ctx, &r);
                r.reserved0 |= IPXG_REC_PRE_EXPORTED;
            }
        // pre_export returns nothing: a failure there is reported by the instance's error(), as
        // after a walk -- the records are handed over, then the engine stops until ipxg_reset
        for (size_t q = 0; q < e->plugins.size() && !e->failed; ++q)
            if (const char* m = e->plugins[q].error ? e->plugins[q].error(e->plugins[q].ctx) : nullptr) {
                e->failed = true;
                e->fail_msg = "process plugin " + std::to_string(q) + " (pre_export): " + m;
            }
    }
    e->ex_head += (uint32_t)k;
    if (k) e->ex6_valid = false;
    if (e->ex_head == e->ex_count) {
        e->ex_head = e->ex_count = 0;
        e->ex6_valid = e->count6_on;
        HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
        e->ex_zero_pending = false;
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    *n = k;
    if (e->failed) return set_err(e, IPXG_EPLUGIN, e->fail_msg);
    return IPXG_OK;
}

// IPFIX basic-template records of n device records at `rec` into the scratch buffers
// (ipf_out: the bytes, ipf_off: n + 1 offsets); no host sync.
static int ipfix_format(ipxg_engine* e, const ipxg_flow_record* rec, uint32_t n, uint32_t dir) {
    int rc;
    const size_t nb = (n + 255) / 256;
    if ((rc = ensure(e, e->ipf_out, (size_t)n * 105 + 16))) return rc;
    if ((rc = ensure(e, e->ipf_tot, (nb + 1) * sizeof(uint64_t)))) return rc;
    if ((rc = ensure(e, e->ipf_off, ((size_t)n + 1) * sizeof(uint64_t)))) return rc;
    launch_ipfix_basic(e->st, rec, n, dir, (uint64_t*)e->ipf_tot.p, (uint8_t*)e->ipf_out.p, (uint64_t*)e->ipf_off.p);
    HIPCHK(e, hipGetLastError());
    return IPXG_OK;
}

int ipxg_ipfix_basic(ipxg_engine* e, const ipxg_flow_record* recs, size_t n, uint32_t dir_bit_field, uint8_t* out,
                     uint64_t* offsets) {
    if (!e || (n && (!recs || !out || !offsets))) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    if (offsets) offsets[0] = 0;
    if (n == 0) return IPXG_OK;
    if (n > IPXG_MAX_BATCH) return set_err(e, IPXG_ETOOBIG, "more records than IPXG_MAX_BATCH");
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if ((rc = ensure(e, e->ipf_rec, n * sizeof(ipxg_flow_record)))) return rc;
    HIPCHK(e, hipMemcpyAsync(e->ipf_rec.p, recs, n * sizeof(ipxg_flow_record), hipMemcpyHostToDevice, e->st));
    if ((rc = ipfix_format(e, (const ipxg_flow_record*)e->ipf_rec.p, (uint32_t)n, dir_bit_field))) return rc;
    HIPCHK(e, hipMemcpyAsync(offsets, e->ipf_off.p, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    HIPCHK(e, hipMemcpyAsync(out, e->ipf_out.p, offsets[n], hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return IPXG_OK;
}

int ipxg_poll_ipfix(ipxg_engine* e, uint32_t dir_bit_field, uint8_t* out, size_t cap, size_t* n, size_t* bytes) {
    if (!e || !n || !bytes || (cap && !out)) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    {
        const int rc1 = join_fmt(e);  // (the IPFIX scratch buffers are the formatting stream's too)
        if (rc1) return rc1;
    }
    *n = *bytes = 0;
    const uint32_t pend = e->ex_count - e->ex_head;
    if (pend == 0) return IPXG_OK;
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if ((rc = ipfix_format(e, e->ex + e->ex_head, pend, dir_bit_field))) return rc;
    std::vector<uint64_t> off((size_t)pend + 1);
    HIPCHK(e, hipMemcpyAsync(off.data(), e->ipf_off.p, off.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    // whole records only: the longest prefix that fits `cap`
    const size_t k = (size_t)(std::upper_bound(off.begin(), off.end(), (uint64_t)cap) - off.begin()) - 1;
    if (k) {
        HIPCHK(e, hipMemcpyAsync(out, e->ipf_out.p, off[k], hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    e->ex_head += (uint32_t)k;
    if (k) e->ex6_valid = false;
    if (e->ex_head == e->ex_count) {
        e->ex_head = e->ex_count = 0;
        e->ex6_valid = e->count6_on;
        HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
        e->ex_zero_pending = false;
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    *n = k;
    *bytes = off[k];
    return IPXG_OK;
}

// ---- IPFIX messages ---------------------------------------------------------------------
// The reference exporter's buffer logic (src/plugins/output/ipfix/src/ipfix.cpp) replayed over
// whole data sets: n4 IPv4-template records, then n6 IPv6-template records, then flush().
// A template buffer takes records while 4 + (k + 1) * len <= mtu - 16 (fill_basic_flow
// :1479/:1497, tmpltMaxBufferSize = mtu - IPFIX_HEADER_SIZE); the record that does not fit
// flushes (export_flow :385-398): the template message if not sent yet (create_template_packet
// :671-728), then data messages (create_data_packet :739-795: walk the template list, newest
// template -- IPv6, 259 -- first, and add every non-empty buffer that still fits the message).
namespace {
constexpr uint32_t IPFIX_LEN[2] = {81, 105};
constexpr uint32_t IPFIX_TMPL_REC = 88;                    // 4 + 18 fields * 4 + 3 enterprise numbers * 4
constexpr uint32_t IPFIX_TMPL_MSG = 16 + 4 + 2 * IPFIX_TMPL_REC;

struct IpfixPlan {
    std::vector<IpfixSet> sets[2];
    std::vector<IpfixMsg> msgs;
    uint64_t bytes = 0;
    bool tmpl = false;  // the template message leads the stream
    uint32_t seq_end = 0;
};

static IpfixPlan ipfix_plan(uint64_t n4, uint64_t n6, const ipxg_ipfix_exporter& x) {
    IpfixPlan P;
    const uint32_t mtu = x.mtu;
    uint64_t b[2] = {0, 0}, emitted[2] = {0, 0};
    uint32_t seq = x.sequence;
    bool tmpl_sent = x.templates_sent != 0;
    auto flush = [&]() {
        if (!tmpl_sent) {
            P.tmpl = true;
            P.bytes += IPFIX_TMPL_MSG;
            tmpl_sent = true;
        }
        for (;;) {
            uint32_t size = 16, flows = 0;
            for (int c : {1, 0}) {  // the template list: IPv6 (259) first, then IPv4 (258)
                const uint32_t sz = 4 + (uint32_t)b[c] * IPFIX_LEN[c];
                if (b[c] > 0 && size + sz <= mtu) {
                    P.sets[c].push_back(IpfixSet{(uint32_t)c, (uint32_t)b[c], emitted[c], P.bytes + size});
                    emitted[c] += b[c];
                    flows += (uint32_t)b[c];
                    size += sz;
                    b[c] = 0;
                }
            }
            if (size == 16) break;
            P.msgs.push_back(IpfixMsg{P.bytes, size, seq});
            P.bytes += size;
            seq += flows;
        }
    };
    const uint64_t n[2] = {n4, n6};
    for (int c : {0, 1}) {
        const uint64_t cap = (mtu - 20) / IPFIX_LEN[c];
        uint64_t rem = n[c];
        while (rem) {
            if (b[c] == cap) flush();
            const uint64_t take = std::min(rem, cap - b[c]);
            b[c] += take;
            rem -= take;
        }
    }
    if (n4 + n6) flush();
    P.seq_end = seq;
    return P;
}

// the template message: header, template set, the IPv6 then the IPv4 basic template records
// (create_template :537-656 with the elements of ipfix-elements.hpp:328-366)
void ipfix_template_msg(uint8_t* m, const ipxg_ipfix_exporter& x) {
    static const uint32_t F[2][18][3] = {
        {{0, 136, 1}, {0, 1, 8}, {29305, 1, 8}, {0, 2, 8}, {29305, 2, 8}, {0, 154, 8}, {0, 155, 8}, {0, 60, 1},
         {0, 4, 1}, {0, 6, 1}, {29305, 6, 1}, {0, 7, 2}, {0, 11, 2}, {0, 10, 4}, {0, 8, 4}, {0, 12, 4}, {0, 56, 6},
         {0, 80, 6}},
        {{0, 136, 1}, {0, 1, 8}, {29305, 1, 8}, {0, 2, 8}, {29305, 2, 8}, {0, 154, 8}, {0, 155, 8}, {0, 60, 1},
         {0, 4, 1}, {0, 6, 1}, {29305, 6, 1}, {0, 7, 2}, {0, 11, 2}, {0, 10, 4}, {0, 27, 16}, {0, 28, 16},
         {0, 56, 6}, {0, 80, 6}}};
    auto be16 = [](uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; };
    auto be32 = [](uint8_t* p, uint32_t v) { for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (24 - 8 * k)); };
    be16(m, 10);
    be16(m + 2, IPFIX_TMPL_MSG);
    be32(m + 4, x.export_time);
    be32(m + 8, x.sequence);
    be32(m + 12, x.odid);
    be16(m + 16, 2);  // TEMPLATE_SET_ID
    be16(m + 18, IPFIX_TMPL_MSG - 16);
    uint32_t p = 20;
    for (int c : {1, 0}) {
        be16(m + p, c ? 259 : 258);
        be16(m + p + 2, 18);
        p += 4;
        for (const auto& f : F[c]) {
            be16(m + p, f[1] | (f[0] ? 0x8000 : 0));
            be16(m + p + 2, f[2]);
            p += 4;
            if (f[0]) {
                be32(m + p, f[0]);
                p += 4;
            }
        }
    }
}
}  // namespace

// n device records at rec -> messages in mb; *bytes, *msgs; updates *x.  n6 >= 0: the
// IPv6-template records among them, known from the export counters (then nothing here waits
// for the device); n6 < 0: counted first (one readback).
static int ipfix_messages(ipxg_engine* e, ipxg_ipfix_exporter* x, const ipxg_flow_record* rec, uint32_t n,
                          int64_t n6, size_t* bytes, size_t* msgs, DevBuf& mb, hipStream_t st) {
    if (x->mtu < 16 + 4 + 105) return set_err(e, IPXG_EINVAL, "IPFIX mtu below one IPv6 basic record");
    int rc;
    const size_t nb = (n + 255) / 256;
    if (n) {
        if ((rc = ensure(e, e->ipf_tot, (nb + 1) * sizeof(uint64_t)))) return rc;
        launch_ipfix_count6(st, rec, n, (uint64_t*)e->ipf_tot.p);  // per-block prefix (the fill needs it)
        HIPCHK(e, hipGetLastError());
        if (n6 < 0) {
            uint64_t c = 0;
            HIPCHK(e, hipMemcpyAsync(&c, (uint64_t*)e->ipf_tot.p + nb, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
            HIPCHK(e, hipStreamSynchronize(st));
            n6 = (int64_t)c;
        }
    } else {
        n6 = 0;
    }
    const IpfixPlan P = ipfix_plan(n - (uint64_t)n6, (uint64_t)n6, *x);
    const size_t ns4 = P.sets[0].size(), ns6 = P.sets[1].size(), nm = P.msgs.size();
    const size_t moff = (ns4 + ns6) * sizeof(IpfixSet), toff = moff + nm * sizeof(IpfixMsg);
    const size_t coff = (toff + IPFIX_TMPL_MSG + 7) & ~(size_t)7;  // {stream bytes, records} (u64 each)
    const size_t pbytes = coff + 2 * sizeof(uint64_t);
    // the pinned staging buffer may still feed the previous plan's upload
    if (e->plan_ev) HIPCHK(e, hipEventSynchronize(e->plan_ev));
    else HIPCHK(e, hipEventCreateWithFlags(&e->plan_ev, hipEventDisableTiming));
    if (e->plan_h_bytes < pbytes) {
        if (e->plan_h) HIPCHK(e, hipHostFree(e->plan_h));
        e->plan_h = nullptr;
        e->plan_h_bytes = 0;
        HIPCHK(e, hipHostMalloc((void**)&e->plan_h, pbytes * 2, hipHostMallocDefault));
        e->plan_h_bytes = pbytes * 2;
    }
    uint8_t* plan = e->plan_h;
    std::memcpy(plan, P.sets[0].data(), ns4 * sizeof(IpfixSet));
    std::memcpy(plan + ns4 * sizeof(IpfixSet), P.sets[1].data(), ns6 * sizeof(IpfixSet));
    std::memcpy(plan + moff, P.msgs.data(), nm * sizeof(IpfixMsg));
    ipfix_template_msg(plan + toff, *x);
    const uint64_t counts[2] = {P.bytes, n};
    std::memcpy(plan + coff, counts, sizeof(counts));
    // the {bytes, records} pair lives at the tail of the message buffer itself (8-byte aligned past
    // the stream), so it stays valid exactly as long as its stream -- the device message buffers
    // alternate (ipxg_device_ipfix_messages), the plan does not
    const size_t cnt_off = (P.bytes + 7) & ~(size_t)7;
    if ((rc = ensure(e, e->ipf_plan, pbytes))) return rc;
    if ((rc = ensure(e, mb, cnt_off + 2 * sizeof(uint64_t)))) return rc;
    uint8_t* out = (uint8_t*)mb.p;
    HIPCHK(e, hipMemcpyAsync(e->ipf_plan.p, plan, pbytes, hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(out + cnt_off, plan + coff, 2 * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIPCHK(e, hipEventRecord(e->plan_ev, st));
    e->ipf_counts = (const uint64_t*)(out + cnt_off);
    if (P.tmpl)
        HIPCHK(e, hipMemcpyAsync(out, (uint8_t*)e->ipf_plan.p + toff, IPFIX_TMPL_MSG, hipMemcpyDeviceToDevice, st));
    const IpfixSet* sets = (const IpfixSet*)e->ipf_plan.p;
    const IpfixMsg* m = (const IpfixMsg*)((uint8_t*)e->ipf_plan.p + moff);
    launch_ipfix_messages(st, rec, n, x->dir_bit_field, (const uint64_t*)e->ipf_tot.p, sets, (uint32_t)ns4,
                          (uint32_t)ns6, m, (uint32_t)nm, x->odid, x->export_time, out);
    HIPCHK(e, hipGetLastError());
    if (P.tmpl) x->templates_sent = 1;
    x->sequence = P.seq_end;
    *bytes = P.bytes;
    *msgs = nm + (P.tmpl ? 1 : 0);
    return IPXG_OK;
}

static int64_t known_v6(ipxg_engine* e) {
    const int64_t k = (e->ex6_valid && e->ex_head == 0) ? (int64_t)e->ex_count6 : -1;
    e->count6_on = true;  // from now on the export kernels count (valid from the next reset)
    return k;
}

void ipxg_ipfix_exporter_init(ipxg_ipfix_exporter* x) {
    if (!x) return;
    std::memset(x, 0, sizeof(*x));
    x->mtu = IPXG_IPFIX_DEFAULT_MTU;
}

uint64_t ipxg_ipfix_bound(uint64_t n) {
    // every record in a message of its own is the worst case: 16 + 4 + 105 per record
    return IPFIX_TMPL_MSG + n * (16 + 4 + 105);
}

int ipxg_ipfix_export(ipxg_engine* e, ipxg_ipfix_exporter* x, const ipxg_flow_record* recs, size_t n, uint8_t* out,
                      size_t cap, size_t* bytes, size_t* msgs) {
    if (!e || !x || !bytes || !msgs || (n && (!recs || !out))) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    {
        const int rc1 = join_fmt(e);  // (the IPFIX scratch buffers are the formatting stream's too)
        if (rc1) return rc1;
    }
    if (n > 0xFFFFFFF0ull) return set_err(e, IPXG_ETOOBIG, "too many records");
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if (n) {
        if ((rc = ensure(e, e->ipf_rec, n * sizeof(ipxg_flow_record)))) return rc;
        HIPCHK(e, hipMemcpyAsync(e->ipf_rec.p, recs, n * sizeof(ipxg_flow_record), hipMemcpyHostToDevice, e->st));
    }
    ipxg_ipfix_exporter y = *x;
    size_t nbytes = 0, nm = 0;
    if ((rc = ipfix_messages(e, &y, (const ipxg_flow_record*)e->ipf_rec.p, (uint32_t)n, -1, &nbytes, &nm, e->ipf_msg, e->st)))
        return rc;
    if (nbytes > cap) return set_err(e, IPXG_ETOOBIG, "output buffer too small for the messages");
    if (nbytes) {
        HIPCHK(e, hipMemcpyAsync(out, e->ipf_msg.p, nbytes, hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    *x = y;
    *bytes = nbytes;
    *msgs = nm;
    return IPXG_OK;
}

int ipxg_device_ipfix_messages(ipxg_engine* e, ipxg_ipfix_exporter* x, const uint8_t** dptr, size_t* n_records,
                               size_t* bytes, size_t* msgs) {
    if (!e || !x || !dptr || !n_records || !bytes || !msgs) return IPXG_EINVAL;
    // An asynchronous batch in flight whose tail (k_fin_list, the first of its kernels to append
    // exports) is still to be launched has written no export: the pending exports are the completed
    // batches', and they are formatted beside its kernels (the tail joins the formatting first) --
    // the batch is not completed here.  Otherwise the batch in flight is completed first.
    const bool beside = e->inflight.on && e->inflight.tail && !e->failed;
    if (!beside) {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    const uint32_t pend = e->ex_count - e->ex_head;
    int rc;
    DevBuf& mb = e->ipf_dmsg[e->ipf_dnext];
    if (!e->fst) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->fst, hipStreamNonBlocking));
        HIPCHK(e, hipEventCreateWithFlags(&e->fmt_fork, hipEventDisableTiming));
        HIPCHK(e, hipEventCreateWithFlags(&e->fmt_done, hipEventDisableTiming));
    }
    if (beside && e->ex_ev_valid) {  // from the in-flight batch's start: not behind its kernels
        HIPCHK(e, hipStreamWaitEvent(e->fst, e->ex_ev, 0));
    } else {  // (beside without ex_ev -- the first call, fst did not exist at the submit: behind the
              // batch's k_bin / k_reduce, which append no export, so the same exports are formatted)
        HIPCHK(e, hipEventRecord(e->fmt_fork, e->st));
        HIPCHK(e, hipStreamWaitEvent(e->fst, e->fmt_fork, 0));
    }
    if ((rc = ipfix_messages(e, x, e->ex + e->ex_head, pend, known_v6(e), bytes, msgs, mb, e->fst))) return rc;
    HIPCHK(e, hipEventRecord(e->fmt_done, e->fst));
    e->fmt_pending = true;
    e->ipf_dnext ^= 1;  // the next call writes the other buffer: this one stays valid until the call after it
    *dptr = (const uint8_t*)mb.p;
    *n_records = pend;
    e->ex_head = e->ex_count = 0;  // consumed
    e->ex6_valid = e->count6_on;
    HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
    e->ex_zero_pending = false;
    return IPXG_OK;
}

int ipxg_device_ipfix_counts(ipxg_engine* e, const uint64_t** dptr) {
    if (!e || !dptr) return IPXG_EINVAL;
    if (!e->ipf_counts) return set_err(e, IPXG_ESTATE, "no ipxg_device_ipfix_messages call yet");
    *dptr = e->ipf_counts;
    return IPXG_OK;
}

int ipxg_poll_ipfix_messages(ipxg_engine* e, ipxg_ipfix_exporter* x, uint8_t* out, size_t cap, size_t* n_records,
                             size_t* bytes, size_t* msgs) {
    if (!e || !x || !n_records || !bytes || !msgs || (cap && !out)) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    {
        const int rc1 = join_fmt(e);  // (the IPFIX scratch buffers are the formatting stream's too)
        if (rc1) return rc1;
    }
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    const uint32_t pend = e->ex_count - e->ex_head;
    ipxg_ipfix_exporter y = *x;
    size_t nbytes = 0, nm = 0;
    int rc;
    if ((rc = ipfix_messages(e, &y, e->ex + e->ex_head, pend, known_v6(e), &nbytes, &nm, e->ipf_msg, e->st))) return rc;
    if (nbytes > cap) return set_err(e, IPXG_ETOOBIG, "output buffer too small for the messages");
    if (nbytes) {
        HIPCHK(e, hipMemcpyAsync(out, e->ipf_msg.p, nbytes, hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    e->ex_head = e->ex_count = 0;
    e->ex6_valid = e->count6_on;
    HIPCHK(e, hipMemsetAsync(e->ex_count_d, 0, 3 * sizeof(uint32_t), e->st));
    e->ex_zero_pending = false;
    HIPCHK(e, hipStreamSynchronize(e->st));
    *x = y;
    *n_records = pend;
    *bytes = nbytes;
    *msgs = nm;
    return IPXG_OK;
}

int ipxg_device_exports(ipxg_engine* e, const ipxg_flow_record** dptr, size_t* n) {
    if (!e || !dptr || !n) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    *dptr = e->ex + e->ex_head;
    *n = e->ex_count - e->ex_head;
    return IPXG_OK;
}

static int clear_exports_impl(ipxg_engine* e) {
    if (!e) return IPXG_EINVAL;
    if (e->pend.on && !e->inflight.on && !e->failed) {
        // a finish (or batch) still pending: its exports are dropped when it completes (and what its
        // completion exports after it), without waiting for it here
        e->pend.clear_after = true;
        e->ex_head = e->ex_count = 0;
        e->ex6_valid = e->count6_on;
        e->ex_zero_pending = true;
        return IPXG_OK;
    }
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    e->ex_head = e->ex_count = 0;
    e->ex6_valid = e->count6_on;
    e->ex_zero_pending = true;  // zeroed on the stream before the next export append (export_view / submit)
    return IPXG_OK;
}

int ipxg_parser_stats(ipxg_engine* e, uint64_t* tcp_ports, uint64_t* udp_ports, ipxg_vlan_stats* vlans) {
    if (!e) return IPXG_EINVAL;
    if (!e->pstat_d) return set_err(e, IPXG_EINVAL, "parser statistics are off (create the engine with ps=true)");
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    std::vector<uint64_t> h(PSTAT_WORDS);
    HIPCHK(e, hipMemcpyAsync(h.data(), e->pstat_d, PSTAT_WORDS * 8, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    static_assert(sizeof(ipxg_vlan_stats) == VS_N * 8, "VlanStats layout");
    for (const std::vector<uint64_t>& hp : e->host_ports)  // the plugin walks' flows, per walk thread
        if (!hp.empty())
            for (size_t k = 0; k < 2 * 65536; ++k) h[k] += hp[k];
    if (tcp_ports) std::memcpy(tcp_ports, h.data(), 65536 * 8);
    if (udp_ports) std::memcpy(udp_ports, h.data() + 65536, 65536 * 8);
    if (vlans) std::memcpy(vlans, h.data() + PSTAT_PORTS, (size_t)IPXG_VLAN_IDS * VS_N * 8);
    return IPXG_OK;
}

// TopPorts::get_top_ports (topPorts.cpp): every TCP port, then every UDP port, in port order,
// goes into a buffer of n entries kept in decreasing frequency, after the entries of equal
// frequency (update_port_buffer's lower_bound on `frequency >= count`); a zero frequency never
// enters.  That is: the ports of non-zero frequency, stably sorted by decreasing frequency,
// the first n.
int ipxg_top_ports(ipxg_engine* e, size_t n, ipxg_port_stat* out, size_t* got) {
    if (!e || (!out && n) || !got) return IPXG_EINVAL;
    std::vector<uint64_t> f(2 * 65536);
    int rc;
    if ((rc = ipxg_parser_stats(e, f.data(), f.data() + 65536, nullptr))) return rc;
    std::vector<uint32_t> idx;
    for (uint32_t k = 0; k < 2 * 65536; ++k)
        if (f[k]) idx.push_back(k);
    const size_t m = std::min(n, idx.size());
    std::partial_sort(idx.begin(), idx.begin() + m, idx.end(), [&](uint32_t a, uint32_t b) {
        return f[a] != f[b] ? f[a] > f[b] : a < b;  // a < b: TCP before UDP, then port order
    });
    for (size_t k = 0; k < m; ++k) {
        std::memset(&out[k], 0, sizeof(out[k]));
        out[k].port = (uint16_t)(idx[k] & 0xFFFF);
        out[k].protocol = idx[k] < 65536 ? 6 : 17;
        out[k].frequency = f[idx[k]];
    }
    *got = m;
    return IPXG_OK;
}

int ipxg_get_stats(ipxg_engine* e, ipxg_stats* out) {
    if (!e || !out) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    std::vector<unsigned long long> h((size_t)STAT_SHARDS * ST_STRIDE);
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    HIPCHK(e, hipMemcpyAsync(h.data(), e->stats_d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    uint64_t s[ST_COUNT] = {};
    for (int sh = 0; sh < STAT_SHARDS; ++sh)
        for (int k = 0; k < ST_COUNT; ++k) s[k] += h[(size_t)sh * ST_STRIDE + k];
    std::memset(out, 0, sizeof(*out));
    out->seen_packets = s[ST_SEEN];
    out->parsed_packets = s[ST_PARSED];
    out->unknown_packets = s[ST_UNKNOWN];
    out->ipv4_packets = s[ST_IPV4];
    out->ipv6_packets = s[ST_IPV6];
    out->tcp_packets = s[ST_TCP];
    out->udp_packets = s[ST_UDP];
    out->mpls_packets = s[ST_MPLS];
    out->pppoe_packets = s[ST_PPPOE];
    out->trill_packets = s[ST_TRILL];
    out->vlan_packets = s[ST_VLAN];
    out->ipv4_bytes = s[ST_IPV4_BYTES];
    out->ipv6_bytes = s[ST_IPV6_BYTES];
    for (int k = 0; k < 5; ++k) s[ST_END_INACTIVE + k] += e->host_end[k];  // the plugin walks' exports
    out->end_inactive = s[ST_END_INACTIVE];
    out->end_active = s[ST_END_ACTIVE];
    out->end_eof = s[ST_END_EOF];
    out->end_forced = s[ST_END_FORCED];
    out->end_no_res = s[ST_END_NO_RES];
    out->flows_in_cache = e->live;
    out->total_exported = s[ST_END_INACTIVE] + s[ST_END_ACTIVE] + s[ST_END_EOF] + s[ST_END_FORCED] +
                          s[ST_END_NO_RES] + e->host_unreasoned;
    out->keyless_packets = s[ST_KEYLESS];
    out->fragmented_packets = s[ST_FRAGMENTED];
    out->fragments_filled = s[ST_FRAG_FILLED];
    out->complex_flows = e->complex_total;
    out->table_capacity = e->strict ? (uint64_t)e->sv.slot_mask + 1 : e->cap;
    out->table_rehashes = e->rehashes;
    out->batches = e->batches;
    out->spilled_packets = e->spilled;
    out->slow_path_packets = e->slow_pkts;
    out->walked_packets = e->walked_pkts;
    out->aggregated_packets = e->agg_pkts;
    for (int k = 0; k < 6; ++k) s[ST_PKTS_1 + k] += e->host_pkts[k];
    out->flows_1_packet = s[ST_PKTS_1];
    out->flows_2_5_packets = s[ST_PKTS_2_5];
    out->flows_6_10_packets = s[ST_PKTS_6_10];
    out->flows_11_20_packets = s[ST_PKTS_11_20];
    out->flows_21_50_packets = s[ST_PKTS_21_50];
    out->flows_51_plus_packets = s[ST_PKTS_51];
    return IPXG_OK;
}

int ipxg_probe_counters(ipxg_engine* e, uint64_t* out) {
    if (!e || !out) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    for (int k = 0; k < 16; ++k) out[k] = e->ctl_h->probe[k];
    return IPXG_OK;
}

int ipxg_profile(ipxg_engine* e, int enable) {
    if (!e) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if ((enable & 0xFF) && !e->evs[0][0])
        for (auto& set : e->evs)
            for (hipEvent_t& ev : set) HIPCHK(e, hipEventCreate(&ev));
    const int level = enable & 0xFF;
    const uint32_t every = ((uint32_t)enable >> 8) & 0xFFFFu;
    e->prof = level != 0;
    e->prof_level = (level == 2 || level == 3) ? level : (level ? 1 : 0);
    e->prof_every = every ? every : 1;
    e->prof_seq = 0;
    e->prof_set[0] = e->prof_set[1] = false;
    if (level) e->tm = ipxg_timing{};
    return IPXG_OK;
}

int ipxg_get_timing(ipxg_engine* e, ipxg_timing* out) {
    if (!e || !out) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    *out = e->tm;
    return IPXG_OK;
}

int ipxg_parse_batch(ipxg_engine* e, const ipxg_batch* batch, ipxg_parsed_pkt* out) {
    if (!e || !batch || !out) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    const uint32_t n = batch->n;
    if (!n) return IPXG_OK;
    int rc;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    if ((rc = check_arena(e, batch))) return rc;
    BatchView bv;
    bv.n = n;
    set_arena_view(bv, batch);
    bv.base_sec = 0;
    if (batch->flags & IPXG_BATCH_DEVICE) {
        bv.arena = batch->arena;
        bv.desc = batch->desc;
    } else {
        if ((rc = ensure(e, e->arena, batch->arena_len + 64))) return rc;
        if ((rc = ensure(e, e->desc, (size_t)n * sizeof(ipxg_pkt_desc)))) return rc;
        HIPCHK(e, hipMemcpyAsync(e->arena.p, batch->arena, batch->arena_len, hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipMemcpyAsync(e->desc.p, batch->desc, (size_t)n * sizeof(ipxg_pkt_desc), hipMemcpyHostToDevice,
                                 e->st));
        bv.arena = (const uint8_t*)e->arena.p;
        bv.desc = (const ipxg_pkt_desc*)e->desc.p;
    }
    ipxg_parsed_pkt* d_out;
    HIPCHK(e, hipMalloc((void**)&d_out, (size_t)n * sizeof(ipxg_parsed_pkt)));
    launch_parse_batch(e->st, bv, e->cfg.datalink, d_out);
    hipError_t le = hipGetLastError();
    if (le == hipSuccess)
        le = hipMemcpyAsync(out, d_out, (size_t)n * sizeof(ipxg_parsed_pkt), hipMemcpyDeviceToHost, e->st);
    if (le == hipSuccess) le = hipStreamSynchronize(e->st);
    (void)hipFree(d_out);
    if (le != hipSuccess) return set_err(e, IPXG_EDEVICE, hipGetErrorString(le));
    return IPXG_OK;
}

int ipxg_xxh64_batch(ipxg_engine* e, const uint8_t* keys, uint32_t keylen, uint32_t n, uint64_t seed,
                     uint64_t* out) {
    if (!e || (n && (!keys || !out))) return IPXG_EINVAL;
    {
        const int rc0 = complete_batch(e);
        if (rc0) return rc0;
    }
    if (!n) return IPXG_OK;
    HIPCHK(e, hipSetDevice(e->cfg.device_id));
    uint8_t* dk;
    uint64_t* dh;
    size_t kb = (size_t)keylen * n;
    HIPCHK(e, hipMalloc((void**)&dk, kb ? kb : 1));
    if (hipMalloc((void**)&dh, (size_t)n * 8) != hipSuccess) {
        (void)hipFree(dk);
        return set_err(e, IPXG_ENOMEM, "hipMalloc failed");
    }
    hipError_t le = kb ? hipMemcpyAsync(dk, keys, kb, hipMemcpyHostToDevice, e->st) : hipSuccess;
    if (le == hipSuccess) {
        launch_xxh64(e->st, dk, keylen, n, seed, dh);
        le = hipGetLastError();
    }
    if (le == hipSuccess) le = hipMemcpyAsync(out, dh, (size_t)n * 8, hipMemcpyDeviceToHost, e->st);
    if (le == hipSuccess) le = hipStreamSynchronize(e->st);
    (void)hipFree(dk);
    (void)hipFree(dh);
    if (le != hipSuccess) return set_err(e, IPXG_EDEVICE, hipGetErrorString(le));
    return IPXG_OK;
}

// The calls that run the engine's C++ host code (containers, the process-plugin walk): no C++
// exception crosses the C ABI (include/ipxg.h: int codes only), and after a process plugin's
// failure (IPXG_EPLUGIN) the engine refuses them until ipxg_reset, as the reference's pipeline
// stops at its first PluginError (workers.cpp:107-112).
extern "C++" template <class F>
static int guarded(ipxg_engine* e, F&& f) {
    if (!e) return IPXG_EINVAL;
    if (e->failed)
        return set_err(e, IPXG_ESTATE, "engine stopped by a process plugin error (ipxg_reset or ipxg_destroy): " +
                                           e->fail_msg);
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_err(e, IPXG_ENOMEM, "host allocation failed");
    } catch (const std::exception& x) {
        return set_err(e, IPXG_EDEVICE, std::string("internal error: ") + x.what());
    } catch (...) {
        return set_err(e, IPXG_EDEVICE, "internal error: unknown exception");
    }
}

int ipxg_submit(ipxg_engine* e, const ipxg_batch* batch) { return guarded(e, [&] { return submit_impl(e, batch); }); }
int ipxg_set_walk_threads(ipxg_engine* e, uint32_t threads) {
    return guarded(e, [&] { return set_walk_threads_impl(e, threads); });
}
int ipxg_add_plugin(ipxg_engine* e, const ipxg_plugin* pl) { return guarded(e, [&] { return add_plugin_impl(e, pl); }); }
int ipxg_expire(ipxg_engine* e, int64_t now_sec) { return guarded(e, [&] { return expire_impl(e, now_sec); }); }
int ipxg_finish(ipxg_engine* e) { return guarded(e, [&] { return finish_impl(e); }); }
int ipxg_pending_exports(ipxg_engine* e, size_t* n) { return guarded(e, [&] { return pending_exports_impl(e, n); }); }
int ipxg_poll_exports(ipxg_engine* e, ipxg_flow_record* out, size_t cap, size_t* n) {
    return guarded(e, [&] { return poll_exports_impl(e, out, cap, n); });
}
int ipxg_clear_exports(ipxg_engine* e) { return guarded(e, [&] { return clear_exports_impl(e); }); }

}  // extern "C"
