// IPFIX export formatting on the device: the data records of the
// reference IPFIX output plugin's basic templates, BASIC_TMPLT_V4 / BASIC_TMPLT_V6
// (include/ipfixprobe/ipfix-elements.hpp:328-366), filled exactly as
// IPFIXExporter::fill_basic_flow (src/plugins/output/ipfix/src/ipfix.cpp:1470-1516) with
// IPFIX_FILL_FIELD (ipfix.cpp:77-96): 1-byte fields copied, 2-byte fields htons, the IPv4
// addresses copied in network order, other 4-byte fields htonl, 8-byte fields byte-swapped,
// everything else (IPv6 addresses, MACs) copied.  Times are 64-bit NTP (MK_NTP_TS,
// ipfix-elements.hpp:50-60); INPUT_INTERFACE is the exporter's dir_bit_field.
//
// Records are written back to back in export order (81 B for ip_version 4, 105 B otherwise:
// the v6 template, as get_template picks it, ipfix.cpp:287-291).  Three kernels: per-block
// byte totals, one exclusive scan over the blocks, then each block stages its records in
// LDS and writes its byte range with consecutive lanes on consecutive bytes.
#include <algorithm>

#include "ipxg_kernels.hpp"

namespace ipxg {

constexpr uint32_t IPFIX_BLOCK = 256;
constexpr uint32_t IPFIX_V4_LEN = 81, IPFIX_V6_LEN = 105;
constexpr uint64_t NTP_EPOCH_DIFF = 2208988800ULL;  // ipfix-elements.hpp:50

__device__ __forceinline__ uint32_t ipfix_len(const ipxg_flow_record& r) {
    return r.ip_version == 4 ? IPFIX_V4_LEN : IPFIX_V6_LEN;
}

__device__ __forceinline__ uint64_t ntp_ts(uint32_t sec, uint32_t usec) {  // MK_NTP_TS
    return (((uint64_t)sec + NTP_EPOCH_DIFF) << 32) | (uint32_t)(((uint64_t)usec << 32) / 1000000u);
}

__device__ __forceinline__ void put_be(uint8_t* p, uint64_t v, int n) {
    for (int k = 0; k < n; ++k) p[k] = (uint8_t)(v >> (8 * (n - 1 - k)));
}

// A record as its 32 words in registers (8 x 16-byte loads): a byte field read through
// ipxg_flow_record's byte members went to memory (global byte loads, or a scratch copy of the
// struct), one load per byte.
struct RecWords {
    uint32_t w[32];
};
__device__ __forceinline__ RecWords load_words(const ipxg_flow_record* r) {
    RecWords x;
    const uint4* q = reinterpret_cast<const uint4*>(r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint4 v = q[k];
        x.w[4 * k] = v.x;
        x.w[4 * k + 1] = v.y;
        x.w[4 * k + 2] = v.z;
        x.w[4 * k + 3] = v.w;
    }
    return x;
}
// byte o / little-endian u16, u32, u64 at byte o of the record (o a compile-time constant)
__device__ __forceinline__ uint32_t rb8(const RecWords& r, int o) { return (r.w[o >> 2] >> (8 * (o & 3))) & 0xFFu; }
__device__ __forceinline__ uint32_t rb16(const RecWords& r, int o) { return rb8(r, o) | (rb8(r, o + 1) << 8); }
__device__ __forceinline__ uint64_t rb64(const RecWords& r, int o) {  // (o a multiple of 4)
    return (uint64_t)r.w[o >> 2] | ((uint64_t)r.w[(o >> 2) + 1] << 32);
}
// offsets in ipxg_flow_record (include/ipxg.h)
enum : int {
    RO_TFS = 8, RO_TFU = 12, RO_TLS = 16, RO_TLU = 20, RO_SBYTES = 24, RO_DBYTES = 32, RO_SPK = 40, RO_DPK = 44,
    RO_SFLAGS = 48, RO_DFLAGS = 49, RO_IPVER = 50, RO_PROTO = 51, RO_SPORT = 52, RO_DPORT = 54, RO_SIP = 56,
    RO_DIP = 72, RO_SMAC = 88, RO_DMAC = 94, RO_END = 102
};
static_assert(offsetof(ipxg_flow_record, src_ip) == RO_SIP && offsetof(ipxg_flow_record, end_reason) == RO_END &&
                  offsetof(ipxg_flow_record, src_mac) == RO_SMAC && offsetof(ipxg_flow_record, src_port) == RO_SPORT,
              "ipxg_flow_record layout");

// one record's basic-template bytes at p (fill_basic_flow's field order)
__device__ __forceinline__ void fill_basic(uint8_t* p, const RecWords& r, uint32_t dir) {
    p[0] = (uint8_t)rb8(r, RO_END);                                          // FLOW_END_REASON   (0, 136, 1)
    put_be(p + 1, rb64(r, RO_SBYTES), 8);                                    // BYTES             (0, 1, 8)
    put_be(p + 9, rb64(r, RO_DBYTES), 8);                                    // BYTES_REV         (29305, 1, 8)
    put_be(p + 17, (uint64_t)r.w[RO_SPK >> 2], 8);                           // PACKETS           (0, 2, 8)
    put_be(p + 25, (uint64_t)r.w[RO_DPK >> 2], 8);                           // PACKETS_REV       (29305, 2, 8)
    put_be(p + 33, ntp_ts(r.w[RO_TFS >> 2], r.w[RO_TFU >> 2]), 8);           // FLOW_START_USEC   (0, 154, 8)
    put_be(p + 41, ntp_ts(r.w[RO_TLS >> 2], r.w[RO_TLU >> 2]), 8);           // FLOW_END_USEC     (0, 155, 8)
    const uint32_t ver = rb8(r, RO_IPVER);
    p[49] = (uint8_t)ver;                                                    // L3_PROTO          (0, 60, 1)
    p[50] = (uint8_t)rb8(r, RO_PROTO);                                       // L4_PROTO          (0, 4, 1)
    p[51] = (uint8_t)rb8(r, RO_SFLAGS);                                      // L4_TCP_FLAGS      (0, 6, 1)
    p[52] = (uint8_t)rb8(r, RO_DFLAGS);                                      // L4_TCP_FLAGS_REV  (29305, 6, 1)
    put_be(p + 53, rb16(r, RO_SPORT), 2);                                    // L4_PORT_SRC       (0, 7, 2)
    put_be(p + 55, rb16(r, RO_DPORT), 2);                                    // L4_PORT_DST       (0, 11, 2)
    put_be(p + 57, dir, 4);                                                  // INPUT_INTERFACE   (0, 10, 4)
    // L3_IPV4/6_ADDR_SRC/DST as stored, then L2_SRC_MAC (0, 56, 6), L2_DST_MAC (0, 80, 6)
    if (ver == 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            p[61 + k] = (uint8_t)rb8(r, RO_SIP + k);
            p[65 + k] = (uint8_t)rb8(r, RO_DIP + k);
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            p[69 + k] = (uint8_t)rb8(r, RO_SMAC + k);
            p[75 + k] = (uint8_t)rb8(r, RO_DMAC + k);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            p[61 + k] = (uint8_t)rb8(r, RO_SIP + k);
            p[77 + k] = (uint8_t)rb8(r, RO_DIP + k);
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            p[93 + k] = (uint8_t)rb8(r, RO_SMAC + k);
            p[99 + k] = (uint8_t)rb8(r, RO_DMAC + k);
        }
    }
}

__global__ __launch_bounds__(IPFIX_BLOCK) void k_ipfix_sizes(const ipxg_flow_record* rec, uint32_t n,
                                                             uint64_t* block_tot) {
    __shared__ uint32_t part[IPFIX_BLOCK / 64];
    const uint32_t i = blockIdx.x * IPFIX_BLOCK + threadIdx.x;
    uint32_t v = i < n ? (rec[i].ip_version == 4 ? IPFIX_V4_LEN : IPFIX_V6_LEN) : 0;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < IPFIX_BLOCK / 64; ++w) t += part[w];
        block_tot[blockIdx.x] = t;
    }
}

// exclusive scan of nb block totals in place (one workgroup); total at block_tot[nb]
__global__ __launch_bounds__(1024) void k_ipfix_scan(uint64_t* block_tot, uint32_t nb) {
    __shared__ uint64_t part[1024];
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t b0 = threadIdx.x * per;
    uint64_t s = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (b0 + k < nb) s += block_tot[b0 + k];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele over the 1024 sums
        const uint64_t x = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
    }
    uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint32_t k = 0; k < per; ++k) {
        if (b0 + k < nb) {
            const uint64_t t = block_tot[b0 + k];
            block_tot[b0 + k] = run;
            run += t;
        }
    }
    if (threadIdx.x == 1023) block_tot[nb] = part[1023];
}

__global__ __launch_bounds__(IPFIX_BLOCK) void k_ipfix_fill(const ipxg_flow_record* rec, uint32_t n, uint32_t dir,
                                                            const uint64_t* block_base, uint8_t* out,
                                                            uint64_t* offsets) {
    __shared__ uint8_t stage[IPFIX_BLOCK * IPFIX_V6_LEN];  // 26.25 KiB
    __shared__ uint32_t wsum[IPFIX_BLOCK / 64];
    const uint32_t i = blockIdx.x * IPFIX_BLOCK + threadIdx.x;
    RecWords r = {};
    uint32_t len = 0;
    if (i < n) {
        r = load_words(rec + i);
        len = rb8(r, RO_IPVER) == 4 ? IPFIX_V4_LEN : IPFIX_V6_LEN;
    }
    // block exclusive scan of the record lengths
    uint32_t x = len;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (uint32_t k = 0; k < IPFIX_BLOCK / 64; ++k) {
        if (k < w) wbase += wsum[k];
        total += wsum[k];
    }
    const uint32_t local = wbase + x - len;
    const uint64_t base = block_base[blockIdx.x];
    if (i < n) {
        fill_basic(stage + local, r, dir);
        offsets[i] = base + local;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) offsets[n] = block_base[gridDim.x];
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < total; k += IPFIX_BLOCK) out[base + k] = stage[k];
}

// ---- messages (ipxg_device_ipfix_messages): the exporter's message stream ----------------
// Records feed the exporter v4-first (stable): a record's place is its rank among the records
// of its template (class 0 = IPv4 template, 1 = IPv6).  The host plans the messages from the
// two counts (IpfixSet / IpfixMsg below, a restatement of IPFIXExporter's buffer logic at the
// granularity of whole data sets) and these kernels write every byte on the device.

// per block: records of class 1 (IPv6 template)
__global__ __launch_bounds__(IPFIX_BLOCK) void k_ipfix_count6(const ipxg_flow_record* rec, uint32_t n,
                                                              uint64_t* block_tot) {
    __shared__ uint32_t part[IPFIX_BLOCK / 64];
    const uint32_t i = blockIdx.x * IPFIX_BLOCK + threadIdx.x;
    const uint64_t m = __ballot(i < n && rec[i].ip_version == 6);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < IPFIX_BLOCK / 64; ++w) t += part[w];
        block_tot[blockIdx.x] = t;
    }
}

// one record per lane: its rank in its class -> its data set (binary search over the class's
// sets, in rank order) -> its destination; the record's bytes are staged in LDS by its lane, then
// each wave writes its 64 records one after the other with consecutive lanes on consecutive
// bytes (written straight from the lanes, 64 records 81 bytes apart per store: 186 us for 100k
// records, the whole step's kernels took 340)
__global__ __launch_bounds__(IPFIX_BLOCK) void k_ipfix_msg_fill(const ipxg_flow_record* rec, uint32_t n, uint32_t dir,
                                                                const uint64_t* block_pre6, const IpfixSet* sets,
                                                                uint32_t nsets4, uint32_t nsets6, uint8_t* out) {
    __shared__ uint8_t stage[IPFIX_BLOCK * IPFIX_V6_LEN];  // 26.25 KiB: record slot k at k * 105
    __shared__ uint32_t wcnt[IPFIX_BLOCK / 64];
    const uint32_t i = blockIdx.x * IPFIX_BLOCK + threadIdx.x;
    const bool act = i < n;
    RecWords r = {};
    if (act) r = load_words(rec + i);
    const bool v6 = act && rb8(r, RO_IPVER) == 6;
    const uint64_t m = __ballot(v6);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t below6 = (uint32_t)__popcll(lane ? (m & (~0ull >> (64 - lane))) : 0ull);
    for (uint32_t k = 0; k < w; ++k) below6 += wcnt[k];
    uint64_t dst = 0;
    uint32_t len = 0;
    if (act) {
        const uint64_t pre6 = block_pre6[blockIdx.x] + below6;             // IPv6 records before i
        const uint64_t ord = v6 ? pre6 : (uint64_t)i - pre6;                // rank in the class
        const IpfixSet* s = v6 ? sets + nsets4 : sets;
        uint32_t lo = 0, hi = v6 ? nsets6 : nsets4;                        // last set with ord0 <= ord
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s[mid].ord0 <= ord) lo = mid;
            else hi = mid;
        }
        len = v6 ? IPFIX_V6_LEN : IPFIX_V4_LEN;
        dst = s[lo].off + 4 + (ord - s[lo].ord0) * len;
        fill_basic(stage + threadIdx.x * IPFIX_V6_LEN, r, dir);
    }
    __syncthreads();
    const uint32_t nw = min(64u, n - min(n, blockIdx.x * IPFIX_BLOCK + w * 64));  // the wave's records
    for (uint32_t j = 0; j < nw; ++j) {  // (wave-uniform)
        const uint64_t dj = __shfl(dst, (int)j);
        const uint32_t lj = __shfl(len, (int)j);
        const uint8_t* src = stage + (w * 64 + j) * IPFIX_V6_LEN;
        for (uint32_t k = lane; k < lj; k += 64) out[dj + k] = src[k];
    }
}

// message headers (fill_ipfix_header) and data set headers (template id, length)
__global__ __launch_bounds__(256) void k_ipfix_msg_headers(const IpfixMsg* msgs, uint32_t nmsgs, const IpfixSet* sets,
                                                           uint32_t nsets, uint32_t odid, uint32_t export_time,
                                                           uint8_t* out) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j < nmsgs) {
        uint8_t* p = out + msgs[j].off;
        put_be(p, 10, 2);
        put_be(p + 2, msgs[j].len, 2);
        put_be(p + 4, export_time, 4);
        put_be(p + 8, msgs[j].seq, 4);
        put_be(p + 12, odid, 4);
    }
    if (j < nsets) {
        const IpfixSet& s = sets[j];
        uint8_t* p = out + s.off;
        put_be(p, s.cls ? 259 : 258, 2);
        put_be(p + 2, 4 + s.count * (s.cls ? IPFIX_V6_LEN : IPFIX_V4_LEN), 2);
    }
}

void launch_ipfix_count6(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint64_t* block_tot) {
    const uint32_t nb = (n + IPFIX_BLOCK - 1) / IPFIX_BLOCK;
    hipLaunchKernelGGL(k_ipfix_count6, dim3(nb), dim3(IPFIX_BLOCK), 0, st, rec, n, block_tot);
    hipLaunchKernelGGL(k_ipfix_scan, dim3(1), dim3(1024), 0, st, block_tot, nb);
}

void launch_ipfix_messages(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint32_t dir,
                           const uint64_t* block_pre6, const IpfixSet* sets, uint32_t nsets4, uint32_t nsets6,
                           const IpfixMsg* msgs, uint32_t nmsgs, uint32_t odid, uint32_t export_time, uint8_t* out) {
    if (n) {
        const uint32_t nb = (n + IPFIX_BLOCK - 1) / IPFIX_BLOCK;
        hipLaunchKernelGGL(k_ipfix_msg_fill, dim3(nb), dim3(IPFIX_BLOCK), 0, st, rec, n, dir, block_pre6, sets, nsets4,
                           nsets6, out);
    }
    const uint32_t nh = std::max(nmsgs, nsets4 + nsets6);
    if (nh)
        hipLaunchKernelGGL(k_ipfix_msg_headers, dim3((nh + 255) / 256), dim3(256), 0, st, msgs, nmsgs, sets,
                           nsets4 + nsets6, odid, export_time, out);
}

void launch_ipfix_basic(hipStream_t st, const ipxg_flow_record* rec, uint32_t n, uint32_t dir, uint64_t* block_tot,
                        uint8_t* out, uint64_t* offsets) {
    const uint32_t nb = (n + IPFIX_BLOCK - 1) / IPFIX_BLOCK;
    hipLaunchKernelGGL(k_ipfix_sizes, dim3(nb), dim3(IPFIX_BLOCK), 0, st, rec, n, block_tot);
    hipLaunchKernelGGL(k_ipfix_scan, dim3(1), dim3(1024), 0, st, block_tot, nb);
    hipLaunchKernelGGL(k_ipfix_fill, dim3(nb), dim3(IPFIX_BLOCK), 0, st, rec, n, dir, block_tot, out, offsets);
}

}  // namespace ipxg
