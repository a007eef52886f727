// ipxg_synth.hip -- device generator of the synthetic packet mixes named by BASELINE.json
// (bench and test infrastructure; not part of the engine).
//
// A mix is a set of frame layouts (header bytes built on the host by tests/synth.py's
// builders, with the offsets of the per-flow and per-packet fields) and a flow table (one
// layout, addresses, ports and VLAN per flow).  Per packet, from a counter-based RNG keyed by
// (seed, global packet index):
//   k_synth_plan   flow (Zipf by CDF binary search, or uniform), direction, frame length (the
//                  layout's size mode: IMIX 64/594/1518 at 7:4:1, QUIC long header for the
//                  flows being opened / short header), TCP flags;
//   (host)         frame offsets = exclusive prefix sum of the lengths rounded up to 64 B
//                  (frames start on a cache line, as in a DPDK mbuf pool);
//   k_synth_write  each workgroup builds 64 frames' headers in LDS (template + addresses,
//                  ports, MACs, VLAN, length fields, flags) and writes the frames (payload zero)
//                  and their 16-byte descriptors with coalesced 16-byte stores.
// Timestamps are t0 + index * dt at nanosecond resolution, truncated to microseconds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SYNTH_TMPL 192

struct SynthLayout {              // 256 bytes
    uint8_t tmpl[SYNTH_TMPL];     // header bytes (+ an L7 prefix)
    uint16_t hdr_len;             // template bytes used
    uint16_t addr_len;            // 4 (IPv4) or 16 (IPv6)
    uint16_t sip_off, dip_off;    // flow-key addresses (the innermost IP header)
    uint16_t sport_off, dport_off;
    uint16_t tcp_flags_off;       // 0: not TCP
    uint16_t vlan_off;            // TCI of the outer VLAN tag (0: none)
    uint16_t patch_off[4];        // 16-bit big-endian length fields = frame_len - patch_bias
    uint16_t patch_bias[4];       // (patch_off 0 = unused)
    uint16_t size_mode;           // 0 IMIX 64/594/1518 7:4:1, 1 QUIC, 2 fixed 64 B
    uint16_t l7_off;              // QUIC: first byte of the QUIC header
    uint16_t min_len;             // shortest frame (>= hdr_len)
    uint16_t alt_len;             // bytes of alt[] written at l7_off in packets of established flows
    uint8_t alt[8];               //   (the protocol's later messages: TLS application data, HTTP body)
    uint16_t blob_len;            // QUIC: the opening flows' long-header packets carry the mix's blob
                                  // (a complete client Initial datagram) at l7_off, blob_len bytes
    uint16_t pad[7];
};
static_assert(sizeof(SynthLayout) == 256, "layout record");

struct SynthFlow {                // 48 bytes
    uint8_t sip[16], dip[16];
    uint16_t sport, dport, layout, vlan;
    uint32_t mac_id;
    uint32_t opening;             // 1: a connection being opened (its packets carry the protocol's
                                  // first message / QUIC long headers); 0: established
};
static_assert(sizeof(SynthFlow) == 48, "flow record");

struct SynthParams {
    const SynthLayout* layouts;
    const SynthFlow* flows;
    const uint64_t* cdf;          // nflows cumulative weights (last = 2^64 - 1); null = uniform
    const uint32_t* rank_flow;    // rank -> flow id (null = identity)
    uint64_t seed;
    uint64_t first_idx;           // global index of the batch's first packet
    uint64_t t0_ns;
    uint32_t nflows, n;
    uint32_t dt_ns;
    uint32_t fwd_q16;             // P(forward direction) * 65536
    uint32_t syn_q16, psh_q16;    // TCP: P(SYN), P(PSH|ACK) * 65536 (else ACK)
    const uint8_t* blob;          // the layouts' blob (blob_len bytes), or null
    uint32_t oshift;              // 4: descriptor offsets in 16-byte units (IPXG_BATCH_OFFSET16), else 0
};

__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// plan[i] = {flow, len | dir << 16 | long_hdr << 17, flags, 0}
__global__ __launch_bounds__(256) void k_synth_plan(SynthParams P, uint4* plan, uint64_t* alen) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= P.n) return;
    const uint64_t g = P.first_idx + i;
    const uint64_t r0 = mix64(P.seed ^ (g * 0xD1B54A32D192ED03ull));
    const uint64_t r1 = mix64(r0 ^ 0x5851F42D4C957F2Dull);
    uint32_t f;
    if (P.cdf) {  // first rank whose cumulative weight exceeds the draw
        uint32_t lo = 0, hi = P.nflows - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (P.cdf[mid] > r0) hi = mid;
            else lo = mid + 1;
        }
        f = lo;
    } else {
        f = (uint32_t)(((r0 >> 32) * (uint64_t)P.nflows) >> 32);
    }
    if (P.rank_flow) f = P.rank_flow[f];
    const SynthLayout& L = P.layouts[P.flows[f].layout];
    const uint32_t u = (uint32_t)(r1 & 0xFFFF);
    const uint32_t dir = ((r1 >> 16) & 0xFFFF) < P.fwd_q16 ? 0u : 1u;
    uint32_t len, lng = 0;
    const uint32_t s12 = (uint32_t)(((r1 >> 32) & 0xFFFF) * 12u >> 16);
    if (L.size_mode == 0) {
        len = s12 < 7 ? 64u : (s12 < 11 ? 594u : 1518u);
    } else if (L.size_mode == 1) {  // QUIC: an opening flow's packets are long-header Initials
        lng = P.flows[f].opening ? 1u : 0u;  // (>= 1200 B datagrams), an established flow's short
                                             // header 1-RTT packets
        const uint32_t ini = L.blob_len > 1200u ? L.blob_len : 1200u;
        len = lng ? L.l7_off + ini : (s12 < 6 ? 80u : 1350u);
    } else {
        len = 64u;
    }
    if (len < L.min_len) len = L.min_len;
    uint32_t flags = 0;
    if (L.tcp_flags_off) flags = u < P.syn_q16 ? 0x02u : (u < P.syn_q16 + P.psh_q16 ? 0x18u : 0x10u);
    plan[i] = make_uint4(f, len | (dir << 16) | (lng << 17), flags, 0);
    alen[i] = (len + 63u) & ~63u;
}

__device__ __forceinline__ void put16(uint8_t* h, uint32_t off, uint32_t v) {
    h[off] = (uint8_t)(v >> 8);
    h[off + 1] = (uint8_t)v;
}

// One workgroup per 64 packets: thread t < 64 builds packet t's header in LDS, then the
// block writes the frames one after another (16 bytes per thread per store).
__global__ __launch_bounds__(256) void k_synth_write(SynthParams P, const uint4* plan, const uint64_t* off,
                                                     uint8_t* arena, uint4* desc) {
    __shared__ uint4 hdr[64][SYNTH_TMPL / 16];
    __shared__ uint32_t meta[64][5];  // offset / 16, len, hdr_len, blob start (l7_off), blob bytes (0: none)
    const uint32_t tid = threadIdx.x;
    const uint32_t base = blockIdx.x * 64u;
    if (tid < 64 && base + tid < P.n) {
        const uint32_t i = base + tid;
        const uint4 pl = plan[i];
        const SynthFlow& F = P.flows[pl.x];
        const SynthLayout& L = P.layouts[F.layout];
        const uint32_t len = pl.y & 0xFFFF, dir = (pl.y >> 16) & 1, lng = (pl.y >> 17) & 1;
        uint8_t* h = reinterpret_cast<uint8_t*>(&hdr[tid][0]);
        const uint4* t4 = reinterpret_cast<const uint4*>(L.tmpl);
        for (int c = 0; c < SYNTH_TMPL / 16; ++c) hdr[tid][c] = t4[c];
        const uint8_t* a = dir ? F.dip : F.sip;
        const uint8_t* b = dir ? F.sip : F.dip;
        for (uint32_t k = 0; k < L.addr_len; ++k) {
            h[L.sip_off + k] = a[k];
            h[L.dip_off + k] = b[k];
        }
        put16(h, L.sport_off, dir ? F.dport : F.sport);
        put16(h, L.dport_off, dir ? F.sport : F.dport);
        // MACs: client 02:00:<id>, server 04:00:<id>; dst first
        const uint32_t m = F.mac_id;
        const uint8_t cm[6] = {0x02, 0x00, (uint8_t)(m >> 24), (uint8_t)(m >> 16), (uint8_t)(m >> 8), (uint8_t)m};
        for (int k = 0; k < 6; ++k) {
            const uint8_t c = cm[k], s = k == 0 ? 0x04 : cm[k];
            h[k] = dir ? c : s;
            h[6 + k] = dir ? s : c;
        }
        if (L.vlan_off) {
            const uint32_t tci = (h[L.vlan_off] << 8 | h[L.vlan_off + 1]) & 0xF000u;
            put16(h, L.vlan_off, tci | (F.vlan & 0x0FFF));
        }
        for (int k = 0; k < 4; ++k)
            if (L.patch_off[k]) put16(h, L.patch_off[k], len - L.patch_bias[k]);
        if (L.tcp_flags_off) h[L.tcp_flags_off] = (uint8_t)pl.z;
        if (L.size_mode == 1 && !lng) h[L.l7_off] = 0x43;  // QUIC short header (1-RTT)
        if (!F.opening)
            for (uint32_t k = 0; k < L.alt_len; ++k) h[L.l7_off + k] = L.alt[k];
        meta[tid][0] = (uint32_t)(off[i] >> 4);  // (frames start on 64 bytes)
        meta[tid][1] = len;
        meta[tid][2] = L.hdr_len;
        meta[tid][3] = L.l7_off;
        meta[tid][4] = lng && P.blob ? L.blob_len : 0u;  // (an opening QUIC flow's Initial)
        const uint64_t t = P.t0_ns + (P.first_idx + i) * (uint64_t)P.dt_ns;
        const uint64_t us = t / 1000u;
        desc[i] = make_uint4((uint32_t)(off[i] >> P.oshift), len | (len << 16), (uint32_t)(us / 1000000u), (uint32_t)(us % 1000000u));
    }
    __syncthreads();
    const uint32_t np = min(64u, P.n - base);
    for (uint32_t q = 0; q < np; ++q) {
        const uint32_t o = meta[q][0], len = meta[q][1], hl = meta[q][2], b0 = meta[q][3], bl = meta[q][4];
        for (uint32_t c = tid; c * 16u < len; c += 256u) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (c * 16u < hl) v = hdr[q][c];
            if (bl && c * 16u + 16u > b0 && c * 16u < b0 + bl) {  // the blob over the template
                uint8_t* vb = reinterpret_cast<uint8_t*>(&v);
                for (uint32_t k = 0; k < 16; ++k) {
                    const uint32_t at = c * 16u + k;
                    if (at >= b0 && at < b0 + bl) vb[k] = P.blob[at - b0];
                }
            }
            *reinterpret_cast<uint4*>(arena + (uint64_t)o * 16u + c * 16u) = v;
        }
    }
}

extern "C" {

int synth_plan(const SynthParams* p, void* plan, void* alen, void* stream) {
    if (!p || p->n == 0) return 0;
    hipLaunchKernelGGL(k_synth_plan, dim3((p->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *p,
                       (uint4*)plan, (uint64_t*)alen);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int synth_write(const SynthParams* p, const void* plan, const void* off, void* arena, void* desc, void* stream) {
    if (!p || p->n == 0) return 0;
    hipLaunchKernelGGL(k_synth_write, dim3((p->n + 63) / 64), dim3(256), 0, (hipStream_t)stream, *p,
                       (const uint4*)plan, (const uint64_t*)off, (uint8_t*)arena, (uint4*)desc);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int synth_layout_size(void) { return (int)sizeof(SynthLayout); }
int synth_flow_size(void) { return (int)sizeof(SynthFlow); }

}  // extern "C"
