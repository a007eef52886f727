// Read-bandwidth microbenchmark for k_bin's access pattern on one MI355X:
//   contig : each wave reads consecutive 16-byte chunks (a float4 stream)
//   frame  : lane = packet; a 16-byte descriptor, then the frame's first 48 bytes at the
//            descriptor's offset (3 x 16-byte loads, dependent on the descriptor)
//   frame_nodesc : the same 48 bytes at i * stride, no descriptor
//   frame_lds : the descriptors, then -- when a wave's 64 frames sit back to back at 64-byte
//            stride (a ballot over the offsets) -- the wave's 4 KB read as 4 contiguous 1 KB
//            loads (lane = 16 bytes) and transposed through the wave's LDS (frames at an 80-byte
//            pitch: conflict-free 16-byte reads), each lane then holding its frame's 48 bytes
// Usage: membench <n_packets> <stride> <blocks> [<LDS KiB per block of the k_tiles runs>]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Desc { uint32_t off, len, s, us; };

__global__ __launch_bounds__(256) void k_contig(const uint4* __restrict__ a, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t base = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; base < n16; base += stride) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = base + k * 256 < n16 ? a[base + k * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// U packets per lane per iteration (all U descriptors, then all 3U head loads in flight)
template <bool DESC, int U = 4, int C = 3>
__global__ __launch_bounds__(256) void k_frame(const uint8_t* __restrict__ arena, const Desc* __restrict__ desc,
                                               uint32_t n, uint32_t fstride, uint32_t* out) {
    uint32_t acc = 0;
    const uint32_t step = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += step * U) {
        uint32_t off[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t i = min(i0 + k * 256, n - 1);
            if (DESC) { const Desc d = desc[i]; off[k] = d.off; acc ^= d.len ^ d.s; }
            else off[k] = i * fstride;
        }
        uint4 h[U][C];
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int c = 0; c < C; ++c) h[k][c] = *reinterpret_cast<const uint4*>(arena + off[k] + 16 * c);
#pragma unroll
        for (int k = 0; k < U; ++k)
#pragma unroll
            for (int c = 0; c < C; ++c) acc ^= h[k][c].x ^ h[k][c].y ^ h[k][c].z ^ h[k][c].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// k_bin's load pattern in its persistent form: tiles of 8 steps x 256 packets, tile t on block
// t % grid; per step the descriptor DA steps ahead and the 48-byte head HA steps ahead (rings in
// registers, buffer loads with `aux`), consumed by an XOR.  LDS `lds_kb` KiB per block (occupancy).
typedef uint32_t mb_u32x4 __attribute__((ext_vector_type(4)));
// W: each tile also stores its 2048 16-byte records (k_bin's record volume): W = 1 sequentially
// (coalesced 1 KB per wave store), W = 2 in 8-record runs spread over 256 partition columns of
// per-block segments (k_bin's layout); store_nt: non-temporal stores
template <int DA, int HA, int W = 0>
__global__ __launch_bounds__(256) void k_tiles(const uint8_t* __restrict__ arena, const Desc* __restrict__ desc,
                                               uint32_t n, uint32_t aux_nt, uint32_t* out, uint4* rec = nullptr,
                                               uint32_t store_nt = 0, uint32_t seg_cap = 0) {
    extern __shared__ uint32_t lds[];
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<Desc*>(desc), 0, (int)(n * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(arena), 0, (int)(n * 64u), 0x00020000);
    const uint32_t tid = threadIdx.x, ntiles = (n + 2047) / 2048;
    uint32_t acc = 0;
    mb_u32x4 Dr[DA];
    mb_u32x4 Hr[HA][3];
    auto ld = [&](uint32_t i) { return __builtin_amdgcn_raw_buffer_load_b128(rd, i < n ? i * 16u : 0xFFFFFF00u, 0, 2); };
    auto lh = [&](const mb_u32x4 d, int c) {
        return aux_nt ? __builtin_amdgcn_raw_buffer_load_b128(ra, d.y ? d.x + 16u * c : 0xFFFFFF00u, 0, 2)
                      : __builtin_amdgcn_raw_buffer_load_b128(ra, d.y ? d.x + 16u * c : 0xFFFFFF00u, 0, 0);
    };
#pragma unroll
    for (int k = 0; k < DA; ++k) Dr[k] = ld(blockIdx.x * 2048 + k * 256 + tid);
#pragma unroll
    for (int h = 0; h < HA; ++h)
#pragma unroll
        for (int c = 0; c < 3; ++c) Hr[h][c] = lh(Dr[h], c);
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint32_t tile = t * 2048, next = (t + gridDim.x) * 2048;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const mb_u32x4 h0 = Hr[j % HA][0], h1 = Hr[j % HA][1], h2 = Hr[j % HA][2];
            const uint32_t ia = j + DA < 8 ? tile + (j + DA) * 256 + tid : next + (j + DA - 8) * 256 + tid;
            const mb_u32x4 dh = Dr[(j + HA) % DA];
#pragma unroll
            for (int c = 0; c < 3; ++c) Hr[j % HA][c] = lh(dh, c);
            Dr[j % DA] = ld(ia);
            acc ^= h0.x ^ h0.y ^ h1.z ^ h2.w;
        }
        if (W) {
            const uint32_t k0 = (t - blockIdx.x) / gridDim.x;  // the block's tile number
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint32_t r = q * 256 + tid;  // record r of the tile
                size_t dst;
                if (W == 1) dst = (size_t)tile + r;
                else if (W == 2) dst = ((size_t)(r >> 3) * gridDim.x + blockIdx.x) * seg_cap + k0 * 8 + (r & 7);  // partition r/8
                else  // W = 3/4/5: the same 8-record runs, each segment starting 5/4/2 records into a line (runs span 2 lines)
                    dst = ((size_t)(r >> 3) * gridDim.x + blockIdx.x) * seg_cap + (W == 3 ? 5 : W == 4 ? 4 : 2) + k0 * 8 + (r & 7);
                const uint4 v = make_uint4(acc, r, t, q);
                if (store_nt) {
                    __builtin_nontemporal_store(v.x, &rec[dst].x);
                    __builtin_nontemporal_store(v.y, &rec[dst].y);
                    __builtin_nontemporal_store(v.z, &rec[dst].z);
                    __builtin_nontemporal_store(v.w, &rec[dst].w);
                } else {
                    rec[dst] = v;
                }
            }
        }
        if (lds[0] == 0xDEADBEEF) __syncthreads();  // (never: keeps the LDS allocation)
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_frame_lds(const uint8_t* __restrict__ arena, const Desc* __restrict__ desc,
                                                   uint32_t n, uint32_t* out) {
    __shared__ uint4 xs[4][64 * 5];  // per wave: 64 frames x 80 bytes
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 256;
    for (uint32_t i0 = blockIdx.x * 256 * 4 + threadIdx.x; i0 < n; i0 += step * 4) {
        uint32_t off[4];
        bool seq[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = min(i0 + k * 256, n - 1);
            const Desc d = desc[i];
            off[k] = d.off;
            acc ^= d.len ^ d.s;
            const uint32_t o0 = __builtin_amdgcn_readfirstlane(d.off);
            seq[k] = __all(d.off == o0 + 64u * lane);
        }
        uint4 h[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t o0 = __builtin_amdgcn_readfirstlane(off[k]);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t a = seq[k] ? o0 + 1024u * c + 16u * lane : (c < 3 ? off[k] + 16u * c : off[k]);
                h[k][c] = *reinterpret_cast<const uint4*>(arena + a);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (seq[k]) {  // chunk (lane & 3) of frame 16c + lane / 4 -> the frame's 80-byte slot
#pragma unroll
                for (int c = 0; c < 4; ++c) xs[w][(16 * c + lane / 4) * 5 + (lane & 3)] = h[k][c];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own LDS stores
#pragma unroll
                for (int c = 0; c < 3; ++c) h[k][c] = xs[w][lane * 5 + c];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) acc ^= h[k][c].x ^ h[k][c].y ^ h[k][c].z ^ h[k][c].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// read back n16 16-byte words (the records a k_tiles<., ., 2> run wrote): k_reduce's input
__global__ __launch_bounds__(256) void k_readback(const uint4* __restrict__ a, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t base = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; base < n16; base += stride) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = base + k * 256 < n16 ? a[base + k * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 10000000;
    const uint32_t fs = argc > 2 ? atoi(argv[2]) : 64;
    const int blocks = argc > 3 ? atoi(argv[3]) : 2048;
    const size_t abytes = (size_t)n * fs + 64;
    uint8_t* arena; Desc* desc; uint32_t* out;
    CHK(hipMalloc(&arena, abytes));
    CHK(hipMalloc(&desc, (size_t)n * sizeof(Desc)));
    CHK(hipMalloc(&out, 16));
    CHK(hipMemset(arena, 1, abytes));
    std::vector<Desc> hd(n);
    for (uint32_t i = 0; i < n; ++i) hd[i] = Desc{i * fs, 64, i, 0};
    CHK(hipMemcpy(desc, hd.data(), (size_t)n * sizeof(Desc), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    auto run = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CHK(hipDeviceSynchronize());
        const int reps = 20;
        CHK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-14s blocks %5d  %8.1f us  %7.0f GB/s (%.0f MB)\n", name, blocks, ms * 1e3, bytes / (ms * 1e-3) / 1e9, bytes / 1e6);
    };
    const size_t n16 = (size_t)n * fs / 16;
    run("contig", (double)n16 * 16, [&] { hipLaunchKernelGGL(k_contig, dim3(blocks), dim3(256), 0, 0, (const uint4*)arena, n16, out); });
    run("frame", (double)n * (48 + 16), [&] { hipLaunchKernelGGL(k_frame<true>, dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    run("frame_nodesc", (double)n * 48, [&] { hipLaunchKernelGGL(k_frame<false>, dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    run("frame_lds", (double)n * (64 + 16), [&] { hipLaunchKernelGGL(k_frame_lds, dim3(blocks), dim3(256), 0, 0, arena, desc, n, out); });
    run("frame_u1", (double)n * (64 + 16), [&] { hipLaunchKernelGGL((k_frame<true, 1>), dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    run("frame_u2", (double)n * (64 + 16), [&] { hipLaunchKernelGGL((k_frame<true, 2>), dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    // the wide walk's 80-byte heads (5 x 16 B) at the frame stride, 4 / 8 packets per lane in flight
    run("frame80_u4", (double)n * (80 + 16), [&] { hipLaunchKernelGGL((k_frame<true, 4, 5>), dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    run("frame80_u8", (double)n * (80 + 16), [&] { hipLaunchKernelGGL((k_frame<true, 8, 5>), dim3(blocks), dim3(256), 0, 0, arena, desc, n, fs, out); });
    if (fs != 64) return 0;  // (the k_tiles runs below assume 64-byte frames)
    const uint32_t lds_kb = argc > 4 ? atoi(argv[4]) : 0;
    if (lds_kb) CHK(hipFuncSetAttribute((const void*)k_tiles<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024));
    if (lds_kb) CHK(hipFuncSetAttribute((const void*)k_tiles<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024));
    if (lds_kb) CHK(hipFuncSetAttribute((const void*)k_tiles<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024));
    const size_t lb = (size_t)(lds_kb ? lds_kb : 1) * 1024;
    uint4* recb;
    const uint32_t seg_cap = ((n + 2047) / 2048 + blocks - 1) / blocks * 8 + 16;
    CHK(hipMalloc(&recb, (size_t)256 * blocks * seg_cap * 16 + (size_t)n * 16));
    if (lds_kb)
        for (const void* f : {(const void*)k_tiles<4, 1, 1>, (const void*)k_tiles<4, 1, 2>, (const void*)k_tiles<4, 1, 3>, (const void*)k_tiles<4, 1, 4>, (const void*)k_tiles<4, 1, 5>})
            CHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kb * 1024));
    for (uint32_t nt : {1u, 0u})
        for (uint32_t snt : {0u, 1u}) {
            char nm[48];
            snprintf(nm, sizeof nm, "w1_%s_st%s", nt ? "nt" : "def", snt ? "nt" : "def");
            run(nm, (double)n * (64 + 16 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1, 1>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, snt, seg_cap); });
            snprintf(nm, sizeof nm, "w2_%s_st%s", nt ? "nt" : "def", snt ? "nt" : "def");
            run(nm, (double)n * (64 + 16 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1, 2>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, snt, seg_cap); });
            snprintf(nm, sizeof nm, "w3_%s_st%s", nt ? "nt" : "def", snt ? "nt" : "def");
            run(nm, (double)n * (64 + 16 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1, 3>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, snt, seg_cap); });
            snprintf(nm, sizeof nm, "w4_%s_st%s", nt ? "nt" : "def", snt ? "nt" : "def");
            run(nm, (double)n * (64 + 16 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1, 4>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, snt, seg_cap); });
            snprintf(nm, sizeof nm, "w5_%s_st%s", nt ? "nt" : "def", snt ? "nt" : "def");
            run(nm, (double)n * (64 + 16 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1, 5>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, snt, seg_cap); });
        }
    // the record round trip: k_tiles<4, 1, 2> (k_bin's loads + its segment stores), then the
    // records read back (timed alone) -- warm (right after) vs cold (after 1.6 GB of other reads)
    {
        const size_t rec16 = (size_t)256 * blocks * seg_cap;
        uint8_t* big;
        const size_t bigb = (size_t)1600 << 20;
        CHK(hipMalloc(&big, bigb));
        CHK(hipMemset(big, 2, bigb));
        for (uint32_t nt : {1u, 0u})
            for (int cold = 0; cold < 2; ++cold) {
                float tot = 0;
                const int reps = 10;
                for (int r = 0; r < reps; ++r) {
                    hipLaunchKernelGGL((k_tiles<4, 1, 2>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out, recb, 0u, seg_cap);
                    if (cold) hipLaunchKernelGGL(k_contig, dim3(blocks), dim3(256), 0, 0, (const uint4*)big, bigb / 16, out);
                    CHK(hipEventRecord(e0));
                    hipLaunchKernelGGL(k_readback, dim3(blocks), dim3(256), 0, 0, (const uint4*)recb, rec16, out);
                    CHK(hipEventRecord(e1));
                    CHK(hipEventSynchronize(e1));
                    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 2) tot += ms;
                }
                const double ms = tot / (reps - 2);
                printf("readback_%s_%s blocks %5d  %8.1f us  %7.0f GB/s (%.0f MB)\n", nt ? "nt" : "def", cold ? "cold" : "warm",
                       blocks, ms * 1e3, rec16 * 16 / (ms * 1e-3) / 1e9, rec16 * 16 / 1e6);
            }
        CHK(hipFree(big));
    }
    for (uint32_t nt : {1u, 0u}) {
        char nm[32];
        snprintf(nm, sizeof nm, "tiles41_%s", nt ? "nt" : "def");
        run(nm, (double)n * (64 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 1>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out); });
        snprintf(nm, sizeof nm, "tiles42_%s", nt ? "nt" : "def");
        run(nm, (double)n * (64 + 16), [&] { hipLaunchKernelGGL((k_tiles<4, 2>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out); });
        snprintf(nm, sizeof nm, "tiles84_%s", nt ? "nt" : "def");
        run(nm, (double)n * (64 + 16), [&] { hipLaunchKernelGGL((k_tiles<8, 4>), dim3(blocks), dim3(256), lb, 0, arena, desc, n, nt, out); });
    }
    return 0;
}
