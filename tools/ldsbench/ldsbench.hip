// LDS throughput microbenchmark for the fold patterns of k_reduce / k_bin (one MI355X):
// 1024-thread workgroups, one per CU, a 112 KiB table of 2048 x 56-byte entries (k_reduce's
// FlowAgg table); every lane issues ITERS operations at pseudo-random entries.  Reports the
// shader cycles of workgroup 0 (s_memtime) and the LDS lane-operations per cycle per CU.
//   op 0  ds_read_b64, random entry (the probe's key read)
//   op 1  ds_add_u64 no-return, random entry (acc fold)
//   op 2  ds_max_u32 no-return, random entry (last1 fold)
//   op 3  ds_add_rtn_u32 on 256 counters, result used (k_bin's partition rank)
//   op 4  ds_write_b32, random entry
//   op 5  ds_add_u64 no-return, lane-private address (no conflicts)
//   op 6  ds_add_u32 no-return, lane-private consecutive words
//   op 7  ops 1+2+2 together (the full udp fold: add64 + 2 x max32), random entry
//   op 8  ds_max_u64 no-return, random entry
//   op 9  random entry, ds_read_b64 then ds_write_b64 (non-atomic RMW, racy; cost only)
//   op 10 ds_max_u32 no-return, lane-private consecutive words (atomic cost without conflicts)
//   op 11 ds_max_u32 no-return, random word of a 4-byte array (struct-of-arrays field)
//   op 12 ds_add_u64 no-return, random word of an 8-byte array (struct-of-arrays field)
//   op 13 ds_read_b32 random word of a 4-byte array
// Usage: ldsbench <op> <iters> <entries (<= 2048)>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int ENT = 2048, ESZ = 56;

template <int OP>
__global__ __launch_bounds__(1024) void k_lds(uint32_t iters, uint32_t nent, unsigned long long* cyc, uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[ENT * ESZ];
    for (uint32_t k = threadIdx.x; k < ENT * ESZ / 4; k += 1024) reinterpret_cast<uint32_t*>(tab)[k] = 0;
    __syncthreads();
    uint32_t x = 0x9E3779B9u * (blockIdx.x * 1024 + threadIdx.x + 1);
    uint64_t acc = 0;
    const uint64_t t0 = __builtin_readcyclecounter();
    for (uint32_t it = 0; it < iters; ++it) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        const uint32_t e = __umulhi(x, nent);
        uint8_t* ent = tab + e * ESZ;
        if constexpr (OP == 0) {
            acc += *reinterpret_cast<volatile unsigned long long*>(ent);
        } else if constexpr (OP == 1) {
            atomicAdd(reinterpret_cast<unsigned long long*>(ent + 8), (1ull << 40) | 64u);
        } else if constexpr (OP == 2) {
            atomicMax(reinterpret_cast<uint32_t*>(ent + 24), it);
        } else if constexpr (OP == 3) {
            acc += atomicAdd(reinterpret_cast<uint32_t*>(tab) + (x & 255), 1u);
        } else if constexpr (OP == 4) {
            *reinterpret_cast<volatile uint32_t*>(ent + 24) = it;
        } else if constexpr (OP == 5) {
            atomicAdd(reinterpret_cast<unsigned long long*>(tab) + threadIdx.x, 1ull);
        } else if constexpr (OP == 6) {
            atomicAdd(reinterpret_cast<uint32_t*>(tab) + threadIdx.x, 1u);
        } else if constexpr (OP == 7) {
            atomicAdd(reinterpret_cast<unsigned long long*>(ent + 8), (1ull << 40) | 64u);
            atomicMax(reinterpret_cast<uint32_t*>(ent + 24), it);
            atomicMax(reinterpret_cast<uint32_t*>(ent + 28), ~it);
        } else if constexpr (OP == 8) {
            atomicMax(reinterpret_cast<unsigned long long*>(ent + 8), (unsigned long long)it);
        } else if constexpr (OP == 10) {
            atomicMax(reinterpret_cast<uint32_t*>(tab) + threadIdx.x, it);
        } else if constexpr (OP == 11) {
            atomicMax(reinterpret_cast<uint32_t*>(tab) + e, it);
        } else if constexpr (OP == 12) {
            atomicAdd(reinterpret_cast<unsigned long long*>(tab) + e, (1ull << 40) | 64u);
        } else if constexpr (OP == 13) {
            acc += reinterpret_cast<volatile uint32_t*>(tab)[e];
        } else if constexpr (OP == 9) {
            volatile unsigned long long* q = reinterpret_cast<volatile unsigned long long*>(ent + 8);
            *q = *q + 1;
        }
    }
    __syncthreads();
    const uint64_t t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    if (acc == 0x123456789ull) sink[0] = (uint32_t)acc;
    if (threadIdx.x == 0) sink[1 + blockIdx.x] = reinterpret_cast<uint32_t*>(tab)[2];
}

template <int OP>
static void run(uint32_t iters, uint32_t nent, int grid) {
    unsigned long long* cyc;
    uint32_t* sink;
    CHK(hipMalloc(&cyc, grid * 8));
    CHK(hipMalloc(&sink, (grid + 1) * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lds<OP>, dim3(grid), dim3(1024), 0, 0, iters, nent, cyc, sink);  // warm
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(k_lds<OP>, dim3(grid), dim3(1024), 0, 0, iters, nent, cyc, sink);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* h = (unsigned long long*)malloc(grid * 8);
    CHK(hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (int i = 0; i < grid; ++i) mean += (double)h[i] / grid;
    const double lane_ops = 1024.0 * iters;
    printf("op %d entries %u iters %u: %.3f ms, %.0f cycles/WG, %.2f lane-ops/cycle/CU, %.1f cycles per wave-instr\n",
           OP, nent, iters, ms, mean, lane_ops / mean, mean / (lane_ops / 64.0));
    free(h);
    CHK(hipFree(cyc));
    CHK(hipFree(sink));
}

int main(int argc, char** argv) {
    const int op = argc > 1 ? atoi(argv[1]) : 1;
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
    const uint32_t nent = argc > 3 ? (uint32_t)atoi(argv[3]) : 2048;
    int cus = 256;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    switch (op) {
        case 0: run<0>(iters, nent, cus); break;
        case 1: run<1>(iters, nent, cus); break;
        case 2: run<2>(iters, nent, cus); break;
        case 3: run<3>(iters, nent, cus); break;
        case 4: run<4>(iters, nent, cus); break;
        case 5: run<5>(iters, nent, cus); break;
        case 6: run<6>(iters, nent, cus); break;
        case 7: run<7>(iters, nent, cus); break;
        case 8: run<8>(iters, nent, cus); break;
        case 9: run<9>(iters, nent, cus); break;
        case 10: run<10>(iters, nent, cus); break;
        case 11: run<11>(iters, nent, cus); break;
        case 12: run<12>(iters, nent, cus); break;
        case 13: run<13>(iters, nent, cus); break;
        default: printf("op 0..13\n"); return 2;
    }
    return 0;
}
