// gapbench: the cost of a dependent kernel boundary on one stream, by what the kernels look like
// (grid, block size, LDS, argument size, dirty bytes left behind, a store into host-mapped
// memory).  Each case launches R back-to-back pairs and reports the wall time per launch from
// HIP events; run under `rocprofv3 --kernel-trace` for the kernels' own durations.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

struct Big {
    unsigned w[128];
};

__global__ void k_nop(unsigned* out) {
    if (out && threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFFu) out[0] = 1;
}
__global__ void k_nop_big(Big b, unsigned* out) {
    if (out && threadIdx.x == 0 && blockIdx.x == b.w[7]) out[0] = b.w[3];
}
__global__ void k_nop_lds(unsigned* out) {
    extern __shared__ unsigned s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (out && s[(threadIdx.x + 1) & 255] == 0xFFFFFFFFu) out[0] = 1;
}
// every thread writes `per` 16-byte words: the kernel leaves `grid * 256 * per * 16` bytes dirty
__global__ void k_write(uint4* dst, unsigned per) {
    const size_t base = ((size_t)blockIdx.x * per) * blockDim.x;
    for (unsigned k = 0; k < per; ++k) dst[base + (size_t)k * blockDim.x + threadIdx.x] = make_uint4(k, 1, 2, 3);
}
__global__ void k_host_store(unsigned* host, unsigned v) {
    if (threadIdx.x < 64 && blockIdx.x == 0) host[threadIdx.x] = v;
}

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t r_ = (x);                                                     \
        if (r_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(r_));              \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 200;
    hipStream_t st;
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    uint4* buf;
    const size_t big = 256ull << 20;
    CHK(hipMalloc(&buf, big));
    unsigned* host;
    CHK(hipHostMalloc((void**)&host, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned* hostd;
    CHK(hipHostGetDevicePointer((void**)&hostd, host, 0));
    Big bg;
    memset(&bg, 0, sizeof(bg));
    bg.w[7] = 0xFFFFFFFFu;
    CHK(hipFuncSetAttribute((const void*)k_nop_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));

    auto run = [&](const char* name, auto&& body) {
        for (int w = 0; w < 10; ++w) body();
        CHK(hipStreamSynchronize(st));
        CHK(hipEventRecord(a, st));
        for (int r = 0; r < R; ++r) body();
        CHK(hipEventRecord(b, st));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        printf("%-44s %8.2f us per iteration\n", name, ms * 1e3 / R);
        fflush(stdout);
    };
    run("nop 512x256", [&] { hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr); });
    run("nop 512x256 x2 (per pair)", [&] {
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
    });
    run("nop 256x1024", [&] { hipLaunchKernelGGL(k_nop, dim3(256), dim3(1024), 0, st, nullptr); });
    run("nop 512x256 512-byte args", [&] { hipLaunchKernelGGL(k_nop_big, dim3(512), dim3(256), 0, st, bg, nullptr); });
    run("nop 512x256 64 KiB LDS", [&] { hipLaunchKernelGGL(k_nop_lds, dim3(512), dim3(256), 65536, st, nullptr); });
    for (unsigned per : {1u, 4u, 16u, 64u, 128u}) {  // (at most 256 MiB: buf)
        char nm[96];
        snprintf(nm, sizeof nm, "write %6.1f MB + nop", 512.0 * 256 * per * 16 / 1e6);
        run(nm, [&] {
            hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, st, buf, per);
            hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
        });
    }
    run("write 8 MB alone", [&] { hipLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, st, buf, 4u); });
    run("host-mapped store + nop", [&] {
        hipLaunchKernelGGL(k_host_store, dim3(1), dim3(64), 0, st, hostd, 1u);
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
    });
    run("memset 64 B + nop", [&] {
        CHK(hipMemsetAsync(buf, 0, 64, st));
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
    });
    hipEvent_t c;
    CHK(hipEventCreate(&c));
    run("event record + nop", [&] {
        CHK(hipEventRecord(c, st));
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
    });
    hipEvent_t dn;
    CHK(hipEventCreateWithFlags(&dn, hipEventDisableTiming));
    run("event record (no timing) + nop", [&] {
        CHK(hipEventRecord(dn, st));
        hipLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, nullptr);
    });
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    run("nop launched with start/stop events (ext)", [&] {
        hipExtLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, e0, e1, 0, (unsigned*)nullptr);
    });
    {
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("  (its own events: %.2f us)\n", ms * 1e3);
    }
    run("write 8 MB + nop, both ext-launched with events", [&] {
        hipExtLaunchKernelGGL(k_write, dim3(512), dim3(256), 0, st, e0, e1, 0, buf, 4u);
        hipExtLaunchKernelGGL(k_nop, dim3(512), dim3(256), 0, st, c, b, 0, (unsigned*)nullptr);
    });
    CHK(hipStreamSynchronize(st));
    return 0;
}
