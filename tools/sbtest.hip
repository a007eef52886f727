// Structured buffer loads past 4 GiB (gfx950): does a record index x stride address beyond
// 4 GiB?  Build: hipcc --offload-arch=gfx950 -O3 tools/sbtest.hip -o tools/sbtest.  Measured on the
// box (round 5): no -- lanes past 4 GiB read the data 4 GiB lower (the address wraps at 32 bits),
// so IPXG_BATCH_OFFSET16 uses per-wave 4 GiB windows of raw resources instead (ipxg_kernels.hpp).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ u32x4 sload(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset, int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v4i32");
__global__ void k(const unsigned char* a, unsigned n16, u32x4* out, unsigned idx) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)a, 16, (int)n16, 0x00020000);
    out[threadIdx.x] = sload(r, (int)(idx + threadIdx.x), 0, 0, 0);
}
int main() {
    const size_t bytes = (size_t)5 << 30;  // 5 GiB
    unsigned char* a; u32x4* out;
    if (hipMalloc(&a, bytes) != hipSuccess) { printf("alloc fail\n"); return 1; }
    hipMalloc(&out, 64 * 16);
    // mark 16-byte units: unit u holds {u, u^0x5a5a, 7, 9} at a few places
    size_t units[4] = {1, ((size_t)1 << 28) - 3, ((size_t)1 << 28) + 5, (bytes / 16) - 64};
    for (size_t u : units) {
        unsigned v[64 * 4];
        for (int l = 0; l < 64; ++l) { v[4*l] = (unsigned)(u + l); v[4*l+1] = (unsigned)((u + l) >> 32); v[4*l+2] = 7; v[4*l+3] = 9; }
        hipMemcpy(a + u * 16, v, sizeof v, hipMemcpyHostToDevice);
    }
    int bad = 0;
    for (size_t u : units) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, a, (unsigned)(bytes / 16), out, (unsigned)u);
        unsigned h[64 * 4];
        hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l) if (h[4*l] != (unsigned)(u + l) || h[4*l+2] != 7) { bad++; if (bad < 5) printf("unit %zu lane %d got %u %u %u\n", u, l, h[4*l], h[4*l+1], h[4*l+2]); }
    }
    // out of range index -> zeros
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, a, (unsigned)(bytes / 16), out, 0xFFFFFFC0u);
    unsigned h[64 * 4];
    hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    int nz = 0; for (int i = 0; i < 256; ++i) nz += h[i] != 0;
    printf("bad %d, oob nonzero %d\n", bad, nz);
    return bad || nz;
}
