// ipxg_sort.hip -- rocPRIM radix sort of 64-bit keys, used only by the two sequential
// fallback paths (fragment ordering per bucket, packet ordering per complex flow).  Kept
// in its own translation unit so the hot kernels compile without rocPRIM.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "ipxg_kernels.hpp"

namespace ipxg {

hipError_t sort_keys_u64(void* temp, size_t& temp_bytes, const uint64_t* in, uint64_t* out,
                         uint32_t n, int end_bit, hipStream_t st) {
    if (end_bit > 64) end_bit = 64;
    return rocprim::radix_sort_keys(temp, temp_bytes, in, out, (size_t)n, 0u, (unsigned)end_bit, st);
}

// strict mode: events by line (stable: equal lines keep packet order)
hipError_t sort_pairs_u32(void* temp, size_t& temp_bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                          uint32_t* vout, uint32_t n, int end_bit, hipStream_t st) {
    if (end_bit > 32) end_bit = 32;
    return rocprim::radix_sort_pairs(temp, temp_bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)end_bit, st);
}

// strict mode: each keyed packet's rank among the keyed packets (its sweep step)
hipError_t exclusive_scan_u32(void* temp, size_t& temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n,
                              hipStream_t st) {
    return rocprim::exclusive_scan(temp, temp_bytes, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
}

// process-plugin bridge: byte offsets of the walked packets' frames
hipError_t exclusive_scan_u64(void* temp, size_t& temp_bytes, const uint64_t* in, uint64_t* out, uint32_t n,
                              hipStream_t st) {
    return rocprim::exclusive_scan(temp, temp_bytes, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), st);
}

}  // namespace ipxg
