// ipxg_sort.hip -- rocPRIM radix sort of 64-bit keys, used only by the two sequential
// fallback paths (fragment ordering per bucket, packet ordering per complex flow).  Kept
// in its own translation unit so the hot kernels compile without rocPRIM.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "ipxg_kernels.hpp"

namespace ipxg {

hipError_t sort_keys_u64(void* temp, size_t& temp_bytes, const uint64_t* in, uint64_t* out,
                         uint32_t n, int end_bit, hipStream_t st) {
    if (end_bit > 64) end_bit = 64;
    return rocprim::radix_sort_keys(temp, temp_bytes, in, out, (size_t)n, 0u, (unsigned)end_bit, st);
}

}  // namespace ipxg
