// Device-wide radix sort for the overflow path (rocPRIM). Keys carry the bucket's base offset in
// their high half, so one sort of all oversized buckets' records leaves every bucket in its own
// range: a Zipf-hot bucket of a million records is sorted by the whole GPU, not by one workgroup
// (a segmented sort gives a segment one block). Kept in its own translation unit (rocPRIM is heavy
// to compile).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "internal.h"

namespace corro {

// keys u64 + values u32, bits [0, end_bit); temp == nullptr -> *temp_bytes = size needed
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s) {
    const hipError_t e = rocprim::radix_sort_pairs(temp, *temp_bytes, ki, ko, vi, vo, n, 0u, end_bit, s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("radix sort: ") + hipGetErrorString(e));
    return CORRO_OK;
}

}  // namespace corro
