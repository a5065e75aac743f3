// Device-wide primitives from rocPRIM, kept in one translation unit (rocPRIM is heavy to compile):
// the overflow path's radix sort and the exclusive scan that turns per-entry need counts into CSR
// offsets for corro_compute_needs' second pass.
//
// Radix sort (overflow path): Keys carry the bucket's base offset in
// their high half, so one sort of all oversized buckets' records leaves every bucket in its own
// range: a Zipf-hot bucket of a million records is sorted by the whole GPU, not by one workgroup
// (a segmented sort gives a segment one block).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

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

using namespace corro;

extern "C" int corro_scan_offsets(corro_ctx *ctx, const uint64_t *counts, uint64_t *offsets, uint64_t n) {
    if (!ctx || (!counts && n) || !offsets) return fail(CORRO_E_INVALID, "NULL argument");
    CORRO_HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    // offsets[0] = 0, offsets[k + 1] = counts[0] + ... + counts[k]
    CORRO_HIP_TRY(hipMemsetAsync(offsets, 0, 8, s));
    if (n) {
        size_t temp = 0;
        CORRO_HIP_TRY(rocprim::inclusive_scan(nullptr, temp, counts, offsets + 1, (size_t)n, rocprim::plus<uint64_t>(), s));
        if (int rc = ctx->d_scan_tmp.ensure(temp + 256)) return rc;
        CORRO_HIP_TRY(rocprim::inclusive_scan(ctx->d_scan_tmp.p, temp, counts, offsets + 1, (size_t)n,
                                              rocprim::plus<uint64_t>(), s));
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    return CORRO_OK;
}
