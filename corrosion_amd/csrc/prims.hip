// Device-wide primitives from rocPRIM, kept in one translation unit (rocPRIM is heavy to compile):
// the overflow path's radix sorts and segmented scans, and the exclusive scan that turns per-entry need counts into CSR
// offsets for corro_compute_needs' second pass.
//
// Radix sort (overflow path): Keys carry the bucket's base offset in
// their high half, so one sort of all oversized buckets' records leaves every bucket in its own
// range: a Zipf-hot bucket of a million records is sorted by the whole GPU, not by one workgroup
// (a segmented sort gives a segment one block).
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <mutex>
#include <vector>

#include "internal.h"
#include "merge_kernels.h"

namespace corro {

// keys u64 + values u32, bits [0, end_bit); temp == nullptr -> *temp_bytes = size needed
int ovf_sort_pairs(void *temp, size_t *temp_bytes, const uint64_t *ki, uint64_t *ko, const uint32_t *vi,
                   uint32_t *vo, uint32_t n, uint32_t end_bit, hipStream_t s) {
    const hipError_t e = rocprim::radix_sort_pairs(temp, *temp_bytes, ki, ko, vi, vo, n, 0u, end_bit, s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("radix sort: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// inclusive max-scan of u64 values segmented by equal consecutive u32 keys (the agent's per-actor
// running max of version ends); temp == nullptr -> *temp_bytes = size needed
int prim_segmax_scan_u64(void *temp, size_t *temp_bytes, const uint32_t *keys, const uint64_t *in, uint64_t *out,
                         uint32_t n, hipStream_t s) {
    const hipError_t e = rocprim::inclusive_scan_by_key(temp, *temp_bytes, keys, in, out, (size_t)n,
                                                        rocprim::maximum<uint64_t>(), rocprim::equal_to<uint32_t>(), s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("segmented scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// inclusive scan of u32 (extraction index group ids); temp == nullptr -> *temp_bytes = size needed
int prim_inclusive_scan_u32(void *temp, size_t *temp_bytes, const uint32_t *in, uint32_t *out, uint32_t n,
                            hipStream_t s) {
    const hipError_t e = rocprim::inclusive_scan(temp, *temp_bytes, in, out, (size_t)n, rocprim::plus<uint32_t>(), s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// inclusive scan of u32 counts into u64 sums (the pk intern's byte offsets); temp == nullptr ->
// *temp_bytes = size needed
struct Widen64 {
    __host__ __device__ inline uint64_t operator()(uint32_t x) const { return x; }
};
int prim_inclusive_scan_u32_u64(void *temp, size_t *temp_bytes, const uint32_t *in, uint64_t *out, uint64_t n,
                                hipStream_t s) {
    const auto wide = rocprim::make_transform_iterator(in, Widen64{});
    const hipError_t e = rocprim::inclusive_scan(temp, *temp_bytes, wide, out, (size_t)n, rocprim::plus<uint64_t>(), s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// inclusive max-scan of u64 (the pk table's ordered rebuild); temp == nullptr -> *temp_bytes = size needed
int prim_inclusive_max_u64(void *temp, size_t *temp_bytes, const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s) {
    const hipError_t e = rocprim::inclusive_scan(temp, *temp_bytes, in, out, (size_t)n, rocprim::maximum<uint64_t>(), s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

struct OvfMax {
    __device__ inline uint32_t operator()(uint32_t x, uint32_t y) const { return x > y ? x : y; }
};

// group start of candidate-sorted index q: the last group head at or before q (heads' indices
// increase, so a plain max-scan of "q if head else 0" finds it; no keys are compared in the scan)
struct OvfHead {
    const uint64_t *k;
    __device__ inline uint32_t operator()(uint32_t q) const { return (q == 0 || k[q - 1] != k[q]) ? q : 0u; }
};

// Segmented scans of the device-wide overflow path (ovf_kernels.h): which = 0 L (exclusive max of
// cl by row), 1 epoch counts (inclusive count of records by row), 2 group start of the candidates
// (plain max-scan over candidate-sorted indices; their running argmax is k_cscan_* in ovf_kernels.h). temp == nullptr ->
// *temp_bytes = the largest size any of them needs.
int ovf_scans(void *temp, size_t *temp_bytes, const OvfDev &d, int which, hipStream_t s) {
    const size_t K = d.K;
    hipError_t e = hipSuccess;
    const rocprim::counting_iterator<uint32_t> idx(0u);
    const auto heads = rocprim::make_transform_iterator(idx, OvfHead{d.ckey_s});
    if (!temp) {
        size_t t0 = 0, t1 = 0, t3 = 0;
        e = rocprim::exclusive_scan_by_key(nullptr, t0, d.rowid, d.cl_s, d.lx, 0u, K, OvfMax{},
                                           rocprim::equal_to<uint32_t>(), s);
        if (e == hipSuccess)
            e = rocprim::inclusive_scan_by_key(nullptr, t1, d.rowid, d.recf, d.epc, K, rocprim::plus<uint32_t>(),
                                               rocprim::equal_to<uint32_t>(), s);
        if (e == hipSuccess) e = rocprim::inclusive_scan(nullptr, t3, heads, d.cgs, K, OvfMax{}, s);
        *temp_bytes = std::max(std::max(t0, t1), t3);
    } else if (which == 0) {
        e = rocprim::exclusive_scan_by_key(temp, *temp_bytes, d.rowid, d.cl_s, d.lx, 0u, K, OvfMax{},
                                           rocprim::equal_to<uint32_t>(), s);
    } else if (which == 1) {
        e = rocprim::inclusive_scan_by_key(temp, *temp_bytes, d.rowid, d.recf, d.epc, K, rocprim::plus<uint32_t>(),
                                           rocprim::equal_to<uint32_t>(), s);
    } else {
        e = rocprim::inclusive_scan(temp, *temp_bytes, heads, d.cgs, (size_t)d.ncand, OvfMax{}, s);
    }
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("segmented scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// inclusive segmented scan of the candidate argmax's tile aggregates (k_cscan_tile)
int ovf_scan_tiles(void *temp, size_t *temp_bytes, const OvfDev &d, const CsAgg *in, CsAgg *out, uint32_t n,
                   hipStream_t s) {
    const hipError_t e = rocprim::inclusive_scan(temp, *temp_bytes, in, out, (size_t)n, CsComb{d.qkey, d.arena, d.qpos}, s);
    if (e != hipSuccess) return fail(CORRO_E_DEVICE, std::string("tile scan: ") + hipGetErrorString(e));
    return CORRO_OK;
}

// First launches of the rocPRIM kernels (the sorts and scans the agent's header passes and the
// overflow fold run) cost tens of milliseconds each: the code objects load and the dispatch
// resolves on first use. Once per process and device, each primitive runs here on a small and a
// large size (the radix sort takes a different kernel set for each), so a node's first gossip batch
// does not pay it. Errors are returned; the inputs are scratch (results discarded).
int prims_warm(corro_ctx *ctx) {
    static std::mutex mu;
    static std::vector<int> done;
    std::lock_guard<std::mutex> lock(mu);
    if (std::find(done.begin(), done.end(), ctx->device) != done.end()) return CORRO_OK;
    hipStream_t s = ctx->stream;
    const uint32_t sizes[2] = {1000u, 1u << 20};
    const uint32_t N = sizes[1];
    DevBuf buf;
    size_t temp = 0;
    for (uint32_t n : sizes) {
        size_t t = 0;
        ovf_sort_pairs(nullptr, &t, nullptr, nullptr, nullptr, nullptr, n, 64, s);
        temp = std::max(temp, t);
        prim_segmax_scan_u64(nullptr, &t, nullptr, nullptr, nullptr, n, s);
        temp = std::max(temp, t);
        prim_inclusive_scan_u32(nullptr, &t, nullptr, nullptr, n, s);
        temp = std::max(temp, t);
        prim_inclusive_scan_u32_u64(nullptr, &t, nullptr, nullptr, n, s);
        temp = std::max(temp, t);
        prim_inclusive_max_u64(nullptr, &t, nullptr, nullptr, n, s);
        temp = std::max(temp, t);
    }
    // keys in/out (u64), values in/out (u32), u32 keys/flags, u64 scan outputs
    const size_t k8 = (size_t)N * 8, k4 = (size_t)N * 4;
    const size_t o_ko = k8, o_vi = 2 * k8, o_vo = o_vi + k4, o_u = o_vo + k4, o_w = o_u + k4, o_t = o_w + k8;
    if (int rc = buf.ensure(o_t + temp + 256)) return rc;
    uint8_t *b = buf.as<uint8_t>();
    CORRO_HIP_TRY(hipMemsetAsync(b, 0, o_t, s));
    auto *ki = reinterpret_cast<uint64_t *>(b), *ko = reinterpret_cast<uint64_t *>(b + o_ko),
         *wo = reinterpret_cast<uint64_t *>(b + o_w);
    auto *vi = reinterpret_cast<uint32_t *>(b + o_vi), *vo = reinterpret_cast<uint32_t *>(b + o_vo),
         *u = reinterpret_cast<uint32_t *>(b + o_u);
    void *tp = b + o_t;
    for (uint32_t n : sizes) {
        size_t t = temp;
        if (int rc = ovf_sort_pairs(tp, &t, ki, ko, vi, vo, n, 64, s)) return rc;
        t = temp;
        if (int rc = prim_segmax_scan_u64(tp, &t, u, ki, wo, n, s)) return rc;
        t = temp;
        if (int rc = prim_inclusive_scan_u32(tp, &t, u, vo, n, s)) return rc;
        t = temp;
        if (int rc = prim_inclusive_scan_u32_u64(tp, &t, u, wo, n, s)) return rc;
        t = temp;
        if (int rc = prim_inclusive_max_u64(tp, &t, ki, wo, n, s)) return rc;
    }
    CORRO_HIP_TRY(hipStreamSynchronize(s));
    buf.release();
    done.push_back(ctx->device);
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
