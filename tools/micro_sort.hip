// Microbenchmark: the overflow fold's row sort (config 5 at 64M: 57.4 M (u64 key, u32 value)
// pairs, 48 key bits) with rocPRIM's gfx950 default onesweep (8 bits per place: 6 passes) against
// wider digits (fewer passes, larger per-block histograms).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/micro_sort.hip -o tools/micro_sort
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <rocprim/device/device_radix_sort.hpp>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t err_ = (x);                                                 \
        if (err_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

template <unsigned Bits, unsigned Ipt, unsigned HB = 512>
using OneCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<HB, 32>, rocprim::kernel_config<512, Ipt>, Bits,
                                        rocprim::block_radix_rank_algorithm::match>>;

template <class Cfg>
int run(const char *name, const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo, uint32_t n,
        unsigned end_bit, const uint64_t *ref) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, ki, ko, vi, vo, n, 0u, end_bit, 0));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; w++) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, ki, ko, vi, vo, n, 0u, end_bit, 0));
    const int reps = 5;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) CK(rocprim::radix_sort_pairs<Cfg>(tmp, tb, ki, ko, vi, vo, n, 0u, end_bit, 0));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    // check against the default-config result
    uint64_t *h = (uint64_t *)malloc(8ULL * n), *hr = (uint64_t *)malloc(8ULL * n);
    CK(hipMemcpy(h, ko, 8ULL * n, hipMemcpyDeviceToHost));
    bool ok = true;
    if (ref) {
        CK(hipMemcpy(hr, ref, 8ULL * n, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n && ok; i++) ok = h[i] == hr[i];
    }
    for (uint32_t i = 1; i < n && ok; i++) ok = h[i - 1] <= h[i];
    printf("%-28s %8.3f ms  temp %6zu MB  %s\n", name, ms / reps, tb >> 20, ok ? "sorted" : "WRONG");
    free(h);
    free(hr);
    CK(hipFree(tmp));
    return 0;
}

int main() {
    const uint32_t n = 57372333;
    const unsigned end_bit = 48;
    uint64_t *ki, *ko, *kref;
    uint32_t *vi, *vo;
    CK(hipMalloc(&ki, 8ULL * n)); CK(hipMalloc(&ko, 8ULL * n)); CK(hipMalloc(&kref, 8ULL * n));
    CK(hipMalloc(&vi, 4ULL * n)); CK(hipMalloc(&vo, 4ULL * n));
    {
        uint64_t *h = (uint64_t *)malloc(8ULL * n);
        uint32_t *hv = (uint32_t *)malloc(4ULL * n);
        uint64_t x = 88172645463325252ULL;
        // row ids in 22 bits (2.3 M rows, Zipf-like: low rows hot), positions in 26 bits
        for (uint32_t i = 0; i < n; i++) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const uint64_t u = x % 2339543;
            const uint64_t row = (u * u) / 2339543;
            h[i] = (row << 26) | (i & ((1u << 26) - 1));
            hv[i] = i;
        }
        CK(hipMemcpy(ki, h, 8ULL * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(vi, hv, 4ULL * n, hipMemcpyHostToDevice));
        free(h);
        free(hv);
    }
    if (run<rocprim::default_config>("default (gfx950: 8 bits)", ki, kref, vi, vo, n, end_bit, nullptr)) return 1;
    if (run<OneCfg<8, 12>>("onesweep 8 bits", ki, ko, vi, vo, n, end_bit, kref)) return 1;
    if (run<OneCfg<10, 8, 256>>("onesweep 10 bits", ki, ko, vi, vo, n, end_bit, kref)) return 1;
    return 0;
}
