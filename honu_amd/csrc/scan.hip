// scan.hip — exclusive prefix sums over u64 columns.
//
// Output offsets are how independent records become one contiguous arena:
// encode scans the exact record sizes into the output offsets (the batch
// form of lani's Grow+Bytes, encode.go:52-58,31-43); decode scans the ACL,
// region and payload counts into table/arena offsets. Three launches
// (tile reduce -> scan of tile sums -> tile scan), each a coalesced sweep;
// at 1M records a scan moves ~16-48 MB, microseconds next to the payloads.
#include "kernels.h"

namespace honu {

template <int K> struct ScanCfg;
template <> struct ScanCfg<1> { static constexpr int ITEMS = 16; };
template <> struct ScanCfg<3> { static constexpr int ITEMS = 4; };

// Inclusive scan across the 256 threads of a block; *total gets the sum.
HONU_DEV uint64_t block_incl_scan(uint64_t v, uint64_t *sh, uint64_t *total) {
    const uint32_t wib = threadIdx.x / HONU_WAVE;
    const uint64_t incl = wave_inclusive_scan(v);
    if (lane_id() == HONU_WAVE - 1) sh[wib] = incl;
    __syncthreads();
    uint64_t add = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < HONU_WAVES_PER_BLOCK; j++) {
        const uint64_t s = sh[j];
        if (j < (int)wib) add += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return incl + add;
}

template <int K>
__global__ __launch_bounds__(HONU_BLOCK) void k_scan_reduce(const uint64_t *__restrict__ in,
                                                            uint64_t n,
                                                            uint64_t *__restrict__ partials) {
    constexpr int ITEMS = ScanCfg<K>::ITEMS;
    __shared__ uint64_t sh[HONU_WAVES_PER_BLOCK];
    const uint64_t base = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) * ITEMS;
    uint64_t s[K];
#pragma unroll
    for (int c = 0; c < K; c++) s[c] = 0;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint64_t row = base + it;
        if (row < n) {
#pragma unroll
            for (int c = 0; c < K; c++) s[c] += in[row * K + c];
        }
    }
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint64_t tot;
        block_incl_scan(s[c], sh, &tot);
        if (threadIdx.x == 0) partials[(uint64_t)blockIdx.x * K + c] = tot;
    }
}

// One block: exclusive scan of the nb tile sums in place; totals[c] = sum.
template <int K>
__global__ __launch_bounds__(HONU_BLOCK) void k_scan_top(uint64_t *__restrict__ partials,
                                                         uint64_t nb,
                                                         uint64_t *__restrict__ totals) {
    __shared__ uint64_t sh[HONU_WAVES_PER_BLOCK];
    const uint64_t per = (nb + HONU_BLOCK - 1) / HONU_BLOCK;
    const uint64_t j0 = threadIdx.x * per;
    const uint64_t j1 = j0 + per < nb ? j0 + per : nb;
    for (int c = 0; c < K; c++) {
        uint64_t local = 0;
        for (uint64_t j = j0; j < j1; j++) local += partials[j * K + c];
        uint64_t tot;
        const uint64_t incl = block_incl_scan(local, sh, &tot);
        uint64_t run = incl - local;
        for (uint64_t j = j0; j < j1; j++) {
            const uint64_t v = partials[j * K + c];
            partials[j * K + c] = run;
            run += v;
        }
        if (threadIdx.x == 0) totals[c] = tot;
    }
}

template <int K>
__global__ __launch_bounds__(HONU_BLOCK) void k_scan_apply(const uint64_t *in, uint64_t n,
                                                           const uint64_t *__restrict__ partials,
                                                           uint64_t *out) {
    constexpr int ITEMS = ScanCfg<K>::ITEMS;
    __shared__ uint64_t sh[HONU_WAVES_PER_BLOCK];
    const uint64_t base = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) * ITEMS;
    uint64_t v[ITEMS][K];
    uint64_t s[K];
#pragma unroll
    for (int c = 0; c < K; c++) s[c] = 0;
#pragma unroll
    for (int it = 0; it < ITEMS; it++) {
        const uint64_t row = base + it;
#pragma unroll
        for (int c = 0; c < K; c++) {
            v[it][c] = row < n ? in[row * K + c] : 0;
            s[c] += v[it][c];
        }
    }
#pragma unroll
    for (int c = 0; c < K; c++) {
        uint64_t tot;
        const uint64_t incl = block_incl_scan(s[c], sh, &tot);
        uint64_t run = incl - s[c] + partials[(uint64_t)blockIdx.x * K + c];
#pragma unroll
        for (int it = 0; it < ITEMS; it++) {
            const uint64_t row = base + it;
            if (row < n) out[row * K + c] = run;
            run += v[it][c];
        }
    }
}

uint64_t scan_partials_len(uint64_t n, int K) {
    const uint64_t tile = (uint64_t)HONU_BLOCK * (K == 1 ? ScanCfg<1>::ITEMS : ScanCfg<3>::ITEMS);
    return ((n + tile - 1) / tile + 1) * (uint64_t)K;
}

template <int K>
static hipError_t scan_k(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *totals,
                         uint64_t *partials, hipStream_t s) {
    const uint64_t tile = (uint64_t)HONU_BLOCK * ScanCfg<K>::ITEMS;
    const uint64_t nb = (n + tile - 1) / tile;
    hipLaunchKernelGGL(k_scan_reduce<K>, dim3((unsigned)nb), dim3(HONU_BLOCK), 0, s, in, n, partials);
    hipLaunchKernelGGL(k_scan_top<K>, dim3(1), dim3(HONU_BLOCK), 0, s, partials, nb, totals);
    hipLaunchKernelGGL(k_scan_apply<K>, dim3((unsigned)nb), dim3(HONU_BLOCK), 0, s, in, n, partials, out);
    return hipGetLastError();
}

hipError_t launch_scan(const uint64_t *in, uint64_t n, int K, uint64_t *out, uint64_t *totals,
                       uint64_t *partials, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(totals, 0, sizeof(uint64_t) * K, s);
    if (K == 1) return scan_k<1>(in, n, out, totals, partials, s);
    if (K == 3) return scan_k<3>(in, n, out, totals, partials, s);
    return hipErrorInvalidValue;
}

}  // namespace honu
