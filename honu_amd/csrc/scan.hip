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

// rows per thread: 3-column scans of small batches use short tiles (more
// workgroups in flight: the scan is latency bound there), large ones long
// tiles (fewer tickets and look-back steps)
constexpr int SCAN_ITEMS_1 = 16, SCAN_ITEMS_3_SHORT = 4, SCAN_ITEMS_3_LONG = 16;
constexpr uint64_t SCAN_LONG_ROWS = 1ull << 19;

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

// One launch: tiles of HONU_BLOCK * ITEMS rows taken in order by an atomic
// ticket (one per workgroup); a tile sums its rows, wave 0 turns the tile's
// column sums into its exclusive prefixes with the decoupled look-back
// (lookback.h) and the workgroup writes its rows. in may alias out.
template <int K, int ITEMS>
__global__ __launch_bounds__(HONU_BLOCK) void k_scan_lb(const uint64_t *in, uint64_t n, uint64_t *out,
                                                        uint64_t *__restrict__ totals, ScanState S) {
    __shared__ uint64_t sh[HONU_WAVES_PER_BLOCK];
    __shared__ uint64_t pre[K];
    __shared__ uint32_t tile_sh;
    const uint32_t ep = lb_epoch(S.lb);
    const uint64_t rows = (uint64_t)HONU_BLOCK * ITEMS;
    const uint64_t ntiles = (n + rows - 1) / rows;
    uint64_t t;
    for (;;) {
        if (threadIdx.x == 0)
            tile_sh = __hip_atomic_fetch_add(&S.lb->ticket, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        t = tile_sh;
        if (t >= ntiles) break;
        const uint64_t base = (t * HONU_BLOCK + threadIdx.x) * ITEMS;
        uint64_t v[ITEMS][K], s[K], x[K], agg[K];
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
        for (int c = 0; c < K; c++) x[c] = block_incl_scan(s[c], sh, &agg[c]) - s[c];
        if (threadIdx.x < HONU_WAVE) {  // wave 0: the tile's prefix across tiles
            uint64_t excl[K];
            lb_scan<K>(S.status, t, ep, agg, excl);
#pragma unroll
            for (int c = 0; c < K; c++) {
                if (threadIdx.x == 0) pre[c] = excl[c];
                if (threadIdx.x == 0 && t == ntiles - 1) totals[c] = excl[c] + agg[c];
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < K; c++) {
            uint64_t run = pre[c] + x[c];
#pragma unroll
            for (int it = 0; it < ITEMS; it++) {
                const uint64_t row = base + it;
                if (row < n) out[row * K + c] = run;
                run += v[it][c];
            }
        }
        __syncthreads();  // pre and tile_sh are rewritten by the next tile
    }
    if (threadIdx.x < HONU_WAVE) lb_finish(S.lb, S.status, S.words, t, ntiles, gridDim.x);
}

uint64_t scan_status_words(uint64_t n) {  // the most K * tiles of any form
    const uint64_t t3 = (n + HONU_BLOCK * SCAN_ITEMS_3_SHORT - 1) / (HONU_BLOCK * SCAN_ITEMS_3_SHORT);
    const uint64_t t1 = (n + HONU_BLOCK * SCAN_ITEMS_1 - 1) / (HONU_BLOCK * SCAN_ITEMS_1);
    return 3 * t3 > t1 ? 3 * t3 + 3 : t1 + 3;
}

template <int K, int ITEMS>
static hipError_t scan_k(const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *totals,
                         const ScanState &S, hipStream_t s) {
    const uint64_t tiles = (n + HONU_BLOCK * ITEMS - 1) / (HONU_BLOCK * ITEMS);
    const uint64_t b = tiles < (uint64_t)S.max_blocks ? tiles : (uint64_t)S.max_blocks;
    hipLaunchKernelGGL((k_scan_lb<K, ITEMS>), dim3((unsigned)b), dim3(HONU_BLOCK), 0, s, in, n,
                       out, totals, S);
    return hipGetLastError();
}

hipError_t launch_scan(const uint64_t *in, uint64_t n, int K, uint64_t *out, uint64_t *totals,
                       const ScanState &S, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(totals, 0, sizeof(uint64_t) * K, s);
    if (K == 1) return scan_k<1, SCAN_ITEMS_1>(in, n, out, totals, S, s);
    if (K == 3)
        return n >= SCAN_LONG_ROWS ? scan_k<3, SCAN_ITEMS_3_LONG>(in, n, out, totals, S, s)
                                   : scan_k<3, SCAN_ITEMS_3_SHORT>(in, n, out, totals, S, s);
    return hipErrorInvalidValue;
}

}  // namespace honu
