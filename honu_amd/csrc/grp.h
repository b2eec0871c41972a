// grp.h — one record per GROUP of G lanes: the shared constants and group
// reductions of the group kernels (grp.hip; A/B build: ab/grp_walk.hip).
#pragma once

#include "kernels.h"
#include "lane.h"

namespace honu {

#define GO_MAX_ALLOC (1ull << 48)  // runtime maxAlloc, linux/amd64

constexpr int GRP = 16;                       // lanes per record
#ifndef FILL_G
#define FILL_G 16                             // decode fill: lanes per record
#endif
#ifndef FILL_K
#define FILL_K 2                              // decode fill: ACL entries per lane in flight
#endif
constexpr uint32_t GCAP = 2048;               // stage window, bytes
constexpr uint32_t GPAD = 16;                 // front pad of the encode stage
constexpr uint32_t GSTAGE = GPAD + GCAP + 32; // + slack for 32-byte windows
constexpr uint32_t GROW = 352;                // honu_meta image
// per-record LDS; the odd multiple of 16 spreads the groups of a wave over
// different banks
constexpr uint32_t GPER = GROW + GSTAGE + 16;
constexpr uint32_t GRECS = HONU_BLOCK / GRP;  // records per workgroup

template <int G> HONU_DEV uint32_t grp_bits(uint64_t ballot) {
    const uint32_t sh = (lane_id() / G) * G;
    return (uint32_t)(ballot >> sh) & (uint32_t)((1ull << G) - 1);
}
template <int G> HONU_DEV uint32_t grp_sum(uint32_t v) {
#pragma unroll
    for (int d = G / 2; d; d >>= 1) v += __shfl_xor(v, d, HONU_WAVE);
    return v;
}
template <int G> HONU_DEV uint64_t grp_sum64(uint64_t v) {
#pragma unroll
    for (int d = G / 2; d; d >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, d, HONU_WAVE);
        const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, HONU_WAVE);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
template <int G> HONU_DEV uint32_t grp_excl_scan(uint32_t v, uint32_t r) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < G; d <<= 1) {
        const uint32_t t = __shfl_up(x, d, G);
        if (r >= (uint32_t)d) x += t;
    }
    return x - v;
}

// bytes [from, to) of an 8-byte word (clamped), as a mask
HONU_DEV uint64_t bytemask64(int from, int to) {
    from = from < 0 ? 0 : (from > 8 ? 8 : from);
    to = to < 0 ? 0 : (to > 8 ? 8 : to);
    if (to <= from) return 0;
    const uint64_t hi = to == 8 ? ~0ull : ((1ull << (8 * to)) - 1);
    return hi & ~((1ull << (8 * from)) - 1);
}

// Row i -> LDS (22 aligned 16-byte chunks over the group).
template <int G> HONU_DEV void grp_stage_row(uint8_t *row, const honu_meta *src, uint32_t r) {
    const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
    u32x4 *d = reinterpret_cast<u32x4 *>(row);
    for (uint32_t c = r; c < GROW / 16; c += G) d[c] = s[c];
}

static inline dim3 grp_grid(uint64_t n, int cap) {
    const uint64_t b = (n * GRP + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(cap > 0 && b > (uint64_t)cap ? (uint64_t)cap : b));
}

}  // namespace honu
