// common.h — device primitives shared by the gfx950 codec kernels.
//
// Wave64 helpers, lani varint arithmetic (restating Go encoding/binary, used by
// lani/encode.go:149-181 and decode.go:127-190) and the byte-stream copy engine
// used for payload movement in both directions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/honu_codec.h"
#include "../../include/honu_bench.h"

#define HONU_WAVE 64
#define HONU_BLOCK 256
#define HONU_WAVES_PER_BLOCK (HONU_BLOCK / HONU_WAVE)

#define HONU_DEV __device__ __forceinline__
#define HONU_HD __host__ __device__ __forceinline__

namespace honu {

// ------------------------------------------------------------------------
// wave helpers
// ------------------------------------------------------------------------
HONU_DEV uint32_t lane_id() { return __lane_id(); }

HONU_DEV uint32_t wave_in_block() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x / HONU_WAVE);
}

HONU_DEV uint64_t uniform64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
HONU_DEV uint32_t uniform32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

HONU_DEV uint32_t readlane32(uint32_t v, uint32_t lane) {
    return __builtin_amdgcn_readlane(v, lane);
}
HONU_DEV uint64_t readlane64(uint64_t v, uint32_t lane) {
    uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Same semantics as HIP's __syncwarp: orders LDS traffic among the lanes of
// one wave. Every per-record loop in this library is wave-uniform.
HONU_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inclusive scan over the 64 lanes.
HONU_DEV uint64_t wave_inclusive_scan(uint64_t v) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int d = 1; d < HONU_WAVE; d <<= 1) {
        uint64_t t = __shfl_up(v, d, HONU_WAVE);
        if (l >= (uint32_t)d) v += t;
    }
    return v;
}
HONU_DEV uint32_t wave_inclusive_scan32(uint32_t v) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int d = 1; d < HONU_WAVE; d <<= 1) {
        uint32_t t = __shfl_up(v, d, HONU_WAVE);
        if (l >= (uint32_t)d) v += t;
    }
    return v;
}
HONU_DEV uint64_t wave_sum(uint64_t v) { return readlane64(wave_inclusive_scan(v), 63); }

// Wave exclusive scan of v (64-bit); *total = the wave's sum.
HONU_DEV uint64_t wave_excl(uint64_t v, uint64_t &total) {
    const uint64_t inc = wave_inclusive_scan(v);
    total = readlane64(inc, 63);
    return inc - v;
}

// Largest lane r with pre(r) <= e, for pre non-decreasing over the lanes
// (each lane its own e; pre read with ds_bpermute).
HONU_DEV uint32_t lane_search(uint64_t pre, uint64_t e) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t mid = lo + step;
        const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pre >> 32), (int)mid) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)pre, (int)mid);
        if (mid < 64 && v <= e) lo = mid;
    }
    return lo;
}
// The same over a 32-bit prefix (one ds_bpermute per step).
HONU_DEV uint32_t lane_search32(uint32_t pre, uint32_t e) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t mid = lo + step;
        const uint32_t v = (uint32_t)__shfl((int)pre, (int)(mid & 63));
        if (mid < 64 && v <= e) lo = mid;
    }
    return lo;
}
// Wave exclusive scan of v (32-bit); *total = the wave's sum.
HONU_DEV uint32_t wave_excl32(uint32_t v, uint32_t &total) {
    const uint32_t inc = wave_inclusive_scan32(v);
    total = __builtin_amdgcn_readlane(inc, 63);
    return inc - v;
}
HONU_DEV uint64_t shfl_xor64(uint64_t v, int d) {
    return ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d) << 32) |
           (uint32_t)__shfl_xor((int)(uint32_t)v, d);
}
HONU_DEV uint64_t shfl64(uint64_t v, uint32_t src) {
    return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src) << 32) |
           (uint32_t)__shfl((int)(uint32_t)v, (int)src);
}


// ------------------------------------------------------------------------
// lani / encoding/binary varint arithmetic
// ------------------------------------------------------------------------
// Length of binary.PutUvarint(x): ceil(bits/7), at least 1.
HONU_HD uint32_t uvarint_len(uint64_t x) {
    uint32_t bits = 64u - (uint32_t)__builtin_clzll(x | 1ull);
    return (bits + 6u) / 7u;
}
// binary.PutVarint zig-zag (encoding/binary/varint.go PutVarint).
HONU_HD uint64_t zigzag(int64_t x) {
    uint64_t ux = (uint64_t)x << 1;
    return x < 0 ? ~ux : ux;
}
HONU_HD int64_t unzigzag(uint64_t ux) {
    int64_t x = (int64_t)(ux >> 1);
    return (ux & 1) ? ~x : x;
}
// Writes binary.PutUvarint(x) through p (any address space).
template <typename P> HONU_DEV uint32_t put_uvarint(P p, uint64_t x) {
    uint32_t i = 0;
    while (x >= 0x80) {
        p[i++] = (uint8_t)(x | 0x80);
        x >>= 7;
    }
    p[i++] = (uint8_t)x;
    return i;
}

// ------------------------------------------------------------------------
// byte-stream copy engine
// ------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16 bytes at any byte address: one global_load_dwordx4 (gfx950 runs with
// unaligned global access enabled)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

// Funnel a 16-byte output chunk out of two aligned 16-byte source chunks: the
// bytes [p, p+16) of lo||hi, p in [0,16). p is wave-uniform, so the switch is
// a uniform branch and each output dword is one v_alignbyte_b32.
HONU_DEV u32x4 funnel16(u32x4 lo, u32x4 hi, uint32_t p) {
    const uint32_t b = p & 3u;
    const uint32_t w0 = lo.x, w1 = lo.y, w2 = lo.z, w3 = lo.w;
    const uint32_t w4 = hi.x, w5 = hi.y, w6 = hi.z, w7 = hi.w;
    u32x4 r;
    switch (p >> 2) {
    case 0:
        r.x = __builtin_amdgcn_alignbyte(w1, w0, b);
        r.y = __builtin_amdgcn_alignbyte(w2, w1, b);
        r.z = __builtin_amdgcn_alignbyte(w3, w2, b);
        r.w = __builtin_amdgcn_alignbyte(w4, w3, b);
        break;
    case 1:
        r.x = __builtin_amdgcn_alignbyte(w2, w1, b);
        r.y = __builtin_amdgcn_alignbyte(w3, w2, b);
        r.z = __builtin_amdgcn_alignbyte(w4, w3, b);
        r.w = __builtin_amdgcn_alignbyte(w5, w4, b);
        break;
    case 2:
        r.x = __builtin_amdgcn_alignbyte(w3, w2, b);
        r.y = __builtin_amdgcn_alignbyte(w4, w3, b);
        r.z = __builtin_amdgcn_alignbyte(w5, w4, b);
        r.w = __builtin_amdgcn_alignbyte(w6, w5, b);
        break;
    default:
        r.x = __builtin_amdgcn_alignbyte(w4, w3, b);
        r.y = __builtin_amdgcn_alignbyte(w5, w4, b);
        r.z = __builtin_amdgcn_alignbyte(w6, w5, b);
        r.w = __builtin_amdgcn_alignbyte(w7, w6, b);
        break;
    }
    return r;
}

template <bool NT> HONU_DEV u32x4 ld16(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT> HONU_DEV void st16(u32x4 *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Byte copy by the lanes of one wave (edges and small spans).
HONU_DEV void wave_copy_bytes(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                              uint64_t n) {
    for (uint64_t k = lane_id(); k < n; k += HONU_WAVE) dst[k] = src[k];
}

// Copy n bytes src -> dst (global, any alignment) with one wave. Interior
// destination chunks are written with 16-byte stores; the partial chunks at
// either end with byte stores, so neighbouring bytes owned by other waves are
// never touched. Source chunks are read with aligned 16-byte loads: an
// aligned 16-byte block holding at least one source byte never crosses a
// page, so the over-read is always mapped.
// NT: non-temporal cache policy, 0 none, 1 loads and stores, 2 loads only,
// 3 stores only; 4: a misaligned source is read with one unaligned 16-byte
// load per chunk instead of two aligned loads and a funnel.
// The head bytes, the tail bytes and the first UNROLL x 64 chunks are all
// loaded before any of them is stored, so a short segment (the common case
// for Small records: 2.5 KB) costs one round trip, not three.
template <int UNROLL = 4, int NT = 0>
HONU_DEV void wave_copy(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, uint64_t n) {
    if (n == 0) return;
    constexpr bool NTL = NT == 1 || NT == 2, NTS = NT == 1 || NT == 3;
    const uint32_t lane = lane_id();
    uint64_t head = (16u - ((uint64_t)dst & 15u)) & 15u;
    if (head > n) head = n;
    const uint64_t chunks = (n - head) >> 4;
    const uint64_t tail = (n - head) & 15u;
    const uint64_t t0 = head + (chunks << 4);
    u32x4 *__restrict__ d4 = reinterpret_cast<u32x4 *>(dst + head);
    const uint8_t *bsrc = src + head;
    const uint32_t p = (uint32_t)((uint64_t)bsrc & 15u);  // wave-uniform
    const u32x4 *__restrict__ s4 = reinterpret_cast<const u32x4 *>(bsrc - p);
    auto load = [&](uint64_t c, u32x4 &a, u32x4 &b) {
        if (NT == 4 && p) {
            a = *reinterpret_cast<const u32x4u *>(bsrc + 16 * c);
        } else {
            a = ld16<NTL>(&s4[c]);
            if (p) b = ld16<NTL>(&s4[c + 1]);
        }
    };
    auto store = [&](uint64_t c, const u32x4 &a, const u32x4 &b) {
        st16<NTS>(&d4[c], (p == 0 || NT == 4) ? a : funnel16(a, b, p));
    };
    // round 0: edges and the first chunks
    uint8_t hv = 0, tv = 0;
    if (lane < head) hv = src[lane];
    if (lane < tail) tv = src[t0 + lane];
    {
        u32x4 a[UNROLL], b[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
            if (lane + u * HONU_WAVE < chunks) load(lane + u * HONU_WAVE, a[u], b[u]);
        if (lane < head) dst[lane] = hv;
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
            if (lane + u * HONU_WAVE < chunks) store(lane + u * HONU_WAVE, a[u], b[u]);
        if (lane < tail) dst[t0 + lane] = tv;
    }
    // the rest: every iteration issues all its loads before any store, with
    // per-chunk predication instead of a serial remainder loop
    for (uint64_t c = lane + UNROLL * HONU_WAVE; c < chunks; c += UNROLL * HONU_WAVE) {
        u32x4 a[UNROLL], b[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
            if (c + u * HONU_WAVE < chunks) load(c + u * HONU_WAVE, a[u], b[u]);
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
            if (c + u * HONU_WAVE < chunks) store(c + u * HONU_WAVE, a[u], b[u]);
    }
}

// ------------------------------------------------------------------------
// honu_record_info as four explicit 8-byte stores (padding bytes included:
// a struct copy may leave them unwritten, and rows are compared bytewise)
// ------------------------------------------------------------------------
HONU_DEV void store_info(honu_record_info *p, const honu_record_info &v) {
    uint64_t *q = reinterpret_cast<uint64_t *>(p);
    q[0] = v.data_off;
    q[1] = v.data_len;
    q[2] = (uint64_t)(uint32_t)v.data_status | ((uint64_t)(uint32_t)v.meta_status << 32);
    q[3] = (uint64_t)v.storage_version | ((uint64_t)v.tombstone << 8);
}

// ------------------------------------------------------------------------
// synthetic payload bytes (shared by host generator and device fill)
// ------------------------------------------------------------------------
HONU_HD uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// 8 payload bytes of record `index` starting at byte 8*word (little endian).
HONU_HD uint64_t payload_word(uint64_t seed, uint64_t index, uint64_t word) {
    return splitmix64((seed * 0xD1B54A32D192ED03ull) ^ (index * 0x8CB92BA72F3D8DD7ull) ^
                      (word * 0x9E3779B97F4A7C15ull) ^ 0x5851F42D4C957F2Dull);
}

// Position-aware digest of a byte run: sum over 8-byte little-endian words
// (zero padded) of splitmix64(word + k * golden), plus the length. Order of
// summation does not matter, so waves reduce it in any grouping.
HONU_HD uint64_t digest_term(uint64_t word, uint64_t k) {
    return splitmix64(word + k * 0x9E3779B97F4A7C15ull);
}

}  // namespace honu
