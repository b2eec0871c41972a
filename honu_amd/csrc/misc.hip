// misc.hip — synthetic payload fill and record digests (bench/test support).
#include "kernels.h"

namespace honu {

HONU_DEV uint8_t payload_byte(uint64_t seed, uint64_t idx, uint64_t k) {
    return (uint8_t)(payload_word(seed, idx, k >> 3) >> (8 * (k & 7)));
}

// Bytes [k0, k0+16) of record idx's payload stream.
HONU_DEV u32x4 payload16(uint64_t seed, uint64_t idx, uint64_t k0) {
    const uint64_t q = k0 >> 3;
    const uint32_t r = (uint32_t)(k0 & 7) * 8;
    const uint64_t w0 = payload_word(seed, idx, q), w1 = payload_word(seed, idx, q + 1);
    uint64_t lo = w0, hi = w1;
    if (r) {
        const uint64_t w2 = payload_word(seed, idx, q + 2);
        lo = (w0 >> r) | (w1 << (64 - r));
        hi = (w1 >> r) | (w2 << (64 - r));
    }
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

__global__ __launch_bounds__(HONU_BLOCK) void k_gen_payload(uint64_t seed, uint64_t first,
                                                            uint64_t n,
                                                            const uint64_t *__restrict__ payload_off,
                                                            uint8_t *__restrict__ payload) {
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    const uint32_t lane = lane_id();
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block(); i < n;
         i += nwaves) {
        const uint64_t s = payload_off[i], len = payload_off[i + 1] - s;
        const uint64_t idx = first + i;
        uint8_t *dst = payload + s;
        uint64_t head = (16u - ((uint64_t)dst & 15u)) & 15u;
        if (head > len) head = len;
        if (lane < head) dst[lane] = payload_byte(seed, idx, lane);
        const uint64_t chunks = (len - head) >> 4;
        u32x4 *d4 = reinterpret_cast<u32x4 *>(dst + head);
        for (uint64_t c = lane; c < chunks; c += HONU_WAVE) d4[c] = payload16(seed, idx, head + 16 * c);
        const uint64_t t0 = head + 16 * chunks;
        if (t0 + lane < len) dst[t0 + lane] = payload_byte(seed, idx, t0 + lane);
    }
}

// digest = splitmix64(len) + sum_k digest_term(word_k, k) over the
// zero-padded little-endian 8-byte words of the run.
__global__ __launch_bounds__(HONU_BLOCK) void k_digest(const uint8_t *__restrict__ arena,
                                                       const uint64_t *__restrict__ off,
                                                       const uint64_t *__restrict__ lens,
                                                       uint64_t n, uint64_t *__restrict__ digest) {
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block(); i < n;
         i += nwaves) {
        const uint64_t s = off[i];
        const uint64_t len = lens ? lens[i] : off[i + 1] - s;
        const uint8_t *p = arena + s;
        const uint64_t nw = (len + 7) >> 3;
        const uint64_t sh = (uint64_t)p & 7u;
        const uint64_t *a = reinterpret_cast<const uint64_t *>(p - sh);
        uint64_t acc = 0;
        constexpr int U = 4;  // words per lane with their loads in flight together
        for (uint64_t k0 = lane_id(); k0 < nw; k0 += U * HONU_WAVE) {
            uint64_t lo[U], hi[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t k = k0 + (uint64_t)u * HONU_WAVE;
                lo[u] = hi[u] = 0;
                if (k < nw) {
                    lo[u] = a[k];
                    if (sh && 8 * k + (8 - sh) < len) hi[u] = a[k + 1];
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t k = k0 + (uint64_t)u * HONU_WAVE;
                if (k < nw) {
                    uint64_t w = lo[u];
                    if (sh) w = (w >> (8 * sh)) | (hi[u] << (64 - 8 * sh));
                    const uint64_t valid = len - 8 * k;
                    if (valid < 8) w &= (1ull << (8 * valid)) - 1;
                    acc += digest_term(w, k);
                }
            }
        }
        acc = wave_sum(acc);
        if (lane_id() == 0) digest[i] = acc + splitmix64(len);
    }
}

hipError_t launch_gen_payload(const LaunchGeom &g, uint64_t seed, uint64_t first, uint64_t n,
                              const uint64_t *payload_off, uint8_t *payload, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t b = (n + 3) / 4;
    if (b > (uint64_t)g.per_record_blocks) b = g.per_record_blocks;
    hipLaunchKernelGGL(k_gen_payload, dim3((unsigned)b), dim3(HONU_BLOCK), 0, s, seed, first, n,
                       payload_off, payload);
    return hipGetLastError();
}

hipError_t launch_digest(const LaunchGeom &g, const uint8_t *arena, const uint64_t *off,
                         const uint64_t *len, uint64_t n, uint64_t *digest, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t b = (n + 3) / 4;
    if (b > (uint64_t)g.per_record_blocks) b = g.per_record_blocks;
    hipLaunchKernelGGL(k_digest, dim3((unsigned)b), dim3(HONU_BLOCK), 0, s, arena, off, len, n,
                       digest);
    return hipGetLastError();
}

}  // namespace honu
