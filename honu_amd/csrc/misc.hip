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


// ------------------------------------------------------------------------
// Round-trip check of a decoded batch against the rows it was encoded from
// (honu_verify_decoded). One wave per record; every byte of the 352-byte row
// is compared with the value the Go decoder must produce from the source
// row: the source byte when the field's struct is present, zero when it is
// nil (fields of nil structs stay zero, metadata.go:202-302), REGIONS_NONNIL
// added (region.go:160). Span offsets index different arenas and are not
// compared; their bytes are. ACL entries and regions are compared entry by
// entry through both rows' list offsets; a list the decode returned in place
// (HONU_ACL_INPLACE, allowed only when every source entry is present) is
// compared with its 18-byte encodings in the records arena, a region list
// returned in place (HONU_REGIONS_INPLACE, any non-empty list) by decoding its
// uvarints there (lani.DecodeUint32: <= 5 bytes, truncated to uint32).
// ------------------------------------------------------------------------
constexpr uint32_t G_ALWAYS = 0, G_IGNORE = 0xFFFFFFFFu, G_ZERO = 0xFFFFFFFEu;

// Presence bit that gates row byte b (G_ALWAYS: unconditional field,
// G_ZERO: padding, G_IGNORE: not compared bytewise).
HONU_DEV uint32_t row_gate(uint32_t b) {
    if (b < 4) return G_IGNORE;  // present: checked as a whole
    if (b < 6) return G_ALWAYS;  // permissions, flags
    if (b == 6) return HONU_HAS_VERSION;  // tombstone
    if (b == 7) return HONU_HAS_COMPRESSION;
    if (b < 11) return HONU_HAS_ENCRYPTION;  // sealing/encryption/signature alg
    if (b < 12) return G_ZERO;
    if (b < 28) return HONU_HAS_VERSION;  // region, vid, pid
    if (b < 40) return HONU_HAS_PARENT;
    if (b < 48) return HONU_HAS_VERSION;  // version_created
    if (b < 60) return HONU_HAS_SCHEMA;
    if (b < 64) return G_ZERO;
    if (b < 72) return HONU_HAS_COMPRESSION;
    if (b < 88) return G_ALWAYS;  // created, modified
    if (b < 96) return G_ZERO;
    if (b < 160) return G_ALWAYS;  // object_id, collection_id, owner, group
    if (b < 192) return HONU_HAS_PUBLISHER;
    if (b < 320) {  // spans: offsets ignored, lengths gated
        if ((b & 15) < 8) return G_IGNORE;
        const uint32_t k = (b - 192) >> 4;  // schema_name, mime, ip, ua, 4 x encryption
        return k == 0 ? HONU_HAS_SCHEMA : k == 1 ? G_ALWAYS : k < 4 ? HONU_HAS_PUBLISHER
                                                             : HONU_HAS_ENCRYPTION;
    }
    if (b < 328 || (b >= 336 && b < 344)) return G_IGNORE;  // list offsets
    return G_ALWAYS;  // acl_count, regions_count
}

// The presence bits the decoder reports for an encoded source row.
HONU_DEV uint32_t decoded_present(uint32_t p) {
    if (!(p & HONU_HAS_META)) return 0;
    p &= 0x7Fu;
    if (!(p & HONU_HAS_VERSION)) p &= ~(uint32_t)HONU_HAS_PARENT;  // Parent lives inside Version
    return p | HONU_REGIONS_NONNIL;
}

__global__ __launch_bounds__(HONU_BLOCK) void k_verify_decoded(
    const honu_meta *__restrict__ src, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ src_acl, const uint32_t *__restrict__ src_reg,
    const uint64_t *__restrict__ payload_off, const uint8_t *__restrict__ rec,
    const honu_meta *__restrict__ dec, const honu_record_info *__restrict__ info,
    const honu_acl *__restrict__ dec_acl, const uint32_t *__restrict__ dec_reg, uint64_t n,
    uint32_t *__restrict__ mismatch) {
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    const uint32_t lane = lane_id();
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block(); i < n;
         i += nwaves) {
        const honu_meta &S = src[i], &D = dec[i];
        const uint8_t *sb = reinterpret_cast<const uint8_t *>(&S);
        const uint8_t *db = reinterpret_cast<const uint8_t *>(&D);
        const uint32_t sp = S.present;
        const uint32_t pr = decoded_present(sp);
        const honu_record_info inf = info[i];
        uint32_t bad = 0;
        if (inf.data_status != HONU_OK || inf.meta_status != HONU_OK) bad |= HONU_VERIFY_STATUS;
        if (inf.data_len != payload_off[i + 1] - payload_off[i]) bad |= HONU_VERIFY_STATUS;
        bool any_nil = false;
        for (uint64_t j = lane; pr && j < S.acl_count; j += HONU_WAVE) any_nil |= !src_acl[S.acl_off + j].present;
        const bool all_present = pr && S.acl_count && !__ballot(any_nil);
        // the in-place region bit: allowed on a non-empty list only
        const bool rinpl = pr && S.regions_count && (D.present & HONU_REGIONS_INPLACE);
        const uint32_t dpr = D.present & ~(rinpl ? (uint32_t)HONU_REGIONS_INPLACE : 0u);
        const bool inpl = all_present && dpr == (pr | HONU_ACL_INPLACE);
        if (dpr != pr && !inpl) bad |= HONU_VERIFY_PRESENT;
        bool row_bad = false;
        for (uint32_t b = lane; b < sizeof(honu_meta); b += HONU_WAVE) {
            const uint32_t g = row_gate(b);
            if (g == G_IGNORE) continue;
            const bool on = pr != 0 && (g == G_ALWAYS || (g != G_ZERO && (pr & g)));
            if (db[b] != (on ? sb[b] : 0)) row_bad = true;
        }
        if (__ballot(row_bad)) bad |= HONU_VERIFY_FIELDS;
        if (bad == 0 && pr) {
            bool span_bad = false;
            const honu_span *ss = &S.schema_name, *ds = &D.schema_name;
            for (int k = 0; k < 8; k++) {
                const uint64_t len = ds[k].len;  // equal to the source's (checked above)
                for (uint64_t j = lane; j < len; j += HONU_WAVE)
                    if (var[ss[k].off + j] != rec[ds[k].off + j]) span_bad = true;
            }
            if (__ballot(span_bad)) bad |= HONU_VERIFY_SPANS;
            bool acl_bad = false;
            for (uint64_t j = lane; inpl && j < S.acl_count; j += HONU_WAVE) {
                const honu_acl &a = src_acl[S.acl_off + j];
                const uint8_t *e = rec + D.acl_off + 18 * j;
                acl_bad |= e[0] != 1 || e[17] != a.permissions;
                for (int q = 0; q < 16; q++) acl_bad |= e[1 + q] != a.client_id[q];
            }
            for (uint64_t j = lane; !inpl && j < S.acl_count; j += HONU_WAVE) {
                const honu_acl &a = src_acl[S.acl_off + j], &e = dec_acl[D.acl_off + j];
                const uint32_t *ew = reinterpret_cast<const uint32_t *>(&e);
                const uint32_t *aw = reinterpret_cast<const uint32_t *>(&a);
                if (a.present) {
                    for (int q = 0; q < 4; q++) acl_bad |= ew[q] != aw[q];
                    acl_bad |= ew[4] != (a.permissions | (1u << 8));
                } else {
                    for (int q = 0; q < 5; q++) acl_bad |= ew[q] != 0;
                }
            }
            if (__ballot(acl_bad)) bad |= HONU_VERIFY_ACL;
            bool reg_bad = false;
            for (uint64_t j = lane; !rinpl && j < S.regions_count; j += HONU_WAVE)
                reg_bad |= src_reg[S.regions_off + j] != dec_reg[D.regions_off + j];
            if (rinpl && lane == 0) {  // the list's uvarints, one after the other
                uint64_t p = D.regions_off;
                for (uint64_t j = 0; j < S.regions_count && !reg_bad; j++) {
                    uint64_t v = 0;
                    uint32_t k = 0, sh = 0;
                    for (; k < 5; k++) {
                        const uint32_t b = rec[p + k];
                        v |= (uint64_t)(b & 0x7F) << sh;
                        sh += 7;
                        if (!(b & 0x80)) break;
                    }
                    reg_bad |= k == 5 || (uint32_t)v != src_reg[S.regions_off + j];
                    p += k + 1;
                }
            }
            if (__ballot(reg_bad)) bad |= HONU_VERIFY_REGIONS;
        }
        if (lane == 0) mismatch[i] = bad;
    }
}

// ------------------------------------------------------------------------
// HBM probe (honu_hbm_probe): the part's achievable streaming rates, for the
// bench's roofline denominator next to the 8 TB/s spec. 16 bytes per lane,
// each wave a contiguous range (the layout of the codec's copy engine) with 8
// chunks per lane in flight, or grid-stride with 4 (the guide's float4 copy).
// ------------------------------------------------------------------------
template <int MODE>  // 0 read, 1 write, 2 copy (wave ranges), 3 copy (grid stride), 4 copy
                     // (wave ranges, non-temporal loads and stores)
__global__ __launch_bounds__(HONU_BLOCK) void k_hbm_probe(const u32x4 *__restrict__ a, u32x4 *__restrict__ b,
                                                          uint64_t n, uint32_t *__restrict__ sink) {
    const uint32_t lane = lane_id();
    if constexpr (MODE == 3) {
        constexpr int U = 4;
        const uint64_t stride = (uint64_t)gridDim.x * HONU_BLOCK * U;
        for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK * U + threadIdx.x; i < n; i += stride) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i + u * HONU_BLOCK < n) v[u] = a[i + u * HONU_BLOCK];
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i + u * HONU_BLOCK < n) b[i + u * HONU_BLOCK] = v[u];
        }
        return;
    }
    constexpr int U = 8;
    const uint64_t W = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    const uint64_t w = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + threadIdx.x / HONU_WAVE;
    const uint64_t lo = n * w / W, hi = n * (w + 1) / W;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = lo + lane; i < hi; i += (uint64_t)HONU_WAVE * U) {
        u32x4 v[U];
        if constexpr (MODE != 1) {
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i + u * HONU_WAVE < hi)
                    v[u] = MODE == 4 ? __builtin_nontemporal_load(a + i + u * HONU_WAVE) : a[i + u * HONU_WAVE];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i + u * HONU_WAVE >= hi) continue;
            if constexpr (MODE == 0) acc ^= v[u];
            else if constexpr (MODE == 1) b[i + u * HONU_WAVE] = u32x4{(uint32_t)i, (uint32_t)u, 1, 2};
            else if constexpr (MODE == 4) __builtin_nontemporal_store(v[u], b + i + u * HONU_WAVE);
            else b[i + u * HONU_WAVE] = v[u];
        }
    }
    if constexpr (MODE == 0)
        if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = 1;  // keeps the loads
}

hipError_t launch_hbm_probe(int mode, const void *src, void *dst, uint64_t bytes, uint32_t blocks,
                            uint32_t *sink, hipStream_t s) {
    const uint64_t n = bytes / 16;
    const u32x4 *a = reinterpret_cast<const u32x4 *>(src);
    u32x4 *b = reinterpret_cast<u32x4 *>(dst);
    switch (mode) {
    case 0: hipLaunchKernelGGL(k_hbm_probe<0>, dim3(blocks), dim3(HONU_BLOCK), 0, s, a, b, n, sink); break;
    case 1: hipLaunchKernelGGL(k_hbm_probe<1>, dim3(blocks), dim3(HONU_BLOCK), 0, s, a, b, n, sink); break;
    case 2: hipLaunchKernelGGL(k_hbm_probe<2>, dim3(blocks), dim3(HONU_BLOCK), 0, s, a, b, n, sink); break;
    case 3: hipLaunchKernelGGL(k_hbm_probe<3>, dim3(blocks), dim3(HONU_BLOCK), 0, s, a, b, n, sink); break;
    default: hipLaunchKernelGGL(k_hbm_probe<4>, dim3(blocks), dim3(HONU_BLOCK), 0, s, a, b, n, sink); break;
    }
    return hipGetLastError();
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

hipError_t launch_verify_decoded(const LaunchGeom &g, const honu_meta *src, const uint8_t *var,
                                 const honu_acl *src_acl, const uint32_t *src_reg,
                                 const uint64_t *payload_off, const uint8_t *rec,
                                 const honu_meta *dec, const honu_record_info *info,
                                 const honu_acl *dec_acl, const uint32_t *dec_reg, uint64_t n,
                                 uint32_t *mismatch, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t b = (n + 3) / 4;
    if (b > (uint64_t)g.per_record_blocks) b = g.per_record_blocks;
    hipLaunchKernelGGL(k_verify_decoded, dim3((unsigned)b), dim3(HONU_BLOCK), 0, s, src, var,
                       src_acl, src_reg, payload_off, rec, dec, info, dec_acl, dec_reg, n,
                       mismatch);
    return hipGetLastError();
}

}  // namespace honu
