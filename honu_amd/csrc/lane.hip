// lane.hip — per-record kernels with one record per LANE (see lane.h for
// why): the header/tail encoder of the default encode (the ACL entries are
// left to k_encode_acl_grp) and the headers-only decode (honu_decode_headers,
// honu_decode_data).
#include "kernels.h"
#include "lane.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))

// ------------------------------------------------------------------------
// encode: header + Metadata tail (object.go:24-45, metadata.go:108-200)
// ------------------------------------------------------------------------
#ifndef ENC_RING
#define ENC_RING 8  // chunks in the writer's LDS ring per lane (0: direct stores)
#endif
// ENC_PF: the prefetching encoder (lane.h encode_record_pf)
#ifndef ENC_PF
#define ENC_PF 0
#endif

// ENC_ROWS_LDS: the wave's 64 rows (contiguous, 22.5 KB) reach the lanes
// through LDS: two passes of 32 rows, each 11 coalesced 1 KB global_load_lds
// instructions, then every lane of the pass reads its row from LDS. Loaded
// per lane, each of a row's 22 16-byte loads touches 64 cache lines (one per
// record); the L1's per-line load path is what bounds this kernel.
#ifndef ENC_ROWS_LDS
#define ENC_ROWS_LDS 0
#endif
#ifndef ENC_ROW_PASS_N
#define ENC_ROW_PASS_N 32
#endif
constexpr uint32_t ENC_ROW_PASS = ENC_ROW_PASS_N;                                   // rows per staging pass
constexpr uint32_t ENC_ROW_BYTES = ENC_ROW_PASS * sizeof(honu_meta);     // 11,264 = 11 x 1 KB
constexpr uint32_t ENC_RING_BYTES = (ENC_RING > 0 ? ENC_RING : 1) * HONU_WAVE * 16;
constexpr uint32_t ENC_WAVE_BYTES = ENC_ROWS_LDS && ENC_ROW_BYTES > ENC_RING_BYTES ? ENC_ROW_BYTES : ENC_RING_BYTES;
static_assert(ENC_ROW_BYTES % 1024 == 0, "whole DMA instructions");

// returns the ACL list position (as acl_out: | ACL_ALL_PRESENT when the
// partial end chunks were written), NO_ACL_POS for a record not encoded
constexpr uint64_t NO_ACL_POS = ~0ull;
template <bool SKIP_ACL>
HONU_DEV uint64_t k_encode_meta_lane_one(uint64_t i, const honu_meta &m, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    uint64_t *__restrict__ acl_out, u32x4 *ring) {
    if (status[i] != HONU_OK) return NO_ACL_POS;
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    if (end > out_cap) {
        status[i] = HONU_ERR_CAPACITY;
        return NO_ACL_POS;
    }
    const uint64_t dlen = payload_off[i + 1] - payload_off[i];
#if ENC_PF
    static_assert(SKIP_ACL, "prefetch form writes the ACL ends only");
    const uint64_t pos = encode_record_pf<ENC_RING>(m, var, acl, reg, dlen, beg, end, out, ring);
#else
    const uint64_t pos = encode_record_lane<SKIP_ACL, SKIP_ACL ? ENC_RING : 0>(m, var, acl, reg, dlen, beg, end,
                                                                           out, ring);
#endif
    if (SKIP_ACL && acl_out) acl_out[i] = pos;
    return pos;
}

// a lane's row straight from global memory (the loads cannot pass the output
// stores, so the whole row is loaded first)
HONU_DEV void load_row(const honu_meta *__restrict__ src, honu_meta &m) {
    const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
    u32x4 *d = reinterpret_cast<u32x4 *>(&m);
#pragma unroll
    for (int k = 0; k < 22; k++) d[k] = s[k];
}

// rows [t0, t0 + 64) of meta (clipped to n) into this lane's m, through the
// wave's LDS area (ENC_ROW_BYTES): wave-uniform call
HONU_DEV void stage_rows(uint8_t *area, const honu_meta *__restrict__ meta, uint64_t t0, uint64_t n,
                         honu_meta &m) {
    const uint32_t lane = lane_id();
    const uint8_t *src = reinterpret_cast<const uint8_t *>(meta + t0);
#pragma unroll 1
    for (uint32_t h = 0; h < HONU_WAVE / ENC_ROW_PASS; h++) {
        const uint64_t r0 = t0 + h * ENC_ROW_PASS;
        const uint64_t rows = r0 >= n ? 0 : (n - r0 < ENC_ROW_PASS ? n - r0 : ENC_ROW_PASS);
        if (!rows) break;  // wave-uniform
        const uint32_t bytes = (uint32_t)rows * (uint32_t)sizeof(honu_meta);
        wave_sync();  // the area's previous reads (ring drains, pass h - 1) are done
#pragma unroll
        for (uint32_t k = 0; k < ENC_ROW_BYTES / 1024; k++)
            if (1024 * k + 16 * lane < bytes)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(src + h * ENC_ROW_BYTES + 1024 * k + 16 * lane),
                    (__attribute__((address_space(3))) void *)(area + 1024 * k), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
        // every lane reads (its own row in its pass), then keeps what is its
        // own by a per-dword select: no branch, so the row lives in one set
        // of registers (a branch per pass kept two copies: 246 VGPRs)
        const bool mine = lane / ENC_ROW_PASS == h;
        const u32x4 *s = reinterpret_cast<const u32x4 *>(area + (lane % ENC_ROW_PASS) * sizeof(honu_meta));
        u32x4 *d = reinterpret_cast<u32x4 *>(&m);
#pragma unroll
        for (int k = 0; k < 22; k++) {
            const u32x4 v = s[k];
            d[k] = u32x4{mine ? v.x : d[k].x, mine ? v.y : d[k].y, mine ? v.z : d[k].z, mine ? v.w : d[k].w};
        }
    }
    wave_sync();  // the area becomes the writer's ring
}

// ------------------------------------------------------------------------
// encode_variant 2: the ACL lists' whole chunks written by the same kernel,
// wave-cooperatively once the tile's 64 records are done, instead of by
// k_encode_acl_grp (which re-reads every row and list position). The lists'
// table rows (20 bytes each, a list contiguous in the table) are staged into
// the wave's LDS area round after round by global_load_lds - each lane's list
// as its own run of 16-byte blocks, as fused.hip's AclStage does for the
// decode - then lane k of a pass builds output chunk k of the round (the
// chunks of the tile's lists in record order, so consecutive lanes store one
// record's consecutive 16 bytes) from the <= 2 entries it straddles.
// (metadata.go:157-162, acls.go:26-39)
// ------------------------------------------------------------------------
// the 18 encoded bytes of the entry whose table row starts at LDS byte q
// (dword aligned) as 4.5 words (acl_enc_words from LDS)
HONU_DEV void acl_enc_lds(const uint8_t *area, uint32_t q, uint32_t d[5]) {
    const __attribute__((address_space(3))) uint32_t *w =
        (const __attribute__((address_space(3))) uint32_t *)(area + q);
    const uint32_t e0 = w[0], e1 = w[1], e2 = w[2], e3 = w[3], e4 = w[4];
    d[0] = 1u | (e0 << 8);
    d[1] = (e0 >> 24) | (e1 << 8);
    d[2] = (e1 >> 24) | (e2 << 8);
    d[3] = (e2 >> 24) | (e3 << 8);
    d[4] = (e3 >> 24) | ((e4 & 0xFF) << 8);
}

// Wave-uniform call: the whole chunks [ceil16(P), floor16(P + 18 na)) of every
// lane whose fl is set (every entry present; its partial end chunks already
// written by the lane), through `area` (slots x 16 bytes of LDS).
HONU_DEV void tile_acl_write(uint8_t *area, uint32_t slots, const honu_acl *__restrict__ acl,
                             uint8_t *__restrict__ out, bool fl, uint64_t P, uint64_t na, uint64_t ao) {
    const uint32_t lane = lane_id();
    const uint64_t X0 = (P + 15) & ~15ull, X1 = (P + 18 * na) & ~15ull;
    const uint64_t nch = fl && X1 > X0 ? (X1 - X0) >> 4 : 0;
    const uint64_t byte0 = ao * sizeof(honu_acl);
    const uint32_t phase = (uint32_t)(byte0 & 15);
    const uint64_t blk0 = byte0 >> 4;
    const uint64_t nbl = nch ? ((byte0 + na * sizeof(honu_acl) + 15) >> 4) - blk0 : 0;
    const bool staged = nch && nbl <= slots;
    if (nch && !staged) {  // a list longer than the staging area: entries straight from memory
        for (uint64_t X = X0; X < X1; X += 16) *reinterpret_cast<u32x4 *>(out + X) = acl_chunk(acl + ao, na, P, X);
    }
    const uint8_t *src = reinterpret_cast<const uint8_t *>(acl);
    uint32_t nbtot;
    const uint32_t nb = staged ? (uint32_t)nbl : 0;
    const uint32_t B = wave_excl32(nb, nbtot);
    uint32_t start = 0, r0 = 0;
    while (start < nbtot) {  // wave-uniform: one staging round
        const uint32_t r1 = (uint32_t)__builtin_popcountll(__ballot(B + nb <= start + slots));
        const uint32_t stop = r1 < HONU_WAVE ? __builtin_amdgcn_readlane(B, r1) : nbtot;
        wave_sync();  // the area's previous readers are done
        for (uint32_t k = 0; k * HONU_WAVE < slots; k++) {  // slot s <- block start + s of the wave's lists
            const uint32_t w0 = start + HONU_WAVE * k;
            if (w0 >= stop) break;  // wave-uniform
            const uint32_t r = (uint32_t)__builtin_popcountll(__ballot(B <= w0)) - 1;
            uint32_t rb = __builtin_amdgcn_readlane(B, r);
            uint64_t rg = readlane64(blk0, r);
            uint64_t heads = __ballot(nb && B > w0 && B < w0 + HONU_WAVE);
            while (heads) {
                const uint32_t h = (uint32_t)__builtin_ctzll(heads);
                heads &= heads - 1;
                const uint32_t hb = __builtin_amdgcn_readlane(B, h);
                const uint64_t hg = readlane64(blk0, h);
                if (lane >= hb - w0) {
                    rb = hb;
                    rg = hg;
                }
            }
            const uint32_t g = w0 + lane;
            if (g < stop)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(src + 16 * (rg + (g - rb))),
                    (__attribute__((address_space(3))) void *)(area + 1024 * k), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
        // the round's chunks: lane e of a pass takes chunk e, in lane order
        const bool in = lane >= r0 && lane < r1 && nb;
        uint32_t ctot;
        const uint32_t cpre = wave_excl32(in ? (uint32_t)nch : 0, ctot);
        const uint32_t lbase = 16 * (B - start) + phase;  // LDS byte of the list's entry 0
        for (uint32_t w0 = 0; w0 < ctot; w0 += HONU_WAVE) {  // wave-uniform
            // the owner of chunk w0: the last lane with cpre <= w0 (cpre is
            // non-decreasing over all lanes; lanes outside the round add 0)
            const uint32_t r = (uint32_t)__builtin_popcountll(__ballot(cpre <= w0)) - 1;
            uint32_t rp = __builtin_amdgcn_readlane(cpre, r), rl = __builtin_amdgcn_readlane(lbase, r);
            uint64_t rP = readlane64(P, r), rX = readlane64(X0, r), rn = readlane64(na, r);
            uint64_t heads = __ballot(in && nch && cpre > w0 && cpre < w0 + HONU_WAVE);
            while (heads) {
                const uint32_t h = (uint32_t)__builtin_ctzll(heads);
                heads &= heads - 1;
                const uint32_t hp = __builtin_amdgcn_readlane(cpre, h), hl = __builtin_amdgcn_readlane(lbase, h);
                const uint64_t hP = readlane64(P, h), hX = readlane64(X0, h), hn = readlane64(na, h);
                if (lane >= hp - w0) {
                    rp = hp;
                    rl = hl;
                    rP = hP;
                    rX = hX;
                    rn = hn;
                }
            }
            const uint32_t e = w0 + lane;
            if (e < ctot) {
                const uint64_t X = rX + 16ull * (e - rp);
                const uint64_t j0 = (X - rP) / 18;
                uint32_t b[10];
                acl_enc_lds(area, rl + 20 * (uint32_t)j0, b);
                b[5] = b[6] = b[7] = b[8] = b[9] = 0;
                if (j0 + 1 < rn) {  // entry j0 + 1 starts at byte 18 of b
                    uint32_t d[5];
                    acl_enc_lds(area, rl + 20 * (uint32_t)j0 + 20, d);
                    b[4] = (b[4] & 0xFFFF) | (d[0] << 16);
                    b[5] = (d[0] >> 16) | (d[1] << 16);
                    b[6] = (d[1] >> 16) | (d[2] << 16);
                    b[7] = (d[2] >> 16) | (d[3] << 16);
                    b[8] = (d[3] >> 16) | (d[4] << 16);
                }
                const uint32_t off = (uint32_t)(X - (rP + 18 * j0));
                const uint32_t q = off >> 2, sh = off & 3;
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    uint32_t w0_ = b[k], w1_ = b[k + 1];
#pragma unroll
                    for (int t = 1; t <= 4; t++)
                        if ((uint32_t)t == q) {
                            w0_ = b[t + k];
                            w1_ = b[t + k + 1];
                        }
                    o[k] = __builtin_amdgcn_alignbyte(w1_, w0_, sh);
                }
                *reinterpret_cast<u32x4 *>(out + X) = u32x4{o[0], o[1], o[2], o[3]};
            }
        }
        start = stop;
        r0 = r1;
    }
    wave_sync();  // the area is the writer's ring again
}

// a list with nil entries, serially by its lane: 00 for a nil entry, else
// 01 | ClientID | Permissions (acls.go:26-39)
HONU_DEV void lane_acl_serial(const honu_acl *__restrict__ A, uint64_t na, uint8_t *__restrict__ out, uint64_t p) {
    for (uint64_t j = 0; j < na; j++) {
        if (A[j].present) {
            uint32_t d[5];
            acl_enc_words(A + j, d);
            for (int b = 0; b < 18; b++) out[p + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
            p += 18;
        } else {
            out[p++] = 0;
        }
    }
}

#ifndef ENC_ACL_SLOTS
#define ENC_ACL_SLOTS 768  // LDS blocks per ACL staging round (encode_variant 2)
#endif

template <bool SKIP_ACL>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_meta_lane(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    uint64_t *__restrict__ acl_out, int acl_in) {
    // per wave: the writer's ring (slot-major, lanes adjacent), with
    // ENC_ROWS_LDS first the row staging, and with acl_in (encode_variant 2)
    // the ACL staging rounds after the tile's records
    constexpr uint32_t AREA = ENC_WAVE_BYTES > ENC_ACL_SLOTS * 16 ? ENC_WAVE_BYTES : ENC_ACL_SLOTS * 16;
    __shared__ __attribute__((aligned(16))) uint8_t smem[HONU_WAVES_PER_BLOCK * AREA];
    uint8_t *area = smem + (threadIdx.x / HONU_WAVE) * AREA;
    u32x4 *ring = reinterpret_cast<u32x4 *>(area) + lane_id();
    // wave-uniform loop over tiles of 64 records (one per lane)
    for (uint64_t t0 = (uint64_t)blockIdx.x * HONU_BLOCK + (threadIdx.x & ~(uint64_t)(HONU_WAVE - 1)); t0 < n;
         t0 += (uint64_t)gridDim.x * HONU_BLOCK) {
        const uint64_t i = t0 + lane_id();
        ESTAMP(0);  // entered
        honu_meta m;
#if ENC_ROWS_LDS
        stage_rows(area, meta, t0, n, m);
#else
        if (i < n) load_row(meta + i, m);
#endif
        uint64_t pos = NO_ACL_POS;
        if (i < n)
            pos = k_encode_meta_lane_one<SKIP_ACL>(i, m, var, acl, reg, payload_off, out, out_cap, out_off,
                                                   status, acl_in ? nullptr : acl_out, ring);
        if (SKIP_ACL && acl_in) {  // wave-uniform
            const uint64_t na = i < n ? m.acl_count : 0;
            const bool enc = pos != NO_ACL_POS && na;
            const bool all = enc && (pos & ACL_ALL_PRESENT);
            if (enc && !all) lane_acl_serial(acl + m.acl_off, na, out, pos);
            tile_acl_write(area, AREA / 16 / HONU_WAVE * HONU_WAVE, acl, out, all, pos & ~ACL_ALL_PRESENT, na,
                           i < n ? m.acl_off : 0);
        }
    }
}

#undef OFF

// ------------------------------------------------------------------------
// headers only: StorageVersion, Data, Tombstone (object.go:47-52,85-134)
// ------------------------------------------------------------------------
// SPANS: also hand the payload's absolute offset (scratch.data_src) and its
// 16-byte aligned size (counts[i], one column) to honu_decode_data's scan and
// copy.
template <bool SPANS>
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_headers(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_record_info *__restrict__ info, DecodeScratch *__restrict__ scratch,
    uint64_t *__restrict__ counts) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK) {
        const uint64_t beg = rec_off[i], end = rec_off[i + 1];
        const uint64_t len = end - beg;
        uint32_t ver = 0;
        int64_t d = -1, b = -1;
        if (len) {
            uint64_t lo, hi;
            lane_fetch16(rec, beg, end, lo, hi);
            ver = (uint32_t)(lo & 0xFF);
            if (len >= 3) {  // dataLength: Uvarint(o[1 : min(11, len-1)])
                const uint32_t wl = (uint32_t)(len - 2 < 10 ? len - 2 : 10);
                uint64_t x;
                const uint32_t k = uvarint_window((lo >> 8) | (hi << 56), hi >> 8, wl, x);
                if (k) {
                    d = (int64_t)x;
                    b = k;
                }
            }
        }
        const bool v1 = ver == HONU_STORAGE_VERSION;
        honu_record_info inf;
        inf.data_off = 0;
        inf.data_len = 0;
        if (!v1) inf.data_status = HONU_ERR_BAD_VERSION;
        else if (d < 0) inf.data_status = HONU_ERR_MALFORMED;
        else if (d == 0) inf.data_status = HONU_OK;
        else if ((uint64_t)d > len - 1 - (uint64_t)b) inf.data_status = HONU_ERR_PANIC;
        else {
            inf.data_status = HONU_OK;
            inf.data_off = beg + 1 + (uint64_t)b;
            inf.data_len = (uint64_t)d;
        }
        inf.meta_status = HONU_UNPARSED;
        inf.storage_version = (uint8_t)ver;
        inf.tombstone = (v1 && d == 0) ? 1 : 0;
#pragma unroll
        for (int k = 0; k < 6; k++) inf._pad[k] = 0;
        if constexpr (SPANS) {
            scratch[i].data_src = inf.data_off;
            counts[i] = (inf.data_len + 15) & ~15ull;
        }
        store_info(info + i, inf);
    }
}

// honu_decode_data, after the scan: data_off relative to the data arena, or
// HONU_ERR_CAPACITY for a payload that does not fit (then nothing is copied).
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_data_place(
    uint64_t n, honu_record_info *__restrict__ info, const uint64_t *__restrict__ offs,
    uint64_t data_cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK) {
        honu_record_info *p = info + i;
        if (p->data_status != HONU_OK || !p->data_len) continue;
        const uint64_t o = offs[i];
        if (o > data_cap || p->data_len > data_cap - o) {
            p->data_status = HONU_ERR_CAPACITY;
            p->data_off = 0;
            p->data_len = 0;
        } else {
            p->data_off = o;
        }
    }
}

static dim3 flat_grid(uint64_t n) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(b > 65536 ? 65536 : b));
}

hipError_t launch_decode_headers(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                 honu_record_info *info, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_headers<false>, flat_grid(n), dim3(HONU_BLOCK), 0, s, rec, rec_off,
                       n, info, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_decode_spans(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_record_info *info, DecodeScratch *scratch, uint64_t *counts,
                               hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_headers<true>, flat_grid(n), dim3(HONU_BLOCK), 0, s, rec, rec_off, n,
                       info, scratch, counts);
    return hipGetLastError();
}

hipError_t launch_decode_data_place(uint64_t n, honu_record_info *info, const uint64_t *offs,
                                    uint64_t data_cap, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_data_place, flat_grid(n), dim3(HONU_BLOCK), 0, s, n, info, offs,
                       data_cap);
    return hipGetLastError();
}

static dim3 lane_grid(uint64_t n, int cap) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(cap > 0 && b > (uint64_t)cap ? (uint64_t)cap : b));
}

hipError_t launch_encode_meta_lane(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                   const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                   uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                   int32_t *status, uint64_t *acl_out, int acl_in, int max_blocks,
                                   hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!acl_out && !acl_in) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_encode_meta_lane<true>, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, var,
                       acl, reg, payload_off, n, out, out_cap, out_off, status, acl_out, acl_in);
    return hipGetLastError();
}

}  // namespace honu

#ifdef HONU_ENC_TIMING
extern "C" int32_t honu_debug_enc_stamps(void *host, uint64_t waves) {
    if (waves > (1 << 16)) waves = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(honu::g_enc_stamps),
                               waves * ENC_STAMPS * sizeof(uint64_t)) == hipSuccess ? 0 : -3;
}
#endif
