// enc.hip — the header + Metadata tail encoder (object.go:24-45,
// metadata.go:108-200) with one record per GROUP of 16 lanes and no serial
// writer: the tail's layout is computed in parallel, its bytes are assembled
// in LDS and leave as aligned 16-byte stores.
//
// The tail is a fixed sequence of 52 slots in grammar order (App. A of
// SURVEY.md; kSlots below): constant and flag bytes, ULIDs and single bytes
// copied from the row, uvarints / zig-zag varints of row fields, frame bodies
// from the var arena, the ACL list and the region list. A slot's encoded
// length depends only on the row (and, for the two lists, on the tables), so
// every lane of the group evaluates 4 slots with the same branch-free code
// (kind, row offset and presence condition come from the table), and a group
// prefix sum places them. The group then builds the output in an LDS image of
// the record's tail (zeroed, every byte OR-ed in by exactly one lane): literal
// slots by the lane that evaluated them, frame bodies as aligned 16-byte
// source blocks spread over the lanes, the ACL list as 16-byte pieces computed
// from the (at most two) table entries each one straddles, region ids by a
// group scan of their lengths. The image leaves as aligned 16-byte stores,
// contiguous over the group's lanes; the chunks shared with the payload (tail
// start) and the next record (tail end) are written byte-exact, so the
// payload copy may run at the same time. Tails longer than the image are
// built in several passes.
//
// Why it exists: the one-record-per-lane encoder (lane.h encode_record_lane
// + the ACL group kernel) touches a different cache line with every lane of
// every load and store and is bound by the L1 miss queue; here
// every access of an instruction covers a few contiguous lines. Measured
// slower all the same (1M Small 2.36 vs 1.09 ms, a Large chunk 142 vs 75 us,
// profiles/r03/encode_group_ab.jsonl): a wave has 4 records in flight instead
// of 64 and each walks ~15 dependent round trips (row, list flags, every
// frame, every ACL round), and the 2 KB image per record in LDS caps a CU at
// ~48 records. So it is encode_variant 1, not the default; the output is the
// same, byte for byte (tests/test_gpu_parity.py runs both).
#include "grp.h"

// Measured slower than the default encoder (below), so it is built only into
// the A/B library (make ab, -DHONU_AB) as encode_variant 1.
#ifdef HONU_AB

namespace honu {

enum : uint8_t {
    S_NONE = 0,
    S_CONST,  // aux
    S_FLAG,   // (present & aux) ? 1 : 0
    S_RAW16,  // 16 row bytes at off
    S_BYTE,   // row byte at off
    S_BOOL,   // row byte at off != 0
    S_UV32,   // uvarint(u32 at off)
    S_UV64,   // uvarint(u64 at off)
    S_ZZ,     // uvarint(zigzag(i64 at off))
    S_FBODY,  // frame body: span at off, bytes from the var arena
    S_ACL,    // the ACL entries
    S_REGS,   // the region uvarints
};

struct SlotDesc {
    uint8_t kind, aux;
    uint16_t off;
    uint32_t cond;  // presence bits that must all be set for the slot to exist
};

#define OFF(f) ((uint16_t)offsetof(honu_meta, f))
#define V HONU_HAS_VERSION
#define PA HONU_HAS_PARENT
#define SC HONU_HAS_SCHEMA
#define PU HONU_HAS_PUBLISHER
#define EN HONU_HAS_ENCRYPTION
#define CO HONU_HAS_COMPRESSION
constexpr int NSLOT = 64;  // 52 used, 4 per lane
constexpr int SLOT_ACL = 24, SLOT_REGS = 26;
__constant__ SlotDesc kSlots[NSLOT] = {
    {S_CONST, 1, 0, 0},                                   // EncodeStruct(meta)    object.go:40
    {S_RAW16, 0, OFF(object_id), 0},                      // metadata.go:110
    {S_RAW16, 0, OFF(collection_id), 0},                  // :115
    {S_FLAG, V, 0, 0},                                    // :120 Version
    {S_UV32, 0, OFF(pid), V},                             // version.go:44-70, scalar.go:106-119
    {S_UV64, 0, OFF(vid), V},
    {S_UV32, 0, OFF(region), V},
    {S_FLAG, PA, 0, V},                                   // Parent
    {S_UV32, 0, OFF(parent_pid), V | PA},
    {S_UV64, 0, OFF(parent_vid), V | PA},
    {S_BOOL, 0, OFF(tombstone), V},
    {S_ZZ, 0, OFF(version_created), V},
    {S_FLAG, SC, 0, 0},                                   // :125 Schema, schema.go:30-53
    {S_UV64, 0, OFF(schema_name) + 8, SC},
    {S_FBODY, 0, OFF(schema_name), SC},
    {S_UV32, 0, OFF(schema_major), SC},
    {S_UV32, 0, OFF(schema_minor), SC},
    {S_UV32, 0, OFF(schema_patch), SC},
    {S_UV64, 0, OFF(mime) + 8, 0},                        // :130 MIME
    {S_FBODY, 0, OFF(mime), 0},
    {S_RAW16, 0, OFF(owner), 0},                          // :135
    {S_RAW16, 0, OFF(group), 0},                          // :140
    {S_BYTE, 0, OFF(permissions), 0},                     // :145
    {S_UV64, 0, OFF(acl_count), 0},                       // :151
    {S_ACL, 0, 0, 0},                                     // :157-162, acls.go:26-39
    {S_UV64, 0, OFF(regions_count), 0},                   // :164, region.go:137-152
    {S_REGS, 0, 0, 0},
    {S_FLAG, PU, 0, 0},                                   // :169 Publisher, provenance.go:34-57
    {S_RAW16, 0, OFF(publisher_id), PU},
    {S_RAW16, 0, OFF(client_id), PU},
    {S_UV64, 0, OFF(ip_address) + 8, PU},
    {S_FBODY, 0, OFF(ip_address), PU},
    {S_UV64, 0, OFF(user_agent) + 8, PU},
    {S_FBODY, 0, OFF(user_agent), PU},
    {S_FLAG, EN, 0, 0},                                   // :174 Encryption, encryption.go:51-89
    {S_UV64, 0, OFF(public_key_id) + 8, EN},
    {S_FBODY, 0, OFF(public_key_id), EN},
    {S_UV64, 0, OFF(encryption_key) + 8, EN},
    {S_FBODY, 0, OFF(encryption_key), EN},
    {S_UV64, 0, OFF(hmac_secret) + 8, EN},
    {S_FBODY, 0, OFF(hmac_secret), EN},
    {S_UV64, 0, OFF(signature) + 8, EN},
    {S_FBODY, 0, OFF(signature), EN},
    {S_BYTE, 0, OFF(sealing_alg), EN},
    {S_BYTE, 0, OFF(encryption_alg), EN},
    {S_BYTE, 0, OFF(signature_alg), EN},
    {S_FLAG, CO, 0, 0},                                   // :179 Compression, compression.go:40-53
    {S_BYTE, 0, OFF(compression_alg), CO},
    {S_ZZ, 0, OFF(compression_level), CO},
    {S_BYTE, 0, OFF(flags), 0},                           // :184
    {S_ZZ, 0, OFF(created), 0},                           // :189
    {S_ZZ, 0, OFF(modified), 0},                          // :194
};
// the frame-body slots, in grammar order
__constant__ uint8_t kBodySlots[8] = {14, 19, 31, 33, 36, 38, 40, 42};
#undef V
#undef PA
#undef SC
#undef PU
#undef EN
#undef CO

#ifndef ENC_WIN
#define ENC_WIN 2048  // image bytes per record (one pass holds tails up to ~ENC_WIN - 16)
#endif
constexpr uint32_t EWIN = ENC_WIN;
constexpr uint32_t EREC = GROW + 4 * NSLOT + EWIN + 32;  // row, slot starts, image + slack
constexpr uint32_t ERECS = HONU_BLOCK / GRP;

// OR the first n (<= 16) bytes of lo||hi into the image at byte rel (any
// int64: dwords outside [0, EWIN) are dropped — another pass owns them).
HONU_DEV void img_or(uint32_t *img, int64_t rel, uint64_t lo, uint64_t hi, uint32_t n) {
    if (n < 16) {
        if (n <= 8) {
            lo &= n == 8 ? ~0ull : ((1ull << (8 * n)) - 1);
            hi = 0;
        } else {
            hi &= (1ull << (8 * (n - 8))) - 1;
        }
    }
    const int64_t d0 = rel >> 2;  // floor
    const uint32_t sh = (uint32_t)(rel & 3) * 8;
    const uint32_t w[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t cur = j < 4 ? w[j] : 0, prev = j > 0 ? w[j - 1] : 0;
        const uint32_t v = sh ? (cur << sh) | (prev >> (32 - sh)) : cur;
        const int64_t d = d0 + j;
        if (v && d >= 0 && d < (int64_t)(EWIN / 4)) atomicOr(&img[d], v);
    }
}

// Length and (for literal slots) bytes of slot d of the row in LDS.
HONU_DEV uint32_t slot_eval(const SlotDesc d, const uint8_t *row, uint32_t pr, uint64_t acl_bytes,
                            uint64_t reg_bytes, uint64_t &lo, uint64_t &hi) {
    const uint32_t a8 = d.off & ~7u, s = (d.off & 7u) * 8;
    const uint64_t x0 = *reinterpret_cast<const uint64_t *>(row + a8);
    const uint64_t x1 = *reinterpret_cast<const uint64_t *>(row + a8 + 8);
    const uint64_t f = s ? (x0 >> s) : x0;  // field bits from off
    uint64_t uv = 0;
    uint32_t len = 1;
    lo = hi = 0;
    switch (d.kind) {
    case S_CONST: lo = d.aux; break;
    case S_FLAG: lo = (pr & d.aux) ? 1 : 0; break;
    case S_RAW16: lo = x0; hi = x1; len = 16; break;  // ULIDs are 16-aligned
    case S_BYTE: lo = f & 0xFF; break;
    case S_BOOL: lo = (f & 0xFF) ? 1 : 0; break;
    case S_UV32: uv = f & 0xFFFFFFFFull; break;
    case S_UV64: uv = x0; break;
    case S_ZZ: uv = zigzag((int64_t)x0); break;
    case S_FBODY: len = (uint32_t)x1; break;  // span.len (bodies: < 2^32, checked by the caller)
    case S_ACL: len = (uint32_t)acl_bytes; break;
    case S_REGS: len = (uint32_t)reg_bytes; break;
    default: len = 0; break;
    }
    if (d.kind == S_UV32 || d.kind == S_UV64 || d.kind == S_ZZ) len = uvarint_bytes(uv, lo, hi);
    if ((pr & d.cond) != d.cond) len = 0;
    return len;
}

template <int G>
HONU_DEV void encode_tail_grp_one(uint64_t i, uint8_t *rs, const honu_meta *__restrict__ meta,
                                  const uint8_t *__restrict__ var, const honu_acl *__restrict__ acl,
                                  const uint32_t *__restrict__ reg,
                                  const uint64_t *__restrict__ payload_off, uint8_t *__restrict__ out,
                                  uint64_t out_cap, const uint64_t *__restrict__ out_off,
                                  int32_t *__restrict__ status) {
    const uint32_t r = lane_id() & (G - 1);
    uint8_t *row = rs;
    uint32_t *starts = reinterpret_cast<uint32_t *>(rs + GROW);
    uint32_t *img = reinterpret_cast<uint32_t *>(rs + GROW + 4 * NSLOT);
    // independent loads first
    const int32_t sti = status[i];
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    const uint64_t dlen = payload_off[i + 1] - payload_off[i];
    grp_stage_row<G>(row, meta + i, r);
    wave_sync();
    const bool go = sti == HONU_OK && end <= out_cap;
    if (sti == HONU_OK && end > out_cap && r == 0) status[i] = HONU_ERR_CAPACITY;
    const honu_meta &m = *reinterpret_cast<const honu_meta *>(row);
    const uint32_t pr = m.present;
    const uint64_t na = go ? m.acl_count : 0, ao = m.acl_off;
    const uint64_t nr = go ? m.regions_count : 0, ro = m.regions_off;
    // the lists' encoded bytes (a nil entry is 1 byte)
    uint64_t ab = 0, rb = 0;
    uint32_t nil = 0;
    for (uint64_t k = r; k < na; k += G) {
        const uint32_t p = acl[ao + k].present;
        ab += p ? 18 : 1;
        nil |= p ? 0 : 1;
    }
    for (uint64_t k = r; k < nr; k += G) rb += uvarint_len(reg[ro + k]);
    ab = grp_sum64<G>(ab);
    rb = grp_sum64<G>(rb);
    nil = grp_sum<G>(nil);
    const uint32_t hn = uvarint_len(dlen);
    const uint64_t T0 = beg + 1 + hn + dlen;
    if (go && end - T0 >= (1ull << 31)) {  // a tail of 2 GiB or more: the lane writer (lane.h)
        if (r == 0) encode_record_lane<false, 0>(m, var, acl, reg, dlen, beg, end, out, nullptr);
        return;
    }
    // slots 4r .. 4r+3: lengths, literal bytes, starts (relative to T0)
    uint64_t slo[4], shi[4];
    uint32_t slen[4];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const SlotDesc d = kSlots[4 * r + k];
        slen[k] = go ? slot_eval(d, row, pr, ab, rb, slo[k], shi[k]) : 0;
        mine += slen[k];
    }
    const uint32_t base = grp_excl_scan<G>(mine, r);
    {
        uint32_t s = base;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            starts[4 * r + k] = s;
            s += slen[k];
        }
    }
    wave_sync();
    if (go && r == 0) {  // header: version byte + uvarint(len data)   object.go:30,35
        uint64_t lo, hi;
        uvarint_bytes(dlen, lo, hi);
        out[beg] = HONU_STORAGE_VERSION;
        for (uint32_t j = 0; j < hn; j++)
            out[beg + 1 + j] = (uint8_t)(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8)));
    }
    const uint64_t X0 = T0 & ~15ull;
    const uint64_t E = go ? end : X0;  // no pass for a record that is not encoded
    const uint32_t acl_at = starts[SLOT_ACL], regs_at = starts[SLOT_REGS];
    for (uint64_t WX = X0; WX < E; WX += EWIN) {  // group-uniform passes
        u32x4 *img4 = reinterpret_cast<u32x4 *>(img);
        for (uint32_t c = r; c < EWIN / 16; c += G) img4[c] = u32x4{0, 0, 0, 0};
        wave_sync();
        const int64_t t0 = (int64_t)(T0 - WX);  // tail start in the image
        // literal slots
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint8_t kind = kSlots[4 * r + k].kind;
            if (slen[k] && kind != S_FBODY && kind != S_ACL && kind != S_REGS)
                img_or(img, t0 + starts[4 * r + k], slo[k], shi[k], slen[k]);
        }
        // frame bodies: aligned 16-byte source blocks over the lanes
        for (int b = 0; b < 8; b++) {
            const uint32_t si = kBodySlots[b];
            const SlotDesc d = kSlots[si];
            if ((pr & d.cond) != d.cond) continue;  // group-uniform
            const honu_span sp = *reinterpret_cast<const honu_span *>(row + d.off);
            if (!sp.len) continue;
            const uint8_t *src = var + sp.off;
            const uint32_t a = (uint32_t)((uint64_t)src & 15);
            const u32x4 *A = reinterpret_cast<const u32x4 *>(src - a);
            const int64_t at = t0 + starts[si] - a;  // image byte of source block 0
            const uint64_t nblk = (a + sp.len + 15) >> 4;
            // only the blocks that land in this pass
            const int64_t k0 = at >= 0 ? 0 : (-at) >> 4;
            for (uint64_t k = k0 + r; k < nblk && at + 16 * (int64_t)k < (int64_t)EWIN; k += G) {
                const u32x4 v = A[k];
                const int lo_b = k == 0 ? (int)a : 0;
                const int64_t hb = (int64_t)a + (int64_t)sp.len - 16 * (int64_t)k;
                const int hi_b = hb > 16 ? 16 : (int)hb;
                const uint64_t lo = (((uint64_t)v.y << 32) | v.x) & bytemask64(lo_b, hi_b);
                const uint64_t hi = (((uint64_t)v.w << 32) | v.z) & bytemask64(lo_b - 8, hi_b - 8);
                img_or(img, at + 16 * (int64_t)k, lo, hi, 16);
            }
        }
        // ACL list
        if (na) {
            const int64_t at = t0 + acl_at;
            if (!nil) {  // 18 bytes per entry: 16-byte pieces from <= 2 entries each
                const uint64_t npc = (18 * na + 15) >> 4;
                const int64_t k0 = at >= 0 ? 0 : (-at) >> 4;
                for (uint64_t k = k0 + r; k < npc && at + 16 * (int64_t)k < (int64_t)EWIN; k += G) {
                    const u32x4 v = acl_chunk(acl + ao, na, 0, 16 * k);
                    const uint64_t rem = 18 * na - 16 * k;
                    img_or(img, at + 16 * (int64_t)k, ((uint64_t)v.y << 32) | v.x,
                           ((uint64_t)v.w << 32) | v.z, rem < 16 ? (uint32_t)rem : 16);
                }
            } else if (r == 0) {  // nil entries: 00, else 01 | ClientID | Permissions
                int64_t p = at;
                for (uint64_t j = 0; j < na; j++) {
                    if (acl[ao + j].present) {
                        uint32_t d5[5];
                        acl_enc_words(acl + ao + j, d5);
                        img_or(img, p, ((uint64_t)d5[1] << 32) | d5[0], ((uint64_t)d5[3] << 32) | d5[2], 16);
                        img_or(img, p + 16, d5[4], 0, 2);
                        p += 18;
                    } else {
                        p += 1;  // the byte stays 0
                    }
                }
            }
        }
        // regions: one uvarint per lane per round, placed by a group scan
        {
            int64_t at = t0 + regs_at;
            for (uint64_t k0 = 0; k0 < nr; k0 += G) {  // group-uniform
                const uint64_t k = k0 + r;
                uint64_t lo = 0, hi = 0;
                const uint32_t l = k < nr ? uvarint_bytes(reg[ro + k], lo, hi) : 0;
                const uint32_t o = grp_excl_scan<G>(l, r);
                if (l) img_or(img, at + o, lo, hi, l);
                at += grp_sum<G>(l);
            }
        }
        wave_sync();
        // the image's chunks [WX, WX + EWIN) ∩ [T0, E) to memory
        const uint64_t wend = WX + EWIN < E ? WX + EWIN : E;
        const uint64_t nch = (wend - WX + 15) >> 4;
        const u32x4 *img4c = reinterpret_cast<const u32x4 *>(img);
        for (uint64_t c = r; c < nch; c += G) {
            const uint64_t X = WX + 16 * c;
            const u32x4 v = img4c[c];
            const uint32_t from = X < T0 ? (uint32_t)(T0 - X) : 0;
            const uint32_t to = X + 16 > E ? (uint32_t)(E - X) : 16;
            if (from == 0 && to == 16) {
                *reinterpret_cast<u32x4 *>(out + X) = v;
            } else if (to > from) {  // shared with the payload or the next record
                LaneWriterT<0>::store_bytes(out + X, from, to, ((uint64_t)v.y << 32) | v.x,
                                            ((uint64_t)v.w << 32) | v.z);
            }
        }
        wave_sync();  // the image is the next pass's
    }
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_tail_grp(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[ERECS * EREC];
    uint8_t *rs = smem + (threadIdx.x / G) * EREC;
    // groups of one wave take consecutive records; the loop is group-uniform
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        encode_tail_grp_one<G>(i, rs, meta, var, acl, reg, payload_off, out, out_cap, out_off, status);
}

hipError_t launch_encode_tail_grp(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                  const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                  uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                  int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_tail_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta,
                       var, acl, reg, payload_off, n, out, out_cap, out_off, status);
    return hipGetLastError();
}

#undef OFF

}  // namespace honu
#endif  // HONU_AB
