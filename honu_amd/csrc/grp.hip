// grp.hip — the per-record metadata kernels with one record per GROUP of G
// lanes (record_variant 2; the size pass and the fill also in variant 0).
//
// Why groups: with one record per lane (lane.hip) each load instruction
// touches 64 different cache lines, one per record, and a CU's 32 KiB L1
// cannot keep the lines of all resident waves from one field to the next, so
// L2 serves every field again (measured at 1M Small: decode parse 0.69 ns,
// decode fill 1.37 ns, encode 1.24 ns per record — 2-6x the HBM time of the
// bytes those kernels move). With one record per wave (encode.hip/decode.hip)
// the serial lani walk is issued once per record for 64 lanes. Here G lanes
// share one record:
//   * the record's bytes move between HBM and LDS once, as aligned 16-byte
//     accesses spread over the group (row image, Metadata tail);
//   * the serial lani walk runs on LDS with every lane of the group in
//     lockstep — the lanes agree on every position, nothing is broadcast;
//   * the lists (ACL entries, regions) and the frame bytes are spread over the
//     group's lanes, positions from group ballots and prefix sums;
//   * the encoder builds the tail in a zeroed LDS stage with OR writes (every
//     byte has exactly one writer, so order does not matter) and leaves it as
//     aligned 16-byte stores; bytes it does not own (payload, neighbours) are
//     never written.
// Tails longer than the stage are built in several windows (encode) or walked
// straight from global memory (decode) by the same code.
#include "kernels.h"
#include "lane.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))
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

// ------------------------------------------------------------------------
// encode stage: OR writes into a zeroed LDS window [W, W + GCAP) of the
// output (absolute offsets); dwords outside the window are dropped.
// ------------------------------------------------------------------------
struct Stage {
    uint32_t *s;  // LDS, GPAD bytes before window offset 0
    uint64_t W;   // absolute output offset of window byte 0 (16-aligned)

    HONU_DEV void or_word(uint64_t dabs, uint32_t v) {  // dabs: 4-aligned
        const uint64_t rel = dabs - W;
        if (v && rel < GCAP) atomicOr(&s[(GPAD + (uint32_t)rel) >> 2], v);
    }
    // OR the 16 little-endian bytes lo||hi (zero beyond their length) at P
    HONU_DEV void or16(uint64_t P, uint64_t lo, uint64_t hi) {
        const uint32_t sh = (uint32_t)(P & 3) * 8;
        const uint64_t D = P & ~3ull;
        const uint32_t w0 = (uint32_t)lo, w1 = (uint32_t)(lo >> 32), w2 = (uint32_t)hi,
                       w3 = (uint32_t)(hi >> 32);
        // out_j = low word of (w_j:w_{j-1}) >> (32 - sh)
        or_word(D, (uint32_t)(((uint64_t)w0 << 32) >> (32 - sh)));
        or_word(D + 4, (uint32_t)((((uint64_t)w1 << 32) | w0) >> (32 - sh)));
        or_word(D + 8, (uint32_t)((((uint64_t)w2 << 32) | w1) >> (32 - sh)));
        or_word(D + 12, (uint32_t)((((uint64_t)w3 << 32) | w2) >> (32 - sh)));
        if (sh) or_word(D + 16, w3 >> (32 - sh));
    }
};

// The serial part of the tail: a LaneWriter (lane.h) whose 16-byte chunks are
// OR-ed into the stage by the group's lead lane; skip() leaves a gap that the
// group fills cooperatively.
struct StageWriter {
    Stage *st;
    bool lead;
    uint64_t pos;     // absolute position of the next byte
    uint64_t a0, a1;  // current chunk [pos & ~15, +16), bytes below pos are 0

    HONU_DEV void init(Stage *s, bool l, uint64_t p) {
        st = s;
        lead = l;
        pos = p;
        a0 = a1 = 0;
    }
    HONU_DEV void flush() {
        if (lead) st->or16(pos & ~15ull, a0, a1);
        a0 = a1 = 0;
    }
    HONU_DEV void put(uint64_t v, uint32_t n) {  // low n (1..8) bytes of v
        const uint32_t f = (uint32_t)(pos & 15);
        const uint32_t s = 8 * f;
        uint64_t t2 = 0;
        if (s < 64) {
            a0 |= v << s;
            if (s) a1 |= v >> (64 - s);
        } else {
            a1 |= v << (s - 64);
            if (s > 64) t2 = v >> (128 - s);
        }
        if (f + n >= 16) {
            flush();  // chunk of the old pos
            a0 = t2;
        }
        pos += n;
    }
    HONU_DEV void byte(uint32_t v) { put(v & 0xFF, 1); }
    HONU_DEV void put16(uint64_t lo, uint64_t hi) {
        put(lo, 8);
        put(hi, 8);
    }
    HONU_DEV void uv(uint64_t x) {
        uint64_t lo, hi;
        const uint32_t n = uvarint_bytes(x, lo, hi);
        put(lo, n < 8 ? n : 8);
        if (n > 8) put(hi, n - 8);
    }
    HONU_DEV void skip(uint64_t len) {
        if (!len) return;
        const uint64_t np = pos + len;
        if ((np & ~15ull) != (pos & ~15ull)) flush();
        pos = np;
    }
    HONU_DEV void finish() {
        if (pos & 15) flush();
    }
};

// src[0, len) (global, any alignment) -> stage at P, aligned 16-byte source
// blocks spread over the group (every block holds a byte of the run, so it is
// mapped).
template <int G>
HONU_DEV void grp_copy_run(Stage &st, uint64_t P, const uint8_t *src, uint64_t len, uint32_t r) {
    if (!len) return;
    const uint32_t a = (uint32_t)((uint64_t)src & 15);
    const u32x4 *A = reinterpret_cast<const u32x4 *>(src - a);
    const uint64_t nblk = (a + len + 15) >> 4;
    for (uint64_t k = r; k < nblk; k += G) {
        const u32x4 v = A[k];
        const int lo_b = k == 0 ? (int)a : 0;
        const int64_t hb = (int64_t)a + (int64_t)len - 16 * (int64_t)k;
        const int hi_b = hb > 16 ? 16 : (int)hb;
        const uint64_t lo = (((uint64_t)v.y << 32) | v.x) & bytemask64(lo_b, hi_b);
        const uint64_t hi = (((uint64_t)v.w << 32) | v.z) & bytemask64(lo_b - 8, hi_b - 8);
        st.or16(P - a + 16 * k, lo, hi);
    }
}

template <int G>
HONU_DEV void grp_frame(StageWriter &W, const uint8_t *var, honu_span sp, uint32_t r) {
    W.uv(sp.len);  // lani Encode :62-77
    grp_copy_run<G>(*W.st, W.pos, var + sp.off, sp.len, r);
    W.skip(sp.len);
}

HONU_DEV uint64_t lds64(const uint8_t *p) { return *reinterpret_cast<const uint64_t *>(p); }

// One window pass of the Metadata tail of record i (metadata.go:108-200).
template <int G>
HONU_DEV void grp_encode_tail(StageWriter &W, const honu_meta &m, const uint8_t *mb,
                              const uint8_t *__restrict__ var, const honu_acl *__restrict__ acl,
                              const uint32_t *__restrict__ reg, uint32_t r) {
    const uint32_t pr = m.present;
    W.byte(1);                                                      // EncodeStruct(meta)
    W.put16(lds64(mb + OFF(object_id)), lds64(mb + OFF(object_id) + 8));          // :110
    W.put16(lds64(mb + OFF(collection_id)), lds64(mb + OFF(collection_id) + 8));  // :115
    if (pr & HONU_HAS_VERSION) {                                    // :120, version.go:44-70
        W.byte(1);
        W.uv(m.pid);
        W.uv(m.vid);
        W.uv(m.region);
        if (pr & HONU_HAS_PARENT) {
            W.byte(1);
            W.uv(m.parent_pid);
            W.uv(m.parent_vid);
        } else {
            W.byte(0);
        }
        W.byte(m.tombstone ? 1 : 0);
        W.uv(zigzag(m.version_created));
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_SCHEMA) {                                     // :125, schema.go:30-53
        W.byte(1);
        grp_frame<G>(W, var, m.schema_name, r);
        W.uv(m.schema_major);
        W.uv(m.schema_minor);
        W.uv(m.schema_patch);
    } else {
        W.byte(0);
    }
    grp_frame<G>(W, var, m.mime, r);                                // :130
    W.put16(lds64(mb + OFF(owner)), lds64(mb + OFF(owner) + 8));    // :135
    W.put16(lds64(mb + OFF(group)), lds64(mb + OFF(group) + 8));    // :140
    W.byte(m.permissions);                                          // :145
    const uint64_t na = m.acl_count, ao = m.acl_off;
    W.uv(na);                                                       // :151
    {  // :157-162, acls.go:26-39: entry j of a round at base + prefix
        uint64_t base = W.pos;
        for (uint64_t t = 0; t < na; t += G) {
            const uint64_t j = t + r;
            const bool valid = j < na;
            uint32_t e0 = 0, e1 = 0, e2 = 0, e3 = 0, e4 = 0;
            if (valid) {
                const uint32_t *e = reinterpret_cast<const uint32_t *>(acl + ao + j);
                e0 = e[0];
                e1 = e[1];
                e2 = e[2];
                e3 = e[3];
                e4 = e[4];
            }
            const bool pres = valid && ((e4 >> 8) & 0xFF);
            const uint32_t mp = grp_bits<G>(__ballot(pres));
            const uint32_t mv = grp_bits<G>(__ballot(valid));
            const uint32_t below = (1u << r) - 1;
            const uint64_t P = base + 18 * __popc(mp & below) + __popc(mv & ~mp & below);
            if (pres) {  // 01 | ulid | perm ; a nil entry is a 00 byte: nothing to OR
                const uint64_t lo = 1ull | ((uint64_t)e0 << 8) | ((uint64_t)e1 << 40);
                const uint64_t hi = (e1 >> 24) | ((uint64_t)e2 << 8) | ((uint64_t)e3 << 40);
                W.st->or16(P, lo, hi);
                W.st->or16(P + 16, (e3 >> 24) | ((e4 & 0xFF) << 8), 0);
            }
            base += 18 * __popc(mp) + __popc(mv & ~mp);
        }
        W.skip(base - W.pos);
    }
    const uint64_t nr = m.regions_count, ro = m.regions_off;
    W.uv(nr);                                                       // :164, region.go:137-152
    {
        uint64_t base = W.pos;
        for (uint64_t t = 0; t < nr; t += G) {
            const uint64_t j = t + r;
            uint64_t lo = 0, hi = 0;
            uint32_t L = 0;
            if (j < nr) L = uvarint_bytes(reg[ro + j], lo, hi);
            const uint32_t pre = grp_excl_scan<G>(L, r);
            if (L) W.st->or16(base + pre, lo, 0);
            base += grp_sum<G>(L);
        }
        W.skip(base - W.pos);
    }
    if (pr & HONU_HAS_PUBLISHER) {                                  // :169, provenance.go:34-57
        W.byte(1);
        W.put16(lds64(mb + OFF(publisher_id)), lds64(mb + OFF(publisher_id) + 8));
        W.put16(lds64(mb + OFF(client_id)), lds64(mb + OFF(client_id) + 8));
        grp_frame<G>(W, var, m.ip_address, r);
        grp_frame<G>(W, var, m.user_agent, r);
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_ENCRYPTION) {                                 // :174, encryption.go:51-89
        W.byte(1);
        grp_frame<G>(W, var, m.public_key_id, r);
        grp_frame<G>(W, var, m.encryption_key, r);
        grp_frame<G>(W, var, m.hmac_secret, r);
        grp_frame<G>(W, var, m.signature, r);
        W.byte(m.sealing_alg);
        W.byte(m.encryption_alg);
        W.byte(m.signature_alg);
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_COMPRESSION) {                                // :179, compression.go:40-53
        W.byte(1);
        W.byte(m.compression_alg);
        W.uv(zigzag(m.compression_level));
    } else {
        W.byte(0);
    }
    W.byte(m.flags);                                                // :184
    W.uv(zigzag(m.created));                                        // :189
    W.uv(zigzag(m.modified));                                       // :194
    W.finish();
}

// Row i -> LDS (22 aligned 16-byte chunks over the group).
template <int G> HONU_DEV void grp_stage_row(uint8_t *row, const honu_meta *src, uint32_t r) {
    const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
    u32x4 *d = reinterpret_cast<u32x4 *>(row);
    for (uint32_t c = r; c < GROW / 16; c += G) d[c] = s[c];
}

// ------------------------------------------------------------------------
// encode: header + Metadata tail (object.go:24-45)
// ------------------------------------------------------------------------
template <int G>
HONU_DEV void k_encode_meta_grp_one(uint64_t i, uint8_t *smem, const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status) {
    const uint32_t r = threadIdx.x & (G - 1);
    if (status[i] != HONU_OK) return;
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    if (end > out_cap) {
        if (r == 0) status[i] = HONU_ERR_CAPACITY;
        return;
    }
    uint8_t *row = smem + (threadIdx.x / G) * GPER;
    uint32_t *stage = reinterpret_cast<uint32_t *>(row + GROW);
    grp_stage_row<G>(row, meta + i, r);
    wave_sync();
    const honu_meta &m = *reinterpret_cast<const honu_meta *>(row);
    const uint64_t dlen = payload_off[i + 1] - payload_off[i];
    {  // header: version byte + uvarint(len data)   object.go:30,35
        uint64_t lo, hi;
        const uint32_t hn = uvarint_bytes(dlen, lo, hi);
        if (r <= hn)
            out[beg + r] = r == 0 ? (uint8_t)HONU_STORAGE_VERSION
                                  : (uint8_t)(r <= 8 ? lo >> (8 * (r - 1)) : hi >> (8 * (r - 9)));
    }
    const uint64_t tstart = beg + 1 + uvarint_len(dlen) + dlen;
    const uint64_t W0 = tstart & ~15ull;
    for (uint64_t W = W0; W < end; W += GCAP) {
        u32x4 *s4 = reinterpret_cast<u32x4 *>(stage);
        for (uint32_t c = r; c < GSTAGE / 16; c += G) s4[c] = u32x4{0, 0, 0, 0};
        wave_sync();
        Stage st{stage, W};
        StageWriter wr;
        wr.init(&st, r == 0, tstart);
        grp_encode_tail<G>(wr, m, row, var, acl, reg, r);
        wave_sync();
        // leave the window: aligned 16-byte stores, byte stores at the ends
        const uint64_t wend = W + GCAP < end ? W + GCAP : end;
        const uint32_t nch = (uint32_t)((wend - W + 15) >> 4);
        const uint8_t *sb = reinterpret_cast<const uint8_t *>(stage) + GPAD;
        for (uint32_t c = r; c < nch; c += G) {
            const uint64_t X = W + 16ull * c;
            if (X >= tstart && X + 16 <= end) {
                *reinterpret_cast<u32x4 *>(out + X) = reinterpret_cast<const u32x4 *>(sb)[c];
            } else {
                for (uint32_t b = 0; b < 16; b++)
                    if (X + b >= tstart && X + b < end) out[X + b] = sb[16 * c + b];
            }
        }
        wave_sync();
    }
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_meta_grp(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[GRECS * GPER];
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_encode_meta_grp_one<G>(i, smem, meta, var, acl, reg, payload_off, n, out, out_cap, out_off, status);
}

// ------------------------------------------------------------------------
// encode size pass (object.go:24-45 / App. A), row image staged in LDS
// ------------------------------------------------------------------------
HONU_DEV bool gspan_in(uint64_t off, uint64_t len, uint64_t var_len) {
    return len == 0 || (off <= var_len && len <= var_len - off);
}
HONU_DEV uint64_t gframe_len(uint64_t len) { return uvarint_len(len) + len; }

template <int G>
HONU_DEV void k_encode_sizes_grp_one(uint64_t i, uint8_t *smem, const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    const uint32_t r = threadIdx.x & (G - 1);
    uint8_t *row = smem + (threadIdx.x / G) * (GROW + 16);
    grp_stage_row<G>(row, meta + i, r);
    wave_sync();
    const honu_meta &m = *reinterpret_cast<const honu_meta *>(row);
    const uint32_t pr = m.present;
    uint64_t size = 0;
    int32_t stc = HONU_OK;
    if (!(pr & HONU_HAS_META)) {
        stc = HONU_ERR_PANIC;  // Marshal(nil, ...): nil deref in Size(), metadata.go:66
    } else {
        bool ok = gspan_in(m.mime.off, m.mime.len, var_len);
        if (pr & HONU_HAS_SCHEMA) ok = ok && gspan_in(m.schema_name.off, m.schema_name.len, var_len);
        if (pr & HONU_HAS_PUBLISHER)
            ok = ok && gspan_in(m.ip_address.off, m.ip_address.len, var_len) &&
                 gspan_in(m.user_agent.off, m.user_agent.len, var_len);
        if (pr & HONU_HAS_ENCRYPTION)
            ok = ok && gspan_in(m.public_key_id.off, m.public_key_id.len, var_len) &&
                 gspan_in(m.encryption_key.off, m.encryption_key.len, var_len) &&
                 gspan_in(m.hmac_secret.off, m.hmac_secret.len, var_len) &&
                 gspan_in(m.signature.off, m.signature.len, var_len);
        const uint64_t na = m.acl_count, nr = m.regions_count;
        const uint64_t ao = m.acl_off, ro = m.regions_off;
        if (na) ok = ok && ao <= acl_len && na <= acl_len - ao;
        if (nr) ok = ok && ro <= reg_len && nr <= reg_len - ro;
        if (!ok) {
            stc = HONU_ERR_INPUT;
        } else {
            uint64_t t = 1 + 32;  // meta flag, ObjectID, CollectionID
            t += 1;               // Version flag
            if (pr & HONU_HAS_VERSION)
                t += uvarint_len(m.pid) + uvarint_len(m.vid) + uvarint_len(m.region) + 1 +
                     ((pr & HONU_HAS_PARENT) ? uvarint_len(m.parent_pid) + uvarint_len(m.parent_vid) : 0) +
                     1 + uvarint_len(zigzag(m.version_created));
            t += 1;  // Schema flag
            if (pr & HONU_HAS_SCHEMA)
                t += gframe_len(m.schema_name.len) + uvarint_len(m.schema_major) +
                     uvarint_len(m.schema_minor) + uvarint_len(m.schema_patch);
            t += gframe_len(m.mime.len) + 33;  // MIME, Owner, Group, Permissions
            t += uvarint_len(na) + uvarint_len(nr);
            uint64_t part = 0;  // this lane's share of the lists
            for (uint64_t k = r; k < na; k += G) part += acl[ao + k].present ? 18 : 1;
            for (uint64_t k = r; k < nr; k += G) part += uvarint_len(reg[ro + k]);
            t += 3;  // Publisher, Encryption, Compression flags
            if (pr & HONU_HAS_PUBLISHER) t += 32 + gframe_len(m.ip_address.len) + gframe_len(m.user_agent.len);
            if (pr & HONU_HAS_ENCRYPTION)
                t += gframe_len(m.public_key_id.len) + gframe_len(m.encryption_key.len) +
                     gframe_len(m.hmac_secret.len) + gframe_len(m.signature.len) + 3;
            if (pr & HONU_HAS_COMPRESSION) t += 1 + uvarint_len(zigzag(m.compression_level));
            t += 1 + uvarint_len(zigzag(m.created)) + uvarint_len(zigzag(m.modified));
            t += grp_sum64<G>(part);
            const uint64_t dlen = payload_off[i + 1] - payload_off[i];
            size = 1 + uvarint_len(dlen) + dlen + t;  // object.go:30,35,40
        }
    }
    if (r == 0) {
        sizes[i] = size;
        if (status) status[i] = stc;
    }
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_sizes_grp(
    const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[GRECS * (GROW + 16)];
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_encode_sizes_grp_one<G>(i, smem, meta, var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
}

// ------------------------------------------------------------------------
// decode parse: Object.Metadata() + Data() + Tombstone() + StorageVersion()
// (object.go:47-134) with the lani walk of metadata.go:202-302 over a byte
// source: the LDS stage of the tail, or global memory for longer tails.
// ------------------------------------------------------------------------
struct SrcGlobal {
    const uint8_t *base;
    HONU_DEV uint32_t u8(uint64_t p) const { return base[p]; }
    HONU_DEV void fetch16(uint64_t p, uint64_t end, uint64_t &lo, uint64_t &hi) const {
        lane_fetch16(base, p, end, lo, hi);
    }
};
struct SrcLds {
    const uint8_t *lds;  // stage byte 0 = absolute offset S
    uint64_t S;
    HONU_DEV uint32_t u8(uint64_t p) const { return lds[p - S]; }
    HONU_DEV void fetch16(uint64_t p, uint64_t, uint64_t &lo, uint64_t &hi) const {
        const uint32_t x = (uint32_t)(p - S);
        const u32x4 *b = reinterpret_cast<const u32x4 *>(lds + (x & ~15u));
        window16(b[0], b[1], x & 15, lo, hi);  // stage slack covers b[1]
    }
};

template <class S> struct GDec {  // lani.Decoder (lani/decode.go), as LaneDec
    S src;
    uint64_t p, end, tstart;

    HONU_DEV int u8(uint32_t &v) {  // DecodeByte :94-103
        if (p >= end) return HONU_ERR_EOF;
        v = src.u8(p);
        p += 1;
        return HONU_OK;
    }
    HONU_DEV int boolean(uint32_t &v) {  // DecodeBool :105-120
        int st = u8(v);
        if (st) return st;
        return v > 1 ? HONU_ERR_PARSE_BOOLEAN : HONU_OK;
    }
    HONU_DEV int uv(uint32_t maxw, int err, uint64_t &v) {
        if (p >= end) return HONU_ERR_EOF;
        const uint64_t avail = end - p;
        const uint32_t n = avail < maxw ? (uint32_t)avail : maxw;
        uint64_t lo, hi;
        src.fetch16(p, end, lo, hi);
        const uint32_t k = uvarint_window(lo, hi, n, v);
        if (!k) return err;
        p += k;
        return HONU_OK;
    }
    HONU_DEV int u32(uint32_t &v) {  // DecodeUint32 :127-146
        uint64_t x = 0;
        int st = uv(5, HONU_ERR_PARSE_VARINT, x);
        v = (uint32_t)x;
        return st;
    }
    HONU_DEV int u64(uint64_t &v) { return uv(10, HONU_ERR_PARSE_VARINT, v); }  // :149-168
    HONU_DEV int i64(int64_t &v) {                                             // :171-190
        uint64_t x = 0;
        int st = uv(10, HONU_ERR_PARSE_VARINT, x);
        v = unzigzag(x);
        return st;
    }
    HONU_DEV int ulid(uint64_t &lo, uint64_t &hi) {  // DecodeULID :209-221
        if (p >= end) return HONU_ERR_EOF;
        if (p + 16 > end) return HONU_ERR_UNEXPECTED_EOF;
        src.fetch16(p, end, lo, hi);
        p += 16;
        return HONU_OK;
    }
    HONU_DEV int frame(uint64_t &off, uint64_t &len) {  // Decode :30-56, readLength :261-282
        uint64_t rl = 0;
        int st = uv(10, HONU_ERR_NO_LENGTH, rl);
        if (st) return st;
        if (rl >= (1ull << 63)) return HONU_ERR_PANIC;  // int(rl) < 0 -> makeslice
        if (rl == 0) {
            off = 0;
            len = 0;
            return HONU_OK;
        }
        if (rl > (uint64_t)INT64_MAX - (p - tstart)) return HONU_ERR_PANIC;  // d.i + rl overflows
        if (p + rl > end) return HONU_ERR_UNEXPECTED_EOF;
        off = p;
        len = rl;
        p += rl;
        return HONU_OK;
    }
};

#define TRY(x)              \
    do {                    \
        st = (x);           \
        if (st) goto done;  \
    } while (0)

// The walk; fields go to the LDS row image R (zeroed; every lane writes the
// same values). Lane r keeps region id r (< 8) in `myreg`.
template <int G, class S>
HONU_DEV int grp_walk(GDec<S> &D, honu_meta *R, uint32_t r, uint64_t &nacl, uint64_t &nreg,
                      uint64_t &acl_pos, uint64_t &reg_pos, uint32_t &myreg) {
    int st = HONU_OK;
    uint32_t f, u;
    uint64_t v, o, l, lo, hi;
    int64_t t;
    uint32_t pr = 0;
    TRY(D.boolean(f));                                      // DecodeStruct(meta) object.go:78
    if (f) {
        pr = HONU_HAS_META;
        TRY(D.ulid(lo, hi));                                // metadata.go:210
        reinterpret_cast<uint64_t *>(R->object_id)[0] = lo;
        reinterpret_cast<uint64_t *>(R->object_id)[1] = hi;
        TRY(D.ulid(lo, hi));                                // :214
        reinterpret_cast<uint64_t *>(R->collection_id)[0] = lo;
        reinterpret_cast<uint64_t *>(R->collection_id)[1] = hi;
        TRY(D.boolean(f));                                  // :219 Version
        if (f) {
            pr |= HONU_HAS_VERSION;
            TRY(D.u32(u)); R->pid = u;                      // scalar.go:121-131
            TRY(D.u64(v)); R->vid = v;
            TRY(D.u32(u)); R->region = u;                   // version.go:80
            TRY(D.boolean(f));                              // :88 Parent
            if (f) {
                pr |= HONU_HAS_PARENT;
                TRY(D.u32(u)); R->parent_pid = u;
                TRY(D.u64(v)); R->parent_vid = v;
            }
            TRY(D.boolean(f)); R->tombstone = (uint8_t)f;   // :96
            TRY(D.i64(t)); R->version_created = t;          // :100
        }
        TRY(D.boolean(f));                                  // :225 Schema
        if (f) {
            pr |= HONU_HAS_SCHEMA;
            TRY(D.frame(o, l)); R->schema_name = honu_span{o, l};     // schema.go:55-73
            TRY(D.u32(u)); R->schema_major = u;
            TRY(D.u32(u)); R->schema_minor = u;
            TRY(D.u32(u)); R->schema_patch = u;
        }
        TRY(D.frame(o, l)); R->mime = honu_span{o, l};      // :231
        TRY(D.ulid(lo, hi));                                // :235
        reinterpret_cast<uint64_t *>(R->owner)[0] = lo;
        reinterpret_cast<uint64_t *>(R->owner)[1] = hi;
        TRY(D.ulid(lo, hi));                                // :239
        reinterpret_cast<uint64_t *>(R->group)[0] = lo;
        reinterpret_cast<uint64_t *>(R->group)[1] = hi;
        TRY(D.u8(u)); R->permissions = (uint8_t)u;          // :243
        TRY(D.u64(nacl));                                   // :249
        if (nacl > 0) {                                     // :254-265
            if (nacl > GO_MAX_ALLOC / 8) TRY(HONU_ERR_PANIC);  // make([]*AccessControl)
            acl_pos = D.p;
            bool fast = false;
            if (18 * nacl <= D.end - D.p) {  // every entry present and inside?
                bool bad = false;
                for (uint64_t k = 0; k < nacl; k += G) {
                    const uint64_t j = k + r;
                    if (j < nacl) bad |= D.src.u8(D.p + 18 * j) != 1;
                }
                fast = grp_bits<G>(__ballot(bad)) == 0;
            }
            if (fast) {
                D.p += 18 * nacl;
                acl_pos |= GRP_ACL_FAST;
            } else {
                for (uint64_t k = 0; k < nacl; k++) {       // acls.go:41-51
                    TRY(D.boolean(f));
                    if (f) {
                        TRY(D.ulid(lo, hi));
                        TRY(D.u8(u));
                    }
                }
            }
            R->acl_count = nacl;
        }
        TRY(D.u64(nreg));                                   // region.go:154-169
        if (nreg > GO_MAX_ALLOC / 4) TRY(HONU_ERR_PANIC);   // make(Regions, length)
        pr |= HONU_REGIONS_NONNIL;
        reg_pos = D.p;
        for (uint64_t k = 0; k < nreg; k++) {
            TRY(D.u32(u));
            if (k == r) myreg = u;
        }
        if (nreg <= 8) reg_pos |= GRP_REG_INLINE;
        R->regions_count = nreg;
        TRY(D.boolean(f));                                  // :271 Publisher
        if (f) {
            pr |= HONU_HAS_PUBLISHER;
            TRY(D.ulid(lo, hi));                            // provenance.go:59-79
            reinterpret_cast<uint64_t *>(R->publisher_id)[0] = lo;
            reinterpret_cast<uint64_t *>(R->publisher_id)[1] = hi;
            TRY(D.ulid(lo, hi));
            reinterpret_cast<uint64_t *>(R->client_id)[0] = lo;
            reinterpret_cast<uint64_t *>(R->client_id)[1] = hi;
            TRY(D.frame(o, l)); R->ip_address = honu_span{o, l};
            TRY(D.frame(o, l)); R->user_agent = honu_span{o, l};
        }
        TRY(D.boolean(f));                                  // :277 Encryption
        if (f) {
            pr |= HONU_HAS_ENCRYPTION;
            TRY(D.frame(o, l)); R->public_key_id = honu_span{o, l};   // encryption.go:91-125
            TRY(D.frame(o, l)); R->encryption_key = honu_span{o, l};
            TRY(D.frame(o, l)); R->hmac_secret = honu_span{o, l};
            TRY(D.frame(o, l)); R->signature = honu_span{o, l};
            TRY(D.u8(u)); R->sealing_alg = (uint8_t)u;
            TRY(D.u8(u)); R->encryption_alg = (uint8_t)u;
            TRY(D.u8(u)); R->signature_alg = (uint8_t)u;
        }
        TRY(D.boolean(f));                                  // :283 Compression
        if (f) {
            pr |= HONU_HAS_COMPRESSION;
            TRY(D.u8(u)); R->compression_alg = (uint8_t)u;  // compression.go:55-67
            TRY(D.i64(t)); R->compression_level = t;
        }
        TRY(D.u8(u)); R->flags = (uint8_t)u;                // :289
        TRY(D.i64(t)); R->created = t;                      // :293
        TRY(D.i64(t)); R->modified = t;                     // :297
    }
    R->present = pr;
done:
    return st;
}
#undef TRY

template <int G> HONU_DEV void grp_zero_row(uint8_t *row, uint32_t r) {
    u32x4 *d = reinterpret_cast<u32x4 *>(row);
    for (uint32_t c = r; c < GROW / 16; c += G) d[c] = u32x4{0, 0, 0, 0};
}

template <int G>
HONU_DEV void k_decode_parse_grp_one(uint64_t i, uint8_t *smem, const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint32_t *__restrict__ reg_inline,
    uint64_t *__restrict__ counts) {
    const uint32_t r = threadIdx.x & (G - 1);
    uint8_t *row = smem + (threadIdx.x / G) * GPER;
    uint8_t *stage = row + GROW;
    const uint64_t beg = rec_off[i], end = rec_off[i + 1];
    const uint64_t len = end - beg;
    uint32_t ver = 0;
    int64_t d = -1, b = -1;
    if (len) {
        uint64_t lo, hi;
        lane_fetch16(rec, beg, end, lo, hi);
        ver = (uint32_t)(lo & 0xFF);
        // dataLength (object.go:114-134): Uvarint(o[1 : min(11, len-1)])
        if (len >= 3) {
            const uint32_t wl = (uint32_t)(len - 2 < 10 ? len - 2 : 10);
            const uint64_t lo1 = (lo >> 8) | (hi << 56), hi1 = hi >> 8;
            uint64_t x;
            const uint32_t k = uvarint_window(lo1, hi1, wl, x);
            if (k) {
                d = (int64_t)x;  // int(rl): negative for rl >= 2^63
                b = k;
            }
        }
    }
    const bool v1 = ver == HONU_STORAGE_VERSION;
    const bool in_range = d >= 0 && (uint64_t)d <= len - 1 - (uint64_t)b;
    int32_t data_status;
    uint64_t data_off = 0, data_len = 0;
    if (!v1) data_status = HONU_ERR_BAD_VERSION;
    else if (d < 0) data_status = HONU_ERR_MALFORMED;
    else if (d == 0) data_status = HONU_OK;
    else if (!in_range) data_status = HONU_ERR_PANIC;  // o[1+b:1+b+d]
    else {
        data_status = HONU_OK;
        data_off = beg + 1 + (uint64_t)b;
        data_len = (uint64_t)d;
    }

    grp_zero_row<G>(row, r);
    wave_sync();
    honu_meta *R = reinterpret_cast<honu_meta *>(row);
    uint64_t nacl = 0, nreg = 0, acl_pos = 0, reg_pos = 0;
    uint32_t myreg = 0;
    int st = HONU_OK;
    if (!v1) st = HONU_ERR_BAD_VERSION;
    else if (d < 0) st = HONU_ERR_MALFORMED;
    else if (!in_range) st = HONU_ERR_PANIC;  // o[1+d+b:]
    else {
        const uint64_t tstart = beg + 1 + (uint64_t)b + (uint64_t)d;
        const uint64_t S = tstart & ~15ull;
        if (end - S <= GCAP) {  // stage [S, end) in LDS
            const uint32_t nch = (uint32_t)((end - S + 15) >> 4);
            const u32x4 *src = reinterpret_cast<const u32x4 *>(rec + S);
            u32x4 *dst = reinterpret_cast<u32x4 *>(stage);
            for (uint32_t c = r; c < nch; c += G) dst[c] = src[c];
            wave_sync();
            GDec<SrcLds> D{SrcLds{stage, S}, tstart, end, tstart};
            st = grp_walk<G>(D, R, r, nacl, nreg, acl_pos, reg_pos, myreg);
        } else {
            GDec<SrcGlobal> D{SrcGlobal{rec}, tstart, end, tstart};
            st = grp_walk<G>(D, R, r, nacl, nreg, acl_pos, reg_pos, myreg);
        }
    }
    wave_sync();
    if (st != HONU_OK) {  // Go returns nil, err
        grp_zero_row<G>(row, r);
        wave_sync();
        nacl = nreg = 0;
        acl_pos = reg_pos = 0;
    }
    {
        const u32x4 *s4 = reinterpret_cast<const u32x4 *>(row);
        u32x4 *d4 = reinterpret_cast<u32x4 *>(meta + i);
        for (uint32_t c = r; c < GROW / 16; c += G) d4[c] = s4[c];
    }
    if (r == 0) {
        honu_record_info inf;
        inf.data_off = data_off;
        inf.data_len = data_len;
        inf.data_status = data_status;
        inf.meta_status = st;
        inf.storage_version = (uint8_t)ver;
        inf.tombstone = (v1 && d == 0) ? 1 : 0;  // Tombstone :103-112
#pragma unroll
        for (int k = 0; k < 6; k++) inf._pad[k] = 0;
        store_info(info + i, inf);
        scratch[i] = DecodeScratch{acl_pos, reg_pos, data_off, end};
        counts[3 * i + 0] = nacl;
        counts[3 * i + 1] = nreg;
        counts[3 * i + 2] = (data_len + 15) & ~15ull;
    }
    if (r < 8 && r < nreg) reg_inline[8 * i + r] = myreg;
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_parse_grp(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint32_t *__restrict__ reg_inline,
    uint64_t *__restrict__ counts) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[GRECS * GPER];
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_decode_parse_grp_one<G>(i, smem, rec, rec_off, n, meta, info, scratch, reg_inline, counts);
}

// ------------------------------------------------------------------------
// decode fill: ACL/region tables and offsets (after the count scans)
// ------------------------------------------------------------------------
template <int G>
HONU_DEV void k_decode_fill_grp_one(uint64_t i, const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint32_t *__restrict__ reg_inline, const uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ offs, honu_acl *__restrict__ acl, uint64_t acl_cap,
    uint32_t *__restrict__ reg, uint64_t reg_cap, uint8_t *__restrict__ data, uint64_t data_cap) {
    const uint32_t r = threadIdx.x & (G - 1);
    honu_record_info *inf = info + i;
    // independent loads first (one round trip)
    const int32_t mst = inf->meta_status;
    const uint64_t na = counts[3 * i], nr = counts[3 * i + 1];
    const uint64_t ao = offs[3 * i], ro = offs[3 * i + 1];
    const DecodeScratch sc = scratch[i];
    if (mst == HONU_OK) {
        if (r == 0) {
            if (na) meta[i].acl_off = ao;
            if (nr) meta[i].regions_off = ro;
        }
        if (ao + na > acl_cap || ro + nr > reg_cap) {
            if (r == 0) inf->meta_status = HONU_ERR_CAPACITY;
        } else if (na + nr) {
            const uint64_t end = sc.rec_end;
            const uint64_t ap = sc.acl_pos & GRP_POS_MASK;
            if (na && (sc.acl_pos & GRP_ACL_FAST)) {
                constexpr int K = FILL_K;  // entries per lane loaded before any store
                for (uint64_t j0 = r; j0 < na; j0 += (uint64_t)G * K) {
                    uint64_t lo[K], hi[K];
                    uint32_t pm[K];
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const uint64_t j = j0 + (uint64_t)G * k;
                        if (j < na) {
                            const uint64_t q = ap + 18 * j;
                            lane_fetch16(rec, q + 1, end, lo[k], hi[k]);
                            pm[k] = rec[q + 17];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const uint64_t j = j0 + (uint64_t)G * k;
                        if (j < na) {
                            uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + j);
                            e[0] = (uint32_t)lo[k];
                            e[1] = (uint32_t)(lo[k] >> 32);
                            e[2] = (uint32_t)hi[k];
                            e[3] = (uint32_t)(hi[k] >> 32);
                            e[4] = pm[k] | (1u << 8);
                        }
                    }
                }
            } else if (na && r == 0) {  // nil entries: walk (validated by the parse)
                uint64_t p = ap;
                for (uint64_t k = 0; k < na; k++) {
                    uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + k);
                    if (rec[p]) {
                        uint64_t lo, hi;
                        lane_fetch16(rec, p + 1, end, lo, hi);
                        e[0] = (uint32_t)lo;
                        e[1] = (uint32_t)(lo >> 32);
                        e[2] = (uint32_t)hi;
                        e[3] = (uint32_t)(hi >> 32);
                        e[4] = rec[p + 17] | (1u << 8);
                        p += 18;
                    } else {
                        e[0] = e[1] = e[2] = e[3] = e[4] = 0;
                        p += 1;
                    }
                }
            }
            if (nr && (sc.regions_pos & GRP_REG_INLINE)) {
                if (r < nr) reg[ro + r] = reg_inline[8 * i + r];
            } else if (nr && r == 0) {
                uint64_t p = sc.regions_pos & GRP_POS_MASK;
                for (uint64_t k = 0; k < nr; k++) {
                    const uint64_t avail = end - p;
                    uint64_t lo, hi, v = 0;
                    lane_fetch16(rec, p, end, lo, hi);
                    const uint32_t kk = uvarint_window(lo, hi, avail < 5 ? (uint32_t)avail : 5, v);
                    reg[ro + k] = (uint32_t)v;
                    p += kk;
                }
            }
        }
    }
    if (r == 0 && data && inf->data_status == HONU_OK && inf->data_len) {
        const uint64_t doff = offs[3 * i + 2];
        if (doff + inf->data_len > data_cap) {
            inf->data_status = HONU_ERR_CAPACITY;
            inf->data_off = 0;
            inf->data_len = 0;
        } else {
            inf->data_off = doff;
        }
    }
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_fill_grp(
    const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint32_t *__restrict__ reg_inline, const uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ offs, honu_acl *__restrict__ acl, uint64_t acl_cap,
    uint32_t *__restrict__ reg, uint64_t reg_cap, uint8_t *__restrict__ data, uint64_t data_cap) {
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_decode_fill_grp_one<G>(i, rec, n, meta, info, scratch, reg_inline, counts, offs, acl, acl_cap, reg, reg_cap, data, data_cap);
}


// ------------------------------------------------------------------------
// encode ACL entries (metadata.go:157-162, acls.go:26-39) into the gap the
// lane encoder left at acl_pos[i]. With every entry present, output byte x of
// the list is byte (x - P) % 18 of entry (x - P) / 18 encoded as
// 01 | ClientID | Permissions, so each lane builds whole aligned 16-byte
// output chunks from the (at most) two entries they straddle: coalesced entry
// loads, one aligned store per chunk, byte stores only at the list's ends.
// A list with nil entries is written serially by the group's lead lane.
// ------------------------------------------------------------------------
template <int G>
HONU_DEV void k_encode_acl_grp_one(uint64_t i, const honu_meta *__restrict__ meta, const honu_acl *__restrict__ acl, uint64_t n,
    uint8_t *__restrict__ out, const int32_t *__restrict__ status,
    const uint64_t *__restrict__ acl_pos) {
    const uint32_t r = threadIdx.x & (G - 1);
    // independent loads first: one round trip before the entries
    const int32_t sti = status[i];
    const uint64_t na = meta[i].acl_count, ao = meta[i].acl_off, pos = acl_pos[i];
    if (sti != HONU_OK || !na) return;
    const honu_acl *A = acl + ao;
    const uint64_t P = pos & ~ACL_ALL_PRESENT;
    if (pos & ACL_ALL_PRESENT) {  // whole chunks [ceil16(P), floor16(E))
        const uint64_t X0 = (P + 15) & ~15ull, X1 = (P + 18 * na) & ~15ull;
        if (X1 <= X0) return;
        const uint64_t nch = (X1 - X0) >> 4;
        constexpr int K = 2;  // chunks per lane computed before any store
        for (uint64_t c0 = r; c0 < nch; c0 += (uint64_t)G * K) {
            u32x4 v[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint64_t c = c0 + (uint64_t)G * k;
                if (c < nch) v[k] = acl_chunk(A, na, P, X0 + 16 * c);
            }
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint64_t c = c0 + (uint64_t)G * k;
                if (c < nch) *reinterpret_cast<u32x4 *>(out + X0 + 16 * c) = v[k];
            }
        }
        return;
    }
    if (r == 0) {  // nil entries: 00 for a nil entry, else 01 | ClientID | Permissions
        uint64_t p = P;
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
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_acl_grp(
    const honu_meta *__restrict__ meta, const honu_acl *__restrict__ acl, uint64_t n,
    uint8_t *__restrict__ out, const int32_t *__restrict__ status,
    const uint64_t *__restrict__ acl_pos) {
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_encode_acl_grp_one<G>(i, meta, acl, n, out, status, acl_pos);
}

#undef OFF

static dim3 grp_grid(uint64_t n, int cap) {
    const uint64_t b = (n * GRP + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(cap > 0 && b > (uint64_t)cap ? (uint64_t)cap : b));
}

hipError_t launch_encode_sizes_grp(const honu_meta *meta, uint64_t var_len, const honu_acl *acl,
                                   uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                                   const uint64_t *payload_off, uint64_t n, uint64_t *sizes,
                                   int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_sizes_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta,
                       var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
    return hipGetLastError();
}

hipError_t launch_encode_meta_grp(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                  const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                  uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                  int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_meta_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, var, acl,
                       reg, payload_off, n, out, out_cap, out_off, status);
    return hipGetLastError();
}

hipError_t launch_encode_acl_grp(const honu_meta *meta, const honu_acl *acl, uint64_t n,
                                 uint8_t *out, const int32_t *status, const uint64_t *acl_pos,
                                 int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_acl_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, acl, n,
                       out, status, acl_pos);
    return hipGetLastError();
}

hipError_t launch_decode_parse_grp(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   honu_meta *meta, honu_record_info *info,
                                   DecodeScratch *scratch, uint32_t *reg_inline, uint64_t *counts,
                                   int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_parse_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, rec, rec_off,
                       n, meta, info, scratch, reg_inline, counts);
    return hipGetLastError();
}

hipError_t launch_decode_fill_grp(const uint8_t *rec, uint64_t n, honu_meta *meta,
                                  honu_record_info *info, const DecodeScratch *scratch,
                                  const uint32_t *reg_inline, const uint64_t *counts,
                                  const uint64_t *offs, honu_acl *acl, uint64_t acl_cap,
                                  uint32_t *reg, uint64_t reg_cap, uint8_t *data,
                                  uint64_t data_cap, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t b = (n * FILL_G + HONU_BLOCK - 1) / HONU_BLOCK;
    const dim3 grid((unsigned)(max_blocks > 0 && b > (uint64_t)max_blocks ? (uint64_t)max_blocks : b));
    hipLaunchKernelGGL(k_decode_fill_grp<FILL_G>, grid, dim3(HONU_BLOCK), 0, s, rec, n, meta,
                       info, scratch, reg_inline, counts, offs, acl, acl_cap, reg, reg_cap, data,
                       data_cap);
    return hipGetLastError();
}

}  // namespace honu
