// lane.h — per-lane lani cursor: one record per LANE.
//
// The Metadata grammar is a serial walk (every field's position depends on
// the previous varint), so a wave that walks one record with 64 lanes in
// lockstep issues the whole walk 64 times over for one record's worth of
// work: measured ~1 ms per 65,536 records, VALU-issue bound. Here each lane
// walks its own record: 64 records per wave-instruction stream.
//
// Bytes come from 16-byte windows: the two aligned 16-byte blocks around the
// cursor, funnel-shifted by the lane's own byte phase. Successive fields of a
// record sit in the same few cache lines, so after the first touch the
// window loads hit L1/L2. Varints are decoded branch-free from the window:
// the terminator is the first byte with a clear top bit (bit mask + ctz) and
// the 7-bit groups are compacted in three shift/mask steps.
#pragma once

#include "common.h"

namespace honu {

// Bytes [s, s+16) of the 32-byte window a||b (s in [0,16)) as two
// little-endian u64: five word picks by the per-lane word offset, then one
// v_alignbyte per output word.
HONU_DEV void window16(const u32x4 a, const u32x4 b, uint32_t s, uint64_t &lo, uint64_t &hi) {
    const uint32_t q4 = s >> 2, sh = s & 3;
    // w[k] = word k of a||b; pick(j) = w[q4 + j] for j in 0..4 (per-lane q4)
    const uint32_t w0 = a.x, w1 = a.y, w2 = a.z, w3 = a.w, w4 = b.x, w5 = b.y, w6 = b.z, w7 = b.w;
    const bool o1 = q4 & 1, o2 = q4 & 2;
#define PICK(j0, j1, j2, j3) (o2 ? (o1 ? (j3) : (j2)) : (o1 ? (j1) : (j0)))
    const uint32_t p0 = PICK(w0, w1, w2, w3);
    const uint32_t p1 = PICK(w1, w2, w3, w4);
    const uint32_t p2 = PICK(w2, w3, w4, w5);
    const uint32_t p3 = PICK(w3, w4, w5, w6);
    const uint32_t p4 = PICK(w4, w5, w6, w7);
#undef PICK
    const uint32_t r0 = __builtin_amdgcn_alignbyte(p1, p0, sh);
    const uint32_t r1 = __builtin_amdgcn_alignbyte(p2, p1, sh);
    const uint32_t r2 = __builtin_amdgcn_alignbyte(p3, p2, sh);
    const uint32_t r3 = __builtin_amdgcn_alignbyte(p4, p3, sh);
    lo = ((uint64_t)r1 << 32) | r0;
    hi = ((uint64_t)r3 << 32) | r2;
}

// Bytes [q, q+16) of the arena as two little-endian u64 (bytes at or beyond
// `end` are unspecified). Requires q < end. The second aligned block is read
// only when it holds a byte below `end`, so no load leaves mapped memory.
HONU_DEV void lane_fetch16(const uint8_t *__restrict__ base, uint64_t q, uint64_t end,
                           uint64_t &lo, uint64_t &hi) {
    const uint64_t A = q & ~15ull;
    const uint32_t s = (uint32_t)(q & 15);
    const u32x4 a = *reinterpret_cast<const u32x4 *>(base + A);
    u32x4 b = {0, 0, 0, 0};
    if (s && A + 16 < end) b = *reinterpret_cast<const u32x4 *>(base + A + 16);
    window16(a, b, s, lo, hi);
}

// Compact the 7-bit groups of up to 8 varint bytes (top bits already clear).
HONU_DEV uint64_t compact7(uint64_t x) {
    x = (x & 0x007F007F007F007Full) | ((x & 0x7F007F007F007F00ull) >> 1);
    x = (x & 0x00003FFF00003FFFull) | ((x & 0x3FFF00003FFF0000ull) >> 2);
    x = (x & 0x000000000FFFFFFFull) | ((x & 0x0FFFFFFF00000000ull) >> 4);
    return x;
}

// binary.Uvarint over the first n (1..10) bytes of the window lo||hi.
// Returns k > 0 (bytes consumed) or 0 when Go's Uvarint returns k <= 0
// (no terminator inside the window, or 64-bit overflow at the 10th byte).
HONU_DEV uint32_t uvarint_window(uint64_t lo, uint64_t hi, uint32_t n, uint64_t &v) {
    const uint64_t tl = ~lo & 0x8080808080808080ull;
    const uint64_t th = ~hi & 0x0000000000008080ull;
    uint32_t k;
    if (tl) k = (uint32_t)(__builtin_ctzll(tl) >> 3) + 1;
    else if (th) k = (uint32_t)(__builtin_ctzll(th) >> 3) + 9;
    else k = 11;
    if (k > n) return 0;
    if (k == 10 && ((hi >> 8) & 0xFF) > 1) return 0;  // overflow (varint.go)
    const uint64_t m = k >= 8 ? lo : (lo & ((1ull << (8 * k)) - 1));
    uint64_t x = compact7(m & 0x7F7F7F7F7F7F7F7Full);
    if (k >= 9) x |= (hi & 0x7F) << 56;
    if (k == 10) x |= ((hi >> 8) & 0x7F) << 63;
    v = x;
    return k;
}

// Row image in registers (NDW dwords: 88 for honu_meta, 92 for
// honu_collection), indices static.
template <int NDW> struct RowT {
    uint32_t d[NDW];
    HONU_DEV void clear() {
#pragma unroll
        for (int i = 0; i < NDW; i++) d[i] = 0;
    }
    HONU_DEV void u8(int off, uint32_t v) { d[off >> 2] |= (v & 0xFF) << (8 * (off & 3)); }
    HONU_DEV void u32(int off, uint32_t v) { d[off >> 2] = v; }
    HONU_DEV void u64(int off, uint64_t v) {
        d[off >> 2] = (uint32_t)v;
        d[(off >> 2) + 1] = (uint32_t)(v >> 32);
    }
    HONU_DEV void bytes16(int off, uint64_t lo, uint64_t hi) {
        u64(off, lo);
        u64(off + 8, hi);
    }
    HONU_DEV void span(int off, uint64_t o, uint64_t l) {
        u64(off, o);
        u64(off + 8, l);
    }
    template <class T> HONU_DEV void store(T *dst) const {
        static_assert(sizeof(T) == 4 * NDW, "row size");
        u32x4 *p = reinterpret_cast<u32x4 *>(dst);
#pragma unroll
        for (int i = 0; i < NDW / 4; i++)
            p[i] = u32x4{d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]};
    }
};
using Row = RowT<88>;

// lani.Decoder (lani/decode.go) over [tstart, end) for one lane.
struct LaneDec {
    const uint8_t *base;
    uint64_t p, end, tstart;

    HONU_DEV int u8(uint32_t &v) {  // DecodeByte :94-103
        if (p >= end) return HONU_ERR_EOF;
        v = base[p];
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
        lane_fetch16(base, p, end, lo, hi);
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
        lane_fetch16(base, p, end, lo, hi);
        p += 16;
        return HONU_OK;
    }
    // Decode :30-56 with readLength :261-282 -> zero-copy span.
    HONU_DEV int frame(uint64_t &off, uint64_t &len) {
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

}  // namespace honu

namespace honu {

// binary.PutUvarint of x as little-endian bytes: lo = bytes 0..7, hi = bytes
// 8..9; returns the length (1..10). Branch-free LEB128 expansion (the inverse
// of compact7) with continuation bits on all but the last byte.
HONU_DEV uint32_t uvarint_bytes(uint64_t x, uint64_t &lo, uint64_t &hi) {
    const uint32_t n = uvarint_len(x);
    uint64_t y = x & 0x00FFFFFFFFFFFFFFull;
    y = (y & 0x000000000FFFFFFFull) | ((y & 0x00FFFFFFF0000000ull) << 4);
    y = (y & 0x00003FFF00003FFFull) | ((y & 0x0FFFC0000FFFC000ull) << 2);
    y = (y & 0x007F007F007F007Full) | ((y & 0x3F803F803F803F80ull) << 1);
    const uint32_t nl = n < 8 ? n : 8;  // bytes in lo
    const uint64_t cont = n > 8 ? 0x8080808080808080ull
                                : (0x8080808080808080ull & ((1ull << (8 * (nl - 1))) - 1));
    lo = (y | cont) & (nl == 8 ? ~0ull : ((1ull << (8 * nl)) - 1));
    hi = 0;
    if (n > 8) hi = ((x >> 56) & 0x7F) | (n > 9 ? 0x80 : 0) | ((x >> 63) << 8);
    return n;
}

// A lane-private byte stream into global memory at an arbitrary offset. Bytes
// gather in a 16-byte register chunk aligned to the destination's 16-byte
// grid. The two partial chunks at the ends (their other bytes belong to
// neighbours) leave as narrower stores, both in finish(): the head chunk is
// parked in registers when it fills, so a put() carries no partial-store code
// (the kernel's size is its instruction-cache footprint).
// R == 0: every full chunk leaves as one 16-byte store where it fills.
// R > 0: full chunks go to a per-lane LDS ring of R chunks (slot-major, lanes
// adjacent) and leave in drain(), which the caller places at points every
// lane passes with fewer than 8 new chunks: the stores then issue from a few
// places with most lanes active, instead of from every put() with the few
// lanes whose chunk just filled (42 % fewer store instructions; the encoder
// is bound by the L1's miss queue, so this bought 1 %: DESIGN §3).
// R == 16 (line drains): drain() lets only the chunks of whole 128-byte lines
// leave; a line's first chunks wait in the ring (<= 7 held + < 8 new) until
// the line is complete or the record ends, so L2 gets every interior line of
// a tail whole, at once, instead of in pieces ~10 us apart (1M Small: HBM
// writes 1.05 -> 0.66 GB and reads 1.28 -> 0.93 GB per launch, 1.09 -> 0.99
// ms; DESIGN §3 "Round 4"). (The whole lines as non-temporal stores: 1M Small
// 0.99 -> 1.37 ms, profiles/r04/ab/enc_line_nt_ab.jsonl.)
template <int R>
struct LaneWriterT {
    uint8_t *out;
    uint64_t cpos;    // absolute offset of the current chunk (16-aligned)
    uint32_t f;       // next byte index in the chunk
    uint32_t first;   // first byte of the chunk this stream owns
    uint64_t a0, a1;  // chunk bytes 0..7, 8..15
    uint64_t hpos;    // parked head chunk (hfirst != 0): offset, first byte, bytes
    uint32_t hfirst;
    uint64_t h0, h1;
    u32x4 *ring;      // R > 0: this lane's slot 0 (slot k at ring[k * HONU_WAVE]: per-wave rings)
    uint32_t nch;     // R > 0: full chunks in the ring, ending just before cpos

    HONU_DEV void init(uint8_t *o, uint64_t pos) {
        out = o;
        cpos = pos & ~15ull;
        f = first = (uint32_t)(pos & 15);
        a0 = a1 = 0;
        hfirst = 0;
        nch = 0;
    }
    HONU_DEV void set_ring(u32x4 *r) { ring = r; }
    // bytes [from, to) of the chunk (b0, b1) at p with the widest aligned
    // stores that fit (at most 6 stores instead of one per byte)
    static HONU_DEV void store_bytes(uint8_t *p, uint32_t from, uint32_t to, uint64_t b0, uint64_t b1) {
        uint32_t j = from;
        auto bytes_at = [&](uint32_t k, uint32_t n) -> uint64_t {  // n <= 8, k + n <= 16
            uint64_t v = k < 8 ? (b0 >> (8 * k)) | (k ? b1 << (64 - 8 * k) : 0) : b1 >> (8 * (k - 8));
            return n == 8 ? v : v & ((1ull << (8 * n)) - 1);
        };
        if ((j & 1) && j < to) { p[j] = (uint8_t)bytes_at(j, 1); j += 1; }
        if ((j & 2) && j + 2 <= to) { *reinterpret_cast<uint16_t *>(p + j) = (uint16_t)bytes_at(j, 2); j += 2; }
        if ((j & 4) && j + 4 <= to) { *reinterpret_cast<uint32_t *>(p + j) = (uint32_t)bytes_at(j, 4); j += 4; }
        if (j + 8 <= to) { *reinterpret_cast<uint64_t *>(p + j) = bytes_at(j, 8); j += 8; }
        if (j + 4 <= to) { *reinterpret_cast<uint32_t *>(p + j) = (uint32_t)bytes_at(j, 4); j += 4; }
        if (j + 2 <= to) { *reinterpret_cast<uint16_t *>(p + j) = (uint16_t)bytes_at(j, 2); j += 2; }
        if (j < to) p[j] = (uint8_t)bytes_at(j, 1);
    }
    HONU_DEV void flush() {
        if (first == 0) {
            const u32x4 v{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)};
            if constexpr (R > 0) {
                ring[((cpos >> 4) & (R - 1)) * HONU_WAVE] = v;
                nch++;
            } else {
                *reinterpret_cast<u32x4 *>(out + cpos) = v;
            }
        } else {  // the head chunk: parked until finish()
            hpos = cpos;
            hfirst = first;
            h0 = a0;
            h1 = a1;
            first = 0;
        }
        cpos += 16;
    }
    // append the low n (1..8) bytes of v (bytes above n must be zero)
    HONU_DEV void put(uint64_t v, uint32_t n) {
        const uint32_t s = 8 * f;
        uint64_t t2 = 0;
        if (s < 64) {
            a0 |= v << s;
            if (s) a1 |= v >> (64 - s);
        } else {
            a1 |= v << (s - 64);
            if (s > 64) t2 = v >> (128 - s);
        }
        f += n;
        if (f >= 16) {
            flush();
            a0 = t2;
            a1 = 0;
            f -= 16;
        }
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
    // raw bytes src[0, len) (global, any alignment). 64 bytes at a time are
    // loaded as five aligned 16-byte blocks before any of them is written out
    // (the output stores may alias for the compiler, so loads cannot move past
    // them on their own); each memory instruction is a per-lane scattered
    // access, so fewer, wider ones are what the address unit needs.
    HONU_DEV void run(const uint8_t *src, uint64_t len) {
        const uint64_t a = (uint64_t)src & 15;
        const u32x4 *w = reinterpret_cast<const u32x4 *>(src - a);
        const uint64_t nw = (a + len + 15) >> 4;  // aligned blocks holding the run
        const uint32_t sh = (uint32_t)(a & 7) * 8, hw = (uint32_t)(a >> 3);
        for (uint64_t k = 0; k < len; k += 64) {
            drain();  // <= R - 1 chunks since the last one (see encode_record_lane)
            const uint64_t q0 = (a + k) >> 4;
            uint64_t x[11];
#pragma unroll
            for (int j = 0; j < 5; j++) {
                u32x4 v{0, 0, 0, 0};
                if (q0 + j < nw) v = w[q0 + j];
                x[2 * j] = ((uint64_t)v.y << 32) | v.x;
                x[2 * j + 1] = ((uint64_t)v.w << 32) | v.z;
            }
            x[10] = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint64_t off = k + 8 * j;
                if (off < len) {
                    const uint64_t take = len - off < 8 ? len - off : 8;
                    const uint64_t lo = hw ? x[j + 1] : x[j], hi = hw ? x[j + 2] : x[j + 1];
                    uint64_t v = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
                    if (take < 8) v &= (1ull << (8 * take)) - 1;
                    put(v, (uint32_t)take);
                }
            }
        }
    }
    HONU_DEV void frame(const uint8_t *var, honu_span sp) {  // lani Encode :62-77
        uv(sp.len);
        run(var + sp.off, sp.len);
    }
    // the ring's chunks to memory (no-op for R == 0)
    HONU_DEV void drain_all() {
        if constexpr (R > 0) {
            const uint64_t p0 = cpos - 16ull * nch;
            for (uint32_t k = 0; k < nch; k++)
                *reinterpret_cast<u32x4 *>(out + p0 + 16 * k) = ring[(((p0 >> 4) + k) & (R - 1)) * HONU_WAVE];
            nch = 0;
        }
    }
    // R == 16: only the chunks of whole 128-byte lines leave (see above)
    HONU_DEV void drain() {
        if constexpr (R == 16) {
            const uint64_t p0 = cpos - 16ull * nch, lim = cpos & ~127ull;
            if (p0 < lim) {
                const uint32_t cnt = (uint32_t)((lim - p0) >> 4);
                for (uint32_t k = 0; k < cnt; k++)
                    *reinterpret_cast<u32x4 *>(out + p0 + 16 * k) = ring[(((p0 >> 4) + k) & (R - 1)) * HONU_WAVE];
                nch -= cnt;
            }
        } else {
            drain_all();
        }
    }
    HONU_DEV void finish() {
        drain_all();
        if (hfirst) store_bytes(out + hpos, hfirst, 16, h0, h1);
        hfirst = 0;
        if (f > first) store_bytes(out + cpos, first, f, a0, a1);
    }
    // absolute position of the next byte
    HONU_DEV uint64_t pos() const { return cpos + f; }
    // continue at `to` (>= pos()); bytes in between are left to another writer
    HONU_DEV void jump(uint64_t to) {
        finish();
        cpos = to & ~15ull;
        f = first = (uint32_t)(to & 15);
        a0 = a1 = 0;
    }
};
using LaneWriter = LaneWriterT<0>;


// Timing build only (-DHONU_ENC_TIMING, tools/enc_timing.py): lane 0 of every
// wave records s_memrealtime at fixed points of its encode.
#ifdef HONU_ENC_TIMING
#define ENC_STAMPS 8
static __device__ uint64_t g_enc_stamps[1 << 16][ENC_STAMPS];  // per translation unit
#define ESTAMP(k)                                                                             \
    do {                                                                                      \
        const uint64_t wid_ = (uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;    \
        if (__lane_id() == 0 && wid_ < (1 << 16)) g_enc_stamps[wid_][k] = wall_clock64();     \
    } while (0)
#else
#define ESTAMP(k) \
    do {          \
    } while (0)
#endif

// ------------------------------------------------------------------------
// encode of one record by one lane (object.go:24-45, metadata.go:108-200),
// shared by the split kernels (lane.hip) and the fused kernel (fused.hip)
// ------------------------------------------------------------------------
HONU_DEV uint64_t frame_len(uint64_t len) { return uvarint_len(len) + len; }
HONU_DEV uint64_t ld64(const uint8_t *p) { return *reinterpret_cast<const uint64_t *>(p); }

// The list kernel (k_encode_acl_grp) writes an all-present ACL list's whole
// ACL_UNIT-byte units, this lane the list's bytes in the partial units at
// its two ends (16: 16-byte chunks; 64: the memory side's write unit, so
// that no unit is written by both kernels).
#ifndef ACL_UNIT
#define ACL_UNIT 16ull
#endif
// HONU_ACL_ENDS 1: the list kernel also writes the list's bytes in the partial
// 16-byte chunks at its two ends (byte stores), so this lane reads no ACL
// entry at all; 0: this lane writes them (ACL_UNIT 16).
#ifndef HONU_ACL_ENDS
#define HONU_ACL_ENDS 0
#endif
// Header + Metadata tail of one record into out[beg, end) (the payload bytes
// in between are the copy engine's). SKIP_ACL: leave the ACL entries to a
// group writer: write the fields up to uvarint(len ACL), return that position
// (| ACL_ALL_PRESENT when every entry is present: the partial 16-byte chunks
// at both ends of the list are then written here) and resume at
// end - (bytes after the list), computed from the row and regions.
// R: the writer's LDS ring (LaneWriterT; ring = this lane's slot 0). Drains
// sit where every lane has written fewer than 112 bytes since the previous one
// (< 8 chunks): between two drains at most one raw-run batch (64 bytes, run()
// drains before each) plus fixed fields of <= 48 bytes, or <= 96 bytes of
// fixed fields (uvarints counted at their 10-byte maximum).
// psrc (honu_encode_records_units): the record's payload bytes; this lane
// then also writes the payload's bytes in its first and last partial 64-byte
// units of the output (PAYLOAD_UNIT), so that the copy (EncodeSegments with
// units) writes whole units only: a 64-byte unit written partly by two
// kernels at different times costs the memory side a read-modify-write
// (DESIGN §3 "the 64-byte write unit"). A compile-time null psrc (the plain
// form's kernel) carries none of it.
template <bool SKIP_ACL, int R>
HONU_DEV uint64_t encode_record_lane(const honu_meta &m, const uint8_t *__restrict__ var,
                                     const honu_acl *__restrict__ acl,
                                     const uint32_t *__restrict__ reg, uint64_t dlen,
                                     uint64_t beg, uint64_t end, uint8_t *__restrict__ out,
                                     u32x4 *ring, const uint8_t *__restrict__ psrc = nullptr) {
    static_assert(R == 0 || ((R == 8 || R == 16) && SKIP_ACL),
                  "drain spacing assumes 8 slots (16 with line drains: <= 7 held + <= 7 new) and no ACL entries");
#define OFF(f) ((int)offsetof(honu_meta, f))
    uint64_t acl_ret = 0;
    ESTAMP(1);  // row loaded
    const uint8_t *mb = reinterpret_cast<const uint8_t *>(&m);
    const uint32_t pr = m.present;
    LaneWriterT<R> W;
    W.set_ring(ring);
    if (psrc) {  // header, then the payload's bytes in its partial end units
        W.init(out, beg);
        W.byte(HONU_STORAGE_VERSION);
        W.uv(dlen);
        const uint64_t a0 = (uint64_t)out + W.pos(), a1 = a0 + dlen;  // absolute payload range
        const uint64_t h_end = ((a0 + PAYLOAD_UNIT - 1) & ~(PAYLOAD_UNIT - 1)) < a1
                                   ? ((a0 + PAYLOAD_UNIT - 1) & ~(PAYLOAD_UNIT - 1)) : a1;
        const uint64_t t_beg = (a1 & ~(PAYLOAD_UNIT - 1)) > h_end ? (a1 & ~(PAYLOAD_UNIT - 1)) : h_end;
        W.run(psrc, h_end - a0);
        if (t_beg > h_end) W.jump(t_beg - (uint64_t)out);
        W.run(psrc + (t_beg - a0), a1 - t_beg);
        W.drain();
    } else {  // header: version byte + uvarint(len data)   object.go:30,35
        uint64_t lo, hi;
        const uint32_t hn = uvarint_bytes(dlen, lo, hi);
        out[beg] = HONU_STORAGE_VERSION;
        for (uint32_t j = 0; j < hn; j++)
            out[beg + 1 + j] = (uint8_t)(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8)));
        W.init(out, beg + 1 + uvarint_len(dlen) + dlen);
    }
    W.byte(1);                                                      // EncodeStruct(meta)
    W.put16(ld64(mb + OFF(object_id)), ld64(mb + OFF(object_id) + 8));          // :110
    W.put16(ld64(mb + OFF(collection_id)), ld64(mb + OFF(collection_id) + 8));  // :115
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
    W.drain();  // <= 33 + 63 bytes
    if (pr & HONU_HAS_SCHEMA) {                                     // :125, schema.go:30-53
        W.byte(1);
        W.frame(var, m.schema_name);
        W.uv(m.schema_major);
        W.uv(m.schema_minor);
        W.uv(m.schema_patch);
    } else {
        W.byte(0);
    }
    W.drain();  // <= 64 + 30
    W.frame(var, m.mime);                                           // :130
    W.drain();  // <= 64
    ESTAMP(2);  // header .. MIME
    W.put16(ld64(mb + OFF(owner)), ld64(mb + OFF(owner) + 8));      // :135
    W.put16(ld64(mb + OFF(group)), ld64(mb + OFF(group) + 8));      // :140
    W.byte(m.permissions);                                          // :145
    const uint64_t na = m.acl_count, ao = m.acl_off;
    W.uv(na);                                                       // :151
    const uint64_t nr = m.regions_count, ro = m.regions_off;
    ESTAMP(3);  // Owner .. ACL count
    if constexpr (SKIP_ACL) {
        const uint64_t P = W.pos();
        uint64_t sfx = uvarint_len(nr) + 3 + 1 + uvarint_len(zigzag(m.created)) +
                       uvarint_len(zigzag(m.modified));
        for (uint64_t k0 = 0; k0 < nr; k0 += 8) {
            uint32_t r8[8];
#pragma unroll
            for (int j = 0; j < 8; j++) r8[j] = k0 + j < nr ? reg[ro + k0 + j] : 0;
#pragma unroll
            for (int j = 0; j < 8; j++) sfx += k0 + j < nr ? uvarint_len(r8[j]) : 0;
        }
        if (pr & HONU_HAS_PUBLISHER) sfx += 32 + frame_len(m.ip_address.len) + frame_len(m.user_agent.len);
        if (pr & HONU_HAS_ENCRYPTION)
            sfx += frame_len(m.public_key_id.len) + frame_len(m.encryption_key.len) +
                   frame_len(m.hmac_secret.len) + frame_len(m.signature.len) + 3;
        if (pr & HONU_HAS_COMPRESSION) sfx += 1 + uvarint_len(zigzag(m.compression_level));
        const uint64_t E = end - sfx;  // the list is [P, E)
        if (na && E - P == 18 * na) {
            // every entry present (a nil entry is 1 byte): this lane writes the
            // list's bytes in the partial 16-byte chunks at both ends, so the
            // group kernel stores whole aligned chunks only
            acl_ret = P | ACL_ALL_PRESENT;
            // the list's bytes up to the first ACL_UNIT boundary and from the
            // last one on (absolute addresses of out, as k_encode_acl_grp)
            const uint64_t ab = (uint64_t)out;
            const uint64_t hu = ((ab + P + ACL_UNIT - 1) & ~(ACL_UNIT - 1)) - ab;
            const uint64_t hend = hu < E ? hu : E;
            const uint64_t tu = ((ab + E) & ~(ACL_UNIT - 1)) - ab;
            const uint64_t T = tu > hend ? tu : hend;
            auto put_n = [&](const u32x4 &v, uint32_t cnt) {  // the first cnt (<= 16) bytes of v
                const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
                if (cnt >= 8) {
                    W.put(lo, 8);
                    if (cnt == 16) W.put(hi, 8);
                    else if (cnt > 8) W.put(hi & ((1ull << (8 * (cnt - 8))) - 1), cnt - 8);
                } else if (cnt) {
                    W.put(lo & ((1ull << (8 * cnt)) - 1), cnt);
                }
            };
            // (acl_chunk: 16 bytes of the list's encoding from x, from the
            // <= 2 entries they straddle)
            if constexpr (HONU_ACL_ENDS && ACL_UNIT == 16) {  // the list kernel's, ends included
                W.jump(E);
            } else if constexpr (ACL_UNIT == 16) {  // one piece of < 16 bytes at each end, both loaded at once
                const u32x4 hv = acl_chunk(acl + ao, na, P, P);
                const u32x4 tv = E > T ? acl_chunk(acl + ao, na, P, T) : u32x4{0, 0, 0, 0};
                put_n(hv, (uint32_t)(hend - P));  // <= 43 + 15 since the drain
                if (T > hend) W.jump(T);  // the whole chunks in between are k_encode_acl_grp's
                put_n(tv, (uint32_t)(E - T));
            } else {
                W.drain();  // the ring holds < 16 chunks
                for (uint64_t x = P; x < hend; x += 16)
                    put_n(acl_chunk(acl + ao, na, P, x), (uint32_t)(hend - x < 16 ? hend - x : 16));
                if (T > hend) W.jump(T);  // the whole units in between are k_encode_acl_grp's
                for (uint64_t x = T; x < E; x += 16)
                    put_n(acl_chunk(acl + ao, na, P, x), (uint32_t)(E - x < 16 ? E - x : 16));
                W.drain();
            }
        } else {
            acl_ret = P;
            W.jump(E);
        }
    } else {
    for (uint64_t k0 = 0; k0 < na; k0 += 8) {                       // :157-162, acls.go:26-39
        uint32_t e[8][5];                                            // 8 entries ahead
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (k0 + j < na) {
                const uint32_t *a = reinterpret_cast<const uint32_t *>(acl + ao + k0 + j);
#pragma unroll
                for (int c = 0; c < 5; c++) e[j][c] = a[c];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (k0 + j < na) {
                if ((e[j][4] >> 8) & 0xFF) {
                    W.byte(1);
                    W.put16(((uint64_t)e[j][1] << 32) | e[j][0], ((uint64_t)e[j][3] << 32) | e[j][2]);
                    W.byte(e[j][4]);
                } else {
                    W.byte(0);
                }
            }
        }
    }
    }
    ESTAMP(4);  // ACL list (ends)
    W.uv(nr);                                                       // :164, region.go:137-152
    for (uint64_t k0 = 0; k0 < nr; k0 += 8) {
        uint32_t r8[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r8[j] = k0 + j < nr ? reg[ro + k0 + j] : 0;
        W.drain();  // <= 15 + 10 before the first batch, <= 40 after one
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (k0 + j < nr) W.uv(r8[j]);
    }
    W.drain();
    ESTAMP(5);  // regions
    if (pr & HONU_HAS_PUBLISHER) {                                  // :169, provenance.go:34-57
        W.byte(1);
        W.put16(ld64(mb + OFF(publisher_id)), ld64(mb + OFF(publisher_id) + 8));
        W.put16(ld64(mb + OFF(client_id)), ld64(mb + OFF(client_id) + 8));
        W.frame(var, m.ip_address);
        W.frame(var, m.user_agent);  // run() drains: <= 33 + 10, then <= 64 + 10
    } else {
        W.byte(0);
    }
    W.drain();  // <= 64
    ESTAMP(6);  // publisher
    if (pr & HONU_HAS_ENCRYPTION) {                                 // :174, encryption.go:51-89
        W.byte(1);
        W.frame(var, m.public_key_id);
        W.frame(var, m.encryption_key);
        W.frame(var, m.hmac_secret);
        W.frame(var, m.signature);
        W.byte(m.sealing_alg);
        W.byte(m.encryption_alg);
        W.byte(m.signature_alg);
    } else {
        W.byte(0);
    }
    W.drain();  // <= 64 + 3; then <= 12 + 1 + 20 to finish()
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
    ESTAMP(7);  // encryption .. end
    return acl_ret;
}
#undef OFF

}  // namespace honu
