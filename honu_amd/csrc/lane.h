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
// grid; full chunks leave as one 16-byte store, the two partial chunks at the
// ends as byte stores (their other bytes belong to neighbours).
struct LaneWriter {
    uint8_t *out;
    uint64_t cpos;    // absolute offset of the current chunk (16-aligned)
    uint32_t f;       // next byte index in the chunk
    uint32_t first;   // first byte of the chunk this stream owns
    uint64_t a0, a1;  // chunk bytes 0..7, 8..15

    HONU_DEV void init(uint8_t *o, uint64_t pos) {
        out = o;
        cpos = pos & ~15ull;
        f = first = (uint32_t)(pos & 15);
        a0 = a1 = 0;
    }
    // bytes [from, to) of the chunk with the widest aligned stores that fit
    // (at most 1 + 1 + 1 + 1 + 1 + 1 stores instead of one per byte)
    HONU_DEV void store_bytes(uint32_t from, uint32_t to) {
        uint8_t *p = out + cpos;
        uint32_t j = from;
        auto bytes_at = [&](uint32_t k, uint32_t n) -> uint64_t {  // n <= 8, k + n <= 16
            uint64_t v = k < 8 ? (a0 >> (8 * k)) | (k ? a1 << (64 - 8 * k) : 0) : a1 >> (8 * (k - 8));
            return n == 8 ? v : v & ((1ull << (8 * n)) - 1);
        };
        if ((j & 1) && j < to) { p[j] = (uint8_t)bytes_at(j, 1); j += 1; }
        if ((j & 2) && j + 2 <= to) { *reinterpret_cast<uint16_t *>(p + j) = (uint16_t)bytes_at(j, 2); j += 2; }
        if ((j & 4) && j + 4 <= to) { *reinterpret_cast<uint32_t *>(p + j) = (uint32_t)bytes_at(j, 4); j += 4; }
        if (j == 0 && to == 16) {
            *reinterpret_cast<u32x4 *>(p) = u32x4{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)};
            return;
        }
        if (j + 8 <= to) { *reinterpret_cast<uint64_t *>(p + j) = bytes_at(j, 8); j += 8; }
        if (j + 4 <= to) { *reinterpret_cast<uint32_t *>(p + j) = (uint32_t)bytes_at(j, 4); j += 4; }
        if (j + 2 <= to) { *reinterpret_cast<uint16_t *>(p + j) = (uint16_t)bytes_at(j, 2); j += 2; }
        if (j < to) p[j] = (uint8_t)bytes_at(j, 1);
    }
    HONU_DEV void flush() {
        if (first == 0)
            *reinterpret_cast<u32x4 *>(out + cpos) =
                u32x4{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)};
        else
            store_bytes(first, 16);
        first = 0;
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
    // raw bytes src[0, len) (global, any alignment). Words are loaded 64 bytes
    // at a time before any of them is written out: the output stores may
    // alias for the compiler, so loads cannot move past them on their own.
    HONU_DEV void run(const uint8_t *src, uint64_t len) {
        const uint64_t a = (uint64_t)src & 7;
        const uint64_t *w = reinterpret_cast<const uint64_t *>(src - a);
        const uint64_t nw = (a + len + 7) >> 3;  // aligned words holding the run
        for (uint64_t k = 0; k < len; k += 64) {
            const uint64_t q0 = (a + k) >> 3;
            uint64_t x[9];
#pragma unroll
            for (int j = 0; j < 9; j++) x[j] = (q0 + j < nw) ? w[q0 + j] : 0;
            const uint32_t sh = (uint32_t)(a & 7) * 8;  // same phase every batch
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint64_t off = k + 8 * j;
                if (off < len) {
                    const uint64_t take = len - off < 8 ? len - off : 8;
                    uint64_t v = sh ? (x[j] >> sh) | (x[j + 1] << (64 - sh)) : x[j];
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
    HONU_DEV void finish() {
        if (f > first) store_bytes(first, f);
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

}  // namespace honu
