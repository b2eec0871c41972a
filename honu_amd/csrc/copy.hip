// copy.hip — the HBM-bound half of the codec: moving payload bytes.
//
// Encode copies each record's `data` (object.go:35, lani Encode's copy,
// encode.go:74) behind its header; materialising decode copies each
// Data() subslice (object.go:97) into a packed, 16-byte aligned arena.
//
// Work is split by BYTES, not by records: the segments lie back to back in a
// "logical" byte space (the source arena for encode, the destination arena
// for decode), and wave w of W owns the logical range [w*B/W, (w+1)*B/W)
// rounded to 16 bytes. A wave binary-searches its first segment once, then
// streams forward across segment boundaries, so every wave moves the same
// number of bytes whatever the record-size mix (XLarge records no longer
// make stragglers) and there is no tail of half-idle CUs at the end of a
// launch. Within a range the copy is 16 bytes per lane, UNROLL chunks in
// flight per lane, realigned with v_alignbyte when source and destination
// phases differ (encode: always, the header length varies).
#include "kernels.h"

namespace honu {

// Segment i of an encode: src = payload[payload_off[i] ...], logical start =
// payload_off[i], dst = out + out_off[i] + 1 + uvarint_len(len).
struct EncodeSegments {
    const uint8_t *payload;
    const uint64_t *payload_off;
    uint8_t *out;
    uint64_t out_cap;
    const uint64_t *out_off;
    const int32_t *status;

    HONU_DEV uint64_t start(uint64_t i) const { return payload_off[i]; }
    HONU_DEV uint64_t lo() const { return payload_off[0]; }
    HONU_DEV uint64_t end(uint64_t i, uint64_t total_abs) const {
        (void)total_abs;
        return payload_off[i + 1];
    }
    bool units;  // honu_encode_payloads_units: the encoder wrote the payload's partial end 64-byte units
    HONU_DEV bool get(uint64_t i, uint64_t &len, const uint8_t *&src, uint8_t *&dst, uint64_t &skip) const {
        // the header/tail encoder may still be running on another stream:
        // its HONU_ERR_CAPACITY is not visible here, so the capacity check
        // is repeated (nothing is written past out_cap)
        // every field loaded unconditionally (all in one round trip)
        const int32_t st = status[i];
        const uint64_t o0 = out_off[i], o1 = out_off[i + 1];
        const uint64_t s = payload_off[i];
        len = payload_off[i + 1] - s;
        src = payload + s;
        dst = out + o0 + 1 + uvarint_len(len);
        skip = 0;
        if (units) {  // the same units as lane.h encode_record_lane (absolute addresses)
            const uint64_t a0 = (uint64_t)dst, a1 = a0 + len;
            const uint64_t h_end = ((a0 + PAYLOAD_UNIT - 1) & ~(PAYLOAD_UNIT - 1)) < a1
                                       ? ((a0 + PAYLOAD_UNIT - 1) & ~(PAYLOAD_UNIT - 1)) : a1;
            const uint64_t t_beg = (a1 & ~(PAYLOAD_UNIT - 1)) > h_end ? (a1 & ~(PAYLOAD_UNIT - 1)) : h_end;
            skip = h_end - a0;
            len = t_beg - h_end;
            src += skip;
            dst += skip;
        }
        return st == HONU_OK && o1 <= out_cap && len != 0;
    }
};

// Segment i of a materialising decode: logical start = offs[3i+2] (the
// destination offset), src = rec + scratch[i].data_src.
struct DecodeSegments {
    const uint8_t *rec;
    const honu_record_info *info;
    const DecodeScratch *scratch;
    const uint64_t *offs;
    uint8_t *data;

    HONU_DEV uint64_t start(uint64_t i) const { return offs[3 * i + 2]; }
    HONU_DEV uint64_t lo() const { return 0; }
    HONU_DEV uint64_t end(uint64_t i, uint64_t total_abs) const { return i + 1 < n_ ? offs[3 * i + 5] : total_abs; }
    uint64_t n_;
    HONU_DEV bool get(uint64_t i, uint64_t &len, const uint8_t *&src, uint8_t *&dst, uint64_t &skip) const {
        skip = 0;
        const int32_t st = info[i].data_status;  // every field in one round trip
        len = info[i].data_len;
        src = rec + scratch[i].data_src;
        dst = data + offs[3 * i + 2];
        return st == HONU_OK && len != 0;
    }
};

// Segment i of honu_decode_data: logical start = offs[i] (one column, the
// destination offset), src = rec + scratch[i].data_src.
struct SpanSegments {
    const uint8_t *rec;
    const honu_record_info *info;
    const DecodeScratch *scratch;
    const uint64_t *offs;
    uint8_t *data;

    HONU_DEV uint64_t start(uint64_t i) const { return offs[i]; }
    HONU_DEV uint64_t lo() const { return 0; }
    HONU_DEV uint64_t end(uint64_t i, uint64_t total_abs) const { (void)total_abs; return offs[i + 1]; }
    HONU_DEV bool get(uint64_t i, uint64_t &len, const uint8_t *&src, uint8_t *&dst, uint64_t &skip) const {
        skip = 0;
        const int32_t st = info[i].data_status;  // every field in one round trip
        len = info[i].data_len;
        src = rec + scratch[i].data_src;
        dst = data + offs[i];
        return st == HONU_OK && len != 0;
    }
};

#define SMALL_SEG_WAVES_FACTOR 4
// average segment bytes from which a launch uses 1 / SMALL_SEG_WAVES_FACTOR of
// its waves
#ifndef COPY_FEW_WAVES_MIN
#define COPY_FEW_WAVES_MIN (64u << 10)
#endif

// TWO (the default; variant 40 of the A/B build without it): a launch of long
// segments on average (>= COPY_FEW_WAVES_MIN) gives its first 1 /
// SMALL_SEG_WAVES_FACTOR of waves the long segments (byte ranges as below,
// short segments skipped) and the other waves, which used to return at once,
// the short ones (each wave a range of segment indices, short segments
// whole): the short records of a mixed batch no longer hold up the few
// streaming waves. 1M Mixed encode + decode 1238-1248 -> 1266-1268 GiB/s on
// one box, 1152-1176 -> 1189-1230 on another (interleaved; every Large and
// XLarge payload is >= 64 KB, so those batches have no short class, and they
// measured equal within the runs' order effect; profiles/r05/copy_classes/).
// (Every wave on every segment instead: Mixed 7 % slower, the long segments'
// streams too many.)
template <class Seg, int UNROLL>
HONU_DEV void copy_short_run(const Seg &seg, uint64_t i0, uint64_t i1, uint64_t short_max) {
    uint64_t len_nx = 0, skip = 0;
    const uint8_t *src_nx = nullptr;
    uint8_t *dst_nx = nullptr;
    bool ok_nx = i0 < i1 && seg.get(i0, len_nx, src_nx, dst_nx, skip);
    for (uint64_t i = i0; i < i1; i++) {
        const uint64_t len = len_nx;
        const uint8_t *src = src_nx;
        uint8_t *dst = dst_nx;
        const bool ok = ok_nx;
        if (i + 1 < i1) ok_nx = seg.get(i + 1, len_nx, src_nx, dst_nx, skip);
        if (ok && len < short_max) wave_copy<UNROLL, 0>(dst, src, len);
    }
}

// tickets (A/B build, variant 46): the index runs' last eighths from a
// counter pair, as the long class's range tails (below)
template <class Seg, int UNROLL, bool TAILS = false>
HONU_DEV void copy_short_class(const Seg &seg, uint64_t n, uint64_t v, uint64_t V, uint64_t short_max,
                               uint32_t *tickets = nullptr) {
    if constexpr (!TAILS) {
        copy_short_run<Seg, UNROLL>(seg, n * v / V, n * (v + 1) / V, short_max);
        (void)tickets;
        return;
    }
    auto cut = [&](uint64_t u) {  // where run u's tail starts
        const uint64_t a = n * u / V, b = n * (u + 1) / V;
        return b - (((b - a) * 8) >> 6);
    };
    copy_short_run<Seg, UNROLL>(seg, n * v / V, cut(v), short_max);
    for (;;) {
        uint32_t t = 0;
        if (__lane_id() == 0) t = atomicAdd(&tickets[0], 1u);
        t = __shfl(t, 0);
        if (t >= V) break;
        copy_short_run<Seg, UNROLL>(seg, cut(t), n * (t + 1) / V, short_max);
    }
    if (__lane_id() == 0 && atomicAdd(&tickets[1], 1u) == (uint32_t)V - 1) {
        atomicExch(&tickets[0], 0u);
        atomicExch(&tickets[1], 0u);
    }
}

// The logical range [lo, hi) of a streaming wave: its first segment by binary
// search, then forward across segment boundaries (skip_short: segments under
// short_max are the short class's).
template <class Seg, int UNROLL, int NT>
HONU_DEV void copy_range(const Seg &seg, uint64_t n, uint64_t lo, uint64_t hi, bool skip_short,
                         uint64_t short_max) {
    if (lo >= hi) return;
    // largest i with start(i) <= lo
    uint64_t a = 0, b = n;  // invariant: start(a) <= lo, answer in [a, b)
    while (b - a > 1) {
        const uint64_t mid = (a + b) >> 1;
        if (seg.start(mid) <= lo) a = mid;
        else b = mid;
    }
    // A segment's descriptors (start, then status / lengths / pointers) are
    // loaded one segment ahead: issued before the current segment's copy, they
    // arrive with its loads, so a short segment costs one round trip instead
    // of three (start -> descriptors -> bytes).
    // (skip: the segment's copy starts that many bytes into it, EncodeSegments
    // with units; its logical range is then [start + skip, + len))
    uint64_t s_nx = seg.start(a), len_nx = 0, skip_nx = 0;
    const uint8_t *src_nx = nullptr;
    uint8_t *dst_nx = nullptr;
    bool ok_nx = seg.get(a, len_nx, src_nx, dst_nx, skip_nx);
    for (uint64_t i = a; i < n; i++) {
        const uint64_t s0 = s_nx, len = len_nx, s = s0 + skip_nx;
        const uint8_t *src = src_nx;
        uint8_t *dst = dst_nx;
        const bool ok = ok_nx;
        if (s0 >= hi) break;
        if (i + 1 < n) {
            s_nx = seg.start(i + 1);
            ok_nx = seg.get(i + 1, len_nx, src_nx, dst_nx, skip_nx);
        }
        if (!ok) continue;
        if (skip_short && len < short_max) continue;  // the short class's
        const uint64_t x = s > lo ? s : lo;
        const uint64_t e = s + len;
        const uint64_t y = e < hi ? e : hi;
        if (x < y)
            wave_copy<UNROLL, NT>(dst + (x - s), src + (x - s), y - x);
    }
}

// Range tails from a counter (tickets: this launch's counter pair, one line of
// a ring of COPY_TICKET_LINES lines in the context that successive copy calls
// take in turn, so copies running at once on different streams never share
// one: ADVICE r05; nullptr: off). In a launch whose segments average at least
// COPY_STEAL_MIN bytes, a streaming wave copies the first 1 - COPY_STEAL / 64
// of its range, then takes the other streaming waves' range tails, in order,
// from tickets[0]: the waves whose ranges hold fewer bytes to copy (a mixed
// batch's short segments are skipped inside them) or that share their CU with
// a metadata kernel take more tails instead of leaving the launch's end to
// the slowest. tickets[1] counts the waves done, and the last one resets both,
// so every launch finds them zero (as the look-back state; a replayed hipGraph
// too). Measured (4 interleaved rounds each, profiles/r05/copy_steal/): 1M
// Mixed encode -1.4 % per step (every copy launch -2 % in the kernel trace),
// Mixed encode + decode -2.9 %, Medium -1.2 % (-3.5 % on another box), Large
// equal; with it on 1M Small too, +1.9 % (2.6 KB payloads: hence the bound).
#define COPY_STEAL_MIN (16u << 10)
#define COPY_STEAL 8u
template <class Seg, int UNROLL, int NT, bool TWO = false, bool STAILS = false>
__global__ __launch_bounds__(HONU_BLOCK) void k_copy_segments(Seg seg, uint64_t n,
                                                               const uint64_t *__restrict__ total_p,
                                                               uint64_t short_max = COPY_FEW_WAVES_MIN,
                                                               uint32_t *tickets = nullptr,
                                                               uint32_t steal = COPY_STEAL,
                                                               uint32_t *short_tickets = nullptr) {
    uint64_t W = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    const uint64_t w = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block();
    const uint64_t base = seg.lo();
    const uint64_t total = *total_p - base;
    // Large segments stream best from few waves (DRAM rows stay open: 2 WG per
    // CU measured best); short segments are latency bound and want every wave
    // the launch has (SMALL_SEG_WAVES_FACTOR x more).
    const bool few = n && total / n >= COPY_FEW_WAVES_MIN;
    if (few) {
        const uint64_t Wall = W;
        W /= SMALL_SEG_WAVES_FACTOR;
        if constexpr (TWO) {
            if (w >= W) {
                copy_short_class<Seg, UNROLL, STAILS>(seg, n, w - W, Wall - W, short_max, short_tickets);
                return;
            }
        }
    }
    if (w >= W) return;
    auto range = [&](uint64_t v, uint64_t &lo, uint64_t &hi) {
        lo = base + ((total * v / W) & ~15ull);
        hi = (v + 1 == W) ? base + total : base + ((total * (v + 1) / W) & ~15ull);
    };
    uint64_t lo, hi;
    range(w, lo, hi);
    if (tickets && n && total / n >= COPY_STEAL_MIN) {  // uniform over the launch
        auto cut = [&](uint64_t l, uint64_t h) {  // where a range's tail starts (steal / 64 of it)
            return h - ((((h - l) * steal) >> 6) & ~15ull);
        };
        copy_range<Seg, UNROLL, NT>(seg, n, lo, cut(lo, hi), TWO && few, short_max);
        for (;;) {
            uint32_t t = 0;
            if (__lane_id() == 0) t = atomicAdd(&tickets[0], 1u);
            t = __shfl(t, 0);
            if (t >= W) break;  // each wave's last take: W of them past the tails
            uint64_t l, h;
            range(t, l, h);
            copy_range<Seg, UNROLL, NT>(seg, n, cut(l, h), h, TWO && few, short_max);
        }
        if (__lane_id() == 0 && atomicAdd(&tickets[1], 1u) == (uint32_t)W - 1) {
            atomicExch(&tickets[0], 0u);  // every wave has taken its last ticket
            atomicExch(&tickets[1], 0u);
        }
        return;
    }
    copy_range<Seg, UNROLL, NT>(seg, n, lo, hi, TWO && few, short_max);
}

#ifdef HONU_AB
// ------------------------------------------------------------------------
// Sweep form: the logical space is cut into tiles of T bytes and wave w
// copies tiles w, w+W, w+2W, ... so that at any moment all waves work inside
// one window of W*T bytes (DRAM rows opened by one wave are hit by its
// neighbours) instead of W scattered streams. A prep kernel maps every tile to
// the first segment overlapping it. T grows with the batch so the map fits
// its fixed capacity.
// ------------------------------------------------------------------------
#define SWEEP_TILE_MIN (16u << 10)

HONU_DEV uint64_t sweep_tile(uint64_t total, uint64_t map_cap) {
    uint64_t t = (total + map_cap - 1) / map_cap;
    t = (t + 4095) & ~4095ull;
    return t < SWEEP_TILE_MIN ? SWEEP_TILE_MIN : t;
}

template <class Seg>
__global__ __launch_bounds__(HONU_BLOCK) void k_tile_map(Seg seg, uint64_t n,
                                                         const uint64_t *__restrict__ total_p,
                                                         uint32_t *__restrict__ map, uint64_t map_cap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t base = seg.lo();
    const uint64_t total = *total_p - base;
    const uint64_t T = sweep_tile(total, map_cap);
    const uint64_t s = seg.start(i) - base, e = seg.end(i, *total_p) - base;
    for (uint64_t t = (s + T - 1) / T; t * T < e; t++) map[t] = (uint32_t)i;
}

template <class Seg, int UNROLL>
__global__ __launch_bounds__(HONU_BLOCK) void k_copy_sweep(Seg seg, uint64_t n,
                                                            const uint64_t *__restrict__ total_p,
                                                            const uint32_t *__restrict__ map,
                                                            uint64_t map_cap) {
    const uint64_t W = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    const uint64_t w = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block();
    const uint64_t base = seg.lo();
    const uint64_t total = *total_p - base;
    const uint64_t T = sweep_tile(total, map_cap);
    const uint64_t ntiles = (total + T - 1) / T;
    for (uint64_t t = w; t < ntiles; t += W) {
        const uint64_t lo = base + t * T;
        const uint64_t hi = lo + T < base + total ? lo + T : base + total;
        for (uint64_t i = map[t]; i < n; i++) {
            uint64_t s = seg.start(i);
            if (s >= hi) break;
            uint64_t len;
            const uint8_t *src;
            uint8_t *dst;
            uint64_t skip;
            if (!seg.get(i, len, src, dst, skip)) continue;
            s += skip;
            const uint64_t x = s > lo ? s : lo;
            const uint64_t e = s + len;
            const uint64_t y = e < hi ? e : hi;
            if (x < y) wave_copy<UNROLL, 0>(dst + (x - s), src + (x - s), y - x);
        }
    }
}

#endif  // HONU_AB

// Copy-engine variants (A/B build only, tools/tune_copy.py): 1-5 contiguous
// per-wave ranges {unroll, non-temporal}; 6-7 the sweep form; 11 / 12
// non-temporal loads only / stores only; 13-15 one unaligned 16-byte load per
// chunk instead of two aligned loads and a funnel; 40 without the short-
// segment class; 44 without the range tails (every variant but 0 and 45 runs
// without them); 45 the tails' share from HONU_COPY_STEAL; 46 the range tails
// and the short class's run tails. The product library has variant 0 only (unroll 4, default
// cache policy, two segment classes: measured fastest).
template <class Seg>
static hipError_t launch_copy(const LaunchGeom &g, const Seg &seg, uint64_t n,
                              const uint64_t *total, uint32_t *tickets, hipStream_t s) {
    const dim3 grid(g.copy_blocks * SMALL_SEG_WAVES_FACTOR), block(HONU_BLOCK);
#ifdef HONU_AB
    if (g.copy_variant >= 6 && g.copy_variant <= 7) {
        if (!g.tile_map) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_tile_map<Seg>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                           seg, n, total, g.tile_map, g.tile_map_cap);
        if (g.copy_variant == 7)
            hipLaunchKernelGGL((k_copy_sweep<Seg, 8>), grid, block, 0, s, seg, n, total, g.tile_map, g.tile_map_cap);
        else
            hipLaunchKernelGGL((k_copy_sweep<Seg, 4>), grid, block, 0, s, seg, n, total, g.tile_map, g.tile_map_cap);
        return hipGetLastError();
    }
    switch (g.copy_variant) {
    case 1: hipLaunchKernelGGL((k_copy_segments<Seg, 8, 0>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 2: hipLaunchKernelGGL((k_copy_segments<Seg, 4, 1>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 3: hipLaunchKernelGGL((k_copy_segments<Seg, 8, 1>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 4: hipLaunchKernelGGL((k_copy_segments<Seg, 2, 0>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 5: hipLaunchKernelGGL((k_copy_segments<Seg, 16, 0>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 11: hipLaunchKernelGGL((k_copy_segments<Seg, 4, 2>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 12: hipLaunchKernelGGL((k_copy_segments<Seg, 4, 3>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 13: hipLaunchKernelGGL((k_copy_segments<Seg, 4, 4>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 14: hipLaunchKernelGGL((k_copy_segments<Seg, 8, 4>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 15: hipLaunchKernelGGL((k_copy_segments<Seg, 2, 4>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 40: hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, false>), grid, block, 0, s, seg, n, total); return hipGetLastError();
    case 45: {  // the range tails' share (/ 64) from the environment (HONU_COPY_STEAL)
        static const uint32_t st = getenv("HONU_COPY_STEAL") ? (uint32_t)atoi(getenv("HONU_COPY_STEAL")) : COPY_STEAL;
        if (st > 64) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, true>), grid, block, 0, s, seg, n, total,
                           (uint64_t)COPY_FEW_WAVES_MIN, tickets, st);
        return hipGetLastError();
    }
    case 46:  // + the short class's run tails (tickets[2..3] of the kind's line)
        hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, true, true>), grid, block, 0, s, seg, n, total,
                           (uint64_t)COPY_FEW_WAVES_MIN, tickets, COPY_STEAL, tickets + 2);
        return hipGetLastError();
    case 44:  // range tails off
        hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, true>), grid, block, 0, s, seg, n, total,
                           (uint64_t)COPY_FEW_WAVES_MIN, nullptr);
        return hipGetLastError();
    case 42: {  // the short class's bound from the environment (bytes)
        static const uint64_t sm = getenv("HONU_COPY_SHORT_MAX") ? strtoull(getenv("HONU_COPY_SHORT_MAX"), nullptr, 10)
                                                                 : (uint64_t)COPY_FEW_WAVES_MIN;
        hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, true>), grid, block, 0, s, seg, n, total, sm);
        return hipGetLastError();
    }
    default: break;
    }
#endif
    hipLaunchKernelGGL((k_copy_segments<Seg, 4, 0, true>), grid, block, 0, s, seg, n, total,
                       (uint64_t)COPY_FEW_WAVES_MIN, g.copy_steal ? tickets : nullptr);
    return hipGetLastError();
}

hipError_t launch_encode_copy(const LaunchGeom &g, const uint8_t *payload,
                              const uint64_t *payload_off, uint64_t n, uint8_t *out,
                              uint64_t out_cap, const uint64_t *out_off, const int32_t *status,
                              bool units, hipStream_t s) {
    if (n == 0) return hipSuccess;
    EncodeSegments seg{payload, payload_off, out, out_cap, out_off, status, units};
    return launch_copy(g, seg, n, payload_off + n, g.copy_tickets, s);
}
// (g.copy_tickets: the launch's own counter line, api.hip copy_geom)

hipError_t launch_span_copy(const LaunchGeom &g, const uint8_t *rec, uint64_t n,
                            const honu_record_info *info, const DecodeScratch *scratch,
                            const uint64_t *offs, uint8_t *data, hipStream_t s) {
    if (n == 0) return hipSuccess;
    SpanSegments seg{rec, info, scratch, offs, data};
    return launch_copy(g, seg, n, offs + n, g.copy_tickets, s);
}

hipError_t launch_decode_copy(const LaunchGeom &g, const uint8_t *rec, uint64_t n,
                              const honu_record_info *info, const DecodeScratch *scratch,
                              const uint64_t *offs, const uint64_t *totals, uint8_t *data,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    DecodeSegments seg{rec, info, scratch, offs, data, n};
    return launch_copy(g, seg, n, totals + 2, g.copy_tickets, s);
}

}  // namespace honu
