// lookback.h — single-pass exclusive scan across a launch (decoupled
// look-back) for the fused codec kernels: one TILE per wave (64 records, one
// per lane), tiles handed out in order by an atomic ticket, so a wave that
// waits on an earlier tile waits on a wave that is already running.
//
// Every tile publishes, per column, a 64-bit status word: its aggregate as
// soon as its own records are counted, then its inclusive prefix once the
// look-back has found it. A waiting wave reads the 64 preceding tiles' words
// at once (one per lane), sums back to the nearest inclusive prefix and
// spins only while a tile in between has not published.
//
// Status word: bits 63:62 flag (0 none, 1 aggregate, 2 inclusive), 61:43 the
// tag: the launch epoch (18 bits) and, above it, the pass (the single-launch
// decode's in-launch recovery pass writes pass-1 words over the pass-0 ones,
// fused.hip), 42:0 the value (< 2^43: the counts are bounded by the bytes of
// one arena). Words of earlier launches carry another epoch, so the
// array is never cleared between launches; the end of a launch resets the
// ticket, advances the epoch and, when the epoch wraps, clears the array:
// lb_finish_blocks (the last workgroup to finish) ends every single-launch
// decode (fused.hip, static tiles and tickets alike); lb_finish (the wave
// holding the last ticket) ends the scans (scan.hip).
// Launch at most as many waves as fit the chip at once: every ticket is one
// atomic on one address, so tickets should be few per wave, not per tile.
// Nothing is passed from the host per launch, so the kernels replay from a
// captured hipGraph.
#pragma once

#include "common.h"

namespace honu {

struct LbState {
    uint32_t ticket;   // next tile
    uint32_t done;     // workgroups finished (static tiles, lb_finish_blocks)
    uint32_t epoch;
    uint32_t misspec;  // speculative decode: a tile published counts that changed (fused.hip)
    uint32_t ticket2;  // next tile of the in-launch recovery pass (fused.hip)
    uint32_t _pad0[27];
    // in-launch recovery counters, polled by the waves that finished early: a
    // line of their own, away from the ticket the other waves still take
    uint32_t tdone;    // tiles of the speculative pass finished
    uint32_t rdone;    // tiles whose stores were released before the recovery pass
    uint32_t _pad1[30];
};
static_assert(sizeof(LbState) == 256, "two 128-byte lines");

constexpr uint32_t LB_EPOCH_BITS = 18;
constexpr uint32_t LB_EPOCH_MASK = (1u << LB_EPOCH_BITS) - 1;
constexpr uint32_t LB_PASS_BIT = 1u << LB_EPOCH_BITS;  // in a tag: the recovery pass
constexpr uint32_t LB_TAG_MASK = (1u << (LB_EPOCH_BITS + 1)) - 1;
constexpr uint32_t LB_TAG_SHIFT = 43;
constexpr uint64_t LB_VAL_MASK = (1ull << LB_TAG_SHIFT) - 1;

// tag: the launch epoch, | LB_PASS_BIT in a recovery pass
HONU_DEV uint64_t lb_word(uint32_t flag, uint32_t tag, uint64_t v) {
    return ((uint64_t)flag << 62) | ((uint64_t)(tag & LB_TAG_MASK) << LB_TAG_SHIFT) | (v & LB_VAL_MASK);
}
// a word of this launch (and pass)?
HONU_DEV bool lb_tagged(uint64_t w, uint32_t tag) {
    return (w >> 62) != 0 && ((uint32_t)(w >> LB_TAG_SHIFT) & LB_TAG_MASK) == (tag & LB_TAG_MASK);
}
HONU_DEV uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
HONU_DEV void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The launch's epoch (wave-uniform; only the launch's last wave changes it).
HONU_DEV uint32_t lb_epoch(LbState *s) {
    return uniform32(__hip_atomic_load(&s->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// The ticket atomic alone (lane 0's return value; read it with
// readlane(v, 0) when needed, so its round trip overlaps other work).
// ctr: &LbState::ticket, or ::ticket2 in a recovery pass.
HONU_DEV uint32_t lb_ticket_issue(uint32_t *ctr) {
    uint32_t t = 0;
    if (lane_id() == 0) t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return t;
}
HONU_DEV uint32_t lb_ticket_issue(LbState *s) { return lb_ticket_issue(&s->ticket); }

// Next tile for this wave (wave-uniform).
HONU_DEV uint64_t lb_ticket(uint32_t *ctr) { return __builtin_amdgcn_readlane(lb_ticket_issue(ctr), 0); }
HONU_DEV uint64_t lb_ticket(LbState *s) { return lb_ticket(&s->ticket); }

// Tile t of the launch with per-column aggregates agg[c] (wave-uniform):
// publishes them, returns the exclusive prefixes of the tile in excl[c] and
// publishes the inclusive ones. status holds K words per tile.
// lb_scan in two halves, so that a wave can do work that needs no offsets
// between publishing its aggregates and waiting for its predecessors.
template <int K>
HONU_DEV void lb_publish(uint64_t *status, uint64_t t, uint32_t ep, const uint64_t (&agg)[K]) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int c = 0; c < K; c++)
        if (lane == (uint32_t)c) lb_store(status + t * K + c, lb_word(t == 0 ? 2 : 1, ep, agg[c]));
}
template <int K>
HONU_DEV void lb_resolve(uint64_t *status, uint64_t t, uint32_t ep, const uint64_t (&agg)[K],
                         uint64_t (&excl)[K]);

template <int K>
HONU_DEV void lb_scan(uint64_t *status, uint64_t t, uint32_t ep, const uint64_t (&agg)[K],
                      uint64_t (&excl)[K]) {
    lb_publish<K>(status, t, ep, agg);
    lb_resolve<K>(status, t, ep, agg, excl);
}

template <int K>
HONU_DEV void lb_resolve(uint64_t *status, uint64_t t, uint32_t ep, const uint64_t (&agg)[K],
                         uint64_t (&excl)[K]) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int c = 0; c < K; c++) excl[c] = 0;
    if (t == 0) return;  // published as inclusive already
    int64_t top[K];
    bool done[K];
#pragma unroll
    for (int c = 0; c < K; c++) {
        top[c] = (int64_t)t - 1;
        done[c] = false;
    }
    for (;;) {
        bool all = true;
#pragma unroll
        for (int c = 0; c < K; c++) {
            if (done[c]) continue;
            const int64_t idx = top[c] - (int64_t)lane;  // lane 0: the nearest tile
            const uint64_t w = idx >= 0 ? lb_load(status + (uint64_t)idx * K + c)
                                        : lb_word(2, ep, 0);  // before tile 0: prefix 0
            const uint32_t fl = (uint32_t)(w >> 62);
            const bool ready = lb_tagged(w, ep);
            const uint64_t nb = __ballot(!ready);
            const uint64_t ib = __ballot(ready && fl == 2);
            const uint32_t p = ib ? (uint32_t)__builtin_ctzll(ib) : 64;  // nearest inclusive
            const uint64_t upto = p >= 63 ? ~0ull : ((2ull << p) - 1);   // lanes 0..p
            if (nb & upto) {  // a tile in between has not published yet
                all = false;
                continue;
            }
            excl[c] += wave_sum(lane <= p ? (w & LB_VAL_MASK) : 0);
            if (p < 64) {
                done[c] = true;
            } else {
                top[c] -= 64;
                all = false;
            }
        }
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int c = 0; c < K; c++)
        if (lane == (uint32_t)c) lb_store(status + t * K + c, lb_word(2, ep, excl[c] + agg[c]));
}

// lb_resolve for launches whose tiles all run at once (static tiles, at most
// LB_GROUPS x 64 tiles). There the decoupled look-back is slow for late
// tiles: every tile publishes its aggregate at about the same time, and the
// inclusive prefixes appear 64 tiles per round trip, so tile t sums back over
// t / 64 windows, one round trip each (~16 for the last tile of a 1,000-tile
// launch). Here tiles are grouped by 64: a tile reads its group's earlier
// aggregates and the previous groups' totals in ONE batch of loads (two per
// lane per column) and spins only on words not yet published; the group's last
// tile publishes the group total (status words gstatus[g * K + c], tagged like
// the tile words) as soon as its group's aggregates are in, before it looks at
// earlier groups, so no total waits on another: a prefix is two round trips
// after the aggregates. Tile words keep their aggregates (no inclusive
// prefixes are written).
//
// need (wave-uniform; both grouped forms): false for a tile that uses none of
// its prefixes (a zero-copy tile with no table entry of its own, and not the
// launch's last tile, which writes the totals): it does not wait for its
// predecessors at all, and excl is then meaningless (the caller zeroes it). A
// group's last tile still publishes the group's aggregate (it waits only for
// its own group's tile aggregates); in the ticket form it publishes the
// group's inclusive prefix only when it needed its own, so a later tile that
// needs offsets may sum further back over aggregates (64 groups per round
// trip). With the ACL and region lists returned in place a zero-copy decode's
// tiles need nothing (fused.hip).
constexpr uint32_t LB_GROUPS = 64;
template <int K>
HONU_DEV void lb_resolve_grouped(uint64_t *status, uint64_t *gstatus, uint64_t t, uint64_t ntiles,
                                 uint32_t ep, const uint64_t (&agg)[K], uint64_t (&excl)[K],
                                 bool need = true) {
    const uint32_t lane = lane_id();
    const uint64_t g = t / HONU_WAVE, r = t % HONU_WAVE;
    const bool closer = r == HONU_WAVE - 1 && t + 1 < ntiles;  // the last group's total is not needed
    // wave-uniform bit masks of the parts still missing: bit c this group's
    // tiles before t (r of them), bit K + c the totals of groups 0 .. g - 1
    uint32_t todo = need || closer ? (1u << K) - 1 : 0;
    if (g && need) todo |= ((1u << K) - 1) << K;
#pragma unroll
    for (int c = 0; c < K; c++) excl[c] = 0;
    for (;;) {
#pragma unroll
        for (int c = 0; c < 2 * K; c++) {
            if (!(todo & (1u << c))) continue;
            const bool grp = c >= K;
            const int col = grp ? c - K : c;
            const uint64_t n_in = grp ? g : r;
            const uint64_t *src = grp ? gstatus + (uint64_t)lane * K + col
                                      : status + (g * HONU_WAVE + lane) * K + col;
            const uint64_t w = lane < n_in ? lb_load(src) : lb_word(1, ep, 0);
            const bool ready = lb_tagged(w, ep);
            if (__ballot(!ready)) continue;
            const uint64_t sum = wave_sum(w & LB_VAL_MASK);
            excl[col] += sum;
            todo &= ~(1u << c);
            if (!grp && closer && lane == 0) lb_store(gstatus + g * K + col, lb_word(1, ep, sum + agg[col]));
        }
        if (!todo) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

// The grouped prefixes for ticket launches (tiles taken in order by running
// waves, more tiles than waves): the group totals get a decoupled look-back of
// their own. Tile words stay aggregates; group g's last tile publishes the
// group total as soon as its group's aggregates are in (flag 1), and its
// inclusive prefix through group g once it has its own prefix (flag 2). A tile
// sums its group's earlier aggregates (one batch of loads) and looks back over
// the group words, 64 groups (4,096 tiles) per round trip, to the nearest
// inclusive one; groups resolve in ticket order, so that is one or two round
// trips where the tile-level look-back took two or three.
template <int K>
HONU_DEV void lb_resolve_grouped_lb(uint64_t *status, uint64_t *gstatus, uint64_t t, uint64_t ntiles,
                                    uint32_t ep, const uint64_t (&agg)[K], uint64_t (&excl)[K],
                                    bool need = true) {
    const uint32_t lane = lane_id();
    const uint64_t g = t / HONU_WAVE, r = t % HONU_WAVE;
    const bool closer = r == HONU_WAVE - 1 && t + 1 < ntiles;
    uint32_t todo = need || closer ? (1u << K) - 1 : 0;  // bit c: this group's tiles before t
    if (g && need) todo |= ((1u << K) - 1) << K;         // bit K + c: the groups before g
    int64_t top[K];
    uint64_t in_sum[K];
#pragma unroll
    for (int c = 0; c < K; c++) {
        excl[c] = 0;
        in_sum[c] = 0;
        top[c] = (int64_t)g - 1;
    }
    for (;;) {
#pragma unroll
        for (int c = 0; c < 2 * K; c++) {
            if (!(todo & (1u << c))) continue;
            if (c < K) {
                const uint64_t w = lane < r ? lb_load(status + (g * HONU_WAVE + lane) * K + c) : lb_word(1, ep, 0);
                const bool ready = lb_tagged(w, ep);
                if (__ballot(!ready)) continue;
                in_sum[c] = wave_sum(w & LB_VAL_MASK);
                excl[c] += in_sum[c];
                todo &= ~(1u << c);
                if (closer && lane == 0) lb_store(gstatus + g * K + c, lb_word(1, ep, in_sum[c] + agg[c]));
            } else {
                const int col = c - K;
                const int64_t idx = top[col] - (int64_t)lane;  // lane 0: the nearest group
                const uint64_t w = idx >= 0 ? lb_load(gstatus + (uint64_t)idx * K + col) : lb_word(2, ep, 0);
                const uint32_t fl = (uint32_t)(w >> 62);
                const bool ready = lb_tagged(w, ep);
                const uint64_t nb = __ballot(!ready), ib = __ballot(ready && fl == 2);
                const uint32_t p = ib ? (uint32_t)__builtin_ctzll(ib) : 64;
                const uint64_t upto = p >= 63 ? ~0ull : ((2ull << p) - 1);
                if (nb & upto) continue;
                excl[col] += wave_sum(lane <= p ? (w & LB_VAL_MASK) : 0);
                if (p < 64) todo &= ~(1u << c);
                else top[col] -= 64;
            }
        }
        if (!todo) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (closer && need) {  // the group's inclusive prefix: this tile's own inclusive one
#pragma unroll
        for (int c = 0; c < K; c++)
            if (lane == (uint32_t)c) lb_store(gstatus + g * K + c, lb_word(2, ep, excl[c] + agg[c]));
    }
}

// Spin (wave-uniform) until *ctr >= target: the in-launch recovery's waits
// for the tiles of a pass, which running waves hold (fused.hip).
HONU_DEV void lb_wait_count(uint32_t *ctr, uint64_t target) {
    for (;;) {
        uint32_t d = 0;
        if (lane_id() == 0) d = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint64_t)__builtin_amdgcn_readlane(d, 0) >= target) return;
        // ~0.9 us between polls: up to ~2,000 waiting waves poll one address
        __builtin_amdgcn_s_sleep(32);
    }
}

// The scans' end (scan.hip; the single-launch decode ends in lb_finish_blocks).
// Called by every wave with the ticket that ended its loop (t_end >= ntiles):
// a wave takes that ticket only after finishing its last tile, so the wave
// holding ticket ntiles + waves - 1 is the last one of the launch. It resets
// the ticket and advances the epoch; on a wrap of the epoch it clears the
// status array (status_words words) first.
HONU_DEV void lb_finish(LbState *s, uint64_t *status, uint64_t status_words, uint64_t t_end,
                        uint64_t ntiles, uint32_t waves) {
    if (t_end != ntiles + waves - 1) return;
    const uint32_t lane = lane_id();
    const uint32_t e = (lb_epoch(s) + 1) & LB_EPOCH_MASK;
    if (e == 0)
        for (uint64_t k = lane; k < status_words; k += HONU_WAVE) lb_store(status + k, 0);
    if (lane == 0) {
        __hip_atomic_store(&s->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->epoch, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Static tiles instead of tickets, for a launch whose tiles all fit its
// resident waves (one tile per wave, tile = the wave's global index). A wave
// waits only on lower-numbered tiles, i.e. on waves of its own or of
// lower-numbered workgroups. Forward progress RELIES ON IN-ORDER WORKGROUP
// DISPATCH (the assumption CUB's blockIdx-tiled decoupled look-back makes):
// the dispatcher launches a grid's workgroups in blockIdx order, so every
// workgroup a waiting wave depends on was dispatched before it and is resident
// or finished, also when kernels of other streams hold part of the chip and
// this grid is not resident all at once (tests/test_lookback.py runs the
// decode in this mode beside a copy that fills the CUs). Saves the launch-time burst of ticket
// atomics on one address (~20 us for 2048 waves). The last workgroup to
// finish (one atomic per workgroup) resets the count and the ticket and
// advances the epoch; on a wrap of the epoch it clears the status array first.
// Also the end of a ticket launch whose waves take their next ticket before
// finishing the current tile (the ticket order alone then no longer tells
// which wave ends last). Called by every thread of the workgroup; flag: one
// word of LDS.
HONU_DEV void lb_finish_blocks(LbState *s, uint64_t *status, uint64_t status_words, uint32_t nblocks,
                               uint32_t *flag, bool clear_misspec = false) {
    __syncthreads();
    if (threadIdx.x == 0)
        *flag = __hip_atomic_fetch_add(&s->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                nblocks - 1;
    __syncthreads();
    if (!*flag) return;
    const uint32_t e = (lb_epoch(s) + 1) & LB_EPOCH_MASK;
    if (e == 0)
        for (uint64_t k = threadIdx.x; k < status_words; k += blockDim.x) lb_store(status + k, 0);
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&s->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->ticket2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->tdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->rdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (clear_misspec) __hip_atomic_store(&s->misspec, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&s->epoch, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace honu
