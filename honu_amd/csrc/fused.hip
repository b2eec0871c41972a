// fused.hip — single-launch Metadata decode (honu_decode_records, and
// honu_decode_batch for large batches).
//
// The split decode (win.hip + scan.hip + grp.hip) hands per-record counts,
// positions and inline region ids between five launches through the context
// scratch; the fill re-reads the ACL bytes from HBM and patches the rows. Here
// one wave owns a tile of 64 consecutive records (one per lane) from the first
// byte to the last: the wave walks its records (win.h), the decoupled
// look-back (lookback.h) turns the counts into table offsets, and the wave
// writes every output with those offsets — rows once, region ids from
// registers, ACL entries re-read right after the walk — with no scratch round
// trips and no launch boundaries.
#include "lookback.h"
#include "win.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))

// ------------------------------------------------------------------------
// decode: Object.Metadata() + Data() + Tombstone() + StorageVersion()
// (object.go:47-134), lani walk metadata.go:202-302, tables and offsets.
// Columns: 0 ACL entries, 1 regions, 2 16-byte aligned payload bytes.
// ------------------------------------------------------------------------
struct DecodeOut {
    honu_meta *meta;
    honu_record_info *info;
    honu_acl *acl;
    uint64_t acl_cap;
    uint32_t *reg;
    uint64_t reg_cap;
    uint64_t data_cap;
    int materialize;          // data offsets into a data arena (else zero-copy)
    DecodeScratch *scratch;   // materialize: payload sources for honu_decode_payloads
    uint64_t *offs;           // materialize: offs[3i+2] = data arena offset
    uint64_t *totals;         // column totals (3)
    bool reg_inplace;         // region lists returned in place (HONU_REGIONS_INPLACE)
};

// Launches of at least this many tiles speculate (publish + ACL flags, below)
// and are followed by the guarded launch: with the flag gather gone the
// speculation pays from ~1000 tiles also with static tiles (62 K Large
// records 0.0876 -> 0.0825 ms, 64 K Small 0.092 -> 0.084; 512 tiles of Medium
// 0.0706 -> 0.0722: the guarded launch's ~4 us weighs more there).
// Measured and not kept (sources in git history, commit 88edda1): rows stored
// field by field during the walk (MemRow, 30 % slower: vmcnt counts stores,
// so every window refill also waited for the row stores); static tiles at
// every batch size (faster, but a wave's second tile would wait on tiles of
// workgroups that need not be resident: not deadlock-free beside another
// launch); the next static tile's head prefetched under the fill (no change);
// ACL entries read as two 16-byte LDS reads and a select chain (FILL_DW 0,
// slower); the measurement knobs that skip the fill, the look-back wait or
// the tickets (HONU_FUSED_DBG). DESIGN §3 has the numbers.
// (Round 4, with the grouped prefixes: 768 still right, no speculation below
// 2049 tiles is 5-7 % slower on 62 K Large / 64 K Small, from 512 equal;
// profiles/r04/ab/dec_spec_min_ab.jsonl.)
#ifndef FUSED_SPEC_MIN_TILES_N  // (A/B builds only)
#define FUSED_SPEC_MIN_TILES_N 768
#endif
constexpr uint64_t FUSED_SPEC_MIN_TILES = FUSED_SPEC_MIN_TILES_N;

// The ACL lists (every entry present) of a tile staged into the wave's LDS
// (its windows, free after the walk) for the table fill: round after round,
// the aligned 16-byte blocks of a run of whole lists, up to STAGE_SLOTS blocks,
// land by global_load_lds (one per-lane source block per slot, 1 KB per
// instruction); the entries are then read from LDS. Lists of more than
// STAGE_SLOTS blocks (over ~1,080 entries) are not staged.
#ifndef STAGE_SLOTS_N
#define STAGE_SLOTS_N 1216
#endif
constexpr uint32_t STAGE_SLOTS = STAGE_SLOTS_N;
static_assert(STAGE_SLOTS % HONU_WAVE == 0, "whole instructions");
// Launch forms: FORM_TICKET (more tiles than resident waves), FORM_STATIC
// (every tile a resident wave). (A third form for launches that need at most
// one workgroup per CU, with twice the staging area so a tile's lists stage in
// one round issued before the look-back wait, measured equal: 62 K Large
// 0.081-0.085 vs 0.082-0.084 ms, 64 K XLarge 0.0735 vs 0.0732 ms,
// profiles/r04/ab/wide_static_ab.jsonl. So was a pair form for launches of at
// most 1,024 tiles, two waves per tile, the second staging and filling every
// second ACL round in its own LDS from a plan and offsets handed over in LDS:
// parity green, 62 K Large 0.076-0.080 vs 0.077-0.080 ms, 64 K / 40 K / 16 K
// Small equal, profiles/r04/ab/dec_pair_fill_ab.jsonl.)
enum { FORM_TICKET = 0, FORM_STATIC = 1 };
template <bool B> struct BoolC { static constexpr bool value = B; };
template <int FORM> constexpr uint32_t form_slots() { return STAGE_SLOTS; }
// a wave's LDS: its windows during the walk, the staging after it
template <int FORM> constexpr uint32_t form_wave_bytes() {
    return form_slots<FORM>() * 16 + 32 > WIN_WAVE_BYTES ? form_slots<FORM>() * 16 + 32 : WIN_WAVE_BYTES;
}
static_assert(2 * HONU_WAVES_PER_BLOCK * form_wave_bytes<FORM_STATIC>() + 64 <= 160 * 1024, "2 workgroups per CU");

template <uint32_t SLOTS>
struct AclStage {
    uint64_t apos;   // this lane's first flag
    uint32_t nb, B;  // this lane's blocks, exclusive prefix over the wave
    uint32_t nacl;   // this lane's staged entries (0: not staged)
    uint32_t nbtot;  // wave-uniform: all blocks
    uint32_t start, stop, r0, r1;  // wave-uniform: the round's blocks and lanes

    HONU_DEV void init(bool fl, uint64_t apos_, uint64_t nacl_) {
        apos = apos_;
        const uint64_t b = fl ? ((apos + 18 * nacl_ + 15) >> 4) - (apos >> 4) : 0;
        const bool st = b && b <= SLOTS;
        nb = st ? (uint32_t)b : 0;
        nacl = st ? (uint32_t)nacl_ : 0;
        B = wave_excl32(nb, nbtot);
        start = 0;
        r0 = 0;
        plan();
    }
    HONU_DEV bool staged() const { return nacl != 0; }
    HONU_DEV bool more() const { return start < nbtot; }
    // the round: lanes [r0, r1) whose blocks end within start + SLOTS
    // (B + nb is non-decreasing over the lanes)
    HONU_DEV void plan() {
        const uint64_t m = __ballot(B + nb <= start + SLOTS);
        r1 = (uint32_t)__builtin_popcountll(m);
        stop = r1 < HONU_WAVE ? __builtin_amdgcn_readlane(B, r1) : nbtot;
    }
    HONU_DEV void advance() {
        start = stop;
        r0 = r1;
        plan();
    }
    // slot s of the round <- block start + s of the wave's list blocks. The
    // 64 slots of instruction k belong to a few lists: the owner of the first
    // slot by one ballot, then the lists that start inside the window in a
    // wave-uniform loop over their lanes (readlane, no lane shuffles).
    HONU_DEV void issue(uint8_t *ws, const uint8_t *__restrict__ rec) const {
        const uint32_t lane = lane_id();
#pragma unroll
        for (uint32_t k = 0; k < SLOTS / HONU_WAVE; k++) {
            const uint32_t w0 = start + HONU_WAVE * k;
            if (w0 >= stop) break;  // wave-uniform
            const uint32_t r = (uint32_t)__builtin_popcountll(__ballot(B <= w0)) - 1;
            uint32_t rb = __builtin_amdgcn_readlane(B, r);
            uint64_t ra = readlane64(apos, r);
            uint64_t heads = __ballot(B > w0 && B < w0 + HONU_WAVE);
            while (heads) {
                const uint32_t h = (uint32_t)__builtin_ctzll(heads);
                heads &= heads - 1;
                const uint32_t hb = __builtin_amdgcn_readlane(B, h);
                const uint64_t ha = readlane64(apos, h);
                if (lane >= hb - w0) {
                    rb = hb;
                    ra = ha;
                }
            }
            const uint32_t g = w0 + lane;
            if (g < stop)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(rec + 16 * ((ra >> 4) + (g - rb))),
                    (__attribute__((address_space(3))) void *)(ws + 1024 * k), 16, 0, 0);
        }
    }
    // the round's entries, from LDS, to the table (records whose ok is false
    // store nothing: capacity); lane e of a pass takes entry e of the round,
    // its list found as in issue()
    // returns true when an entry flag of the round is not 1 (checked only
    // with chk: the walk speculated that every entry is present)
    // (an entry is five aligned dword LDS reads and four v_alignbyte: 1M Small
    // 0.760 -> 0.747 ms against two 16-byte reads and window16's select chain.
    // Round 4, measured and not kept: two or four entries per lane per pass,
    // one list walk per pass (equal); and as measurement-only builds, the
    // table stores left out (1M Small 0.708 -> 0.560 ms, 62 K Large 0.082 ->
    // 0.072 ms) or the same bytes as contiguous 16-byte stores (0.693 ms,
    // 0.079 ms): the table's bytes, not the store pattern, are the cost.
    // profiles/r04/ab/dec_fill_*.jsonl)
    template <class AfterWait>
    HONU_DEV bool store(const uint8_t *ws, honu_acl *__restrict__ acl, uint64_t ao, bool ok,
                        bool chk, AfterWait after_wait) const {
        const uint32_t lane = lane_id();
        __builtin_amdgcn_s_waitcnt(0);  // the round's blocks have landed
        wave_sync();
        WSTAMP(14);  // fill: the round's wait (its DMA, and every store before it)
        after_wait();
        const bool in = lane >= r0 && lane < r1;
        uint32_t etot;
        const uint32_t epre = wave_excl32(in ? nacl : 0, etot);
        // per list: LDS offset of its first flag, table offset, capacity verdict
        const uint32_t lbase = 16 * (B - start) + (uint32_t)(apos & 15);
        const uint64_t tdst = ok ? ao : ~0ull;
        bool bad = false;
        for (uint32_t w0 = 0; w0 < etot; w0 += HONU_WAVE) {  // wave-uniform
            const uint32_t r = (uint32_t)__builtin_popcountll(__ballot(epre <= w0)) - 1;
            uint32_t rp = __builtin_amdgcn_readlane(epre, r);
            uint32_t rl = __builtin_amdgcn_readlane(lbase, r);
            uint64_t rt = readlane64(tdst, r);
            uint64_t heads = __ballot(epre > w0 && epre < w0 + HONU_WAVE);
            while (heads) {
                const uint32_t h = (uint32_t)__builtin_ctzll(heads);
                heads &= heads - 1;
                const uint32_t hp = __builtin_amdgcn_readlane(epre, h);
                const uint32_t hl = __builtin_amdgcn_readlane(lbase, h);
                const uint64_t ht = readlane64(tdst, h);
                if (lane >= hp - w0) {
                    rp = hp;
                    rl = hl;
                    rt = ht;
                }
            }
            const uint32_t e = w0 + lane;
            const uint32_t j = e - rp;
            // the ClientID's first byte in LDS, Permissions 16 bytes on
            const uint32_t q = rl + 18 * j + 1;
            uint64_t lo, hi;
            uint32_t pm;
            const uint32_t sh = q & 3u;
            const __attribute__((address_space(3))) uint32_t *w =
                (const __attribute__((address_space(3))) uint32_t *)(ws + (q & ~3u));
            const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
            lo = ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
            hi = ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, sh) << 32) | __builtin_amdgcn_alignbyte(d3, d2, sh);
            pm = (d4 >> (8 * sh)) & 0xFF;
            if (chk && e < etot)
                bad |= ((const __attribute__((address_space(3))) uint8_t *)ws)[q - 1] != 1;
            if (e < etot && rt != ~0ull) {
                uint32_t *d = reinterpret_cast<uint32_t *>(acl + rt + j);
                d[0] = (uint32_t)lo;
                d[1] = (uint32_t)(lo >> 32);
                d[2] = (uint32_t)hi;
                d[3] = (uint32_t)(hi >> 32);
                d[4] = pm | (1u << 8);
            }
        }
        WSTAMP(15);  // fill: the round's passes
        wave_sync();  // the LDS is the next round's (or the next tile's windows)
        return bad;
    }
};

// In-place ACL lists (HONU_ACL_INPLACE): the speculative walk took every list
// that fits as all present; its flags are checked here. flag_gather fetches
// the dwords holding flags [from, from + 64) of every lane's list (base: the
// list's first flag, cnt: its entries, 0 for none) into the wave's LDS, 256
// bytes per list: instruction k has lane j fetch flag j of lane k's list (a
// few cache lines per instruction, the lines the list occupies anyway).
// (lane k's flags in LDS row k, FLAG_ROW apart: win.h)
HONU_DEV void flag_gather(uint8_t *ws, const uint8_t *__restrict__ rec, uint64_t base, uint64_t cnt,
                          uint64_t from) {
    const uint32_t lane = lane_id();
    const uint64_t b = base + 18 * from;
    const uint32_t m = cnt > from ? (uint32_t)(cnt - from < HONU_WAVE ? cnt - from : HONU_WAVE) : 0;
#pragma unroll 4
    for (uint32_t k = 0; k < HONU_WAVE; k++) {
        const uint32_t mk = __builtin_amdgcn_readlane(m, k);
        if (!mk) continue;  // wave-uniform
        const uint64_t bk = readlane64(b, k);
        if (lane < mk)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(rec + ((bk + 18ull * lane) & ~3ull)),
                (__attribute__((address_space(3))) void *)(ws + FLAG_ROW * k), 4, 0, HONU_BURST_AUX);
    }
}
// After flag_gather(.., 0): true when a flag of this lane's list (chk) is not
// 1 (a nil entry or a bad flag: the walk then read the fields after the list
// at the wrong place). Lists of more than 64 entries take further bursts.
// Leaves the LDS free.
HONU_DEV bool flag_check(uint8_t *ws, const uint8_t *__restrict__ rec, bool chk, uint64_t base,
                         uint64_t cnt) {
    const uint32_t lane = lane_id();
    bool bad = false;
    for (uint64_t from = 0;; from += HONU_WAVE) {
        __builtin_amdgcn_s_waitcnt(0);  // the burst has landed
        wave_sync();
        if (chk && cnt > from) {
            const uint32_t m = (uint32_t)(cnt - from < HONU_WAVE ? cnt - from : HONU_WAVE);
            const uint64_t b = base + 18 * from;
            const __attribute__((address_space(3))) uint8_t *fl =
                (const __attribute__((address_space(3))) uint8_t *)(ws + FLAG_ROW * lane);
#pragma unroll
            for (uint32_t j = 0; j < HONU_WAVE; j++)
                if (j < m) bad |= fl[4 * j + (uint32_t)((b + 18ull * j) & 3)] != 1;
        }
        if (!__ballot(chk && cnt > from + HONU_WAVE)) break;
        wave_sync();  // every lane has read its flags before the next burst lands
        flag_gather(ws, rec, chk ? base : 0, chk ? cnt : 0, from + HONU_WAVE);
    }
    wave_sync();
    return bad;
}

// Speculative publish (the walk's early hook): a tile's counts go to the
// look-back as soon as its regions are read, ~18 us per tile before the walk
// ends, so successors wait less. A record failing in a later field has its
// counts changed to 0; its tile then raises LbState.misspec, and the guarded
// launch that follows every speculative one redoes the whole batch without
// speculation (it returns at once when the flag is clear).
struct SpecPub {
    bool on;
    bool spec_acl;  // the walk leaves the ACL entry flags to the fill (win.h NoEarly)
    uint64_t *status;
    uint64_t t;
    uint32_t ep;
    uint64_t c0, c1;            // this lane's published counts
    uint64_t x[3], agg[3];      // in-tile exclusive prefixes, tile aggregates
    HONU_DEV void counts(uint64_t a, uint64_t r, uint64_t d) {
        if (!on) return;
        c0 = a;
        c1 = r;
        x[0] = wave_excl(a, agg[0]);
        x[1] = wave_excl(r, agg[1]);
        x[2] = wave_excl(d, agg[2]);
        lb_publish<3>(status, t, ep, agg);
    }
};

// MODE 0: plain; 1: speculative publish; 2: guarded recovery (runs only when
// the speculative launch before it raised misspec). Three instantiations, so
// profiles tell the launches apart. FORM (FORM_*, chosen at launch): static
// forms give every tile a resident wave of its own (tiles <= waves): static
// tiles and grouped prefixes instead of tickets and the look-back over group
// totals (lookback.h); each form a kernel of its own, so none pays another's
// registers or LDS.
//
// In-launch recovery (ticket form, MODE 1 with `inline_rec`): instead of a
// guarded second launch, the speculative launch itself finishes the job. A
// wave whose ticket loop ends counts its tiles into LbState::tdone and waits
// until every tile of the pass is counted (the tiles it waits for are held
// by running waves: tickets are only taken by running waves, so this cannot
// deadlock, also when the grid is not resident at once); misspec is final
// then. Clean (the usual case): the wave ends. Misspeculated: every wave
// releases its stores (agent scope: the pass-1 stores of the same outputs,
// maybe from another XCD, must land after them), counts its tiles into
// rdone, and once all are released the waves decode the batch again without
// speculation from a second ticket counter, with look-back words tagged as
// pass 1 (lookback.h). No second launch waits for CU resources behind other
// kernels (a no-op guard of 78 KB workgroups spent up to
// 1.4 ms queued beside the bench's copies and encoder; the guard is now
// k_decode_guard below). Measured slower in the clean case, so off. Static
// tiles keep the guarded launch: their waves may wait on workgroups that are
// not resident yet, so a launch-wide wait could deadlock beside another
// persistent kernel.
//
// The recovery count (a measurement, honu_ctx_get_param "recoveries") in the
// context's pinned word: one thread of one wave updates it per recovery, so a
// plain load and store, no read-modify-write atomic over PCIe (which needs
// platform atomics support: ADVICE r05).
HONU_DEV void count_recovery(uint32_t *recoveries) {
    if (!recoveries) return;
    const uint32_t v = __hip_atomic_load(recoveries, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(recoveries, v + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// WPB: waves per workgroup (4; the guarded launch, k_decode_guard below: 1).
template <int MODE, int FORM, bool INPL, int WPB>
HONU_DEV void decode_fused_body(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    DecodeOut O, LbState *lb, uint64_t *lb_status, uint64_t *lb_gstatus, uint64_t lb_words,
    uint32_t *spec_seen, uint32_t *recoveries, bool inline_rec) {
    constexpr int mode = MODE;
    if (mode == 2 && __hip_atomic_load(&lb->misspec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        return;  // every wave of the launch returns: the look-back state is untouched
    // a recovery that runs tells the host (the context's pinned word), which
    // then decodes the context's next calls without speculation (api.hip)
    if (mode == 2 && spec_seen && blockIdx.x == 0 && threadIdx.x == 0) {
        __hip_atomic_store(spec_seen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        count_recovery(recoveries);  // (a count apart from the back-off flag, for measurements)
    }
    constexpr bool STAT = FORM != FORM_TICKET;
    constexpr uint32_t WAVE_BYTES = form_wave_bytes<FORM>();
    __shared__ __attribute__((aligned(16))) uint8_t smem[WPB * WAVE_BYTES];
    __shared__ uint32_t last_flag;
    __shared__ uint32_t wg_ticket;
    uint8_t *ws = smem + (threadIdx.x / HONU_WAVE) * WAVE_BYTES;
    const uint32_t lane = lane_id();
    const uint32_t ep = lb_epoch(lb);
    const uint64_t ntiles = (n + HONU_WAVE - 1) / HONU_WAVE;
    const bool ir = MODE == 1 && FORM == FORM_TICKET && inline_rec;  // in-launch recovery
    const uint64_t waves = (uint64_t)gridDim.x * WPB;
    // every tile has a resident wave of its own: static tiles (lookback.h)
    // (measured: taking the next ticket and loading its bounds before the
    // look-back wait, to overlap them with it, doubled the wait: tiles are
    // then handed out ~40 us before their waves start them, which spreads the
    // publish times of consecutive tiles)
    constexpr bool stat_idx = STAT;
    uint64_t k_static = (uint64_t)blockIdx.x * WPB + threadIdx.x / HONU_WAVE;
    WSTAMP_START();
    // ticket mode: the next tile's ticket is requested once the current tile's
    // last ACL staging round has landed (its table stores and the rest of the
    // tile then hide the atomic's round trip: -0.8 %), or at the tile's end
    // when it staged nothing. A workgroup takes the first tiles of its waves
    // with one atomic (4 tickets), so a launch starts with 512 ticket atomics
    // on the one address instead of 2,048 (1M Small 0.780 -> 0.757 ms, 262 K
    // Large 0.258 -> 0.238 ms, profiles/r03/ab/wg_ticket_ab.jsonl).
    uint32_t tk = 0;
    bool tk_pending = false;
    if constexpr (!stat_idx) {  // the same in every wave of the workgroup
        if (threadIdx.x == 0)
            wg_ticket = __hip_atomic_fetch_add(&lb->ticket, (uint32_t)WPB, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        tk = wg_ticket + threadIdx.x / HONU_WAVE;
        tk_pending = true;
    }
    uint32_t my_tiles = 0;  // tiles of pass 0 this wave decoded
    // one pass over the tiles; SPEC (compile time): speculative publish and
    // ACL flags (mode 1's first pass), so each pass is specialised
    auto tiles = [&](auto spec_c, uint32_t pass) {
    constexpr bool spec = decltype(spec_c)::value;
    const uint32_t tag = pass ? (ep | LB_PASS_BIT) : ep;  // look-back words of this pass
    uint32_t *tctr = pass ? &lb->ticket2 : &lb->ticket;
    for (;;) {
        uint64_t t;
        if constexpr (stat_idx) {
            t = k_static;
            k_static += waves;
        } else if (tk_pending) {
            t = __builtin_amdgcn_readlane(tk, 0);
            tk_pending = false;
        } else {
            t = lb_ticket(tctr);
        }
        if (t >= ntiles) break;
        if (pass == 0) my_tiles++;
        // the recovery pass tells the host (once: the wave holding its first tile)
        if (pass == 1 && t == 0 && spec_seen && lane == 0) {
            __hip_atomic_store(spec_seen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            count_recovery(recoveries);
        }
        const uint64_t i0 = t * HONU_WAVE, i = i0 + lane;
        const uint64_t lim = i0 + HONU_WAVE < n ? i0 + HONU_WAVE : n;  // the tile's records are [i0, lim)
        const bool valid = i < lim;
        TileHead H;
        tile_head_bounds(i0, rec_off, lim, H);
        tile_head_bytes(rec, H);
        WinParse P;
        RegRow R;
        SpecPub early;
        early.on = spec;
        early.spec_acl = early.on;
        early.status = lb_status;
        early.t = t;
        early.ep = tag;
        win_walk(i0, ws, rec, lim, H, R, P, early, INPL, O.reg_inplace);

        // counts -> offsets: wave scan + look-back across tiles
        uint64_t agg[3], excl[3], x0, x1, x2;
        if (early.on) {  // published during the walk; a changed count: misspeculation
            x0 = early.x[0];
            x1 = early.x[1];
            x2 = early.x[2];
            agg[0] = early.agg[0];
            agg[1] = early.agg[1];
            agg[2] = early.agg[2];
            if (__ballot(P.ntab != early.c0 || P.nreg != early.c1) && lane == 0)
                __hip_atomic_store(&lb->misspec, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const uint64_t c0 = P.ntab, c1 = P.nreg, c2 = (P.data_len + 15) & ~15ull;
            x0 = wave_excl(c0, agg[0]);
            x1 = wave_excl(c1, agg[1]);
            x2 = wave_excl(c2, agg[2]);
            // publish, then write the rows while the predecessors finish
            // (their list offsets are patched in below)
            lb_publish<3>(lb_status, t, tag, agg);
        }
        rows_out<true>(ws, R, i0, lim, O.meta);
        // table form (acl_inplace 0): the ACL lists with every entry present
        // go to the table from LDS; the first round of their blocks is staged
        // now, before the wait, as it needs no offsets
        const bool fl = !INPL && valid && P.st == HONU_OK && P.ntab && (P.acl_pos & GRP_ACL_FAST);
        AclStage<form_slots<FORM>()> S;
        S.init(fl, P.acl_pos & GRP_POS_MASK, P.ntab);
        if (S.more()) S.issue(ws, rec);
        // in-place form: a speculated list stays where it is, but its entry
        // flags must be 1. The first 64 flags of every such list come in ONE
        // burst now (instruction k: lane j fetches the dword holding flag j of
        // lane k's list into LDS), checked after the look-back wait, so the
        // round trip hides under the wait and no table bytes are written.
        // (The two forms never stage at once: an in-place list has ntab 0.)
        // (the first GRP_ACL_A0 flags the walk checked from its window)
        // (and its last GRP_ACL_TL, from the window after the list)
        const bool ichk = INPL && early.spec_acl && valid && P.st == HONU_OK &&
                          P.nacl > GRP_ACL_A0(P.acl_pos) + GRP_ACL_TL(P.acl_pos) && (P.acl_pos & GRP_ACL_FAST);
        const bool igather = INPL && early.spec_acl && __ballot(ichk);  // wave-uniform
        if (igather)
            flag_gather(ws, rec, ichk ? (P.acl_pos & GRP_POS_MASK) + 18 * GRP_ACL_A0(P.acl_pos) : 0,
                        ichk ? P.nacl - GRP_ACL_A0(P.acl_pos) - GRP_ACL_TL(P.acl_pos) : 0, 0);
        WSTAMP(10);  // publish + rows out + first staging round issued
#if defined(HONU_STAGE_TIMING) && defined(HONU_STAGE_DRAIN)
        // (timing variant: the wave's outstanding stores and loads drained
        // first, stamped as stage 14, so stage 11 is the look-back alone.
        // Measured: the drain is 0.08 us of a tile, the wait is the look-back
        // itself, 9.6 us on 1M Small, 7.3 us on a 62 K Large chunk; the
        // look-back's first loads issued before the row stores changed
        // nothing: profiles/r05/lookback/)
        if (INPL) {
            __builtin_amdgcn_s_waitcnt(0);
            WSTAMP(14);
        }
#endif
        // zero copy: a tile with no table entry (ACL and region lists in
        // place) uses none of its prefixes, so it does not wait for its
        // predecessors (the launch's last tile does, for the totals). A
        // materialising decode waits in every tile: each record's data-arena
        // offset (offs[3i+2], also for an empty payload) is the copy's sorted
        // segment start (copy.hip DecodeSegments).
        const bool need = t == ntiles - 1 || agg[0] || agg[1] || O.materialize;
        if constexpr (STAT)  // every tile runs at once: grouped prefixes (lookback.h)
            lb_resolve_grouped<3>(lb_status, lb_gstatus, t, ntiles, tag, agg, excl, need);
        else  // tickets: a decoupled look-back over the group totals (the plain
              // one over tile words, lb_resolve, measured 3 % slower on 1M Small)
            lb_resolve_grouped_lb<3>(lb_status, lb_gstatus, t, ntiles, tag, agg, excl, need);
        if (!need) excl[0] = excl[1] = excl[2] = 0;  // (offsets of zero entries: unused)
        WSTAMP(11);  // look-back wait
        // nothing is staged in the in-place form: the next ticket is requested
        // here, and the rest of the tile hides its round trip
        if (!stat_idx && igather) {
            tk = lb_ticket_issue(tctr);
            tk_pending = true;
        }
        if (t == ntiles - 1 && lane < 3)
            O.totals[lane] = lane == 0 ? excl[0] + agg[0] : (lane == 1 ? excl[1] + agg[1] : excl[2] + agg[2]);
        const uint64_t ao = excl[0] + x0, ro = excl[1] + x1, doff = excl[2] + x2;

        int32_t mst = P.st;
        if (mst == HONU_OK) {  // as honu_decode_tables: offsets first, then the capacity check
            if (P.ntab) O.meta[i].acl_off = ao;
            if (P.nreg) O.meta[i].regions_off = ro;
            if (ao + P.ntab > O.acl_cap || ro + P.nreg > O.reg_cap) mst = HONU_ERR_CAPACITY;
        }
        int32_t dst_ = P.data_status;
        uint64_t doff_out = P.data_off, dlen_out = P.data_len;
        if (O.materialize && dst_ == HONU_OK && P.data_len) {
            if (doff + P.data_len > O.data_cap) {
                dst_ = HONU_ERR_CAPACITY;
                doff_out = dlen_out = 0;
            } else {
                doff_out = doff;
            }
        }
        if (valid) {
            store_info(O.info + i, make_info(P, doff_out, dlen_out, dst_, mst));
            if (O.materialize) {
                O.scratch[i].data_src = P.data_off;
                O.offs[3 * i + 2] = doff;
            }
        }

        // region table: ids the walk kept in registers, else re-read
        const bool ok = valid && mst == HONU_OK;
        if (ok && P.nreg) {
            if (P.reg_pos & GRP_REG_INLINE) {
#pragma unroll
                for (int k = 0; k < REG_INLINE; k++)
                    if ((uint64_t)k < P.nreg) O.reg[ro + k] = P.regs[k];
            } else {
                uint64_t p = P.reg_pos & GRP_POS_MASK;
                for (uint64_t k = 0; k < P.nreg; k++) {
                    const uint64_t avail = P.end - p;
                    uint64_t lo, hi, v = 0;
                    lane_fetch16(rec, p, P.end, lo, hi);
                    const uint32_t kk = uvarint_window(lo, hi, avail < 5 ? (uint32_t)avail : 5, v);
                    O.reg[ro + k] = (uint32_t)v;
                    p += kk;
                }
            }
        }
        // ACL table, lists the staging does not take (nil entries, or longer
        // than one round): the lane walks its list from global memory
        const uint64_t apos = P.acl_pos & GRP_POS_MASK;
        bool acl_bad = false;  // spec_acl: an entry flag that is not 1
        if (ok && P.ntab && !S.staged()) {
            uint64_t p = apos;
            const bool fast_list = (P.acl_pos & GRP_ACL_FAST) != 0;
            for (uint64_t k = 0; k < P.ntab; k++) {
                uint32_t *d = reinterpret_cast<uint32_t *>(O.acl + ao + k);
                if (early.spec_acl && fast_list && rec[p] != 1) acl_bad = true;
                if (rec[p]) {
                    uint64_t lo, hi;
                    lane_fetch16(rec, p + 1, P.end, lo, hi);
                    d[0] = (uint32_t)lo;
                    d[1] = (uint32_t)(lo >> 32);
                    d[2] = (uint32_t)hi;
                    d[3] = (uint32_t)(hi >> 32);
                    d[4] = rec[p + 17] | (1u << 8);
                    p += 18;
                } else {
                    d[0] = d[1] = d[2] = d[3] = d[4] = 0;
                    p += 1;
                }
            }
        } else if (early.spec_acl && valid && P.st == HONU_OK && P.ntab && (P.acl_pos & GRP_ACL_FAST) &&
                   !S.staged()) {
            // the record failed the capacity check, so nothing is stored, but
            // its speculated list's flags still decide whether the walk read
            // the fields after the list at the right place (staged lists are
            // checked by S.store whatever the capacity verdict)
            for (uint64_t k = 0; k < P.nacl; k++)
                if (rec[apos + 18 * k] != 1) {
                    acl_bad = true;
                    break;
                }
        }
        WSTAMP(12);  // info, regions, lists with nil entries
        if (igather)
            acl_bad |= flag_check(ws, rec, ichk, (P.acl_pos & GRP_POS_MASK) + 18 * GRP_ACL_A0(P.acl_pos),
                                  P.nacl - GRP_ACL_A0(P.acl_pos) - GRP_ACL_TL(P.acl_pos));
        // staged lists: round by round, lane e of a pass takes entry e of the
        // round's entries (one run of the table per record), reads its 17
        // bytes from LDS and stores the 20-byte row
        while (S.more()) {
            const bool last = S.stop >= S.nbtot;  // wave-uniform
            acl_bad |= S.store(ws, O.acl, ao, ok, early.spec_acl, [&]() {
                if (last && !stat_idx) {
                    tk = lb_ticket_issue(tctr);
                    tk_pending = true;
                }
            });
            S.advance();
            if (S.more()) S.issue(ws, rec);
        }
        // a speculated list had an entry that is not present (nil, or a bad
        // flag): the walk read the fields after it at the wrong place. A
        // record that failed after a speculated list is not filled, so its
        // flags are unchecked: its failure may come from the speculation
        // itself, so it counts as misspeculated too (malformed input only).
        if (early.spec_acl && valid && P.st != HONU_OK && (P.acl_pos & GRP_ACL_FAST)) acl_bad = true;
        if (early.spec_acl && __ballot(acl_bad) && lane == 0)
            __hip_atomic_store(&lb->misspec, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        WSTAMP(13);  // ACL fill
    }
    };  // tiles
    tiles(BoolC<MODE == 1>{}, 0u);
    if constexpr (MODE == 1 && FORM == FORM_TICKET) {
        if (ir) {
            // in-launch recovery (above): the speculative pass is over for
            // this wave; its misspec store (sc1) has completed before its
            // tiles are counted
            __builtin_amdgcn_s_waitcnt(0);
            if (lane == 0) __hip_atomic_fetch_add(&lb->tdone, my_tiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lb_wait_count(&lb->tdone, ntiles);
            uint32_t ms = 0;
            if (lane == 0) ms = __hip_atomic_load(&lb->misspec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readlane(ms, 0)) {  // misspeculated (else: done)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // pass-0 stores reach memory
                if (lane == 0)
                    __hip_atomic_fetch_add(&lb->rdone, my_tiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lb_wait_count(&lb->rdone, ntiles);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                tk_pending = false;
                tiles(BoolC<false>{}, 1u);
            }
        }
    }
    WSTAMP_FLUSH();
    lb_finish_blocks(lb, lb_status, lb_words, gridDim.x, &last_flag, mode == 2 || ir);
}

#define HONU_FUSED_PARAMS                                                                             \
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n, DecodeOut O,   \
        LbState *lb, uint64_t *lb_status, uint64_t *lb_gstatus, uint64_t lb_words, uint32_t *spec_seen, \
        uint32_t *recoveries, bool inline_rec
#define HONU_FUSED_ARGS rec, rec_off, n, O, lb, lb_status, lb_gstatus, lb_words, spec_seen, recoveries, inline_rec

template <int MODE, int FORM, bool INPL>
__global__ __launch_bounds__(HONU_BLOCK, 2) void k_decode_fused(HONU_FUSED_PARAMS) {
    decode_fused_body<MODE, FORM, INPL, HONU_WAVES_PER_BLOCK>(HONU_FUSED_ARGS);
}

// The guarded launch (MODE 2, ticket tiles) in one-wave workgroups of 19 KB
// LDS (the four-wave ones take 78 KB). Where a no-op guard still waits is
// registers, not LDS: beside the other slot's tail encoder (k_encode_meta_lane,
// 180 VGPRs at 2 waves per SIMD: 144 of a SIMD's 512 free) no decode wave fits
// (227-255 VGPRs; capped by amdgpu_num_vgpr the walk still needs 169 with 105
// spilled), so it waits 25-60 us for an encoder wave to end in every Small
// step; beside the copies and the other kernels it takes 4-6 us (1M Mixed:
// every guard, profiles/r05/guard). VERDICT r04 item 5.
template <bool INPL>
__global__ __launch_bounds__(HONU_WAVE) void k_decode_guard(
    HONU_FUSED_PARAMS) {
    decode_fused_body<2, FORM_TICKET, INPL, 1>(HONU_FUSED_ARGS);
}

#ifdef HONU_STAGE_TIMING
extern "C" int32_t honu_debug_stage_times(void *host, uint64_t waves, int32_t reset) {
    if (reset) {
        static uint64_t zero[1 << 16][STAGES_MAX];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_stage), zero, sizeof zero) != hipSuccess) return -1;
        return 0;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stage), waves * STAGES_MAX * sizeof(uint64_t)) ==
                   hipSuccess
               ? 0
               : -1;
}
#endif

// Which of a speculated list's entry flags the walk checks itself (win.h), as
// this translation unit was built: bit 0 the first ones (window 1), bit 1 the
// last ones (window 2). Read back as the context param "walk_flag_checks", so
// tests know which nil entries cost a recovery launch.
int decode_walk_flag_checks() { return (HONU_GATHER_SKIP_WIN ? 1 : 0) | (HONU_GATHER_SKIP_WIN2 ? 2 : 0); }

hipError_t launch_decode_fused(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_meta *meta, honu_record_info *info, honu_acl *acl,
                               uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, int materialize,
                               uint64_t data_cap, DecodeScratch *scratch, uint64_t *offs,
                               uint64_t *totals, LbState *lb, uint64_t *lb_status,
                               uint64_t *lb_gstatus, uint64_t lb_words, int max_blocks, uint32_t *spec_seen,
                               uint32_t *recoveries, bool allow_spec, bool inplace, bool reg_inplace,
                               bool inline_rec, int guard_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    // (32-record tiles for batches whose 64-record tiles fill at most half the
    // resident waves, so that every SIMD walks records, measured slower with
    // the grouped prefixes too: 62 K Large 0.0742 -> 0.0774 ms, 64 K XLarge
    // zero copy 0.0766 -> 0.0803 ms; the walk's latency, not the idle SIMDs,
    // sets a short batch's time. DESIGN §3 "Round 4".)
    const uint64_t tiles = (n + HONU_WAVE - 1) / HONU_WAVE;
    uint64_t b = (tiles + HONU_WAVES_PER_BLOCK - 1) / HONU_WAVES_PER_BLOCK;
    if (max_blocks > 0 && b > (uint64_t)max_blocks) b = (uint64_t)max_blocks;
    DecodeOut O{meta, info, acl, acl_cap, reg, reg_cap, data_cap, materialize, scratch, offs, totals, reg_inplace};
    // speculation pays where tiles queue for tickets (1M Small 0.866 -> 0.840
    // ms with the publish alone, -> 0.778 with the ACL flags too) and, since
    // the flag gather is gone, in static-tile launches of ~1000 tiles and more
    // (profiles/r03/fused_spec_ab.jsonl, spec_acl_ab*.jsonl)
    const bool stat = tiles <= b * HONU_WAVES_PER_BLOCK && tiles <= (uint64_t)HONU_WAVE * LB_GROUPS;
    const dim3 grid((unsigned)b), block(HONU_BLOCK);
#define HONU_FUSED_LAUNCH_F(M, F, I)                                                                      \
    hipLaunchKernelGGL((k_decode_fused<M, F, I>), grid, block, 0, s, rec, rec_off, n, O, lb, lb_status,    \
                       lb_gstatus, lb_words, spec_seen, recoveries, inline_rec && !stat)
#define HONU_FUSED_LAUNCH(M)                                                                               \
    do {                                                                                                   \
        if (stat && inplace) HONU_FUSED_LAUNCH_F(M, FORM_STATIC, true);                                     \
        else if (stat) HONU_FUSED_LAUNCH_F(M, FORM_STATIC, false);                                          \
        else if (inplace) HONU_FUSED_LAUNCH_F(M, FORM_TICKET, true);                                        \
        else HONU_FUSED_LAUNCH_F(M, FORM_TICKET, false);                                                    \
    } while (0)
    if (tiles < FUSED_SPEC_MIN_TILES || !allow_spec) {
        HONU_FUSED_LAUNCH(0);
        return hipGetLastError();
    }
    // speculative launch, then (static tiles, or inline recovery off) the
    // guarded recovery launch (a no-op unless a record failed after publishing
    // its counts or a speculated ACL list holds a nil entry)
    HONU_FUSED_LAUNCH(1);
    if (stat || !inline_rec) {
        // one-wave workgroups, as many waves as the speculative launch had
        // (guard_blocks > 0: that many), ticket tiles whatever the batch
        // (deadlock-free with any grid, static or not)
        uint64_t gw = b * HONU_WAVES_PER_BLOCK;
        if (guard_blocks > 0 && (uint64_t)guard_blocks < gw) gw = (uint64_t)guard_blocks;
        const dim3 g2((unsigned)gw), b2(HONU_WAVE);
#ifdef HONU_AB  // (A/B build: HONU_GUARD_WIDE=1, the round-4 guard of four-wave workgroups)
        static const bool wide = getenv("HONU_GUARD_WIDE") && atoi(getenv("HONU_GUARD_WIDE")) == 1;
        if (wide) {
            HONU_FUSED_LAUNCH(2);
            return hipGetLastError();
        }
#endif
        if (inplace)
            hipLaunchKernelGGL((k_decode_guard<true>), g2, b2, 0, s, rec, rec_off, n, O, lb, lb_status,
                               lb_gstatus, lb_words, spec_seen, recoveries, false);
        else
            hipLaunchKernelGGL((k_decode_guard<false>), g2, b2, 0, s, rec, rec_off, n, O, lb, lb_status,
                               lb_gstatus, lb_words, spec_seen, recoveries, false);
    }
#undef HONU_FUSED_LAUNCH_F
#undef HONU_FUSED_LAUNCH
    return hipGetLastError();
}


#undef OFF

}  // namespace honu
