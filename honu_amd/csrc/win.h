// win.h — the Metadata walk with one record per LANE reading through per-lane
// LDS windows, shared by the split parse (win.hip) and the fused decode
// (fused.hip).
//
// One record per lane keeps the serial lani walk cheap (64 records per
// wave-instruction stream), but a lane that fetches its own bytes makes every
// load instruction touch 64 cache lines (one per record): measured TA-bound,
// ~50 L1 tag lookups per load instruction and 3-6x L2 read amplification.
// Here the wave moves each lane's next bytes into a per-lane LDS window with
// global_load_lds (16 consecutive lanes of one instruction read one record's
// 256 contiguous bytes) and the lanes walk from LDS.
//
// A window is a RING of 16 blocks of 16 bytes: block B of the arena lives in
// slot B % 16, so moving the window forward fetches only the blocks it did not
// hold, and blocks at or past the record's end are never fetched (the walk
// never reads them; a field that straddles the end fails on the length check
// before its bytes matter). Windows move at fixed points of the grammar where
// the whole wave is converged: the start of the tail, every ~14 ACL entries
// while the entry flags are checked, after the ACL list and after the
// signature. A field outside the lane's window is read from global memory, so
// the window placement only affects speed, never results.
#pragma once

#include "kernels.h"
#include "lane.h"

namespace honu {

#define GO_MAX_ALLOC (1ull << 48)  // runtime maxAlloc, linux/amd64

// The pad slot of every window (slot 16, there for bank spreading) holds a
// copy of ring slot 0, so a 16-byte field read is five aligned dword reads
// with no wrap and four v_alignbyte, not two 16-byte reads and a per-lane
// select chain (1M Small zero copy 0.751 -> 0.736 ms, 262 K Large 239 -> 234
// us, split parse of 16 K Small 63.2 -> 61.8 us;
// profiles/r03/ab/win_mirror_ab.jsonl)
constexpr uint32_t WB = 256;           // window bytes per lane (16 blocks)
constexpr uint32_t WSL = WB / 16 + 1;  // LDS stride in 16-byte slots: one pad slot per
                                       // window puts the lanes of a ds_read_b128 group
                                       // on different banks
constexpr uint32_t WS = WSL * 16;
constexpr uint64_t NOWIN = ~0ull;
// Where a window starts: the 64-byte unit holding the walk's position, so
// that a window ends on a unit boundary and the next refill does not fetch
// its last line's rest again (16: the block; 128: the line, which leaves too
// little of the window ahead, 1.5-4 % slower). HONU_GATHER_SKIP_WIN: below,
// at the ACL flag burst. Both defaults measured in round 6
// (profiles/r06/gather_skip/): the decode reads 1.625 -> 1.448 GB per 1M
// records zero copy and 1.627 -> 1.461 GB materialising at equal time; the
// line model (tools/decode_line_model.py) predicts both within 1 %.
// Cache policy of the window refills and of the ACL flag bursts (the aux
// operand of global_load_lds): 2 = nt, evict first, so that the lines read
// twice — a record's last line is the next record's header line, which the
// tile head read with the default policy — stay in the L2 longer (1M records
// zero copy: reads 1.447 -> 1.354 GB at equal time, profiles/r06/nt/; 0 for
// the default policy).
#ifndef HONU_WIN_AUX
#define HONU_WIN_AUX 2
#endif
#ifndef HONU_BURST_AUX
#define HONU_BURST_AUX 2
#endif
#ifndef HONU_GATHER_SKIP_WIN
#define HONU_GATHER_SKIP_WIN 1
#endif
#ifndef HONU_GATHER_SKIP_WIN2
#define HONU_GATHER_SKIP_WIN2 0
#endif
#ifndef HONU_WIN_ALIGN
#define HONU_WIN_ALIGN 64
#endif
static_assert(HONU_WIN_ALIGN >= 16 && HONU_WIN_ALIGN <= 128 && (HONU_WIN_ALIGN & (HONU_WIN_ALIGN - 1)) == 0,
              "a power of two from a block to half the window");
HONU_DEV uint64_t win_base(uint64_t p) { return p & ~(uint64_t)(HONU_WIN_ALIGN - 1); }
// windows + per-lane wanted base, previous base and fetch limit
constexpr uint32_t WIN_WAVE_BYTES = HONU_WAVE * WS + 3 * HONU_WAVE * 8;
// The ACL flag gathers (the walk below, fused.hip flag_gather): lane k's flags
// land in LDS row k; rows are 65 dwords apart, so when every lane reads flag j
// of its own row the 64 reads fall on 64 different banks (with 64-dword rows
// they all hit bank j, a 64-way conflict per flag: 1M Small zero copy
// 2.5 % slower, profiles/r05/lds/).
constexpr uint32_t FLAG_ROW = 4 * (HONU_WAVE + 1);
static_assert(FLAG_ROW * HONU_WAVE <= WIN_WAVE_BYTES, "the flag rows fit a wave's windows");
// region ids of a record kept in registers by the walk (the generator writes
// at most 9); longer lists are re-read from the record by the fill
constexpr int REG_INLINE = 9;

struct LaneWin {
    uint8_t *wave;      // this wave's windows (LDS)
    uint64_t *wants;    // 64 requested bases (LDS)
    uint64_t *olds;     // 64 previous bases (LDS)
    uint64_t *lims;     // 64 fetch limits: blocks starting at or past them are not fetched
    const uint8_t *rec;
    uint64_t wb;        // absolute offset of this lane's window start, NOWIN if none
    uint32_t lane;

    HONU_DEV void init(uint8_t *wave_smem, const uint8_t *records, uint64_t lim) {
        wave = wave_smem;
        wants = reinterpret_cast<uint64_t *>(wave + HONU_WAVE * WS);
        olds = wants + HONU_WAVE;
        lims = olds + HONU_WAVE;
        rec = records;
        wb = NOWIN;
        lane = lane_id();
        lims[lane] = lim;
    }
    HONU_DEV const uint8_t *mine() const { return wave + lane * WS; }
    HONU_DEV const uint8_t *slot(uint64_t blk) const { return mine() + (uint32_t)(blk & 15) * 16; }

    // All 64 lanes: lane L's window becomes [want_L, want_L + WB) unless
    // want_L == NOWIN (want 16-aligned). Slot s of the wave's window array is
    // window s / WSL, ring slot s % WSL; instruction k writes slots 64k .. 64k+63.
    HONU_DEV void refill(uint64_t want) {
        wants[lane] = want;
        olds[lane] = wb;
        wave_sync();
#pragma unroll
        for (uint32_t k = 0; k < WSL; k++) {
            const uint32_t s = 64 * k + lane;
            const uint32_t L = s / WSL, c = s % WSL;
            const uint64_t b = wants[L];
            if (b != NOWIN) {  // slot 16 mirrors ring slot 0 (fetch16 reads across the wrap)
                const uint64_t w0 = b >> 4;
                const uint64_t blk = w0 + (((c & 15) - w0) & 15);  // the block of [w0, w0+16) in slot c
                const uint64_t o = olds[L];
                const bool held = o != NOWIN && blk >= (o >> 4) && blk < (o >> 4) + 16;
                if (!held && 16 * blk < lims[L])
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void *)(rec + 16 * blk),
                        (__attribute__((address_space(3))) void *)(wave + 1024 * k), 16, 0, HONU_WIN_AUX);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
        if (want != NOWIN) wb = want;
    }
    HONU_DEV bool in(uint64_t p) const { return wb != NOWIN && p >= wb && p - wb < WB; }
    HONU_DEV uint32_t at(uint64_t p) const {  // in(p)
        return ((const __attribute__((address_space(3))) uint8_t *)slot(p >> 4))[p & 15];
    }
    // The LDS and the global read stay two instructions of their own address
    // spaces: a select between the two pointers compiles to flat_load_ubyte
    // (counted by both vmcnt and lgkmcnt, LDS hits at flat latency).
    HONU_DEV uint32_t u8(uint64_t p) const {
        if (in(p)) return at(p);
        return ((const __attribute__((address_space(1))) uint8_t *)rec)[p];
    }
    HONU_DEV void fetch16(uint64_t p, uint64_t end, uint64_t &lo, uint64_t &hi) const {
        if (wb != NOWIN && p >= wb && p - wb <= WB - 16) {
            // [p, p + 16) as five aligned dwords of the lane's slots (slot 16
            // mirrors slot 0, so the run never wraps) and four v_alignbyte
            const uint32_t o = ((uint32_t)(p >> 4) & 15) * 16 + (uint32_t)(p & 15);
            const uint32_t sh = o & 3;
            const __attribute__((address_space(3))) uint32_t *w =
                (const __attribute__((address_space(3))) uint32_t *)(mine() + (o & ~3u));
            const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
            lo = ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32) | __builtin_amdgcn_alignbyte(d1, d0, sh);
            hi = ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, sh) << 32) | __builtin_amdgcn_alignbyte(d3, d2, sh);
            return;
        }
        lane_fetch16(rec, p, end, lo, hi);
    }
};

struct WDec {  // lani.Decoder (lani/decode.go) over [tstart, end), as LaneDec
    const LaneWin *w;
    uint64_t p, end, tstart;

    HONU_DEV int u8(uint32_t &v) {  // DecodeByte :94-103
        if (p >= end) return HONU_ERR_EOF;
        v = w->u8(p);
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
        w->fetch16(p, end, lo, hi);
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
        w->fetch16(p, end, lo, hi);
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

#define HONU_SKIP 0x7fffffff  // lane without a walk (past n)

// Timing build only (-DHONU_WALK_TIMING, tools/walk_timing.py): lane 0 of every
// wave records s_memrealtime (100 MHz) at fixed points of its first walk.
#ifdef HONU_WALK_TIMING
#define WALK_STAMPS 10
static __device__ uint64_t g_walk_stamps[1 << 16][WALK_STAMPS];  // per translation unit
#define WSTAMP(k)                                                                          \
    do {                                                                                   \
        const uint64_t wid_ = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + threadIdx.x / 64; \
        if (lane_id() == 0 && wid_ < (1 << 16)) g_walk_stamps[wid_][k] = wall_clock64();      \
    } while (0)
#elif defined(HONU_STAGE_TIMING)
// Timing build only (-DHONU_STAGE_TIMING, tools/fused_timing.py): lane 0 of
// every wave ADDS the time since its previous stamp to stage k, over every tile
// the wave takes, so the sums divided by the tiles give the stage costs under
// full load (the single-launch decode stamps its post-walk stages as 10..15).
// The sums live in LDS until the wave ends (WSTAMP_FLUSH): a stamp waits only
// for LDS and scalar reads (lgkmcnt), not for the wave's outstanding global
// loads and stores (vmcnt), so it does not add waits of its own. (Until round
// 4 the sums were read-modify-written in global memory, and every stamp waited
// for all the wave's stores: the stages after a store burst looked longer.)
#define STAGES_MAX 16
static __device__ uint64_t g_stage[1 << 16][STAGES_MAX];
static __shared__ uint64_t s_stage[HONU_WAVES_PER_BLOCK][STAGES_MAX + 1];  // + the last stamp
#define STAGE_WID() ((uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + threadIdx.x / 64)
#define WSTAMP(k)                                                          \
    do {                                                                   \
        if (lane_id() == 0) {                                              \
            uint64_t *s_ = s_stage[threadIdx.x / 64];                      \
            const uint64_t now_ = wall_clock64();                          \
            s_[k] += now_ - s_[STAGES_MAX];                                \
            s_[STAGES_MAX] = now_;                                         \
        }                                                                  \
    } while (0)
#define WSTAMP_START()                                                     \
    do {                                                                   \
        if (lane_id() == 0) {                                              \
            uint64_t *s_ = s_stage[threadIdx.x / 64];                      \
            for (int k_ = 0; k_ < STAGES_MAX; k_++) s_[k_] = 0;            \
            s_[STAGES_MAX] = wall_clock64();                               \
        }                                                                  \
    } while (0)
#define WSTAMP_FLUSH()                                                     \
    do {                                                                   \
        const uint64_t wid_ = STAGE_WID();                                 \
        if (lane_id() == 0 && wid_ < (1 << 16))                            \
            for (int k_ = 0; k_ < STAGES_MAX; k_++)                        \
                g_stage[wid_][k_] += s_stage[threadIdx.x / 64][k_];        \
    } while (0)
#else
#define WSTAMP(k) \
    do {          \
    } while (0)
#endif
#ifndef WSTAMP_START
#define WSTAMP_START() \
    do {               \
    } while (0)
#endif
#ifndef WSTAMP_FLUSH
#define WSTAMP_FLUSH() \
    do {               \
    } while (0)
#endif

// Where the walk puts the decoded row (metadata.go:202-302 field by field):
// the whole 352-byte row in 88 registers, out in one coalesced pass afterwards
// (rows_out). (Rows stored field by field as they are decoded free the
// registers but were 30 % slower: vmcnt counts stores, so every window refill
// waited for them; DESIGN §3, source in git history at 88edda1.)
struct RegRow : Row {
    HONU_DEV void begin() { clear(); }
    template <int OFF, int LEN> HONU_DEV void zero() {}  // begin() cleared it
    HONU_DEV void finish(bool st_ok, bool hm, uint32_t pr) {
        (void)hm;
        u32((int)offsetof(honu_meta, present), pr);
        if (!st_ok) clear();
    }
};

// The walk's early hook (wave-uniform call, every lane): the record's ACL
// entry and region counts once the regions are read (0 for a record that has
// failed so far) and its aligned payload bytes. spec_acl: the walk takes a
// list that fits the record (18 bytes per entry) as all present WITHOUT
// checking its entry flags; the caller must then check them (the fused
// decode does, while it fills the table, and redoes the batch when one is
// not 1). NoEarly: nothing, flags checked in the walk.
struct NoEarly {
    bool spec_acl = false;
    HONU_DEV void counts(uint64_t, uint64_t, uint64_t) {}
};

// What the walk of one record leaves in the lane's registers.
struct WinParse {
    int st;             // Metadata() status; HONU_SKIP for a lane past n
    uint64_t nacl;
    uint64_t nreg;      // region table entries: the list's length, 0 for a list returned in place
    uint64_t ntab;      // ACL table entries: nacl, or 0 for a list returned in place
    uint64_t acl_pos;   // first ACL entry flag, | GRP_ACL_FAST when every entry is present
    uint64_t reg_pos;   // first region varint, | GRP_REG_INLINE when nreg <= REG_INLINE
    uint32_t regs[REG_INLINE];
    uint64_t end;       // record end (absolute)
    uint64_t data_off, data_len;  // Data() subslice (absolute), when data_status == OK
    int32_t data_status;
    uint32_t ver;
    uint32_t tomb;
};

// The first bytes of a tile's records: the record bounds and the 16 bytes at
// each record's start (header). Loaded apart from the walk so that a wave can
// issue the next tile's loads while it finishes the current one.
struct TileHead {
    uint64_t beg, end;
    u32x4 a, b;  // the aligned blocks holding [beg, beg + 16) (b only when needed)
};
// rec_off[i], rec_off[i + 1] of record i0 + lane (0, 0 past n)
HONU_DEV void tile_head_bounds(uint64_t i0, const uint64_t *__restrict__ rec_off, uint64_t n,
                               TileHead &H) {
    const uint64_t i = i0 + lane_id();
    H.beg = H.end = 0;
    if (i < n) {
        H.beg = rec_off[i];
        H.end = rec_off[i + 1];
    }
}
// the header blocks (lane_fetch16 without the funnel)
HONU_DEV void tile_head_bytes(const uint8_t *__restrict__ rec, TileHead &H) {
    H.a = u32x4{0, 0, 0, 0};
    H.b = u32x4{0, 0, 0, 0};
    if (H.end > H.beg) {
        const uint64_t A = H.beg & ~15ull;
        H.a = *reinterpret_cast<const u32x4 *>(rec + A);
        // the version byte and dataLength's <= 10 bytes (object.go:114-134)
        // are [beg, beg + 11): the next block only when they cross into it
        if ((H.beg & 15) > 5 && A + 16 < H.end) H.b = *reinterpret_cast<const u32x4 *>(rec + A + 16);
    }
}

// Object.Metadata() + Data() + Tombstone() + StorageVersion() (object.go:47-134)
// of record i0 + lane, the lani walk of metadata.go:202-302. Wave-uniform
// call (every lane of the wave, i0 the same): the window refills need the
// whole wave. H: the tile's bounds and header bytes (tile_head_*). The row
// goes to R (RegRow; acl_off / regions_off only for lists returned in place,
// the table forms' offsets are the caller's). inplace (wave-uniform): a list
// whose entries are all present is returned in place (HONU_ACL_INPLACE,
// acl_off = its absolute position, no table entries); with early.spec_acl
// that is speculated like the rest of the list's layout and the caller checks
// the flags. reg_inplace: every non-empty region list is returned in place
// (HONU_REGIONS_INPLACE, regions_off = its first varint's absolute position;
// every varint still validated here), so P.nreg, the region TABLE entries, is
// 0 and nothing is kept in P.regs.
template <class RowT, class EarlyT>
HONU_DEV void win_walk(uint64_t i0, uint8_t *wave_smem, const uint8_t *__restrict__ rec,
                       uint64_t n, const TileHead &H, RowT &R, WinParse &P, EarlyT &early,
                       bool inplace, bool reg_inplace) {
#define OFF(f) ((int)offsetof(honu_meta, f))
#define STEP(x)                      \
    do {                             \
        if (st == HONU_OK) st = (x); \
    } while (0)
    const uint32_t lane = lane_id();
    const uint64_t i = i0 + lane;
    const bool valid = i < n;
    WSTAMP(0);  // walk entered
    const uint64_t beg = H.beg, end = H.end;
    LaneWin W;
    WSTAMP(1);  // rec_off loaded
    W.init(wave_smem, rec, end);
    const uint64_t len = end - beg;
    uint32_t ver = 0;
    int64_t d = -1, b = -1;
    if (valid && len) {
        uint64_t lo, hi;
        window16(H.a, H.b, (uint32_t)(beg & 15), lo, hi);
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
    P.data_off = 0;
    P.data_len = 0;
    if (!v1) P.data_status = HONU_ERR_BAD_VERSION;
    else if (d < 0) P.data_status = HONU_ERR_MALFORMED;
    else if (d == 0) P.data_status = HONU_OK;
    else if (!in_range) P.data_status = HONU_ERR_PANIC;  // o[1+b:1+b+d]
    else {
        P.data_status = HONU_OK;
        P.data_off = beg + 1 + (uint64_t)b;
        P.data_len = (uint64_t)d;
    }
    P.ver = ver;
    P.tomb = (v1 && d == 0) ? 1 : 0;  // Tombstone :103-112
    P.end = end;

    R.begin();
    uint64_t nacl = 0, nreg = 0, acl_pos = 0, reg_pos = 0;
#pragma unroll
    for (int k = 0; k < REG_INLINE; k++) P.regs[k] = 0;
    int st = HONU_OK;
    if (!valid) st = HONU_SKIP;
    else if (!v1) st = HONU_ERR_BAD_VERSION;
    else if (d < 0) st = HONU_ERR_MALFORMED;
    else if (!in_range) st = HONU_ERR_PANIC;  // o[1+d+b:]
    WDec D;
    D.w = &W;
    D.end = end;
    D.tstart = st == HONU_OK ? beg + 1 + (uint64_t)b + (uint64_t)d : 0;
    D.p = D.tstart;
    WSTAMP(2);  // header read
    W.refill(st == HONU_OK ? win_base(D.p) : NOWIN);
    WSTAMP(3);  // first window

    uint32_t f = 0, u = 0, pr = 0;
    uint64_t v = 0, o = 0, l = 0, lo = 0, hi = 0;
    int64_t t = 0;
    STEP(D.boolean(f));                                     // DecodeStruct(meta) object.go:78
    const bool hm = st == HONU_OK && f;
    bool has_enc = false;
    if (hm) {
        pr = HONU_HAS_META;
        STEP(D.ulid(lo, hi)); R.bytes16(OFF(object_id), lo, hi);       // metadata.go:210
        STEP(D.ulid(lo, hi)); R.bytes16(OFF(collection_id), lo, hi);   // :214
        STEP(D.boolean(f));                                 // :219 Version
        if (st == HONU_OK && f) {
            pr |= HONU_HAS_VERSION;
            STEP(D.u32(u)); R.u32(OFF(pid), u);             // scalar.go:121-131
            STEP(D.u64(v)); R.u64(OFF(vid), v);
            STEP(D.u32(u)); R.u32(OFF(region), u);          // version.go:80
            STEP(D.boolean(f));                             // :88 Parent
            if (st == HONU_OK && f) {
                pr |= HONU_HAS_PARENT;
                STEP(D.u32(u)); R.u32(OFF(parent_pid), u);
                STEP(D.u64(v)); R.u64(OFF(parent_vid), v);
            } else {
                R.template zero<OFF(parent_pid), 12>();
            }
            STEP(D.boolean(f)); R.u8(OFF(tombstone), f);    // :96
            STEP(D.i64(t)); R.u64(OFF(version_created), (uint64_t)t);  // :100
        } else {
            R.template zero<OFF(region), 36>();  // region .. version_created
        }
        STEP(D.boolean(f));                                 // :225 Schema
        if (st == HONU_OK && f) {
            pr |= HONU_HAS_SCHEMA;
            STEP(D.frame(o, l)); R.span(OFF(schema_name), o, l);       // schema.go:55-73
            STEP(D.u32(u)); R.u32(OFF(schema_major), u);
            STEP(D.u32(u)); R.u32(OFF(schema_minor), u);
            STEP(D.u32(u)); R.u32(OFF(schema_patch), u);
        } else {
            R.template zero<OFF(schema_major), 12>();
            R.template zero<OFF(schema_name), 16>();
        }
        STEP(D.frame(o, l)); R.span(OFF(mime), o, l);       // :231
        STEP(D.ulid(lo, hi)); R.bytes16(OFF(owner), lo, hi);   // :235
        STEP(D.ulid(lo, hi)); R.bytes16(OFF(group), lo, hi);   // :239
        STEP(D.u8(u)); R.u8(OFF(permissions), u);           // :243
        STEP(D.u64(nacl));                                  // :249
        WSTAMP(4);  // fields up to the ACL count
        if (st == HONU_OK && nacl > GO_MAX_ALLOC / 8) st = HONU_ERR_PANIC;  // make([]*AccessControl)
    }
    // ACL entries (:254-265, acls.go:41-51): speculate every entry present
    // (flags at p + 18 j). The first 64 flags of every lane's list are
    // gathered in ONE round trip: the windows' LDS is free at this point (the
    // walk is past every byte it holds), and instruction k of a 64-instruction
    // burst of dword global_load_lds has lane j fetch flag j of lane k's list
    // (one list per instruction: 64 flags 18 bytes apart, a few cache lines);
    // every lane then checks its own flags with independent LDS reads. Flags
    // past the 64th are checked window by window.
    bool fast = false;
    if (hm && st == HONU_OK && nacl > 0) {
        acl_pos = D.p;
        fast = 18 * nacl <= D.end - D.p;
    }
    uint64_t ak = 0;
    const bool spec_acl = early.spec_acl;  // wave-uniform
    // HONU_GATHER_SKIP_WIN 1: the flags the lane's window already holds (the
    // list's start, <= 15 entries) are checked from LDS first and the burst
    // (here, or the speculative decode's after its publish: the count rides
    // in acl_pos, GRP_ACL_A0) gathers only the ones after them, so it does
    // not fetch the window's lines a second time. A flag that is not 1 here
    // sends the list to the entry-by-entry walk below, speculative or not.
    uint32_t a0 = 0;
#if HONU_GATHER_SKIP_WIN
    if (fast && W.in(acl_pos)) {
        const uint64_t room = (W.wb + WB - acl_pos + 17) / 18;
        a0 = (uint32_t)(nacl < room ? nacl : room);
        bool ok = true;
#pragma unroll
        for (uint32_t j = 0; j < (WB + 17) / 18; j++)
            if (j < a0) ok &= W.at(acl_pos + 18ull * j) == 1;
        if (!ok) fast = false;  // the entries are walked one by one below
        ak = fast ? a0 : 0;
    }
#endif
    // HONU_GATHER_SKIP_WIN2 1: likewise the list's last flags (<= 4) that
    // window 2, placed at the list's end, will hold: checked from it after its
    // refill (a flag that is not 1 there reverts the list to the
    // entry-by-entry walk), their count riding in acl_pos (GRP_ACL_TL).
    uint32_t tl = 0;
#if HONU_GATHER_SKIP_WIN2
    if (fast) {
        const uint64_t w2b = win_base(acl_pos + 18 * nacl);
        uint64_t jb = w2b > acl_pos ? (w2b - acl_pos + 17) / 18 : 0;  // the first flag at >= w2b
        if (jb < a0) jb = a0;
        tl = (uint32_t)(jb < nacl ? nacl - jb : 0);
    }
#endif
    const uint64_t nhead = nacl - tl;  // the flags checked before window 2
    if (!spec_acl && __ballot(fast && ak < nhead)) {
        const uint64_t gbase = fast ? acl_pos + 18ull * a0 : 0;
        const uint32_t gcnt = fast ? (uint32_t)(nhead - a0 < 64 ? nhead - a0 : 64) : 0;
        wave_sync();  // the windows' last reads are done
#pragma unroll 4
        for (uint32_t k = 0; k < HONU_WAVE; k++) {
            const uint64_t base = readlane64(gbase, k);  // lane k's list, to every lane
            if (lane < __builtin_amdgcn_readlane(gcnt, k))
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(rec + ((base + 18ull * lane) & ~3ull)),
                    (__attribute__((address_space(3))) void *)(W.wave + FLAG_ROW * k), 4, 0, HONU_BURST_AUX);
        }
        __builtin_amdgcn_s_waitcnt(0);
        wave_sync();
        W.wb = NOWIN;  // the windows' bytes are gone
        if (fast) {
            const uint32_t m = gcnt;
            const __attribute__((address_space(3))) uint8_t *fl =
                (const __attribute__((address_space(3))) uint8_t *)(W.wave + FLAG_ROW * lane);
            bool ok = true;
#pragma unroll
            for (uint32_t j = 0; j < 64; j++)
                if (j < m) ok &= fl[4 * j + (uint32_t)((gbase + 18ull * j) & 3)] == 1;
            ak = a0 + m;
            if (!ok) fast = false;  // the entries are walked one by one below
        }
        wave_sync();  // the gather area becomes windows again
    }
    if (!spec_acl) {
        bool chk = fast && ak < nhead;
        while (__ballot(chk)) {
            W.refill(chk ? win_base(D.p + 18 * ak) : NOWIN);
            if (chk) {
                // the flags this window holds (at most 15), read independently
                const uint64_t q = D.p + 18 * ak;
                const uint64_t room = W.in(q) ? (W.wb + WB - q + 17) / 18 : 0;
                const uint32_t cnt = (uint32_t)(nhead - ak < room ? nhead - ak : room);
                bool ok = true;
#pragma unroll
                for (uint32_t j = 0; j < (WB + 17) / 18; j++)
                    if (j < cnt) ok &= W.at(q + 18 * j) == 1;
                ak += cnt;
                if (!ok) fast = false;  // the entries are walked one by one below
                if (!fast || ak == nhead) chk = false;
            }
        }
    }
    bool inpl = false;  // returned in place
    if (hm && st == HONU_OK && nacl > 0) {
        if (fast) {
            D.p += 18 * nacl;
            if (inplace) {  // metadata.go:254-266 without the copy: the entries stay where they are
                inpl = true;
                pr |= HONU_ACL_INPLACE;
                R.u64(OFF(acl_off), acl_pos);
            }
            acl_pos |= GRP_ACL_FAST | ((uint64_t)a0 << GRP_ACL_A0_SHIFT) |
                       ((uint64_t)tl << GRP_ACL_TL_SHIFT);  // for the fill
        } else {
            for (uint64_t k = 0; k < nacl && st == HONU_OK; k++) {
                STEP(D.boolean(f));
                if (st == HONU_OK && f) {
                    STEP(D.ulid(lo, hi));
                    STEP(D.u8(u));
                }
            }
        }
    }
    WSTAMP(5);  // ACL flags checked
    W.refill(hm && st == HONU_OK ? win_base(D.p) : NOWIN);
    WSTAMP(6);  // window after the list
#if HONU_GATHER_SKIP_WIN2
    if (fast && tl) {  // the last flags, from window 2 (or memory, W.u8)
        const uint64_t ap = acl_pos & GRP_POS_MASK;
        bool ok = true;
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (j < tl) ok &= W.u8(ap + 18 * (nacl - tl + j)) == 1;
        if (!ok) {  // a nil entry among them: the list is walked entry by entry after all
            fast = false;
            inpl = false;
            pr &= ~(uint32_t)HONU_ACL_INPLACE;
            acl_pos = ap;
            D.p = ap;
            for (uint64_t k = 0; k < nacl && st == HONU_OK; k++) {
                STEP(D.boolean(f));
                if (st == HONU_OK && f) {
                    STEP(D.ulid(lo, hi));
                    STEP(D.u8(u));
                }
            }
        }
    }
#endif
    if (hm) R.u64(OFF(acl_count), nacl);  // 0 for an empty list (metadata.go:254)
    if (hm) {
        STEP(D.u64(nreg));                                  // region.go:154-169
        if (st == HONU_OK && nreg > GO_MAX_ALLOC / 4) st = HONU_ERR_PANIC;  // make(Regions, n)
        pr |= HONU_REGIONS_NONNIL;
        reg_pos = D.p;
        if (reg_inplace) {  // region.go:154-169 without the copy: validated, not kept
            for (uint64_t k = 0; k < nreg && st == HONU_OK; k++) STEP(D.u32(u));
            if (st == HONU_OK && nreg) {
                pr |= HONU_REGIONS_INPLACE;
                R.u64(OFF(regions_off), reg_pos);
            }
        } else {
#pragma unroll
            for (int k = 0; k < REG_INLINE; k++) {
                if ((uint64_t)k < nreg) {
                    STEP(D.u32(u));
                    P.regs[k] = u;
                }
            }
            for (uint64_t k = REG_INLINE; k < nreg && st == HONU_OK; k++) STEP(D.u32(u));
        }
        if (nreg <= REG_INLINE) reg_pos |= GRP_REG_INLINE;
        R.u64(OFF(regions_count), nreg);
    }
    // both list counts are known here; a later field can still fail the
    // record (its counts then become 0): the early hook publishes them
    // tentatively (fused.hip speculative decode)
    early.counts(hm && st == HONU_OK && !inpl ? nacl : 0, hm && st == HONU_OK && !reg_inplace ? nreg : 0,
                 (P.data_len + 15) & ~15ull);
    if (hm) {
        STEP(D.boolean(f));                                 // :271 Publisher
        if (st == HONU_OK && f) {
            pr |= HONU_HAS_PUBLISHER;
            STEP(D.ulid(lo, hi)); R.bytes16(OFF(publisher_id), lo, hi);   // provenance.go:59-79
            STEP(D.ulid(lo, hi)); R.bytes16(OFF(client_id), lo, hi);
            STEP(D.frame(o, l)); R.span(OFF(ip_address), o, l);
            STEP(D.frame(o, l)); R.span(OFF(user_agent), o, l);
        } else {
            R.template zero<OFF(publisher_id), 32>();
            R.template zero<OFF(ip_address), 32>();
        }
        STEP(D.boolean(f));                                 // :277 Encryption
        if (st == HONU_OK && f) {
            pr |= HONU_HAS_ENCRYPTION;
            has_enc = true;
            STEP(D.frame(o, l)); R.span(OFF(public_key_id), o, l);     // encryption.go:91-125
            STEP(D.frame(o, l)); R.span(OFF(encryption_key), o, l);
            STEP(D.frame(o, l)); R.span(OFF(hmac_secret), o, l);
            STEP(D.frame(o, l)); R.span(OFF(signature), o, l);
        } else {
            R.template zero<OFF(public_key_id), 64>();
        }
    }
    WSTAMP(7);  // regions .. signature
    W.refill(hm && st == HONU_OK ? win_base(D.p) : NOWIN);
    WSTAMP(8);  // window after the signature
    if (hm) {
        if (has_enc) {
            STEP(D.u8(u)); R.u8(OFF(sealing_alg), u);
            STEP(D.u8(u)); R.u8(OFF(encryption_alg), u);
            STEP(D.u8(u)); R.u8(OFF(signature_alg), u);
        }
        STEP(D.boolean(f));                                 // :283 Compression
        if (st == HONU_OK && f) {
            pr |= HONU_HAS_COMPRESSION;
            STEP(D.u8(u)); R.u8(OFF(compression_alg), u);   // compression.go:55-67
            STEP(D.i64(t)); R.u64(OFF(compression_level), (uint64_t)t);
        } else {
            R.template zero<OFF(compression_level), 8>();
        }
        STEP(D.u8(u)); R.u8(OFF(flags), u);                 // :289
        STEP(D.i64(t)); R.u64(OFF(created), (uint64_t)t);   // :293
        STEP(D.i64(t)); R.u64(OFF(modified), (uint64_t)t);  // :297
    }
    R.finish(st == HONU_OK, hm, pr);
    if (st != HONU_OK) {  // Go returns nil, err
        nacl = nreg = 0;
    }
    WSTAMP(9);  // walk done
    P.st = st;
    P.nacl = nacl;
    P.ntab = inpl ? 0 : nacl;
    P.nreg = reg_inplace ? 0 : nreg;  // region table entries
    P.acl_pos = acl_pos;
    P.reg_pos = reg_pos;
#undef STEP
#undef OFF
}

// The wave's 64 rows out through its LDS windows (free after the walk): 32
// rows per pass, written as contiguous 16-byte stores. NT: non-temporal
// stores (the single-launch decode, whose rows nothing in the launch reads
// again: 1M Small zero copy 0.704-0.711 -> 0.691-0.694 ms, 62 K Large 0.080-0.084
// -> 0.079-0.080 ms, profiles/r04/ab/dec_nt_stores_ab.jsonl; the split parse's
// rows are read back by its table kernel, so it keeps plain stores). (The ACL
// table as non-temporal stores too: 1M Small equal to rows alone, 62 K Large
// 0.085 ms, slower.)
template <bool NT = false>
HONU_DEV void rows_out(uint8_t *wave_smem, const Row &R, uint64_t i0, uint64_t n,
                       honu_meta *__restrict__ meta) {
    const uint32_t lane = lane_id();
    for (uint32_t h = 0; h < 2; h++) {
        wave_sync();
        if ((lane >> 5) == h) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(wave_smem + (lane & 31) * sizeof(honu_meta));
#pragma unroll
            for (int c = 0; c < 22; c++)
                dst[c] = u32x4{R.d[4 * c], R.d[4 * c + 1], R.d[4 * c + 2], R.d[4 * c + 3]};
        }
        wave_sync();
        const uint64_t r0 = i0 + 32 * h;
        const uint64_t rows = r0 >= n ? 0 : (n - r0 < 32 ? n - r0 : 32);
        const u32x4 *src = reinterpret_cast<const u32x4 *>(wave_smem);
        u32x4 *out = reinterpret_cast<u32x4 *>(meta + r0);
        for (uint32_t s = lane; s < rows * 22; s += HONU_WAVE) {
            if constexpr (NT) __builtin_nontemporal_store(src[s], out + s);
            else out[s] = src[s];
        }
    }
    wave_sync();
}

HONU_DEV honu_record_info make_info(const WinParse &P, uint64_t data_off, uint64_t data_len,
                                    int32_t data_status, int32_t meta_status) {
    honu_record_info inf;
    inf.data_off = data_off;
    inf.data_len = data_len;
    inf.data_status = data_status;
    inf.meta_status = meta_status;
    inf.storage_version = (uint8_t)P.ver;
    inf.tombstone = (uint8_t)P.tomb;
#pragma unroll
    for (int k = 0; k < 6; k++) inf._pad[k] = 0;
    return inf;
}

}  // namespace honu
