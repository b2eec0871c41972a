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
#include <stdlib.h>

#include "lookback.h"
#include "win.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))
#ifndef FILL_U
#define FILL_U 4  // ACL entries per lane in flight in the fill
#endif

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
    int dbg;                  // A/B measurement knobs (HONU_FUSED_DBG): 1 no ACL fill,
                              // 2 no look-back wait, 4 static tiles (with 2)
};

__global__ __launch_bounds__(HONU_BLOCK, 2) void k_decode_fused(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    DecodeOut O, LbState *lb, uint64_t *lb_status, uint64_t lb_words) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[HONU_WAVES_PER_BLOCK * WIN_WAVE_BYTES];
    __shared__ uint32_t last_flag;
    uint8_t *ws = smem + (threadIdx.x / HONU_WAVE) * WIN_WAVE_BYTES;
    const uint32_t lane = lane_id();
    const uint32_t ep = lb_epoch(lb);
    const uint64_t ntiles = (n + HONU_WAVE - 1) / HONU_WAVE;
    const uint64_t waves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    // every tile has a resident wave of its own: static tiles (lookback.h)
    const bool stat = ntiles <= waves && !(O.dbg & 4);
    uint64_t t;
    uint64_t k_static = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + threadIdx.x / HONU_WAVE;
    for (;;) {
        if (stat || (O.dbg & 4)) {  // dbg 4: measurement only (with 2), static tiles at any size
            t = k_static;
            k_static += waves;
        } else {
            t = lb_ticket(lb);
        }
        if (t >= ntiles) break;
        const uint64_t i0 = t * HONU_WAVE, i = i0 + lane;
        const bool valid = i < n;
        WinParse P;
        win_walk(i0, ws, rec, rec_off, n, P);

        // counts -> offsets: wave scan + look-back across tiles
        const uint64_t c0 = P.nacl, c1 = P.nreg, c2 = (P.data_len + 15) & ~15ull;
        uint64_t agg[3], excl[3];
        const uint64_t x0 = wave_excl(c0, agg[0]);
        const uint64_t x1 = wave_excl(c1, agg[1]);
        const uint64_t x2 = wave_excl(c2, agg[2]);
        // publish, then write the rows while the predecessors finish (their
        // list offsets are patched in below), then wait
        if (!(O.dbg & 2)) lb_publish<3>(lb_status, t, ep, agg);
        rows_out(ws, P.R, i0, n, O.meta);
        if (O.dbg & 2) {
            excl[0] = excl[1] = excl[2] = 0;
        } else {
            lb_resolve<3>(lb_status, t, ep, agg, excl);
        }
        if (t == ntiles - 1 && lane < 3)
            O.totals[lane] = lane == 0 ? excl[0] + agg[0] : (lane == 1 ? excl[1] + agg[1] : excl[2] + agg[2]);
        const uint64_t ao = excl[0] + x0, ro = excl[1] + x1, doff = excl[2] + x2;

        int32_t mst = P.st;
        if (mst == HONU_OK) {  // as honu_decode_tables: offsets first, then the capacity check
            if (P.nacl) O.meta[i].acl_off = ao;
            if (P.nreg) O.meta[i].regions_off = ro;
            if (ao + P.nacl > O.acl_cap || ro + P.nreg > O.reg_cap) mst = HONU_ERR_CAPACITY;
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
        // ACL table. Lists with every entry present: the wave's entries are one
        // run of the table; lane e of a round takes entry e of that run (record
        // by a search over the lanes' prefixes), reads the 17 bytes after its
        // flag (the walk fetched them moments ago) and stores the 20-byte row.
        const bool fast = ok && P.nacl && (P.acl_pos & GRP_ACL_FAST);
        const uint64_t apos = P.acl_pos & GRP_POS_MASK;
        if (ok && P.nacl && !fast) {  // nil entries: the lane walks its list (validated)
            uint64_t p = apos;
            for (uint64_t k = 0; k < P.nacl; k++) {
                uint32_t *d = reinterpret_cast<uint32_t *>(O.acl + ao + k);
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
        }
        uint64_t ftot;
        const uint64_t fpre = wave_excl(fast ? P.nacl : 0, ftot);
        constexpr int U = FILL_U;  // entries per lane in flight
        if (!(O.dbg & 1))
        for (uint64_t e0 = 0; e0 < ftot; e0 += U * HONU_WAVE) {  // wave-uniform
            u32x4 id[U];
            uint32_t pm[U];
            uint64_t dst[U];
#pragma unroll
            for (int k = 0; k < U; k++) {
                const uint64_t e = e0 + lane + HONU_WAVE * k;
                const uint32_t r = lane_search(fpre, e < ftot ? e : 0);
                const uint64_t rp = shfl64(fpre, r), ra = shfl64(apos, r), rao = shfl64(ao, r);
                const uint64_t j = e - rp;
                const uint64_t q = ra + 18 * j + 1;  // ClientID, then Permissions at q + 16
                dst[k] = rao + j;
                if (e < ftot) {  // one unaligned 16-byte load + one byte
                    id[k] = *reinterpret_cast<const u32x4u *>(rec + q);
                    pm[k] = rec[q + 16];
                }
            }
#pragma unroll
            for (int k = 0; k < U; k++) {
                const uint64_t e = e0 + lane + HONU_WAVE * k;
                if (e < ftot) {
                    uint32_t *d = reinterpret_cast<uint32_t *>(O.acl + dst[k]);
                    d[0] = id[k].x;
                    d[1] = id[k].y;
                    d[2] = id[k].z;
                    d[3] = id[k].w;
                    d[4] = pm[k] | (1u << 8);
                }
            }
        }
    }
    if (stat)
        lb_finish_blocks(lb, lb_status, lb_words, gridDim.x, &last_flag);
    else if (!(O.dbg & 4))
        lb_finish(lb, lb_status, lb_words, t, ntiles, (uint32_t)waves);
}

hipError_t launch_decode_fused(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_meta *meta, honu_record_info *info, honu_acl *acl,
                               uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, int materialize,
                               uint64_t data_cap, DecodeScratch *scratch, uint64_t *offs,
                               uint64_t *totals, LbState *lb, uint64_t *lb_status,
                               uint64_t lb_words, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t tiles = (n + HONU_WAVE - 1) / HONU_WAVE;
    uint64_t b = (tiles + HONU_WAVES_PER_BLOCK - 1) / HONU_WAVES_PER_BLOCK;
    if (max_blocks > 0 && b > (uint64_t)max_blocks) b = (uint64_t)max_blocks;
#ifdef HONU_AB  // measurement knobs, A/B library only (they break the results)
    static const int dbg = getenv("HONU_FUSED_DBG") ? atoi(getenv("HONU_FUSED_DBG")) : 0;
#else
    const int dbg = 0;
#endif
    DecodeOut O{meta, info, acl, acl_cap, reg, reg_cap, data_cap, materialize, scratch, offs, totals, dbg};
    hipLaunchKernelGGL(k_decode_fused, dim3((unsigned)b), dim3(HONU_BLOCK), 0, s, rec, rec_off, n,
                       O, lb, lb_status, lb_words);
    return hipGetLastError();
}


#undef OFF

}  // namespace honu
