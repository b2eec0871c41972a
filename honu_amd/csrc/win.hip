// win.hip — the split decode parse (honu_decode_parse, record_variant 0):
// one record per LANE reading through per-lane LDS windows (win.h). Rows go
// out through LDS; the per-record list positions, counts and inline region ids
// go to the context scratch for honu_decode_tables (scan + group fill).
#include "win.h"

namespace honu {

#ifdef HONU_WALK_TIMING
}  // namespace honu
extern "C" int32_t honu_debug_walk_stamps(void *host, uint64_t waves) {
    if (waves > (1 << 16)) waves = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(honu::g_walk_stamps),
                               waves * WALK_STAMPS * sizeof(uint64_t)) == hipSuccess ? 0 : -3;
}
namespace honu {
#endif

__global__ __launch_bounds__(HONU_BLOCK) void k_decode_parse_win(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint32_t *__restrict__ reg_inline,
    uint64_t *__restrict__ counts, bool inplace, bool reg_inplace) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[HONU_WAVES_PER_BLOCK * WIN_WAVE_BYTES];
    const uint32_t wv = threadIdx.x / HONU_WAVE;
    uint8_t *ws = smem + wv * WIN_WAVE_BYTES;
    // one wave per 64 records, grid-stride over the batch (the loop is wave-uniform)
    for (uint64_t i0 = (uint64_t)blockIdx.x * HONU_BLOCK + wv * HONU_WAVE; i0 < n;
         i0 += (uint64_t)gridDim.x * HONU_BLOCK) {
        WinParse P;
        TileHead H;
        tile_head_bounds(i0, rec_off, n, H);
        tile_head_bytes(rec, H);
        RegRow R;
        NoEarly none;
        win_walk(i0, ws, rec, n, H, R, P, none, inplace, reg_inplace);
        rows_out(ws, R, i0, n, meta);
        const uint64_t i = i0 + lane_id();
        if (i >= n) continue;
        store_info(info + i, make_info(P, P.data_off, P.data_len, P.data_status, P.st));
        // the group fill takes inline regions from reg_inline (8 per record)
        const uint64_t rp = P.nreg > 8 ? (P.reg_pos & GRP_POS_MASK) : P.reg_pos;
        scratch[i] = DecodeScratch{P.acl_pos, rp, P.data_off, P.end};
#pragma unroll
        for (int k = 0; k < 8; k++)
            if ((uint64_t)k < P.nreg) reg_inline[8 * i + k] = P.regs[k];
        counts[3 * i + 0] = P.ntab;  // 0 for a list returned in place
        counts[3 * i + 1] = P.nreg;  // 0 for a list returned in place
        counts[3 * i + 2] = (P.data_len + 15) & ~15ull;
    }
}

static dim3 win_grid(uint64_t n, int cap) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(cap > 0 && b > (uint64_t)cap ? (uint64_t)cap : b));
}

hipError_t launch_decode_parse_win(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   honu_meta *meta, honu_record_info *info,
                                   DecodeScratch *scratch, uint32_t *reg_inline, uint64_t *counts,
                                   int max_blocks, bool inplace, bool reg_inplace, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_parse_win, win_grid(n, max_blocks),
                       dim3(HONU_BLOCK), 0, s, rec, rec_off, n, meta, info, scratch, reg_inline,
                       counts, inplace, reg_inplace);
    return hipGetLastError();
}

}  // namespace honu
