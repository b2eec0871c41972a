// lane.hip — per-record kernels with one record per LANE (see lane.h for
// why): the header/tail encoder of the default encode (the ACL entries are
// left to k_encode_acl_grp) and the headers-only decode (honu_decode_headers,
// honu_decode_data).
#include "kernels.h"
#include "lane.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))

// ------------------------------------------------------------------------
// encode: header + Metadata tail (object.go:24-45, metadata.go:108-200)
// ------------------------------------------------------------------------
// The ring: RING 16-byte chunks per lane, slot-major with the wave's lanes
// adjacent (ring slot k of lane L at area + 16 (64 k + L)). Two forms, chosen
// at launch: RING 8 (drains of every full chunk; 32 KB of LDS per workgroup,
// the registers allow 3 waves per SIMD) where a launch has at most as many
// tiles as the line form has resident waves, RING 16 (line drains, lane.h;
// 64 KB per workgroup: 2 waves per SIMD) above that. Measured (interleaved,
// profiles/r04/ab/enc_line_drain_ab.jsonl): 1M Small 1.09 -> 0.99 ms, 262 K
// Small 0.298 -> 0.265 ms; 64 K Small 0.074 -> 0.078 ms and a 62 K Large chunk
// 0.082 -> 0.086 ms (latency-bound: fewer records in flight per SIMD and
// lines held back lengthen a tile), hence the switch.
// The switch: more tiles than the line form's resident waves, i.e. 4 waves x
// min(the launch's workgroups, 2 per CU) (launch_encode_meta_lane; a
// lane_blocks cap lowers it). ENC_LINE_MIN_TILES_N fixes it instead (A/B
// builds only).
template <int RING> constexpr uint32_t enc_wave_bytes() { return (RING > 0 ? RING : 1) * HONU_WAVE * 16; }

template <bool SKIP_ACL, int RING>
HONU_DEV void k_encode_meta_lane_one(uint64_t i, const honu_meta &m, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    EncAclPos *__restrict__ acl_out, u32x4 *ring, const uint8_t *__restrict__ payload) {
    if (status[i] != HONU_OK) return;
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    if (end > out_cap) {
        status[i] = HONU_ERR_CAPACITY;
        return;
    }
    const uint64_t dlen = payload_off[i + 1] - payload_off[i];
    const uint64_t pos = encode_record_lane<SKIP_ACL, SKIP_ACL ? RING : 0>(
        m, var, acl, reg, dlen, beg, end, out, ring, payload ? payload + payload_off[i] : nullptr);
    if constexpr (SKIP_ACL)
        acl_out[i] = EncAclPos{pos, m.acl_off, m.acl_count,
                               m.acl_bytes | ((m.present & HONU_ACL_SIZED) ? ENC_ACL_SIZED : 0)};
}

// a lane's row straight from global memory (the loads cannot pass the output
// stores, so the whole row is loaded first)
HONU_DEV void load_row(const honu_meta *__restrict__ src, honu_meta &m) {
    const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
    u32x4 *d = reinterpret_cast<u32x4 *>(&m);
#pragma unroll
    for (int k = 0; k < 22; k++) d[k] = s[k];
}

template <bool SKIP_ACL, int RING, bool UNITS = false>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_meta_lane(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    EncAclPos *__restrict__ acl_out, const uint8_t *__restrict__ payload) {
    constexpr uint32_t WAVE_BYTES = enc_wave_bytes<RING>();
    __shared__ __attribute__((aligned(16))) uint8_t smem[HONU_WAVES_PER_BLOCK * WAVE_BYTES];
    uint8_t *area = smem + (threadIdx.x / HONU_WAVE) * WAVE_BYTES;
    u32x4 *ring = reinterpret_cast<u32x4 *>(area) + lane_id();
    // wave-uniform loop over tiles of 64 records (one per lane)
    for (uint64_t t0 = (uint64_t)blockIdx.x * HONU_BLOCK + (threadIdx.x & ~(uint64_t)(HONU_WAVE - 1)); t0 < n;
         t0 += (uint64_t)gridDim.x * HONU_BLOCK) {
        const uint64_t i = t0 + lane_id();
        ESTAMP(0);  // entered
        honu_meta m;
        if (i < n) {
            load_row(meta + i, m);
            k_encode_meta_lane_one<SKIP_ACL, RING>(i, m, var, acl, reg, payload_off, out, out_cap, out_off, status,
                                             acl_out, ring, UNITS ? payload : nullptr);
        }
    }
}

#undef OFF

// ------------------------------------------------------------------------
// headers only: StorageVersion, Data, Tombstone (object.go:47-52,85-134)
// ------------------------------------------------------------------------
// SPANS: also hand the payload's absolute offset (scratch.data_src) and its
// 16-byte aligned size (counts[i], one column) to honu_decode_data's scan and
// copy.
template <bool SPANS>
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_headers(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_record_info *__restrict__ info, DecodeScratch *__restrict__ scratch,
    uint64_t *__restrict__ counts) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK) {
        const uint64_t beg = rec_off[i], end = rec_off[i + 1];
        const uint64_t len = end - beg;
        uint32_t ver = 0;
        int64_t d = -1, b = -1;
        if (len) {
            uint64_t lo, hi;
            lane_fetch16(rec, beg, end, lo, hi);
            ver = (uint32_t)(lo & 0xFF);
            if (len >= 3) {  // dataLength: Uvarint(o[1 : min(11, len-1)])
                const uint32_t wl = (uint32_t)(len - 2 < 10 ? len - 2 : 10);
                uint64_t x;
                const uint32_t k = uvarint_window((lo >> 8) | (hi << 56), hi >> 8, wl, x);
                if (k) {
                    d = (int64_t)x;
                    b = k;
                }
            }
        }
        const bool v1 = ver == HONU_STORAGE_VERSION;
        honu_record_info inf;
        inf.data_off = 0;
        inf.data_len = 0;
        if (!v1) inf.data_status = HONU_ERR_BAD_VERSION;
        else if (d < 0) inf.data_status = HONU_ERR_MALFORMED;
        else if (d == 0) inf.data_status = HONU_OK;
        else if ((uint64_t)d > len - 1 - (uint64_t)b) inf.data_status = HONU_ERR_PANIC;
        else {
            inf.data_status = HONU_OK;
            inf.data_off = beg + 1 + (uint64_t)b;
            inf.data_len = (uint64_t)d;
        }
        inf.meta_status = HONU_UNPARSED;
        inf.storage_version = (uint8_t)ver;
        inf.tombstone = (v1 && d == 0) ? 1 : 0;
#pragma unroll
        for (int k = 0; k < 6; k++) inf._pad[k] = 0;
        if constexpr (SPANS) {
            scratch[i].data_src = inf.data_off;
            counts[i] = (inf.data_len + 15) & ~15ull;
        }
        store_info(info + i, inf);
    }
}

// honu_decode_data, after the scan: data_off relative to the data arena, or
// HONU_ERR_CAPACITY for a payload that does not fit (then nothing is copied).
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_data_place(
    uint64_t n, honu_record_info *__restrict__ info, const uint64_t *__restrict__ offs,
    uint64_t data_cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK) {
        honu_record_info *p = info + i;
        if (p->data_status != HONU_OK || !p->data_len) continue;
        const uint64_t o = offs[i];
        if (o > data_cap || p->data_len > data_cap - o) {
            p->data_status = HONU_ERR_CAPACITY;
            p->data_off = 0;
            p->data_len = 0;
        } else {
            p->data_off = o;
        }
    }
}

static dim3 flat_grid(uint64_t n) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(b > 65536 ? 65536 : b));
}

hipError_t launch_decode_headers(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                 honu_record_info *info, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_headers<false>, flat_grid(n), dim3(HONU_BLOCK), 0, s, rec, rec_off,
                       n, info, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_decode_spans(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_record_info *info, DecodeScratch *scratch, uint64_t *counts,
                               hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_headers<true>, flat_grid(n), dim3(HONU_BLOCK), 0, s, rec, rec_off, n,
                       info, scratch, counts);
    return hipGetLastError();
}

hipError_t launch_decode_data_place(uint64_t n, honu_record_info *info, const uint64_t *offs,
                                    uint64_t data_cap, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_data_place, flat_grid(n), dim3(HONU_BLOCK), 0, s, n, info, offs,
                       data_cap);
    return hipGetLastError();
}

static dim3 lane_grid(uint64_t n, int cap) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(cap > 0 && b > (uint64_t)cap ? (uint64_t)cap : b));
}

hipError_t launch_encode_meta_lane(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                   const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                   uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                   int32_t *status, EncAclPos *acl_out, int max_blocks, int num_cu,
                                   const uint8_t *payload, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!acl_out) return hipErrorInvalidValue;
    const dim3 grid = lane_grid(n, max_blocks);
#ifdef ENC_LINE_MIN_TILES_N
    const uint64_t line_min_tiles = ENC_LINE_MIN_TILES_N;
    (void)num_cu;
#else
    const uint64_t resident_blocks = grid.x < 2u * (uint64_t)num_cu ? grid.x : 2u * (uint64_t)num_cu;
    const uint64_t line_min_tiles = HONU_WAVES_PER_BLOCK * resident_blocks;
#endif
    const bool line = (n + HONU_WAVE - 1) / HONU_WAVE > line_min_tiles;
#define HONU_META_LANE(RG, U)                                                                        \
    hipLaunchKernelGGL((k_encode_meta_lane<true, RG, U>), grid, dim3(HONU_BLOCK), 0, s, meta, var, acl, \
                       reg, payload_off, n, out, out_cap, out_off, status, acl_out, payload)
    if (line && payload) HONU_META_LANE(16, true);
    else if (line) HONU_META_LANE(16, false);
    else if (payload) HONU_META_LANE(8, true);
    else HONU_META_LANE(8, false);
#undef HONU_META_LANE
    return hipGetLastError();
}

}  // namespace honu

#ifdef HONU_ENC_TIMING
extern "C" int32_t honu_debug_enc_stamps(void *host, uint64_t waves) {
    if (waves > (1 << 16)) waves = 1 << 16;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(honu::g_enc_stamps),
                               waves * ENC_STAMPS * sizeof(uint64_t)) == hipSuccess ? 0 : -3;
}
#endif
