// kernels.h — launch wrappers shared between the kernel translation units and
// the C ABI (api.hip). Every wrapper is asynchronous on `stream` and returns a
// hipError_t from the launch.
#pragma once

#include "common.h"
#include "lookback.h"

// LDS budget per wave for the Metadata tail writer (encode.hip) and the
// decode window (decode.hip). Generated tails are 0.15-1.8 KB; longer tails
// take the in-place fallback (encode) or re-stage the window (decode).
#define ENC_TAIL_LDS 4096
#define DEC_WIN 2048

namespace honu {

// Per-record scratch handed from honu_decode_parse to honu_decode_fill.
struct DecodeScratch {
    uint64_t acl_pos;     // absolute offset of the first ACL entry flag
    uint64_t regions_pos; // absolute offset of the first region varint
    uint64_t data_src;    // absolute offset of the payload (Data() subslice)
    uint64_t rec_end;     // absolute end of the record
};

// Flag bits on DecodeScratch::acl_pos / regions_pos, set by the lane and group
// parses for the group fill (positions are < 2^62).
#define GRP_ACL_FAST (1ull << 63)    // acl_pos: every entry present, entry j at acl_pos + 18 j
#define GRP_REG_INLINE (1ull << 62)  // regions_pos: region ids in reg_inline[8 i ..]
// acl_pos bits 56-59 (GRP_ACL_FAST lists, HONU_GATHER_SKIP_WIN): how many of
// the list's first flags the walk already checked from its window (win.h)
#define GRP_ACL_A0_SHIFT 56
#define GRP_ACL_A0(pos) (((pos) >> GRP_ACL_A0_SHIFT) & 15ull)
// bits 53-55 (HONU_GATHER_SKIP_WIN2): how many of its last flags it checked
// from the window after the list
#define GRP_ACL_TL_SHIFT 53
#define GRP_ACL_TL(pos) (((pos) >> GRP_ACL_TL_SHIFT) & 7ull)
#define GRP_POS_MASK ((1ull << GRP_ACL_TL_SHIFT) - 1)  // positions < 2^53
// Flag on the lane encoder's ACL list position: every entry present, and the
// list's partial end chunks are already written (the group kernel stores the
// whole chunks in between).
#define ACL_ALL_PRESENT (1ull << 63)
// The memory side's write unit: a 64-byte unit that leaves L2 partly written
// costs a read-modify-write (tools/partial_write_probe.hip). The units form of
// the encode (honu_encode_*_units): the encoder writes a payload's partial end
// units, the copy the whole ones (lane.h encode_record_lane, copy.hip
// EncodeSegments).
#define PAYLOAD_UNIT 64ull

// 01 | ClientID | Permissions, the 18 encoded bytes of a present
// *AccessControl (acls.go:26-39), as 4.5 little-endian words.
HONU_DEV void acl_enc_words(const honu_acl *e, uint32_t d[5]) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(e);
    const uint32_t e0 = w[0], e1 = w[1], e2 = w[2], e3 = w[3], e4 = w[4];
    d[0] = 1u | (e0 << 8);
    d[1] = (e0 >> 24) | (e1 << 8);
    d[2] = (e1 >> 24) | (e2 << 8);
    d[3] = (e2 >> 24) | (e3 << 8);
    d[4] = (e3 >> 24) | ((e4 & 0xFF) << 8);
}

// 16 output bytes at absolute X >= P of the list at P (every entry present)
HONU_DEV u32x4 acl_chunk(const honu_acl *A, uint64_t na, uint64_t P, uint64_t X) {
    const uint64_t j0 = (X - P) / 18;
    uint32_t b[10];
    acl_enc_words(A + j0, b);
    b[5] = b[6] = b[7] = b[8] = b[9] = 0;
    if (j0 + 1 < na) {  // entry j0 + 1 starts at byte 18 of b
        uint32_t d[5];
        acl_enc_words(A + j0 + 1, d);
        b[4] = (b[4] & 0xFFFF) | (d[0] << 16);
        b[5] = (d[0] >> 16) | (d[1] << 16);
        b[6] = (d[1] >> 16) | (d[2] << 16);
        b[7] = (d[2] >> 16) | (d[3] << 16);
        b[8] = (d[3] >> 16) | (d[4] << 16);
    }
    // chunk byte k = byte (X - P - 18 j0) + k of b (X >= P)
    const uint32_t off = (uint32_t)(X - (P + 18 * j0));
    const uint32_t q = off >> 2, sh = off & 3;
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t w0 = b[k], w1 = b[k + 1];
#pragma unroll
        for (int t = 1; t <= 4; t++)
            if ((uint32_t)t == q) {
                w0 = b[t + k];
                w1 = b[t + k + 1];
            }
        o[k] = __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

struct LaunchGeom {
    int num_cu;
    int per_record_blocks;  // cap on blocks for one-wave-per-record kernels
    int lane_blocks;        // cap on blocks for the lane / group / window kernels
                            // (0: one block per 256 lanes of work, no cap)
    int copy_blocks;        // blocks of the byte-balanced copy kernel
    int copy_variant;       // copy engine variant (copy.hip: unroll depth / cache policy)
    int encode_variant;     // header/tail encoder: 0 lane writer + ACL group kernel (lane.hip,
                            // grp.hip; default), 1 group layout (enc.hip, A/B build only)
    int record_variant;     // per-record kernels: 0 auto (the fastest measured form
                            // of each; honu_decode_batch single-launch from 48 K
                            // records), 5 split decode, 6 single-launch decode
                            // at every size (the rejected one-record-per-wave /
                            // per-group / per-lane forms 1-4: DESIGN §3)
    uint32_t *tile_map;     // sweep-form tile -> segment map (context scratch)
    uint64_t tile_map_cap;
    uint32_t *copy_tickets; // the copies' range-tail counters (copy.hip): in the context's
                            // geometry the ring's first line, in a launch's copy its own line
    int copy_steal;         // 1: range tails from the counters (default), 0: off
};
#define COPY_TICKET_STRIDE 32u  // uint32 words: one 128-byte line per copy launch
#define COPY_TICKET_LINES 64u   // the ring: copy calls in flight at once on one context

hipError_t launch_encode_copy(const LaunchGeom &g, const uint8_t *payload,
                              const uint64_t *payload_off, uint64_t n, uint8_t *out,
                              uint64_t out_cap, const uint64_t *out_off, const int32_t *status,
                              bool units, hipStream_t s);

hipError_t launch_decode_copy(const LaunchGeom &g, const uint8_t *rec, uint64_t n,
                              const honu_record_info *info, const DecodeScratch *scratch,
                              const uint64_t *offs, const uint64_t *totals, uint8_t *data,
                              hipStream_t s);
hipError_t launch_decode_keys(const LaunchGeom &g, const honu_meta *meta,
                              const honu_record_info *info, uint64_t n, uint8_t *keys,
                              int32_t *key_status, hipStream_t s);

// The lane encoder's hand-over to the ACL list kernel, one per record: where
// the list goes (| ACL_ALL_PRESENT) and the row fields the list kernel needs,
// so that it reads 32 bytes per record instead of two lines of the row.
struct EncAclPos {
    uint64_t pos;        // the list's first byte in the output (| ACL_ALL_PRESENT)
    uint64_t acl_off;    // the row's acl_off / acl_count
    uint64_t acl_count;
    uint64_t carried;    // the row's acl_bytes | ENC_ACL_SIZED when HONU_ACL_SIZED is set
};
#define ENC_ACL_SIZED (1ull << 63)

// acl_out != null: the ACL entries are left out (hand-over in acl_out) for
// launch_encode_acl_grp
hipError_t launch_encode_meta_lane(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                   const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                   uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                   int32_t *status, EncAclPos *acl_out, int max_blocks, int num_cu,
                                   const uint8_t *payload, hipStream_t s);
hipError_t launch_encode_acl_grp(const honu_meta *meta, const honu_acl *acl, uint64_t n,
                                 uint8_t *out, int32_t *status, const EncAclPos *acl_pos,
                                 int max_blocks, hipStream_t s);
// the same with the lists placed by the kernel itself (no acl_pos), so that it
// can run beside launch_encode_meta_lane
hipError_t launch_encode_acl_grp_self(const honu_meta *meta, const honu_acl *acl, const uint64_t *payload_off,
                                      uint64_t n, uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                      int32_t *status, int max_blocks, hipStream_t s);
// header + Metadata tail, ACL entries included, one record per 16-lane group
// (enc.hip; encode_variant 1, A/B build only)
hipError_t launch_encode_tail_grp(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                  const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                  uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                  int32_t *status, int max_blocks, hipStream_t s);

hipError_t launch_encode_sizes_grp(const honu_meta *meta, uint64_t var_len, const honu_acl *acl,
                                   uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                                   const uint64_t *payload_off, uint64_t n, uint64_t *sizes,
                                   int32_t *status, int max_blocks, hipStream_t s);
hipError_t launch_decode_fill_grp(const uint8_t *rec, uint64_t n, honu_meta *meta,
                                  honu_record_info *info, const DecodeScratch *scratch,
                                  const uint32_t *reg_inline, const uint64_t *counts,
                                  const uint64_t *offs, honu_acl *acl, uint64_t acl_cap,
                                  uint32_t *reg, uint64_t reg_cap, uint8_t *data,
                                  uint64_t data_cap, int max_blocks, hipStream_t s);

// fused.hip: one launch from records to rows, record info and tables
// (materialize: also the data-arena offsets honu_decode_payloads copies to)
int decode_walk_flag_checks();  // fused.hip: bit 0 window 1's flags, bit 1 window 2's
hipError_t launch_decode_fused(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_meta *meta, honu_record_info *info, honu_acl *acl,
                               uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, int materialize,
                               uint64_t data_cap, DecodeScratch *scratch, uint64_t *offs,
                               uint64_t *totals, LbState *lb, uint64_t *lb_status,
                               uint64_t *lb_gstatus, uint64_t lb_words, int max_blocks, uint32_t *spec_seen,
                               uint32_t *recoveries, bool allow_spec, bool inplace, bool reg_inplace,
                               bool inline_rec, int guard_blocks, hipStream_t s);

hipError_t launch_decode_parse_win(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   honu_meta *meta, honu_record_info *info,
                                   DecodeScratch *scratch, uint32_t *reg_inline, uint64_t *counts,
                                   int max_blocks, bool inplace, bool reg_inplace, hipStream_t s);

hipError_t launch_system_sizes(const honu_collection *rows, uint64_t var_len, const honu_acl *acl,
                               uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                               const honu_index *idx, uint64_t idx_len, uint64_t n,
                               uint64_t *sizes, int32_t *status, hipStream_t s);
hipError_t launch_system_encode(const honu_collection *rows, const uint8_t *var,
                                const honu_acl *acl, const uint32_t *reg, const honu_index *idx,
                                uint64_t n, uint8_t *out, uint64_t out_cap,
                                const uint64_t *out_off, int32_t *status, hipStream_t s);
hipError_t launch_system_parse(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               bool headless, honu_collection *rows, int32_t *status,
                               DecodeScratch *scratch, uint64_t *counts, hipStream_t s);
hipError_t launch_system_fill(const uint8_t *rec, uint64_t n, honu_collection *rows,
                              int32_t *status, const DecodeScratch *scratch,
                              const uint64_t *counts, const uint64_t *offs, honu_acl *acl,
                              uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, honu_index *idx,
                              uint64_t idx_cap, hipStream_t s);

hipError_t launch_decode_headers(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                 honu_record_info *info, hipStream_t s);
hipError_t launch_decode_spans(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_record_info *info, DecodeScratch *scratch, uint64_t *counts,
                               hipStream_t s);
hipError_t launch_decode_data_place(uint64_t n, honu_record_info *info, const uint64_t *offs,
                                    uint64_t data_cap, hipStream_t s);
hipError_t launch_span_copy(const LaunchGeom &g, const uint8_t *rec, uint64_t n,
                            const honu_record_info *info, const DecodeScratch *scratch,
                            const uint64_t *offs, uint8_t *data, hipStream_t s);

// Exclusive scan of K interleaved u64 columns: out[i*K+c] = sum_{j<i} in[j*K+c];
// totals[c] = full sum. One launch (decoupled look-back over tiles); the
// state is the context's (scan_status_words(n) status words).
struct ScanState {
    LbState *lb;
    uint64_t *status;
    uint64_t words;
    int max_blocks;
};
uint64_t scan_status_words(uint64_t n);
hipError_t launch_scan(const uint64_t *in, uint64_t n, int K, uint64_t *out, uint64_t *totals,
                       const ScanState &S, hipStream_t s);

hipError_t launch_hbm_probe(int mode, const void *src, void *dst, uint64_t bytes, uint32_t blocks,
                            uint32_t *sink, hipStream_t s);
hipError_t launch_gen_payload(const LaunchGeom &g, uint64_t seed, uint64_t first, uint64_t n,
                              const uint64_t *payload_off, uint8_t *payload, hipStream_t s);
hipError_t launch_verify_decoded(const LaunchGeom &g, const honu_meta *src, const uint8_t *var,
                                 const honu_acl *src_acl, const uint32_t *src_reg,
                                 const uint64_t *payload_off, const uint8_t *rec,
                                 const honu_meta *dec, const honu_record_info *info,
                                 const honu_acl *dec_acl, const uint32_t *dec_reg, uint64_t n,
                                 uint32_t *mismatch, hipStream_t s);
hipError_t launch_digest(const LaunchGeom &g, const uint8_t *arena, const uint64_t *off,
                         const uint64_t *len, uint64_t n, uint64_t *digest, hipStream_t s);

}  // namespace honu
