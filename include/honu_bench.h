/*
 * honu_bench.h — measurement and test support of libhonu_codec.so: the
 * synthetic workload generator (the reference benchmark's shapes), payload
 * digests, the decoded-batch verifier and the HBM streaming probe. These are
 * exported by the same library but are not part of the drop-in boundary a
 * binding vendors (include/honu_codec.h): bench.py, the tests
 * and honu_amd/c_abi_demo.c use them.
 */
#ifndef HONU_BENCH_H
#define HONU_BENCH_H

#include "honu_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Synthetic workload (bench/test support; mirrors the reference benchmark   */
/* generator object_test.go:195-386 with a seeded counter-based PRNG).       */
/* ------------------------------------------------------------------------ */
typedef enum honu_shape {
    HONU_SHAPE_SMALL = 0,  /* payload U[512, 4608)        object_test.go:376 */
    HONU_SHAPE_MEDIUM = 1, /* payload U[8192, 40960)      :378 */
    HONU_SHAPE_LARGE = 2,  /* payload U[65536, 327680)    :380 */
    HONU_SHAPE_XLARGE = 3, /* payload U[1048576, 5242880) :382 */
    HONU_SHAPE_MIXED = 4   /* per record: S .50 / M .30 / L .19 / XL .01 */
} honu_shape;

/* Host-side sizing pass for records [first, first+n) of the synthetic batch
 * (seed, shape): totals of var-arena bytes, ACL entries, region entries and
 * payload bytes, so the caller can allocate before honu_gen_meta. */
void honu_gen_totals(uint64_t seed, int32_t shape, uint64_t first, uint64_t n,
                     uint64_t totals[4]);

/* Host-side: fill HOST arrays for records [first, first+n): rows, var arena,
 * ACL table, region table and the CSR payload offsets (n+1, starting at 0).
 * Offsets in rows are relative to the given arrays. */
void honu_gen_meta(uint64_t seed, int32_t shape, uint64_t first, uint64_t n, honu_meta *meta,
                   uint8_t *var_arena, honu_acl *acl, uint32_t *regions, uint64_t *payload_off);

/* Payload bytes of record `index` of the synthetic batch are
 * honu_payload_byte(seed, index, k) for k in [0, len). Host and device
 * produce identical bytes. */
void honu_gen_payload_host(uint64_t seed, uint64_t first, uint64_t n, const uint64_t *payload_off,
                           uint8_t *payload);
int32_t honu_gen_payload(honu_ctx *ctx, uint64_t seed, uint64_t first, uint64_t n,
                         const uint64_t *d_payload_off, uint8_t *d_payload, void *stream);

/* ------------------------------------------------------------------------ */
/* Verification helpers (device, used by tests and bench at full size)       */
/* ------------------------------------------------------------------------ */

/* Position-aware 64-bit digest of every record's bytes: splitmix64(len) +
 * sum over the zero-padded little-endian 8-byte words w_k of
 * splitmix64(w_k + k * 0x9E3779B97F4A7C15). d_digest[i] covers
 * d_arena[d_off[i], d_off[i+1]) or, when d_len != NULL,
 * [d_off[i], d_off[i]+d_len[i]) with d_off of length n. */
int32_t honu_digest_records(honu_ctx *ctx, const uint8_t *d_arena, const uint64_t *d_off,
                            const uint64_t *d_len, uint64_t n, uint64_t *d_digest, void *stream);
/* Round trip check of a decoded batch against the encode input it came from
 * (bench and tests at full size, where the CPU oracle is too slow): record i
 * was encoded from source row d_src[i] (spans into d_var, lists into d_src_acl
 * / d_src_regions, payload length d_payload_off[i+1] - d_payload_off[i]) and
 * decoded into d_dec[i] / d_info[i] (spans into the records arena d_rec,
 * lists into d_dec_acl / d_dec_regions). d_mismatch[i] gets an OR of
 * HONU_VERIFY_* bits, 0 when every row byte, span byte, ACL entry and region
 * equals what the Go decoder returns for that input (nil structs zero,
 * REGIONS_NONNIL set, nil ACL entries all-zero). Payload bytes are checked
 * with honu_digest_records. */
enum {
    HONU_VERIFY_STATUS = 1u << 0,   /* a status is not OK, or len(Data()) differs */
    HONU_VERIFY_PRESENT = 1u << 1,  /* presence bits */
    HONU_VERIFY_FIELDS = 1u << 2,   /* a fixed row byte (scalars, ULIDs, span lengths, counts) */
    HONU_VERIFY_SPANS = 1u << 3,    /* bytes of a MIME/schema/publisher/encryption span */
    HONU_VERIFY_ACL = 1u << 4,      /* an ACL table entry */
    HONU_VERIFY_REGIONS = 1u << 5   /* a region table entry */
};
int32_t honu_verify_decoded(honu_ctx *ctx, const honu_meta *d_src, const uint8_t *d_var,
                            const honu_acl *d_src_acl, const uint32_t *d_src_regions,
                            const uint64_t *d_payload_off, const uint8_t *d_rec,
                            const honu_meta *d_dec, const honu_record_info *d_info,
                            const honu_acl *d_dec_acl, const uint32_t *d_dec_regions, uint64_t n,
                            uint32_t *d_mismatch, void *stream);
/* The same digest of one host byte run. */
uint64_t honu_digest_host(const uint8_t *p, uint64_t len);

/* Measurement: the part's achievable HBM streaming rates (bench.py's
 * roofline denominator beside the 8 TB/s spec). mode 0 reads bytes of d_src,
 * 1 writes bytes of d_dst, 2 copies d_src -> d_dst with each wave on a
 * contiguous range (the codec copy engine's layout, 8 x 16 B per lane in
 * flight), 3 the same copy grid-stride (4 x 16 B per lane), 4 mode 2 with
 * non-temporal loads and stores (tools/copy_sweep.hip: the fastest plain copy
 * form measured on this part, at 4 workgroups per CU). bytes is rounded
 * down to 16; buffers 16-byte aligned; blocks_per_cu 0 = 2. Asynchronous on
 * stream; time it with events. */
int32_t honu_hbm_probe(honu_ctx *ctx, int32_t mode, const void *d_src, void *d_dst, uint64_t bytes,
                       uint32_t blocks_per_cu, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HONU_BENCH_H */
