/*
 * honu_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single thread) of the Go reference's object-record
 * codec: rotationalio/honu pkg/store/object, pkg/store/lani, pkg/store/metadata,
 * pkg/store/lamport (Scalar codec) and pkg/region (Regions codec), plus the
 * Go stdlib encoding/binary varint routines they call (Go 1.25.1, go.mod:3;
 * not under /root/reference, restated from the published algorithm).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the CPU baseline. The product
 * (honu_amd/) never links or calls it.
 *
 * Parity pinning: the Go toolchain is absent from this image, so the reference
 * cannot be run. The restatement is pinned by the reference's own known-answer
 * tests (tests/test_oracle_golden.py): the 1264-byte fixture object
 * (object_test.go:29) with its full byte map, Scalar{42,198} -> 2a c6 01
 * (lamport/scalar_test.go:78), the varint size tables (lani/encode_test.go:
 * 270-362), frame sizes, single-byte encodings, the decoder error vectors
 * (lani/decode_test.go:44-70,175-182), the nil/malformed object cases
 * (object_test.go:60-83) and the Size() fixtures of every metadata type.
 *
 * Records use the product's row layout (include/honu_codec.h) so outputs can be
 * compared byte for byte; the grammar walk itself shares no code with the
 * product.
 */
#ifndef HONU_ORACLE_H
#define HONU_ORACLE_H

#include <stdint.h>
#include "../include/honu_codec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Go encoding/binary (varint.go) */
int oracle_put_uvarint(uint8_t *buf, uint64_t x);                  /* PutUvarint */
int oracle_uvarint(const uint8_t *buf, uint64_t n, uint64_t *out);  /* Uvarint -> k */
int oracle_put_varint(uint8_t *buf, int64_t x);                    /* PutVarint */
int oracle_varint(const uint8_t *buf, uint64_t n, int64_t *out);    /* Varint -> k */

/* lani.Encodable.Size() upper bounds (the Grow hint): metadata.go:62-106,
 * version.go:31-42, schema.go:24-28, acls.go:19-21, provenance.go:25-31,
 * encryption.go:42-51, compression.go:27-29. which: 0 Metadata, 1 Version,
 * 2 SchemaVersion, 3 AccessControl, 4 Publisher, 5 Encryption, 6 Compression. */
int64_t oracle_size_bound(int which, const honu_meta *m);

/* object.Marshal (object.go:24-45) of one record. Writes at most `cap` bytes
 * to out (out may be NULL with cap 0 to size only) and returns the exact
 * encoded length in *out_len. Returns an honu_status (PANIC for a nil
 * Metadata, INPUT for spans outside their arenas, CAPACITY when cap is short). */
int oracle_marshal(const honu_meta *m, const uint8_t *var, uint64_t var_len, const honu_acl *acl,
                   uint64_t acl_len, const uint32_t *regions, uint64_t regions_len,
                   const uint8_t *data, uint64_t data_len, uint8_t *out, uint64_t cap,
                   uint64_t *out_len);

/* Decode output forms (bits of `forms` below), the product's context params
 * "acl_inplace" and "regions_inplace" (include/honu_codec.h). */
#define ORACLE_ACL_INPLACE 1
#define ORACLE_REGIONS_INPLACE 2

/* Object.Metadata() + Object.Data() + Tombstone() + StorageVersion()
 * (object.go:47-134) of one record `o` of length len, located at absolute
 * offset `base` of its arena (spans and data_off are reported absolute).
 * ACL entries / regions are appended to acl_out / regions_out (capacities
 * given); *acl_n / *regions_n receive the counts decoded. On a Metadata error
 * the row is zeroed (Go returns nil, err) and counts are 0. forms &
 * ORACLE_ACL_INPLACE: an ACL list whose entries are all present is returned in
 * place, as the product does by default (include/honu_codec.h
 * HONU_ACL_INPLACE): acl_off is the absolute offset of its first entry and
 * nothing goes to acl_out. forms & ORACLE_REGIONS_INPLACE: a non-empty region
 * list likewise (HONU_REGIONS_INPLACE, regions_off absolute, every uvarint
 * still decoded with DecodeUint32's checks). */
void oracle_decode(const uint8_t *o, uint64_t len, uint64_t base, honu_meta *m,
                   honu_record_info *info, honu_acl *acl_out, uint64_t acl_cap,
                   uint32_t *regions_out, uint64_t regions_cap, uint64_t *acl_n,
                   uint64_t *regions_n, int forms);

/* Batch drivers with the same output conventions as the HIP path
 * (honu_marshal_batch / honu_decode_batch): sequential offsets == exclusive
 * scans; when data != NULL payloads are materialised at 16-byte aligned
 * offsets of `data`. out_off has n+1 entries. Return 0 or HONU_ERR_CAPACITY. */
int oracle_marshal_batch(const honu_meta *meta, const uint8_t *var, uint64_t var_len,
                         const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                         uint64_t regions_len, const uint8_t *payload,
                         const uint64_t *payload_off, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, int32_t *status);

int oracle_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n, honu_meta *meta,
                        honu_record_info *info, honu_acl *acl, uint64_t acl_cap,
                        uint32_t *regions, uint64_t regions_cap, uint8_t *data, uint64_t data_cap,
                        uint64_t totals[3], int forms);

/* keys.New(oid, &Version.Scalar) (keys/keys.go:42-51) for a decoded row. */
int oracle_key(const honu_meta *m, int32_t meta_status, uint8_t key[29]);

/* System objects (object/system.go:10-45) with metadata.Collection
 * (collection.go), Index (index.go) and Field (field.go). */
int64_t oracle_field_size(uint64_t name_len);                /* Field.Size */
int64_t oracle_index_size(const honu_index *x);              /* Index.Size */
int64_t oracle_collection_size(const honu_collection *c, const honu_acl *acl,
                               const honu_index *idx);       /* Collection.Size */
/* MarshalSystem of one collection row (no HONU_HAS_COLLECTION: MarshalSystem(nil)) */
int oracle_system_marshal(const honu_collection *c, const uint8_t *var, uint64_t var_len,
                          const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                          uint64_t regions_len, const honu_index *idx, uint64_t idx_len,
                          uint8_t *out, uint64_t cap, uint64_t *out_len);
/* UnmarshalSystem(obj, &Collection{}) of one record at absolute offset base;
 * counts = ACL entries, regions, indexes appended to the tables. */
int oracle_system_decode(const uint8_t *o, uint64_t len, uint64_t base, honu_collection *c,
                         honu_acl *acl_out, uint64_t acl_cap, uint32_t *regions_out,
                         uint64_t regions_cap, honu_index *idx_out, uint64_t idx_cap,
                         uint64_t counts[3]);
int oracle_system_marshal_batch(const honu_collection *rows, const uint8_t *var, uint64_t var_len,
                                const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                                uint64_t regions_len, const honu_index *idx, uint64_t idx_len,
                                uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                                int32_t *status);
int oracle_system_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_collection *rows, int32_t *status, honu_acl *acl,
                               uint64_t acl_cap, uint32_t *regions, uint64_t regions_cap,
                               honu_index *idx, uint64_t idx_cap, uint64_t totals[3]);
/* lani.Unmarshal(raw, &metadata.Collection{}) (lani.go:29-33) per record:
 * Collection.Decode (collection.go:240-356) from byte 0 of the raw value, as
 * store.go:367 calls it on a bbolt value that holds a whole system object. */
int oracle_collection_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   honu_collection *rows, int32_t *status, honu_acl *acl,
                                   uint64_t acl_cap, uint32_t *regions, uint64_t regions_cap,
                                   honu_index *idx, uint64_t idx_cap, uint64_t totals[3]);

#ifdef __cplusplus
}
#endif
#endif
