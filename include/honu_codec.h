/*
 * honu_codec.h — C ABI of the MI355X-native batch object-record codec.
 *
 * This is the drop-in boundary for Honu's reflection-free object codec
 * (rotationalio/honu, pkg/store/object + pkg/store/lani + pkg/store/metadata).
 * The reference has no FFI at all (it is pure Go, CGO_ENABLED=0); the entry
 * points below are what a cgo shim behind a `honu_hip` build tag binds so that
 * pkg/store keeps its Go API (see INTEGRATION.md for the cgo stub).
 *
 *   reference (Go, one record per call)               this ABI (one batch per call)
 *   -----------------------------------------------   ------------------------------------------
 *   object.Marshal(meta, data)  object.go:24-45        honu_encode_sizes + honu_exclusive_scan
 *                                                       + honu_encode   (or honu_marshal_batch)
 *   Object.Metadata()           object.go:66-83        honu_decode_parse + honu_decode_fill
 *   Object.Data()               object.go:85-99          (or honu_decode_batch); per-record
 *   Object.Tombstone()          object.go:103-112        results land in honu_record_info
 *   Object.StorageVersion()     object.go:47-52
 *   Object.Key()                object.go:57-64        honu_decode_keys (29-byte keys.Key column)
 *   lani.Encodable.Size()       lani/lani.go:9-12      (host only; Size() is a Grow hint, not bytes)
 *
 * Conventions
 *   - Every pointer argument named d_* is DEVICE memory (hipMalloc / torch
 *     tensor storage) unless stated; every call is asynchronous on `stream`
 *     (a hipStream_t passed as void*, NULL = the null stream). No call
 *     allocates, frees or synchronises, so a sequence of calls can be
 *     captured into a hipGraph.
 *   - Batches are CSR: record i occupies bytes [off[i], off[i+1]) of an arena.
 *   - Functions return an honu_status for argument errors (HONU_E_ARG,
 *     HONU_E_WORKSPACE, HONU_E_HIP); per-record outcomes are written to device
 *     status arrays using the same enum.
 *   - The library is gfx950-only; it fails loudly (HONU_E_NO_DEVICE) when no
 *     gfx950 device is present. There is no CPU fallback.
 */
#ifndef HONU_CODEC_H
#define HONU_CODEC_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HONU_ABI_VERSION 6u  /* 6: region lists returned in place (HONU_REGIONS_INPLACE);
                                5: honu_encode_*_units; 4: ACL lists returned in place (HONU_ACL_INPLACE) */
#define HONU_STORAGE_VERSION 1u /* object.StorageVersion, object.go:14 */
#define HONU_ULID_LEN 16
#define HONU_KEY_LEN 29         /* keys.keySize, keys/keys.go:14 */

/* ------------------------------------------------------------------------ */
/* Status codes. Per-record codes map 1:1 to the Go sentinels.              */
/* ------------------------------------------------------------------------ */
typedef enum honu_status {
    HONU_OK = 0,
    HONU_ERR_BAD_VERSION = 1,    /* object.ErrBadVersion     object/errors.go:6 */
    HONU_ERR_MALFORMED = 2,      /* object.ErrMalformed      object/errors.go:7 */
    HONU_ERR_EOF = 3,            /* io.EOF                   lani/decode.go:95,129,151,173,195,211 */
    HONU_ERR_UNEXPECTED_EOF = 4, /* io.ErrUnexpectedEOF      lani/decode.go:47,200,215 */
    HONU_ERR_NO_LENGTH = 5,      /* lani.ErrNoLength         lani/errors.go:8 */
    HONU_ERR_PARSE_BOOLEAN = 6,  /* lani.ErrParseBoolean     lani/errors.go:9 */
    HONU_ERR_PARSE_VARINT = 7,   /* lani.ErrParseVarInt      lani/errors.go:10 */
    HONU_ERR_PANIC = 8,          /* input on which the Go reference panics (slice
                                    out of range object.go:77,97; makeslice
                                    decode.go:50, metadata.go:255, region.go:160;
                                    nil *Metadata in Marshal metadata.go:66) */
    HONU_ERR_CAPACITY = 9,       /* an output arena/table was too small (ABI only) */
    HONU_ERR_INPUT = 10,         /* an encode input span/list points outside its arena (ABI only) */
    HONU_UNPARSED = 11,          /* meta_status of honu_decode_headers: Metadata() not evaluated */
    /* call-level errors (returned, never written per record) */
    HONU_E_ARG = -1,
    HONU_E_WORKSPACE = -2,       /* n exceeds the context's reserved record count */
    HONU_E_HIP = -3,             /* a HIP runtime call failed */
    HONU_E_NO_DEVICE = -4        /* no gfx950 device / kernels not loadable */
} honu_status;

/* ------------------------------------------------------------------------ */
/* Data layout                                                               */
/* ------------------------------------------------------------------------ */

/* A byte range inside an arena. Zero length == nil == empty: lani frames of
 * length 0 decode to nil (lani/decode.go:37-39) and nil/empty encode alike. */
typedef struct honu_span {
    uint64_t off;
    uint64_t len;
} honu_span;

/* Presence bits of honu_meta.present (the lani nil-flag bytes). */
enum {
    HONU_HAS_META = 1u << 0,        /* object-level Metadata nil flag (object.go:40) */
    HONU_HAS_VERSION = 1u << 1,     /* Metadata.Version      metadata.go:20 */
    HONU_HAS_PARENT = 1u << 2,      /* Version.Parent        version.go:17 */
    HONU_HAS_SCHEMA = 1u << 3,      /* Metadata.Schema       metadata.go:21 */
    HONU_HAS_PUBLISHER = 1u << 4,   /* Metadata.Publisher    metadata.go:28 */
    HONU_HAS_ENCRYPTION = 1u << 5,  /* Metadata.Encryption   metadata.go:29 */
    HONU_HAS_COMPRESSION = 1u << 6, /* Metadata.Compression  metadata.go:30 */
    HONU_REGIONS_NONNIL = 1u << 7,  /* set by decode: Regions.Decode always makes a
                                       (possibly empty) slice, region.go:160 */
    HONU_ACL_INPLACE = 1u << 8,     /* set by decode (honu_meta only): the ACL list is
                                       returned in place, see honu_meta.acl_off */
    HONU_REGIONS_INPLACE = 1u << 9, /* set by decode (honu_meta only): the region list
                                       is returned in place, see honu_meta.regions_off */
    HONU_ACL_SIZED = 1u << 10       /* encode input (honu_meta only): acl_bytes holds the
                                       ACL list's encoded length, see honu_meta.acl_bytes */
};

/* One metadata.Metadata (metadata.go:17-35) flattened into a fixed 352-byte
 * row. Rows are the encode input and the decode output.
 *   encode: spans index `var_arena`, acl_off/acl_count index the ACL table,
 *           regions_off/regions_count index the region table.
 *   decode: spans are ABSOLUTE offsets into the records arena (zero copy, like
 *           lani.DecodeFixed), regions_off indexes the output region table.
 *           The ACL list comes back in one of two forms:
 *           - in place (HONU_ACL_INPLACE set in `present`; the default, context
 *             param "acl_inplace" 1): every entry of the list is present, and
 *             acl_off is the ABSOLUTE offset in the records arena of the first
 *             entry's encoding; entry j is the 18 bytes at acl_off + 18*j:
 *             0x01 | ClientID[16] | Permissions (acls.go:26-51), so
 *             ACL[j] = &AccessControl{rec[acl_off+18j+1 : +17], rec[acl_off+18j+17]};
 *           - table (HONU_ACL_INPLACE clear, acl_count > 0): a list holding a
 *             nil entry, or every list when "acl_inplace" is 0: acl_off indexes
 *             the honu_acl output table (present == 0 is a nil entry).
 *           Go copies every entry into a new *AccessControl either way
 *           (metadata.go:254-266); the in-place form leaves that copy to the
 *           binding, as Data() and the string spans already do.
 *           The region list likewise:
 *           - in place (HONU_REGIONS_INPLACE set; the default, context param
 *             "regions_inplace" 1, every non-empty list): regions_off is the
 *             ABSOLUTE offset in the records arena of the first region's
 *             uvarint; the regions_count uvarints follow back to back, each
 *             decoded as lani.DecodeUint32 does (at most 5 bytes, the value
 *             truncated to uint32: decode.go:127-146). The decode has already
 *             validated every one of them (a bad varint fails the record), so
 *             the binding's Regions.Decode loop (region.go:154-169) cannot fail;
 *           - table (HONU_REGIONS_INPLACE clear, regions_count > 0; every list
 *             when "regions_inplace" is 0): regions_off indexes the uint32
 *             output region table.
 *           In-place lists and spans point into the records arena: the row is
 *           valid while that arena is. Encode input rows must use the table
 *           forms: a row with HONU_ACL_INPLACE or HONU_REGIONS_INPLACE set gets
 *           HONU_ERR_INPUT from honu_encode_sizes.
 *   encode, HONU_ACL_SIZED (optional, what a binding's flatten sets while it
 *           copies m.ACL): acl_bytes = sum over the list of 18 per present
 *           entry and 1 per nil one (acls.go:26-39, encode.go:210-226), so the
 *           size pass reads no ACL table entry (the list kernel reads every
 *           entry anyway and checks the length: a row whose acl_bytes is not
 *           the list's length gets HONU_ERR_INPUT from the records call and
 *           its range of the output holds unspecified bytes; a value outside
 *           [acl_count, 18 * acl_count] is rejected by honu_encode_sizes).
 *           Without the bit the size pass reads the list from the table.
 * Times are Go UnixNano with 0 <=> time.Time{}.IsZero() (lani/encode.go:201-206,
 * decode.go:224-237). Fields of absent (nil) sub-structs are zero on decode. */
typedef struct honu_meta {
    uint32_t present;            /*   0 HONU_HAS_* bits */
    uint8_t permissions;         /*   4 Metadata.Permissions */
    uint8_t flags;               /*   5 Metadata.Flags */
    uint8_t tombstone;           /*   6 Version.Tombstone (bool, 0/1) */
    uint8_t compression_alg;     /*   7 Compression.Algorithm */
    uint8_t sealing_alg;         /*   8 Encryption.SealingAlgorithm */
    uint8_t encryption_alg;      /*   9 Encryption.EncryptionAlgorithm */
    uint8_t signature_alg;       /*  10 Encryption.SignatureAlgorithm */
    uint8_t _pad0;               /*  11 */
    uint32_t region;             /*  12 Version.Region */
    uint64_t vid;                /*  16 Version.Scalar.VID */
    uint32_t pid;                /*  24 Version.Scalar.PID */
    uint32_t parent_pid;         /*  28 Version.Parent.PID */
    uint64_t parent_vid;         /*  32 Version.Parent.VID */
    int64_t version_created;     /*  40 Version.Created */
    uint32_t schema_major;       /*  48 SchemaVersion.Major */
    uint32_t schema_minor;       /*  52 */
    uint32_t schema_patch;       /*  56 */
    uint32_t _pad1;              /*  60 */
    int64_t compression_level;   /*  64 Compression.Level */
    int64_t created;             /*  72 Metadata.Created */
    int64_t modified;            /*  80 Metadata.Modified */
    uint64_t acl_bytes;          /*  88 encode input with HONU_ACL_SIZED: the ACL
                                        list's encoded length; 0 on decode */
    uint8_t object_id[16];       /*  96 Metadata.ObjectID */
    uint8_t collection_id[16];   /* 112 Metadata.CollectionID */
    uint8_t owner[16];           /* 128 Metadata.Owner */
    uint8_t group[16];           /* 144 Metadata.Group */
    uint8_t publisher_id[16];    /* 160 Publisher.PublisherID */
    uint8_t client_id[16];       /* 176 Publisher.ClientID */
    honu_span schema_name;       /* 192 SchemaVersion.Name */
    honu_span mime;              /* 208 Metadata.MIME */
    honu_span ip_address;        /* 224 Publisher.IPAddress (net.IP bytes) */
    honu_span user_agent;        /* 240 Publisher.UserAgent */
    honu_span public_key_id;     /* 256 Encryption.PublicKeyID */
    honu_span encryption_key;    /* 272 Encryption.EncryptionKey */
    honu_span hmac_secret;       /* 288 Encryption.HMACSecret */
    honu_span signature;         /* 304 Encryption.Signature */
    uint64_t acl_off;            /* 320 first entry in the ACL table, or (decode,
                                        HONU_ACL_INPLACE) in the records arena */
    uint64_t acl_count;          /* 328 len(Metadata.ACL); 0 <=> nil */
    uint64_t regions_off;        /* 336 first entry in the region table, or (decode,
                                        HONU_REGIONS_INPLACE) in the records arena */
    uint64_t regions_count;      /* 344 len(Metadata.WriteRegions) */
} honu_meta;                     /* 352 */

/* One *metadata.AccessControl (acls.go:12-15); present==0 is a nil pointer
 * in the ACL slice (encoded as a single 0x00 flag byte). */
typedef struct honu_acl {
    uint8_t client_id[16];
    uint8_t permissions;
    uint8_t present;
    uint8_t _pad[2];
} honu_acl; /* 20 */

/* Per-record decode results: the Object methods object.go:47-112. */
typedef struct honu_record_info {
    uint64_t data_off;       /* payload: absolute offset in the records arena
                                (zero copy, like Data()'s subslice) or in the
                                data arena when materialising */
    uint64_t data_len;       /* len(Data()); 0 also for nil */
    int32_t data_status;     /* error of Object.Data() */
    int32_t meta_status;     /* error of Object.Metadata() */
    uint8_t storage_version; /* Object.StorageVersion() */
    uint8_t tombstone;       /* Object.Tombstone() */
    uint8_t _pad[6];
} honu_record_info; /* 32 */

/* ------------------------------------------------------------------------ */
/* Context                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct honu_ctx honu_ctx;

/* Create a context on HIP device `device` with scratch for batches of up to
 * `max_records` records (scan partials, decode list positions). Allocation
 * happens here and only here. Returns NULL and sets *err on failure.
 * The scratch is per context: calls that use it (scans, decodes and the decode
 * payload copies, which read the decode's scratch) issued on different
 * streams concurrently need one context each. The encode payload copies
 * (honu_encode_payloads*) use none and may run concurrently on one context:
 * every copy call takes its own range-tail counter line from a ring of 64
 * (param "copy_steal"), so up to 64 copies may be in flight at once on one
 * context. The library reads no environment variable: a
 * context is configured through honu_ctx_set_param only. Arenas: the records
 * arena, the materialised data arena and row arrays must be 16-byte aligned,
 * ACL and region tables 4-byte aligned (hipMalloc gives 256). */
honu_ctx *honu_ctx_create(int device, uint64_t max_records, int32_t *err);
void honu_ctx_destroy(honu_ctx *ctx);
uint64_t honu_ctx_max_records(const honu_ctx *ctx);

/* The single-launch decode and the one-launch scans keep decoupled look-back
 * state in the context (a tile ticket, a finished-workgroup count and a launch
 * epoch) that each launch leaves clean for the next, so nothing is cleared
 * per call and the calls replay from a captured hipGraph. A launch that did
 * not run to completion (its stream was torn down, the device reset) can leave
 * it dirty: a context that saw a HIP error (HONU_E_HIP) must be reset with
 * honu_ctx_reset, on a stream with no other work of this context in flight,
 * before its next decode or scan (it returns when the reset is done). */
int32_t honu_ctx_reset(honu_ctx *ctx, void *stream);

/* Launch-geometry knobs (defaults suit MI355X): "copy_blocks" (workgroups of
 * the payload copy kernel, default 2 per CU), "record_blocks" (cap on
 * workgroups of the one-wave-per-record kernels, default 8 per CU),
 * "lane_blocks" (cap on workgroups of the lane, group and window kernels;
 * default 0 = no cap — a cap leaves room for a concurrent payload copy),
 * "copy_variant" (copy-engine variant, default 0), "copy_steal" (1, the
 * default: in a copy whose payloads average >= 16 KB each streaming wave
 * copies 7/8 of its byte range, then the ranges' last eighths from a counter
 * in the context; 0: fixed ranges only), "record_variant" (how the
 * per-record metadata kernels map records to lanes: 0 auto — the fastest
 * measured form per kernel, with honu_decode_batch running the single-launch
 * decode for batches of 48 K records or more; 5 the split decode at every
 * size; 6 the single-launch decode at every size), "encode_variant" (the
 * header/tail encoder of honu_encode_records: 0 one record per lane + the ACL
 * lists by 16-lane groups, the default; 1 one record per 16-lane group laid
 * out by a prefix sum over the grammar's slots, same bytes), "speculate" (the
 * single-launch decode's speculation, see honu_decode_records: 2 auto, the
 * default — only in materialising calls and the table forms, where it hides
 * look-back waits; 1 in every call; 0 off), "speculate_backoff" (0..16: the calls left without
 * speculation after a recovery; setting it also forgets a recovery the host
 * has not seen yet), "encode_fork" (honu_encode_records: 1 runs the ACL lists'
 * kernel, which then places the lists itself, on a stream of the context's own
 * beside the header/tail encoder, forked from and joined back into the
 * caller's stream by events; 0 after it; 2, the default, forks when
 * "lane_blocks" caps the encoder's grid and the caller's stream has neither a
 * CU mask nor a non-default priority, which the fork's stream would escape).
 * "acl_inplace" (1 default, 0 off): the decode calls
 * (honu_decode_parse/fill/tables/records/batch) return an ACL list whose
 * entries are all present in place (HONU_ACL_INPLACE, see honu_meta) instead
 * of copying it into the ACL table; 0 returns every list in the table.
 * "regions_inplace" (1 default, 0 off): the same calls return every
 * non-empty region list in place (HONU_REGIONS_INPLACE) instead of in the
 * region table; 0 returns every list in the table. With both in place a
 * zero-copy batch whose ACL lists hold no nil entry writes no table entry,
 * and the single-launch decode's 64-record tiles then need no offsets from
 * their predecessors (only the batch's last tile resolves them, for
 * d_totals).
 * "inline_recovery" (0 default, 1 on): a speculative single-launch decode
 * with more 64-record tiles than resident waves redoes a misspeculated batch
 * inside the same launch instead of in a guarded second launch (one-wave
 * workgroups, placed as registers free up beside other kernels even when it
 * has nothing to do); launches whose tiles all fit keep the guarded launch. Measured slower
 * in the common, clean case (DESIGN §3 "Round 5"), hence off. "recoveries"
 * (get only): the recovery passes or launches the context has run. */
int32_t honu_ctx_set_param(honu_ctx *ctx, const char *name, int64_t value);

/* The current value of a parameter of honu_ctx_set_param, and
 * "speculate_backoff": how many of the context's next decode calls run
 * without speculation (16 once a recovery launch has run, see
 * honu_decode_records; the count drops by one per call), and
 * "walk_flag_checks" (as built): which entry flags of a speculated ACL list
 * the walk checks itself, so that a nil entry there costs no recovery launch —
 * bit 0 the first ones (the window at the tail's start), bit 1 the last ones
 * (the window after the list); the flags in between are the burst's. */
int32_t honu_ctx_get_param(const honu_ctx *ctx, const char *name, int64_t *value);

/* ABI self-description, used by bindings to check struct layouts. */
uint32_t honu_abi_version(void);
uint64_t honu_sizeof_meta(void);
uint64_t honu_sizeof_acl(void);
uint64_t honu_sizeof_collection(void);
uint64_t honu_sizeof_index(void);
uint64_t honu_sizeof_record_info(void);
const char *honu_status_string(int32_t status);
/* Text of the last call-level failure on this thread (HIP error text etc.). */
const char *honu_last_error(void);

/* ------------------------------------------------------------------------ */
/* Encode: object.Marshal over a batch (object.go:24-45)                     */
/* ------------------------------------------------------------------------ */

/* Exact encoded length of every record: 1 + uvarint(len data) + len data +
 * 1 + len(Metadata encoding) (object.go:30,35,40). A record that cannot be
 * encoded gets size 0 and d_status[i] = HONU_ERR_PANIC when HONU_HAS_META is
 * clear (Marshal(nil, …) dereferences nil, metadata.go:66) or HONU_ERR_INPUT
 * when a span or list lies outside its arena; otherwise d_status[i] = HONU_OK.
 * Arguments as for honu_encode. */
int32_t honu_encode_sizes(honu_ctx *ctx, const honu_meta *d_meta, uint64_t var_len,
                          const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                          uint64_t regions_len, const uint64_t *d_payload_off, uint64_t n,
                          uint64_t *d_sizes, int32_t *d_status, void *stream);

/* Exclusive prefix sum: d_out[i] = sum(d_in[0..i)), d_out[n] = total.
 * d_out must hold n+1 values and may alias d_in only if equal. */
int32_t honu_exclusive_scan(honu_ctx *ctx, const uint64_t *d_in, uint64_t n, uint64_t *d_out,
                            void *stream);

/* Encode record i into d_out[d_out_off[i], d_out_off[i+1]). d_out_off comes
 * from honu_encode_sizes + honu_exclusive_scan and d_status from
 * honu_encode_sizes: records whose status is not HONU_OK are skipped, records
 * whose range exceeds out_cap get HONU_ERR_CAPACITY; nothing is written for a
 * failed record.
 *   d_var, var_len:        byte arena indexed by honu_meta spans
 *   d_acl, acl_len:        ACL table indexed by acl_off/acl_count
 *   d_regions, regions_len: uint32 region table
 *   d_payload, d_payload_off: CSR payload arena (the `data` argument)
 * honu_encode = honu_encode_records (header + Metadata tail of every record)
 * followed by honu_encode_payloads (the payload bytes, object.go:35); the two
 * phases are exported separately so they can be scheduled and timed apart. */
int32_t honu_encode(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var, uint64_t var_len,
                    const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                    uint64_t regions_len, const uint8_t *d_payload, const uint64_t *d_payload_off,
                    uint64_t n, uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                    int32_t *d_status, void *stream);
int32_t honu_encode_records(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                            const honu_acl *d_acl, const uint32_t *d_regions,
                            const uint64_t *d_payload_off, uint64_t n, uint8_t *d_out,
                            uint64_t out_cap, const uint64_t *d_out_off, int32_t *d_status,
                            void *stream);
/* honu_encode_payloads needs only d_out_off and the size pass's d_status, so it
 * may run on another stream beside honu_encode_records (each writes only its
 * own bytes of the shared 16-byte chunks); it repeats the out_cap check
 * itself and copies nothing for a record that ends past out_cap. */
int32_t honu_encode_payloads(honu_ctx *ctx, const uint8_t *d_payload, const uint64_t *d_payload_off,
                             uint64_t n, uint8_t *d_out, uint64_t out_cap,
                             const uint64_t *d_out_off, const int32_t *d_status, void *stream);
/* The same two phases split at the memory side's 64-byte write unit (ABI 5):
 * honu_encode_records_units also writes each payload's bytes in the partial
 * 64-byte units at its two ends (from d_payload), and honu_encode_payloads_units
 * writes the whole units between, so no 64-byte unit of the records arena is
 * written partly by both phases (a unit that leaves L2 partly written costs a
 * read-modify-write: DESIGN §3 "the 64-byte write unit"; 1M Small step -1.6 %).
 * Units are counted on absolute addresses of d_out. Records encoded by one of
 * the pair are completed only by the other: never mix the two forms on a
 * batch. honu_encode (one call) uses this form. */
int32_t honu_encode_records_units(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                                  const honu_acl *d_acl, const uint32_t *d_regions,
                                  const uint8_t *d_payload, const uint64_t *d_payload_off, uint64_t n,
                                  uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                                  int32_t *d_status, void *stream);
int32_t honu_encode_payloads_units(honu_ctx *ctx, const uint8_t *d_payload, const uint64_t *d_payload_off,
                                   uint64_t n, uint8_t *d_out, uint64_t out_cap,
                                   const uint64_t *d_out_off, const int32_t *d_status, void *stream);

/* sizes + scan + encode in one call; d_out_off (n+1) is produced here. */
int32_t honu_marshal_batch(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                           uint64_t var_len, const honu_acl *d_acl, uint64_t acl_len,
                           const uint32_t *d_regions, uint64_t regions_len,
                           const uint8_t *d_payload, const uint64_t *d_payload_off, uint64_t n,
                           uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                           int32_t *d_status, void *stream);

/* ------------------------------------------------------------------------ */
/* Decode: Object.Metadata() + Object.Data() over a batch (object.go:66-99)  */
/* ------------------------------------------------------------------------ */

/* Phase 1: parse every record of the CSR batch (d_rec, d_rec_off[n+1]):
 * header, payload descriptor and the full Metadata walk with the exact
 * lani error semantics. Writes d_meta rows (list counts set, list offsets
 * not yet) and d_info. List positions and counts are kept in the context. */
int32_t honu_decode_parse(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                          uint64_t n, honu_meta *d_meta, honu_record_info *d_info, void *stream);

/* Phase 2: assign table offsets (exclusive scans over the counts), fill
 * the ACL and region tables, and when d_data != NULL assign every payload a
 * 16-byte aligned offset in d_data (d_info[i].data_off is then relative to
 * d_data) and copy the payloads there (honu_decode_payloads). d_totals
 * (device, 3 x u64) receives the totals the batch needs: ACL table entries
 * (lists returned in place take none), region table entries (likewise),
 * data-arena bytes (the latter also in zero-copy mode). Rows returned with
 * in-place lists (and every span) point into d_rec: keep the records arena
 * alive while the rows are used. Records whose
 * outputs do not fit get HONU_ERR_CAPACITY in meta_status / data_status. */
int32_t honu_decode_fill(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                         uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                         honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                         uint64_t regions_cap, uint8_t *d_data, uint64_t data_cap,
                         uint64_t *d_totals, void *stream);
/* honu_decode_fill without the payload copy, and the copy alone (after
 * honu_decode_tables with the same d_data and d_totals). */
int32_t honu_decode_tables(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n, honu_meta *d_meta,
                           honu_record_info *d_info, honu_acl *d_acl, uint64_t acl_cap,
                           uint32_t *d_regions, uint64_t regions_cap, uint8_t *d_data,
                           uint64_t data_cap, uint64_t *d_totals, void *stream);
int32_t honu_decode_payloads(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n,
                             const honu_record_info *d_info, uint8_t *d_data,
                             const uint64_t *d_totals, void *stream);

/* Parse + tables in ONE launch (the default batch decode): every output of
 * honu_decode_parse + honu_decode_tables — rows with their list offsets,
 * record info, ACL and region tables, d_totals — from a single pass over each
 * record's header and Metadata tail. With materialize != 0 every payload also
 * gets its 16-byte aligned data-arena offset (d_info[i].data_off, checked
 * against data_cap) and honu_decode_payloads (same context, same d_totals)
 * then copies the payloads; with materialize == 0 Data() stays the zero-copy
 * subslice of the records arena (Object.Data, object.go:85-99). Results are
 * identical to the split path's. Launches of 768 or more 64-record tiles
 * speculate (counts published before the walk ends, ACL entry flags checked
 * by the table fill or a gather after the publish) when the param
 * "speculate" allows it — by default materialising calls and the table forms,
 * not a zero-copy call with both lists in place; a batch holding any record that fails after its counts
 * were published, or a nil ACL entry past the list's first bytes (those the
 * walk has at hand are checked at once), is decoded a second time without
 * speculation inside the same call, so such a batch costs about twice a
 * clean one (malformed input and nil entries only; results are exact either
 * way). A recovery that ran sets a pinned word of the context, and the
 * context's next 16 calls after the host sees it do not speculate (no
 * recovery launch: about 1.1x a speculative clean call), so a stream of such
 * batches does not pay twice per batch. */
int32_t honu_decode_records(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                            uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                            honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                            uint64_t regions_cap, int32_t materialize, uint64_t data_cap,
                            uint64_t *d_totals, void *stream);

/* parse + fill in one call: from 48 K records honu_decode_records (+
 * honu_decode_payloads when d_data != NULL), below the split phases. */
int32_t honu_decode_batch(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                          uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                          honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                          uint64_t regions_cap, uint8_t *d_data, uint64_t data_cap,
                          uint64_t *d_totals, void *stream);

/* Object.StorageVersion() / Data() / Tombstone() (object.go:47-52,85-112)
 * without Metadata(): every honu_record_info field but meta_status, which is
 * HONU_UNPARSED. Reads only each record's header (version byte + the
 * dataLength varint): the Collection.Exists path (collection.go:55-65). */
int32_t honu_decode_headers(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                            uint64_t n, honu_record_info *d_info, void *stream);

/* Object.Data() (object.go:85-99) of every record materialised into a packed
 * data arena, without Metadata(): Data() needs only the header, so this runs
 * beside (on another stream and context) or without a Metadata() parse. d_info
 * is written as by honu_decode_headers, except that data_off is relative to
 * d_data: payloads are 16-byte aligned and back to back in record order, the
 * offsets honu_decode_fill assigns. A payload that does not fit data_cap gets
 * HONU_ERR_CAPACITY in data_status and is not copied. d_totals (optional,
 * device, 1 x u64) receives the data-arena bytes the batch needs. */
int32_t honu_decode_data(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                         uint64_t n, honu_record_info *d_info, uint8_t *d_data, uint64_t data_cap,
                         uint64_t *d_totals, void *stream);
/* honu_decode_data in two phases, to schedule or time the copy apart: place
 * (header walk, offsets, capacity; d_info complete after it) and the payload
 * copy (same ctx and d_info, after place on the same stream). */
int32_t honu_decode_data_place(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                               uint64_t n, honu_record_info *d_info, uint64_t data_cap,
                               uint64_t *d_totals, void *stream);
int32_t honu_decode_data_copy(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n,
                              const honu_record_info *d_info, uint8_t *d_data, void *stream);

/* Object.Key() (object.go:57-64 -> keys.New, keys/keys.go:42-51) for every
 * decoded record: 0x01 | ObjectID | BE64(VID) | BE32(PID), 29 bytes per
 * record at d_keys + 29*i. d_key_status[i] = meta_status, or HONU_ERR_PANIC
 * when the decoded Version is nil (metadata.go:54 dereferences it). */
int32_t honu_decode_keys(honu_ctx *ctx, const honu_meta *d_meta, const honu_record_info *d_info,
                         uint64_t n, uint8_t *d_keys, int32_t *d_key_status, void *stream);

/* ------------------------------------------------------------------------ */
/* System objects (object/system.go): metadata.Collection with its Indexes.  */
/* ------------------------------------------------------------------------ */

/* Presence bit 0 of honu_collection.present: the EncodeStruct flag that
 * MarshalSystem writes for the collection (system.go:22); bits 1-7 as for
 * honu_meta (Version, Parent, Schema, Publisher, Encryption, Compression,
 * non-nil WriteRegions). */
#define HONU_HAS_COLLECTION HONU_HAS_META

/* One metadata.Collection (collection.go:16-33) as a fixed 352-byte row.
 * Field meanings, spans, list descriptors and time encoding as honu_meta;
 * index_off/index_count describe Collection.Indexes in a honu_index table. */
typedef struct honu_collection {
    uint32_t present;            /*   0 HONU_HAS_* bits */
    uint8_t permissions;         /*   4 Collection.Permissions */
    uint8_t flags;               /*   5 Collection.Flags */
    uint8_t tombstone;           /*   6 Version.Tombstone */
    uint8_t compression_alg;     /*   7 */
    uint8_t sealing_alg;         /*   8 */
    uint8_t encryption_alg;      /*   9 */
    uint8_t signature_alg;       /*  10 */
    uint8_t _pad0;               /*  11 */
    uint32_t region;             /*  12 Version.Region */
    uint64_t vid;                /*  16 */
    uint32_t pid;                /*  24 */
    uint32_t parent_pid;         /*  28 */
    uint64_t parent_vid;         /*  32 */
    int64_t version_created;     /*  40 */
    uint32_t schema_major;       /*  48 */
    uint32_t schema_minor;       /*  52 */
    uint32_t schema_patch;       /*  56 */
    uint32_t _pad1;              /*  60 */
    int64_t compression_level;   /*  64 */
    int64_t created;             /*  72 Collection.Created */
    int64_t modified;            /*  80 Collection.Modified */
    uint64_t _pad2;              /*  88 */
    uint8_t id[16];              /*  96 Collection.ID */
    uint8_t owner[16];           /* 112 */
    uint8_t group[16];           /* 128 */
    uint8_t publisher_id[16];    /* 144 */
    uint8_t client_id[16];       /* 160 */
    uint8_t _pad3[16];           /* 176 */
    honu_span name;              /* 192 Collection.Name */
    honu_span schema_name;       /* 208 */
    honu_span ip_address;        /* 224 */
    honu_span user_agent;        /* 240 */
    honu_span public_key_id;     /* 256 */
    honu_span encryption_key;    /* 272 */
    honu_span hmac_secret;       /* 288 */
    honu_span signature;         /* 304 */
    uint64_t acl_off;            /* 320 */
    uint64_t acl_count;          /* 328 len(ACL); 0 <=> nil */
    uint64_t regions_off;        /* 336 */
    uint64_t regions_count;      /* 344 */
    uint64_t index_off;          /* 352 first entry in the index table */
    uint64_t index_count;        /* 360 len(Indexes); 0 <=> nil */
} honu_collection;               /* 368 */

/* One *metadata.Index (index.go:16-22) with its Field / Ref (field.go:12-16).
 * present == 0 is a nil pointer in the Indexes slice. */
typedef struct honu_index {
    uint8_t present;             /*   0 */
    uint8_t type;                /*   1 IndexType */
    uint8_t has_field;           /*   2 Field != nil */
    uint8_t field_type;          /*   3 Field.Type (FieldType) */
    uint8_t has_ref;             /*   4 Ref != nil */
    uint8_t ref_type;            /*   5 Ref.Type */
    uint8_t _pad[10];            /*   6 */
    uint8_t id[16];              /*  16 Index.ID */
    uint8_t field_collection[16];/*  32 Field.Collection */
    uint8_t ref_collection[16];  /*  48 Ref.Collection */
    honu_span name;              /*  64 Index.Name */
    honu_span field_name;        /*  80 Field.Name */
    honu_span ref_name;          /*  96 Ref.Name */
} honu_index;                    /* 112 */

/* ------------------------------------------------------------------------ */
/* System objects on the GPU                                                 */
/* ------------------------------------------------------------------------ */

/* object.MarshalSystem(collection) (system.go:10-31) for n collections:
 * 0x01 | EncodeStruct(collection) | 0x00. Exact encoded lengths in d_sizes,
 * statuses as honu_encode_sizes (HONU_ERR_INPUT for spans or lists outside
 * their arenas). A row without HONU_HAS_COLLECTION encodes MarshalSystem(nil)
 * = 01 00 00. */
int32_t honu_system_sizes(honu_ctx *ctx, const honu_collection *d_rows, uint64_t var_len,
                          const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                          uint64_t regions_len, const honu_index *d_index, uint64_t index_len,
                          uint64_t n, uint64_t *d_sizes, int32_t *d_status, void *stream);
/* Writes records at d_out + d_out_off[i] (offsets from honu_exclusive_scan of
 * the sizes); skips records whose status is not HONU_OK. */
int32_t honu_system_encode(honu_ctx *ctx, const honu_collection *d_rows, const uint8_t *d_var,
                           const honu_acl *d_acl, const uint32_t *d_regions,
                           const honu_index *d_index, uint64_t n, uint8_t *d_out,
                           uint64_t out_cap, const uint64_t *d_out_off, int32_t *d_status,
                           void *stream);
/* sizes + scan (d_out_off has n+1 entries) + encode. */
int32_t honu_system_marshal_batch(honu_ctx *ctx, const honu_collection *d_rows,
                                  const uint8_t *d_var, uint64_t var_len, const honu_acl *d_acl,
                                  uint64_t acl_len, const uint32_t *d_regions,
                                  uint64_t regions_len, const honu_index *d_index,
                                  uint64_t index_len, uint64_t n, uint8_t *d_out,
                                  uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status,
                                  void *stream);
/* object.UnmarshalSystem(obj, &metadata.Collection{}) (system.go:33-45) for
 * n records: decodes obj[1 : len-1] (the storage version byte is not checked,
 * the trailing nil-metadata byte is not read). Rows as honu_meta decode
 * (spans absolute in the records arena; fields of nil structs zero; a nil
 * collection leaves a zero row). ACL entries, regions and index rows go to
 * the tables (capacities in entries); d_status[i] is the UnmarshalSystem
 * error, HONU_ERR_PANIC for records shorter than 2 bytes (slice bounds) and
 * for counts Go's make() rejects. d_totals (3 u64, device): ACL entries,
 * regions, indexes. */
int32_t honu_system_decode_batch(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                                 uint64_t n, honu_collection *d_rows, int32_t *d_status,
                                 honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                                 uint64_t regions_cap, honu_index *d_index, uint64_t index_cap,
                                 uint64_t *d_totals, void *stream);
/* lani.Unmarshal(raw, &metadata.Collection{}) (lani/lani.go:29-33) for n
 * records: Collection.Decode (collection.go:240-356) from byte 0 of each raw
 * value to its end, as the store calls it on the bbolt value of a system
 * object (store.go:367, whose storage-version and struct-flag bytes are then
 * read as the first bytes of the ID). Rows, tables and statuses as
 * honu_system_decode_batch; a row that decodes has HONU_HAS_COLLECTION set
 * (the target is never nil). store.go:155 passes a nil *Collection, on which
 * Collection.Decode always panics (nil dereference, collection.go:242): no
 * batch call is needed to reproduce that. */
int32_t honu_collection_decode_batch(honu_ctx *ctx, const uint8_t *d_rec,
                                     const uint64_t *d_rec_off, uint64_t n,
                                     honu_collection *d_rows, int32_t *d_status, honu_acl *d_acl,
                                     uint64_t acl_cap, uint32_t *d_regions, uint64_t regions_cap,
                                     honu_index *d_index, uint64_t index_cap, uint64_t *d_totals,
                                     void *stream);

/* ------------------------------------------------------------------------ */
/* Read feed: the local-storage read path (iterator/cursor.go:31-38 copies    */
/* each bbolt value; Collection.Exists, collection.go:55-65, asks Tombstone). */
/* Records are appended into pinned host memory; each submitted batch is      */
/* copied to the device, decoded (zero copy) and keyed on its own stream      */
/* while the next batch fills: two slots, so the H2D copy, the kernels and    */
/* the D2H copies of one batch overlap the host filling the other.            */
/* ------------------------------------------------------------------------ */
typedef struct honu_feed honu_feed;

enum {
    HONU_FEED_HEADERS = 1u << 0  /* StorageVersion/Data/Tombstone only (honu_decode_headers) */
};

/* Host views of a decoded batch, valid until the next append/reserve into the
 * same slot (one more submit). Spans in meta rows and info.data_off are
 * absolute offsets into `records` (the batch's pinned arena), so Data() is the
 * subslice records[data_off : data_off + data_len], as in the reference. */
typedef struct honu_feed_result {
    uint64_t n;                       /* records in the batch */
    const uint8_t *records;           /* pinned arena holding the batch's records */
    const uint64_t *rec_off;          /* n + 1 offsets into records */
    const honu_meta *meta;            /* n rows (NULL with HONU_FEED_HEADERS) */
    const honu_record_info *info;     /* n */
    const honu_acl *acl;              /* acl_n entries (never more than the table holds) */
    uint64_t acl_n;
    const uint32_t *regions;          /* regions_n entries (likewise) */
    uint64_t regions_n;
    const uint8_t *keys;              /* 29 * n bytes, Object.Key() (NULL with HEADERS) */
    const int32_t *key_status;        /* n */
    uint64_t acl_needed;              /* entries the batch needed; > acl_n when the table
                                         overflowed (those records: HONU_ERR_CAPACITY) */
    uint64_t regions_needed;
} honu_feed_result;

/* A feed with two slots of batch_records records / batch_bytes bytes each.
 * The decoded ACL / region tables hold batch_bytes/8 + 1024 and
 * batch_bytes/4 + 1024 entries per batch; a batch that needs more reports
 * HONU_ERR_CAPACITY in the meta_status of the records that did not fit. */
honu_feed *honu_feed_create(int device, uint64_t batch_records, uint64_t batch_bytes,
                            uint32_t flags, int32_t *err);
void honu_feed_destroy(honu_feed *feed);
/* Copy one record into the current batch: HONU_ERR_CAPACITY when it does not
 * fit (submit, then append again), HONU_E_ARG when the slot still holds a
 * batch that was submitted but not waited for. */
int32_t honu_feed_append(honu_feed *feed, const uint8_t *rec, uint64_t len);
/* honu_feed_append for records 0..n-1 of a host CSR arena (record i =
 * arena[off[i], off[i+1]): a cursor page), stopping at the first record that
 * does not fit; *appended = records taken. */
int32_t honu_feed_append_batch(honu_feed *feed, const uint8_t *arena, const uint64_t *off,
                               uint64_t n, uint64_t *appended);
/* Reserve len bytes for the next record in pinned memory and return the
 * pointer (the caller writes the record there), or NULL with *err set. */
uint8_t *honu_feed_reserve(honu_feed *feed, uint64_t len, int32_t *err);
/* Records in the current (filling) batch. */
uint64_t honu_feed_pending(const honu_feed *feed);
/* Start decoding the current batch (asynchronous); *ticket identifies it.
 * The other slot becomes the filling one. */
int32_t honu_feed_submit(honu_feed *feed, uint64_t *ticket);
/* Wait for a submitted batch and describe its results. */
int32_t honu_feed_wait(honu_feed *feed, uint64_t ticket, honu_feed_result *out);

/* ------------------------------------------------------------------------ */
/* Write feed: the local-storage write path (a store Put marshals one record */
/* per call today: object.Marshal, object.go:24-45, from store.go:226,530).  */
/* Records (row + the bytes it references + payload) are appended into      */
/* pinned memory; each submitted batch is copied to the device, marshalled   */
/* and copied back on its own stream while the next batch fills (two slots). */
/* ------------------------------------------------------------------------ */
typedef struct honu_put_feed honu_put_feed;

/* Host views of a marshalled batch, valid until the slot is refilled (one
 * more submit). Record i is records[rec_off[i], rec_off[i+1]) when
 * status[i] == HONU_OK (Marshal's []byte); a failed record has an empty range
 * and its error (HONU_ERR_PANIC for Marshal(nil, ...)). */
typedef struct honu_put_result {
    uint64_t n;
    const uint8_t *records;
    const uint64_t *rec_off;  /* n + 1 */
    const int32_t *status;    /* n */
} honu_put_result;

/* A feed with two slots of batch_records records each; batch_bytes bounds a
 * batch's input bytes: the bytes its rows' spans reference + payloads + 20
 * per ACL entry + 4 per region. */
honu_put_feed *honu_put_feed_create(int device, uint64_t batch_records, uint64_t batch_bytes,
                                    int32_t *err);
void honu_put_feed_destroy(honu_put_feed *feed);
/* Append object.Marshal(meta, data) for one record. `row` is the record's
 * honu_meta: its spans index var[0, var_len), acl_off/acl_count index
 * acl[0, acl_len), regions_off/regions_count index regions[0, regions_len)
 * (a caller may pass whole batch tables or the record's own). Only the bytes
 * and entries the row references are copied (spans of absent sub-structs are
 * ignored). HONU_ERR_CAPACITY: the batch is full (submit, then append again);
 * HONU_ERR_INPUT: a span or list lies outside its array (nothing appended);
 * HONU_E_ARG: the filling slot still holds a batch that was not waited for.
 * data == NULL with data_len == 0 is a nil payload (a tombstone). */
int32_t honu_put_feed_append(honu_put_feed *feed, const honu_meta *row, const uint8_t *var,
                             uint64_t var_len, const honu_acl *acl, uint64_t acl_len,
                             const uint32_t *regions, uint64_t regions_len, const uint8_t *data,
                             uint64_t data_len);
/* honu_put_feed_append for records 0..n-1 of a host CSR batch (payload i =
 * payload[payload_off[i], payload_off[i+1])), stopping at the first record
 * that does not go in; *appended = records taken. */
int32_t honu_put_feed_append_batch(honu_put_feed *feed, const honu_meta *rows, uint64_t n,
                                   const uint8_t *var, uint64_t var_len, const honu_acl *acl,
                                   uint64_t acl_len, const uint32_t *regions, uint64_t regions_len,
                                   const uint8_t *payload, const uint64_t *payload_off,
                                   uint64_t *appended);
uint64_t honu_put_feed_pending(const honu_put_feed *feed);
int32_t honu_put_feed_submit(honu_put_feed *feed, uint64_t *ticket);
int32_t honu_put_feed_wait(honu_put_feed *feed, uint64_t ticket, honu_put_result *out);

/* ------------------------------------------------------------------------ */
/* Host memory helpers (pinned buffers for the host<->device path)          */
/* ------------------------------------------------------------------------ */
void *honu_host_alloc(uint64_t bytes);  /* hipHostMalloc, NULL on failure */
void honu_host_free(void *p);
void *honu_device_alloc(uint64_t bytes); /* hipMalloc on the current device */
void honu_device_free(void *p);
int32_t honu_memcpy_h2d(void *d_dst, const void *h_src, uint64_t bytes, void *stream);
int32_t honu_memcpy_d2h(void *h_dst, const void *d_src, uint64_t bytes, void *stream);
int32_t honu_stream_sync(void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HONU_CODEC_H */
