/*
 * honu_oracle.c — TEST INFRASTRUCTURE ONLY (see honu_oracle.h).
 *
 * A deliberately plain, serial restatement of the Go reference. Each function
 * names the reference lines it follows. Nothing here is tuned; the only goals
 * are exactness and readability.
 */
#include "honu_oracle.h"

#include <string.h>

#define MAX_VARINT_LEN64 10 /* binary.MaxVarintLen64 */
#define MAX_VARINT_LEN32 5  /* binary.MaxVarintLen32 */
#define GO_MAX_ALLOC (1ull << 48) /* runtime maxAlloc on linux/amd64 + arm64 */

/* ===================================================================== */
/* Go stdlib encoding/binary varint.go (Go 1.25.1)                        */
/* ===================================================================== */

/* binary.PutUvarint: minimal LEB128. */
int oracle_put_uvarint(uint8_t *buf, uint64_t x) {
    int i = 0;
    while (x >= 0x80) {
        buf[i] = (uint8_t)x | 0x80;
        x >>= 7;
        i++;
    }
    buf[i] = (uint8_t)x;
    return i + 1;
}

/* binary.Uvarint: returns k > 0 bytes read, 0 if buf too small, -(i+1) on
 * 64-bit overflow (10th byte > 1, or an 11th byte reached). */
int oracle_uvarint(const uint8_t *buf, uint64_t n, uint64_t *out) {
    uint64_t x = 0;
    unsigned s = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (i == MAX_VARINT_LEN64) {
            *out = 0;
            return -(int)(i + 1);
        }
        uint8_t b = buf[i];
        if (b < 0x80) {
            if (i == MAX_VARINT_LEN64 - 1 && b > 1) {
                *out = 0;
                return -(int)(i + 1);
            }
            *out = x | ((uint64_t)b << s);
            return (int)(i + 1);
        }
        x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    *out = 0;
    return 0;
}

/* binary.PutVarint: zig-zag then PutUvarint. */
int oracle_put_varint(uint8_t *buf, int64_t x) {
    uint64_t ux = (uint64_t)x << 1;
    if (x < 0) ux = ~ux;
    return oracle_put_uvarint(buf, ux);
}

/* binary.Varint: Uvarint then un-zig-zag (continues on error like Go). */
int oracle_varint(const uint8_t *buf, uint64_t n, int64_t *out) {
    uint64_t ux;
    int k = oracle_uvarint(buf, n, &ux);
    int64_t x = (int64_t)(ux >> 1);
    if (ux & 1) x = ~x;
    *out = x;
    return k;
}

/* ===================================================================== */
/* Size() upper bounds                                                    */
/* ===================================================================== */

int64_t oracle_size_bound(int which, const honu_meta *m) {
    /* Scalar.Size() = MaxVarintLen32 + MaxVarintLen64 (lamport/scalar.go:41,102-104) */
    const int64_t scalar = MAX_VARINT_LEN32 + MAX_VARINT_LEN64;
    /* Version.Size (version.go:29-42): 12 + Scalar + Parent? */
    int64_t version = 12 + scalar + ((m->present & HONU_HAS_PARENT) ? scalar : 0);
    /* SchemaVersion.Size (schema.go:22-28): 25 + len(Name) */
    int64_t schema = 25 + (int64_t)m->schema_name.len;
    int64_t acl = 17; /* AccessControl.Size (acls.go:17-21) */
    /* Publisher.Size (provenance.go:23-31): 52 + len(IP) + len(UA) */
    int64_t publisher = 52 + (int64_t)m->ip_address.len + (int64_t)m->user_agent.len;
    /* Encryption.Size (encryption.go:40-51): 43 + frames */
    int64_t encryption = 43 + (int64_t)(m->public_key_id.len + m->encryption_key.len +
                                        m->hmac_secret.len + m->signature.len);
    int64_t compression = 11; /* compression.go:19-29 */
    switch (which) {
    case 0: {
        /* Metadata.Size (metadata.go:60-106). ACL entries are all counted as
         * non-nil here (callers pass present ACLs); acl_count * (10 + 1 + 17). */
        int64_t s = 121;
        if (m->present & HONU_HAS_VERSION) s += version;
        if (m->present & HONU_HAS_SCHEMA) s += schema;
        s += (int64_t)m->mime.len;
        s += (int64_t)m->acl_count * MAX_VARINT_LEN64;
        s += (int64_t)m->acl_count * (1 + acl);
        s += (int64_t)m->regions_count * MAX_VARINT_LEN32;
        if (m->present & HONU_HAS_PUBLISHER) s += publisher;
        if (m->present & HONU_HAS_ENCRYPTION) s += encryption;
        if (m->present & HONU_HAS_COMPRESSION) s += compression;
        return s;
    }
    case 1: return version;
    case 2: return schema;
    case 3: return acl;
    case 4: return publisher;
    case 5: return encryption;
    case 6: return compression;
    default: return -1;
    }
}

/* ===================================================================== */
/* Encoder (lani/encode.go). A bounded writer: the bytes written are a    */
/* pure function of the values (Grow/capacity never changes them).        */
/* ===================================================================== */

typedef struct {
    uint8_t *buf;
    uint64_t cap;
    uint64_t len;
} owriter;

static void w_bytes(owriter *w, const uint8_t *p, uint64_t n) {
    if (w->buf && w->len + n <= w->cap && n) memcpy(w->buf + w->len, p, n);
    w->len += n;
}
static void w_byte(owriter *w, uint8_t c) { w_bytes(w, &c, 1); } /* EncodeByte :124-131 */
static void w_bool(owriter *w, int b) { w_byte(w, b ? 0x01 : 0x00); } /* EncodeBool :134-139 */
static void w_uvarint(owriter *w, uint64_t x) { /* EncodeUint32/Uint64 :149-170 */
    uint8_t tmp[MAX_VARINT_LEN64];
    int k = oracle_put_uvarint(tmp, x);
    w_bytes(w, tmp, (uint64_t)k);
}
static void w_varint(owriter *w, int64_t x) { /* EncodeInt64 :172-181 */
    uint8_t tmp[MAX_VARINT_LEN64];
    int k = oracle_put_varint(tmp, x);
    w_bytes(w, tmp, (uint64_t)k);
}
static void w_frame(owriter *w, const uint8_t *p, uint64_t n) { /* Encode :62-77 */
    w_uvarint(w, n);
    w_bytes(w, p, n);
}
static void w_time(owriter *w, int64_t ns) { /* EncodeTime :201-206; 0 <=> IsZero */
    w_varint(w, ns);
}

/* span -> pointer inside var arena, or NULL when out of range */
static const uint8_t *span_ptr(const uint8_t *var, uint64_t var_len, honu_span s, int *bad) {
    if (s.len == 0) return var; /* any pointer; no bytes read */
    if (s.off > var_len || s.len > var_len - s.off) {
        *bad = 1;
        return var;
    }
    return var + s.off;
}

/* Metadata.Encode (metadata.go:108-200) preceded by its EncodeStruct flag. */
static int encode_meta(owriter *w, const honu_meta *m, const uint8_t *var, uint64_t var_len,
                       const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                       uint64_t regions_len) {
    int bad = 0;
    const uint8_t *name = span_ptr(var, var_len, m->schema_name, &bad);
    const uint8_t *mime = span_ptr(var, var_len, m->mime, &bad);
    const uint8_t *ip = span_ptr(var, var_len, m->ip_address, &bad);
    const uint8_t *ua = span_ptr(var, var_len, m->user_agent, &bad);
    const uint8_t *pk = span_ptr(var, var_len, m->public_key_id, &bad);
    const uint8_t *ek = span_ptr(var, var_len, m->encryption_key, &bad);
    const uint8_t *hs = span_ptr(var, var_len, m->hmac_secret, &bad);
    const uint8_t *sg = span_ptr(var, var_len, m->signature, &bad);
    if (m->acl_count && (m->acl_off > acl_len || m->acl_count > acl_len - m->acl_off)) bad = 1;
    if (m->regions_count &&
        (m->regions_off > regions_len || m->regions_count > regions_len - m->regions_off))
        bad = 1;
    /* a decode output row: encode takes the table forms */
    if (m->present & (HONU_ACL_INPLACE | HONU_REGIONS_INPLACE)) bad = 1;
    /* a carried list length (HONU_ACL_SIZED) must lie in [count, 18 count]
     * (include/honu_codec.h; the exact check: oracle_marshal_batch) */
    if ((m->present & HONU_ACL_SIZED) &&
        (m->acl_bytes < m->acl_count || m->acl_bytes > 18 * m->acl_count))
        bad = 1;
    if (bad) return HONU_ERR_INPUT;

    w_bool(w, 1);                         /* EncodeStruct(meta) flag, encode.go:210-216 */
    w_bytes(w, m->object_id, 16);         /* :110 EncodeULID */
    w_bytes(w, m->collection_id, 16);     /* :115 */
    if (m->present & HONU_HAS_VERSION) {  /* :120 EncodeStruct(Version) */
        w_bool(w, 1);
        w_uvarint(w, m->pid);             /* Scalar.Encode scalar.go:106-119 */
        w_uvarint(w, m->vid);
        w_uvarint(w, m->region);          /* version.go:51 EncodeUint32(Region) */
        if (m->present & HONU_HAS_PARENT) { /* :56 EncodeStruct(Parent) */
            w_bool(w, 1);
            w_uvarint(w, m->parent_pid);
            w_uvarint(w, m->parent_vid);
        } else {
            w_bool(w, 0);
        }
        w_bool(w, m->tombstone != 0);     /* :61 EncodeBool */
        w_time(w, m->version_created);    /* :66 EncodeTime */
    } else {
        w_bool(w, 0);
    }
    if (m->present & HONU_HAS_SCHEMA) {   /* :125; schema.go:30-53 */
        w_bool(w, 1);
        w_frame(w, name, m->schema_name.len);
        w_uvarint(w, m->schema_major);
        w_uvarint(w, m->schema_minor);
        w_uvarint(w, m->schema_patch);
    } else {
        w_bool(w, 0);
    }
    w_frame(w, mime, m->mime.len);        /* :130 EncodeString(MIME) */
    w_bytes(w, m->owner, 16);             /* :135 */
    w_bytes(w, m->group, 16);             /* :140 */
    w_byte(w, m->permissions);            /* :145 */
    w_uvarint(w, m->acl_count);           /* :151 EncodeUint64(len ACL) */
    for (uint64_t i = 0; i < m->acl_count; i++) { /* :157-162, acls.go:26-39 */
        const honu_acl *a = &acl[m->acl_off + i];
        if (a->present) {
            w_bool(w, 1);
            w_bytes(w, a->client_id, 16);
            w_byte(w, a->permissions);
        } else {
            w_bool(w, 0);
        }
    }
    w_uvarint(w, m->regions_count);       /* :164 Regions.Encode region.go:137-152 */
    for (uint64_t i = 0; i < m->regions_count; i++) w_uvarint(w, regions[m->regions_off + i]);
    if (m->present & HONU_HAS_PUBLISHER) { /* :169; provenance.go:34-57 */
        w_bool(w, 1);
        w_bytes(w, m->publisher_id, 16);
        w_bytes(w, m->client_id, 16);
        w_frame(w, ip, m->ip_address.len);
        w_frame(w, ua, m->user_agent.len);
    } else {
        w_bool(w, 0);
    }
    if (m->present & HONU_HAS_ENCRYPTION) { /* :174; encryption.go:51-89 */
        w_bool(w, 1);
        w_frame(w, pk, m->public_key_id.len);
        w_frame(w, ek, m->encryption_key.len);
        w_frame(w, hs, m->hmac_secret.len);
        w_frame(w, sg, m->signature.len);
        w_byte(w, m->sealing_alg);
        w_byte(w, m->encryption_alg);
        w_byte(w, m->signature_alg);
    } else {
        w_bool(w, 0);
    }
    if (m->present & HONU_HAS_COMPRESSION) { /* :179; compression.go:40-53 */
        w_bool(w, 1);
        w_byte(w, m->compression_alg);
        w_varint(w, m->compression_level);
    } else {
        w_bool(w, 0);
    }
    w_byte(w, m->flags);                  /* :184 */
    w_time(w, m->created);                /* :189 */
    w_time(w, m->modified);               /* :194 */
    return HONU_OK;
}

int oracle_marshal(const honu_meta *m, const uint8_t *var, uint64_t var_len, const honu_acl *acl,
                   uint64_t acl_len, const uint32_t *regions, uint64_t regions_len,
                   const uint8_t *data, uint64_t data_len, uint8_t *out, uint64_t cap,
                   uint64_t *out_len) {
    *out_len = 0;
    /* Marshal(nil, ...) panics in meta.Size() (metadata.go:66). */
    if (!(m->present & HONU_HAS_META)) return HONU_ERR_PANIC;
    owriter w = {out, cap, 0};
    w_byte(&w, HONU_STORAGE_VERSION);     /* object.go:30 EncodeUint8(StorageVersion) */
    w_frame(&w, data, data_len);          /* object.go:35 Encode(data) */
    int st = encode_meta(&w, m, var, var_len, acl, acl_len, regions, regions_len); /* :40 */
    if (st != HONU_OK) return st;
    *out_len = w.len;
    if (out && w.len > cap) return HONU_ERR_CAPACITY;
    return HONU_OK;
}

/* ===================================================================== */
/* Decoder (lani/decode.go)                                               */
/* ===================================================================== */

typedef struct {
    const uint8_t *buf;
    uint64_t len;
    uint64_t i;
} oreader;

/* DecodeByte :94-103 */
static int r_byte(oreader *r, uint8_t *c) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    *c = r->buf[r->i++];
    return HONU_OK;
}
/* DecodeBool :105-120 */
static int r_bool(oreader *r, int *b) {
    uint8_t c;
    int st = r_byte(r, &c);
    if (st) return st;
    if (c == 0) *b = 0;
    else if (c == 1) *b = 1;
    else return HONU_ERR_PARSE_BOOLEAN;
    return HONU_OK;
}
/* DecodeUint32 :127-146 (5-byte window, truncating) */
static int r_u32(oreader *r, uint32_t *v) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    uint64_t j = r->i + MAX_VARINT_LEN32;
    if (j > r->len) j = r->len;
    uint64_t x;
    int k = oracle_uvarint(r->buf + r->i, j - r->i, &x);
    if (k <= 0) return HONU_ERR_PARSE_VARINT;
    r->i += (uint64_t)k;
    *v = (uint32_t)x;
    return HONU_OK;
}
/* DecodeUint64 :149-168 */
static int r_u64(oreader *r, uint64_t *v) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    uint64_t j = r->i + MAX_VARINT_LEN64;
    if (j > r->len) j = r->len;
    int k = oracle_uvarint(r->buf + r->i, j - r->i, v);
    if (k <= 0) return HONU_ERR_PARSE_VARINT;
    r->i += (uint64_t)k;
    return HONU_OK;
}
/* DecodeInt64 :171-190 */
static int r_i64(oreader *r, int64_t *v) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    uint64_t j = r->i + MAX_VARINT_LEN64;
    if (j > r->len) j = r->len;
    int k = oracle_varint(r->buf + r->i, j - r->i, v);
    if (k <= 0) return HONU_ERR_PARSE_VARINT;
    r->i += (uint64_t)k;
    return HONU_OK;
}
/* DecodeULID :209-221 */
static int r_ulid(oreader *r, uint8_t out[16]) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    if (r->i + 16 > r->len) return HONU_ERR_UNEXPECTED_EOF;
    memcpy(out, r->buf + r->i, 16);
    r->i += 16;
    return HONU_OK;
}
/* Decode :30-56 via readLength :261-282. The frame becomes a span (absolute
 * offset = base + position); length 0 is nil (span {0,0}). */
static int r_frame(oreader *r, uint64_t base, honu_span *s) {
    if (r->i >= r->len) return HONU_ERR_EOF;
    uint64_t j = r->i + MAX_VARINT_LEN64;
    if (j > r->len) j = r->len;
    uint64_t rl;
    int k = oracle_uvarint(r->buf + r->i, j - r->i, &rl);
    if (k <= 0) return HONU_ERR_NO_LENGTH;
    r->i += (uint64_t)k;
    /* int(rl) is negative for rl >= 2^63: make([]byte, rl) panics (:50). */
    if (rl >= (1ull << 63)) return HONU_ERR_PANIC;
    if (rl == 0) {
        s->off = 0;
        s->len = 0;
        return HONU_OK;
    }
    /* j := d.i + rl overflows int for rl > MaxInt64 - d.i, so the bounds check
     * passes and make([]byte, rl) panics. */
    if (rl > (uint64_t)INT64_MAX - r->i) return HONU_ERR_PANIC;
    if (r->i + rl > r->len) return HONU_ERR_UNEXPECTED_EOF;
    s->off = base + r->i;
    s->len = rl;
    r->i += rl;
    return HONU_OK;
}

typedef struct {
    honu_acl *acl_out;
    uint64_t acl_cap, acl_n;
    uint32_t *reg_out;
    uint64_t reg_cap, reg_n;
} olists;

#define TRY(x) do { int st_ = (x); if (st_) return st_; } while (0)

/* Metadata.Decode (metadata.go:202-302) after its nil flag. forms &
 * ORACLE_ACL_INPLACE: a list whose entries are all present is returned in
 * place (HONU_ACL_INPLACE, acl_off = absolute offset of its first entry)
 * instead of in the table; forms & ORACLE_REGIONS_INPLACE: a non-empty region
 * list is returned in place (HONU_REGIONS_INPLACE, regions_off = absolute
 * offset of its first uvarint; every uvarint decoded and checked as below). */
static int decode_meta_body(oreader *r, uint64_t base, honu_meta *m, olists *L, int forms) {
    const int acl_inplace = forms & ORACLE_ACL_INPLACE, reg_inplace = forms & ORACLE_REGIONS_INPLACE;
    int b;
    TRY(r_ulid(r, m->object_id));                    /* :210 */
    TRY(r_ulid(r, m->collection_id));                /* :214 */
    TRY(r_bool(r, &b));                              /* :219 DecodeStruct(Version) */
    if (b) {                                         /* version.go:74-103 */
        m->present |= HONU_HAS_VERSION;
        TRY(r_u32(r, &m->pid));                      /* Scalar.Decode scalar.go:121-131 */
        TRY(r_u64(r, &m->vid));
        TRY(r_u32(r, &m->region));                   /* :80 */
        TRY(r_bool(r, &b));                          /* :88 DecodeStruct(Parent) */
        if (b) {
            m->present |= HONU_HAS_PARENT;
            TRY(r_u32(r, &m->parent_pid));
            TRY(r_u64(r, &m->parent_vid));
        }
        TRY(r_bool(r, &b));                          /* :96 Tombstone */
        m->tombstone = (uint8_t)b;
        TRY(r_i64(r, &m->version_created));          /* :100 DecodeTime */
    }
    TRY(r_bool(r, &b));                              /* :225 DecodeStruct(Schema) */
    if (b) {                                         /* schema.go:55-73 */
        m->present |= HONU_HAS_SCHEMA;
        TRY(r_frame(r, base, &m->schema_name));
        TRY(r_u32(r, &m->schema_major));
        TRY(r_u32(r, &m->schema_minor));
        TRY(r_u32(r, &m->schema_patch));
    }
    TRY(r_frame(r, base, &m->mime));                 /* :231 */
    TRY(r_ulid(r, m->owner));                        /* :235 */
    TRY(r_ulid(r, m->group));                        /* :239 */
    TRY(r_byte(r, &m->permissions));                 /* :243 */
    uint64_t nacl;
    TRY(r_u64(r, &nacl));                            /* :249 */
    if (nacl > 0) {                                  /* :254-265 */
        /* make([]*AccessControl, nACLs): 8-byte elements > maxAlloc panics */
        if (nacl > GO_MAX_ALLOC / 8) return HONU_ERR_PANIC;
        /* Every entry present (flag 1, then 16 + 1 bytes) with the list inside
         * the record: exactly the lists Go decodes without a nil entry and
         * without an error, 18 bytes per entry. */
        int all = acl_inplace && nacl <= (r->len - r->i) / 18;
        for (uint64_t i = 0; all && i < nacl; i++)
            if (r->buf[r->i + 18 * i] != 1) all = 0;
        if (all) {
            m->present |= HONU_ACL_INPLACE;
            m->acl_off = base + r->i;
            r->i += 18 * nacl;
        } else {
            m->acl_off = L->acl_n;
            for (uint64_t i = 0; i < nacl; i++) {
                honu_acl a;
                memset(&a, 0, sizeof a);
                TRY(r_bool(r, &b));                  /* DecodeStruct(o.ACL[i]) */
                if (b) {
                    a.present = 1;
                    TRY(r_ulid(r, a.client_id));     /* acls.go:41-51 */
                    TRY(r_byte(r, &a.permissions));
                }
                if (L->acl_n < L->acl_cap) L->acl_out[L->acl_n] = a;
                L->acl_n++;
            }
        }
        m->acl_count = nacl;
    }
    uint64_t nreg;
    TRY(r_u64(r, &nreg));                            /* Regions.Decode region.go:154-169 */
    if (nreg > GO_MAX_ALLOC / 4) return HONU_ERR_PANIC; /* make(Regions, length) */
    m->present |= HONU_REGIONS_NONNIL;
    m->regions_off = L->reg_n;
    const uint64_t reg_at = base + r->i;
    for (uint64_t i = 0; i < nreg; i++) {
        uint32_t v;
        TRY(r_u32(r, &v));
        if (reg_inplace) continue;  /* validated; the list stays where it is */
        if (L->reg_n < L->reg_cap) L->reg_out[L->reg_n] = v;
        L->reg_n++;
    }
    m->regions_count = nreg;
    if (nreg == 0) m->regions_off = 0;
    else if (reg_inplace) {
        m->present |= HONU_REGIONS_INPLACE;
        m->regions_off = reg_at;
    }
    TRY(r_bool(r, &b));                              /* :271 DecodeStruct(Publisher) */
    if (b) {                                         /* provenance.go:59-79 */
        m->present |= HONU_HAS_PUBLISHER;
        TRY(r_ulid(r, m->publisher_id));
        TRY(r_ulid(r, m->client_id));
        TRY(r_frame(r, base, &m->ip_address));
        TRY(r_frame(r, base, &m->user_agent));
    }
    TRY(r_bool(r, &b));                              /* :277 DecodeStruct(Encryption) */
    if (b) {                                         /* encryption.go:91-125 */
        m->present |= HONU_HAS_ENCRYPTION;
        TRY(r_frame(r, base, &m->public_key_id));
        TRY(r_frame(r, base, &m->encryption_key));
        TRY(r_frame(r, base, &m->hmac_secret));
        TRY(r_frame(r, base, &m->signature));
        TRY(r_byte(r, &m->sealing_alg));
        TRY(r_byte(r, &m->encryption_alg));
        TRY(r_byte(r, &m->signature_alg));
    }
    TRY(r_bool(r, &b));                              /* :283 DecodeStruct(Compression) */
    if (b) {                                         /* compression.go:55-67 */
        m->present |= HONU_HAS_COMPRESSION;
        TRY(r_byte(r, &m->compression_alg));
        TRY(r_i64(r, &m->compression_level));
    }
    TRY(r_byte(r, &m->flags));                       /* :289 */
    TRY(r_i64(r, &m->created));                      /* :293 */
    TRY(r_i64(r, &m->modified));                     /* :297 */
    return HONU_OK;
}

/* Object.dataLength (object.go:114-134): (-1,-1) on empty or invalid. The
 * window o[1:min(11, len-1)] never includes the record's last byte. */
static void data_length(const uint8_t *o, uint64_t len, int64_t *d, int64_t *b) {
    *d = -1;
    *b = -1;
    if (len == 0) return;
    int64_t j = 1 + MAX_VARINT_LEN64;
    if (j > (int64_t)len - 1) j = (int64_t)len - 1;
    if (j < 1) return;
    uint64_t rl;
    int k = oracle_uvarint(o + 1, (uint64_t)(j - 1), &rl);
    if (k <= 0) return;
    *d = (int64_t)rl; /* int(rl): negative for rl >= 2^63 */
    *b = k;
}

void oracle_decode(const uint8_t *o, uint64_t len, uint64_t base, honu_meta *m,
                   honu_record_info *info, honu_acl *acl_out, uint64_t acl_cap,
                   uint32_t *regions_out, uint64_t regions_cap, uint64_t *acl_n,
                   uint64_t *regions_n, int forms) {
    memset(m, 0, sizeof *m);
    memset(info, 0, sizeof *info);
    *acl_n = 0;
    *regions_n = 0;
    uint8_t ver = len ? o[0] : 0;                    /* StorageVersion :47-52 */
    info->storage_version = ver;
    int64_t d, b;
    data_length(o, len, &d, &b);
    info->tombstone = (ver == HONU_STORAGE_VERSION && d == 0); /* Tombstone :103-112 */

    /* Data() :85-99 */
    if (ver != HONU_STORAGE_VERSION) info->data_status = HONU_ERR_BAD_VERSION;
    else if (d < 0) info->data_status = HONU_ERR_MALFORMED;
    else if (d == 0) info->data_status = HONU_OK;    /* nil, nil */
    else if ((uint64_t)d > len - 1 - (uint64_t)b) info->data_status = HONU_ERR_PANIC; /* o[1+b:1+b+d] */
    else {
        info->data_status = HONU_OK;
        info->data_off = base + 1 + (uint64_t)b;
        info->data_len = (uint64_t)d;
    }

    /* Metadata() :66-83 */
    if (ver != HONU_STORAGE_VERSION) { info->meta_status = HONU_ERR_BAD_VERSION; return; }
    if (d < 0) { info->meta_status = HONU_ERR_MALFORMED; return; }
    if ((uint64_t)d > len - 1 - (uint64_t)b) { info->meta_status = HONU_ERR_PANIC; return; } /* o[1+d+b:] */
    uint64_t t = 1 + (uint64_t)d + (uint64_t)b;
    oreader r = {o + t, len - t, 0};
    olists L = {acl_out, acl_cap, 0, regions_out, regions_cap, 0};
    int present;
    int st = r_bool(&r, &present);                   /* DecodeStruct(meta) :78 */
    if (st == HONU_OK && present) {
        m->present = HONU_HAS_META;
        st = decode_meta_body(&r, base + t, m, &L, forms);
    }
    info->meta_status = st;
    if (st != HONU_OK) {
        memset(m, 0, sizeof *m);                     /* Go returns nil, err */
        return;
    }
    *acl_n = L.acl_n;
    *regions_n = L.reg_n;
}

/* ===================================================================== */
/* Batch drivers                                                          */
/* ===================================================================== */

/* The ACL list's encoded length from the table: 18 per present entry, 1 per
 * nil one (acls.go:26-39, encode.go:210-226). */
static uint64_t acl_list_bytes(const honu_meta *m, const honu_acl *acl) {
    uint64_t b = 0;
    for (uint64_t j = 0; j < m->acl_count; j++) b += acl[m->acl_off + j].present ? 18 : 1;
    return b;
}

int oracle_marshal_batch(const honu_meta *meta, const uint8_t *var, uint64_t var_len,
                         const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                         uint64_t regions_len, const uint8_t *payload,
                         const uint64_t *payload_off, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, int32_t *status) {
    uint64_t pos = 0;
    int any_cap = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *data = payload + payload_off[i];
        uint64_t dlen = payload_off[i + 1] - payload_off[i];
        uint64_t sz = 0;
        /* size pass: a record that cannot be encoded (PANIC, INPUT) has size 0 */
        int st = oracle_marshal(&meta[i], var, var_len, acl, acl_len, regions, regions_len, data,
                                dlen, NULL, 0, &sz);
        /* a row carrying its ACL list's length (HONU_ACL_SIZED) is sized by
         * that length without reading the table (honu_encode_sizes); one whose
         * length is not the list's gets HONU_ERR_INPUT from the encode and its
         * range stays unwritten here (unspecified bytes on the GPU) */
        if (st == HONU_OK && (meta[i].present & HONU_ACL_SIZED)) {
            const uint64_t actual = acl_list_bytes(&meta[i], acl);
            if (actual != meta[i].acl_bytes) {
                sz = sz - actual + meta[i].acl_bytes;
                st = -HONU_ERR_INPUT; /* (marks the record for the encode pass) */
            }
        }
        out_off[i] = pos;
        pos += sz;
        if (status) status[i] = st;
    }
    out_off[n] = pos;
    for (uint64_t i = 0; i < n; i++) {
        if (status && status[i] == -HONU_ERR_INPUT) {
            status[i] = out_off[i + 1] > out_cap ? HONU_ERR_CAPACITY : HONU_ERR_INPUT;
            continue;
        }
        if (status && status[i] != HONU_OK) continue;
        uint64_t beg = out_off[i], end = out_off[i + 1];
        if (end > out_cap) {
            if (status) status[i] = HONU_ERR_CAPACITY;
            any_cap = 1;
            continue;
        }
        uint64_t sz;
        int st = oracle_marshal(&meta[i], var, var_len, acl, acl_len, regions, regions_len,
                                payload + payload_off[i], payload_off[i + 1] - payload_off[i],
                                out + beg, end - beg, &sz);
        if (status) status[i] = st;
    }
    return any_cap ? HONU_ERR_CAPACITY : HONU_OK;
}

int oracle_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n, honu_meta *meta,
                        honu_record_info *info, honu_acl *acl, uint64_t acl_cap,
                        uint32_t *regions, uint64_t regions_cap, uint8_t *data, uint64_t data_cap,
                        uint64_t totals[3], int forms) {
    uint64_t acl_pos = 0, reg_pos = 0, data_pos = 0;
    int any_cap = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t an, rn;
        uint64_t beg = rec_off[i], len = rec_off[i + 1] - rec_off[i];
        honu_acl *ao = acl ? acl + (acl_pos < acl_cap ? acl_pos : acl_cap) : NULL;
        uint32_t *ro = regions ? regions + (reg_pos < regions_cap ? reg_pos : regions_cap) : NULL;
        uint64_t acap = acl && acl_pos < acl_cap ? acl_cap - acl_pos : 0;
        uint64_t rcap = regions && reg_pos < regions_cap ? regions_cap - reg_pos : 0;
        oracle_decode(rec + beg, len, beg, &meta[i], &info[i], ao, acap, ro, rcap, &an, &rn,
                      forms);
        if (info[i].meta_status == HONU_OK) {
            if (an) meta[i].acl_off = acl_pos;
            if (rn) meta[i].regions_off = reg_pos;  /* (a list in place keeps its own) */
            if (acl_pos + an > acl_cap || reg_pos + rn > regions_cap) {
                info[i].meta_status = HONU_ERR_CAPACITY;
                any_cap = 1;
            }
            acl_pos += an;
            reg_pos += rn;
        }
        if (info[i].data_status == HONU_OK && info[i].data_len) {
            uint64_t dl = info[i].data_len;
            uint64_t src = info[i].data_off;
            if (!data) { /* zero copy: only count the arena bytes a copy would need */
                data_pos += (dl + 15) & ~15ull;
                continue;
            }
            info[i].data_off = data_pos;
            if (data_pos + dl > data_cap) {
                info[i].data_status = HONU_ERR_CAPACITY;
                info[i].data_off = 0;
                info[i].data_len = 0;
                any_cap = 1;
            } else {
                memcpy(data + data_pos, rec + src, dl);
            }
            data_pos += (dl + 15) & ~15ull;
        }
    }
    if (totals) {
        totals[0] = acl_pos;
        totals[1] = reg_pos;
        totals[2] = data_pos;
    }
    return any_cap ? HONU_ERR_CAPACITY : HONU_OK;
}

int oracle_key(const honu_meta *m, int32_t meta_status, uint8_t key[29]) {
    memset(key, 0, 29);
    if (meta_status != HONU_OK) return meta_status;
    if (!(m->present & HONU_HAS_VERSION)) return HONU_ERR_PANIC; /* &o.Version.Scalar, nil */
    key[0] = 0x01;                                   /* keys.go:44 keyVersion */
    memcpy(key + 1, m->object_id, 16);
    for (int i = 0; i < 8; i++) key[17 + i] = (uint8_t)(m->vid >> (56 - 8 * i)); /* BigEndian */
    for (int i = 0; i < 4; i++) key[25 + i] = (uint8_t)(m->pid >> (24 - 8 * i));
    return HONU_OK;
}

/* ===================================================================== */
/* System objects: object/system.go with metadata.Collection              */
/* (collection.go), Index (index.go) and Field (field.go).                */
/* ===================================================================== */

/* Size() upper bounds: Field.Size field.go:38-40 (27 + len Name),
 * Index.Size index.go:47-56 (29 + len Name + Field + Ref),
 * Collection.Size collection.go:81-135 (115 + ...). */
int64_t oracle_field_size(uint64_t name_len) { return 27 + (int64_t)name_len; }

int64_t oracle_index_size(const honu_index *x) {
    int64_t s = 29 + (int64_t)x->name.len;
    if (x->has_field) s += oracle_field_size(x->field_name.len);
    if (x->has_ref) s += oracle_field_size(x->ref_name.len);
    return s;
}

int64_t oracle_collection_size(const honu_collection *c, const honu_acl *acl,
                               const honu_index *idx) {
    const int64_t scalar = MAX_VARINT_LEN32 + MAX_VARINT_LEN64;
    int64_t s = 115 + (int64_t)c->name.len;
    if (c->present & HONU_HAS_VERSION)
        s += 12 + scalar + ((c->present & HONU_HAS_PARENT) ? scalar : 0);
    s += (int64_t)c->acl_count * MAX_VARINT_LEN64;
    for (uint64_t i = 0; i < c->acl_count; i++) s += 1 + (acl[c->acl_off + i].present ? 17 : 0);
    s += (int64_t)c->regions_count * MAX_VARINT_LEN64;
    s += (int64_t)c->regions_count * MAX_VARINT_LEN32;
    if (c->present & HONU_HAS_PUBLISHER)
        s += 52 + (int64_t)c->ip_address.len + (int64_t)c->user_agent.len;
    if (c->present & HONU_HAS_SCHEMA) s += 25 + (int64_t)c->schema_name.len;
    if (c->present & HONU_HAS_ENCRYPTION)
        s += 43 + (int64_t)(c->public_key_id.len + c->encryption_key.len + c->hmac_secret.len +
                            c->signature.len);
    if (c->present & HONU_HAS_COMPRESSION) s += 11;
    s += (int64_t)c->index_count * MAX_VARINT_LEN64;
    for (uint64_t i = 0; i < c->index_count; i++) {
        const honu_index *x = &idx[c->index_off + i];
        s += 1 + (x->present ? oracle_index_size(x) : 0);
    }
    return s;
}

/* Field.Encode field.go:42-60 after its EncodeStruct flag */
static void encode_field(owriter *w, const uint8_t *name, uint64_t name_len, uint8_t type,
                         const uint8_t col[16]) {
    w_frame(w, name, name_len);                      /* EncodeString(Name) */
    w_byte(w, type);                                 /* EncodeUint8(Type) */
    w_bytes(w, col, 16);                             /* EncodeULID(Collection) */
}

/* Collection.Encode (collection.go:137-237) preceded by its EncodeStruct flag */
static int encode_collection(owriter *w, const honu_collection *c, const uint8_t *var,
                             uint64_t var_len, const honu_acl *acl, uint64_t acl_len,
                             const uint32_t *regions, uint64_t regions_len, const honu_index *idx,
                             uint64_t idx_len) {
    int bad = 0;
    const uint8_t *name = span_ptr(var, var_len, c->name, &bad);
    const uint8_t *sname = span_ptr(var, var_len, c->schema_name, &bad);
    const uint8_t *ip = span_ptr(var, var_len, c->ip_address, &bad);
    const uint8_t *ua = span_ptr(var, var_len, c->user_agent, &bad);
    const uint8_t *pk = span_ptr(var, var_len, c->public_key_id, &bad);
    const uint8_t *ek = span_ptr(var, var_len, c->encryption_key, &bad);
    const uint8_t *hs = span_ptr(var, var_len, c->hmac_secret, &bad);
    const uint8_t *sg = span_ptr(var, var_len, c->signature, &bad);
    if (c->acl_count && (c->acl_off > acl_len || c->acl_count > acl_len - c->acl_off)) bad = 1;
    if (c->regions_count &&
        (c->regions_off > regions_len || c->regions_count > regions_len - c->regions_off))
        bad = 1;
    if (c->index_count && (c->index_off > idx_len || c->index_count > idx_len - c->index_off))
        bad = 1;
    for (uint64_t i = 0; !bad && i < c->index_count; i++) {
        const honu_index *x = &idx[c->index_off + i];
        if (!x->present) continue;
        span_ptr(var, var_len, x->name, &bad);
        if (x->has_field) span_ptr(var, var_len, x->field_name, &bad);
        if (x->has_ref) span_ptr(var, var_len, x->ref_name, &bad);
    }
    if (bad) return HONU_ERR_INPUT;

    w_bool(w, 1);                                    /* EncodeStruct(obj) system.go:22 */
    w_bytes(w, c->id, 16);                           /* :139 EncodeULID(ID) */
    w_frame(w, name, c->name.len);                   /* :144 EncodeString(Name) */
    if (c->present & HONU_HAS_VERSION) {             /* :149 EncodeStruct(Version) */
        w_bool(w, 1);
        w_uvarint(w, c->pid);
        w_uvarint(w, c->vid);
        w_uvarint(w, c->region);
        if (c->present & HONU_HAS_PARENT) {
            w_bool(w, 1);
            w_uvarint(w, c->parent_pid);
            w_uvarint(w, c->parent_vid);
        } else {
            w_bool(w, 0);
        }
        w_bool(w, c->tombstone != 0);
        w_time(w, c->version_created);
    } else {
        w_bool(w, 0);
    }
    w_bytes(w, c->owner, 16);                        /* :154 */
    w_bytes(w, c->group, 16);                        /* :159 */
    w_byte(w, c->permissions);                       /* :164 */
    w_uvarint(w, c->acl_count);                      /* :170 EncodeUint64(len ACL) */
    for (uint64_t i = 0; i < c->acl_count; i++) {    /* :176-181 */
        const honu_acl *a = &acl[c->acl_off + i];
        if (a->present) {
            w_bool(w, 1);
            w_bytes(w, a->client_id, 16);
            w_byte(w, a->permissions);
        } else {
            w_bool(w, 0);
        }
    }
    w_uvarint(w, c->regions_count);                  /* :183 WriteRegions.Encode */
    for (uint64_t i = 0; i < c->regions_count; i++) w_uvarint(w, regions[c->regions_off + i]);
    if (c->present & HONU_HAS_PUBLISHER) {           /* :188 */
        w_bool(w, 1);
        w_bytes(w, c->publisher_id, 16);
        w_bytes(w, c->client_id, 16);
        w_frame(w, ip, c->ip_address.len);
        w_frame(w, ua, c->user_agent.len);
    } else {
        w_bool(w, 0);
    }
    if (c->present & HONU_HAS_SCHEMA) {              /* :193 */
        w_bool(w, 1);
        w_frame(w, sname, c->schema_name.len);
        w_uvarint(w, c->schema_major);
        w_uvarint(w, c->schema_minor);
        w_uvarint(w, c->schema_patch);
    } else {
        w_bool(w, 0);
    }
    if (c->present & HONU_HAS_ENCRYPTION) {          /* :198 */
        w_bool(w, 1);
        w_frame(w, pk, c->public_key_id.len);
        w_frame(w, ek, c->encryption_key.len);
        w_frame(w, hs, c->hmac_secret.len);
        w_frame(w, sg, c->signature.len);
        w_byte(w, c->sealing_alg);
        w_byte(w, c->encryption_alg);
        w_byte(w, c->signature_alg);
    } else {
        w_bool(w, 0);
    }
    if (c->present & HONU_HAS_COMPRESSION) {         /* :203 */
        w_bool(w, 1);
        w_byte(w, c->compression_alg);
        w_varint(w, c->compression_level);
    } else {
        w_bool(w, 0);
    }
    w_byte(w, c->flags);                             /* :208 */
    w_uvarint(w, c->index_count);                    /* :214 EncodeUint64(len Indexes) */
    for (uint64_t i = 0; i < c->index_count; i++) {  /* :220-225; index.go:58-86 */
        const honu_index *x = &idx[c->index_off + i];
        if (!x->present) {
            w_bool(w, 0);
            continue;
        }
        w_bool(w, 1);
        w_bytes(w, x->id, 16);
        w_frame(w, span_ptr(var, var_len, x->name, &bad), x->name.len);
        w_byte(w, x->type);
        if (x->has_field) {
            w_bool(w, 1);
            encode_field(w, span_ptr(var, var_len, x->field_name, &bad), x->field_name.len,
                         x->field_type, x->field_collection);
        } else {
            w_bool(w, 0);
        }
        if (x->has_ref) {
            w_bool(w, 1);
            encode_field(w, span_ptr(var, var_len, x->ref_name, &bad), x->ref_name.len,
                         x->ref_type, x->ref_collection);
        } else {
            w_bool(w, 0);
        }
    }
    w_time(w, c->created);                           /* :227 */
    w_time(w, c->modified);                          /* :232 */
    return HONU_OK;
}

int oracle_system_marshal(const honu_collection *c, const uint8_t *var, uint64_t var_len,
                          const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                          uint64_t regions_len, const honu_index *idx, uint64_t idx_len,
                          uint8_t *out, uint64_t cap, uint64_t *out_len) {
    *out_len = 0;
    owriter w = {out, cap, 0};
    w_byte(&w, HONU_STORAGE_VERSION);                /* system.go:17 EncodeUint8 */
    if (c->present & HONU_HAS_COLLECTION) {          /* :22 EncodeStruct(obj) */
        int st = encode_collection(&w, c, var, var_len, acl, acl_len, regions, regions_len, idx,
                                   idx_len);
        if (st != HONU_OK) return st;
    } else {
        w_bool(&w, 0);
    }
    w_bool(&w, 0);                                   /* :27 EncodeStruct(nil) */
    *out_len = w.len;
    if (out && w.len > cap) return HONU_ERR_CAPACITY;
    return HONU_OK;
}

typedef struct {
    honu_acl *acl_out;
    uint64_t acl_cap, acl_n;
    uint32_t *reg_out;
    uint64_t reg_cap, reg_n;
    honu_index *idx_out;
    uint64_t idx_cap, idx_n;
} osyslists;

/* Field.Decode field.go:62-80 */
static int decode_field(oreader *r, uint64_t base, honu_span *name, uint8_t *type,
                        uint8_t col[16]) {
    TRY(r_frame(r, base, name));
    TRY(r_byte(r, type));
    TRY(r_ulid(r, col));
    return HONU_OK;
}

/* Collection.Decode (collection.go:240-356) after its nil flag */
static int decode_collection_body(oreader *r, uint64_t base, honu_collection *c, osyslists *L) {
    int b;
    TRY(r_ulid(r, c->id));                           /* :248 */
    TRY(r_frame(r, base, &c->name));                 /* :252 DecodeString */
    TRY(r_bool(r, &b));                              /* :257 DecodeStruct(Version) */
    if (b) {
        c->present |= HONU_HAS_VERSION;
        TRY(r_u32(r, &c->pid));
        TRY(r_u64(r, &c->vid));
        TRY(r_u32(r, &c->region));
        TRY(r_bool(r, &b));
        if (b) {
            c->present |= HONU_HAS_PARENT;
            TRY(r_u32(r, &c->parent_pid));
            TRY(r_u64(r, &c->parent_vid));
        }
        TRY(r_bool(r, &b));
        c->tombstone = (uint8_t)b;
        TRY(r_i64(r, &c->version_created));
    }
    TRY(r_ulid(r, c->owner));                        /* :263 */
    TRY(r_ulid(r, c->group));                        /* :267 */
    TRY(r_byte(r, &c->permissions));                 /* :271 */
    uint64_t nacl;
    TRY(r_u64(r, &nacl));                            /* :277 */
    if (nacl > 0) {                                  /* :282-293 */
        if (nacl > GO_MAX_ALLOC / 8) return HONU_ERR_PANIC;
        c->acl_off = L->acl_n;
        for (uint64_t i = 0; i < nacl; i++) {
            honu_acl a;
            memset(&a, 0, sizeof a);
            TRY(r_bool(r, &b));
            if (b) {
                a.present = 1;
                TRY(r_ulid(r, a.client_id));
                TRY(r_byte(r, &a.permissions));
            }
            if (L->acl_n < L->acl_cap) L->acl_out[L->acl_n] = a;
            L->acl_n++;
        }
        c->acl_count = nacl;
    }
    uint64_t nreg;
    TRY(r_u64(r, &nreg));                            /* :295 WriteRegions.Decode */
    if (nreg > GO_MAX_ALLOC / 4) return HONU_ERR_PANIC;
    c->present |= HONU_REGIONS_NONNIL;
    c->regions_off = L->reg_n;
    for (uint64_t i = 0; i < nreg; i++) {
        uint32_t v;
        TRY(r_u32(r, &v));
        if (L->reg_n < L->reg_cap) L->reg_out[L->reg_n] = v;
        L->reg_n++;
    }
    c->regions_count = nreg;
    if (nreg == 0) c->regions_off = 0;
    TRY(r_bool(r, &b));                              /* :299 DecodeStruct(Publisher) */
    if (b) {
        c->present |= HONU_HAS_PUBLISHER;
        TRY(r_ulid(r, c->publisher_id));
        TRY(r_ulid(r, c->client_id));
        TRY(r_frame(r, base, &c->ip_address));
        TRY(r_frame(r, base, &c->user_agent));
    }
    TRY(r_bool(r, &b));                              /* :305 DecodeStruct(Schema) */
    if (b) {
        c->present |= HONU_HAS_SCHEMA;
        TRY(r_frame(r, base, &c->schema_name));
        TRY(r_u32(r, &c->schema_major));
        TRY(r_u32(r, &c->schema_minor));
        TRY(r_u32(r, &c->schema_patch));
    }
    TRY(r_bool(r, &b));                              /* :311 DecodeStruct(Encryption) */
    if (b) {
        c->present |= HONU_HAS_ENCRYPTION;
        TRY(r_frame(r, base, &c->public_key_id));
        TRY(r_frame(r, base, &c->encryption_key));
        TRY(r_frame(r, base, &c->hmac_secret));
        TRY(r_frame(r, base, &c->signature));
        TRY(r_byte(r, &c->sealing_alg));
        TRY(r_byte(r, &c->encryption_alg));
        TRY(r_byte(r, &c->signature_alg));
    }
    TRY(r_bool(r, &b));                              /* :317 DecodeStruct(Compression) */
    if (b) {
        c->present |= HONU_HAS_COMPRESSION;
        TRY(r_byte(r, &c->compression_alg));
        TRY(r_i64(r, &c->compression_level));
    }
    TRY(r_byte(r, &c->flags));                       /* :323 */
    uint64_t nidx;
    TRY(r_u64(r, &nidx));                            /* :329 */
    if (nidx > 0) {                                  /* :334-345 */
        if (nidx > GO_MAX_ALLOC / 8) return HONU_ERR_PANIC; /* make([]*Index, n) */
        c->index_off = L->idx_n;
        for (uint64_t i = 0; i < nidx; i++) {
            honu_index x;
            memset(&x, 0, sizeof x);
            TRY(r_bool(r, &b));                      /* DecodeStruct(c.Indexes[i]) */
            if (b) {                                 /* Index.Decode index.go:88-120 */
                x.present = 1;
                TRY(r_ulid(r, x.id));
                TRY(r_frame(r, base, &x.name));
                TRY(r_byte(r, &x.type));
                TRY(r_bool(r, &b));                  /* DecodeStruct(o.Field) */
                if (b) {
                    x.has_field = 1;
                    TRY(decode_field(r, base, &x.field_name, &x.field_type, x.field_collection));
                }
                TRY(r_bool(r, &b));                  /* DecodeStruct(o.Ref) */
                if (b) {
                    x.has_ref = 1;
                    TRY(decode_field(r, base, &x.ref_name, &x.ref_type, x.ref_collection));
                }
            }
            if (L->idx_n < L->idx_cap) L->idx_out[L->idx_n] = x;
            L->idx_n++;
        }
        c->index_count = nidx;
    }
    TRY(r_i64(r, &c->created));                      /* :347 DecodeTime */
    TRY(r_i64(r, &c->modified));                     /* :351 */
    return HONU_OK;
}

/* headless = 0: object.UnmarshalSystem(obj, &Collection{}) (system.go:36-45);
 * headless = 1: lani.Unmarshal(obj, &Collection{}) (lani.go:29-33), i.e.
 * Collection.Decode from byte 0 of the raw value as store.go:367 calls it
 * (the storage version byte and the struct flag are read as the ID). */
static int collection_decode(const uint8_t *o, uint64_t len, uint64_t base, int headless,
                             honu_collection *c, honu_acl *acl_out, uint64_t acl_cap,
                             uint32_t *regions_out, uint64_t regions_cap, honu_index *idx_out,
                             uint64_t idx_cap, uint64_t counts[3]) {
    memset(c, 0, sizeof *c);
    counts[0] = counts[1] = counts[2] = 0;
    osyslists L = {acl_out, acl_cap, 0, regions_out, regions_cap, 0, idx_out, idx_cap, 0};
    int st;
    if (headless) {
        oreader r = {o, len, 0};
        c->present = HONU_HAS_COLLECTION;           /* the target itself, never nil */
        st = decode_collection_body(&r, base, c, &L);
    } else {
        /* obj[1 : len(obj)-1] (system.go:40) panics for len < 2 */
        if (len < 2) return HONU_ERR_PANIC;
        oreader r = {o + 1, len - 2, 0};
        int present;
        st = r_bool(&r, &present);                   /* DecodeStruct(v) :41 */
        if (st == HONU_OK && present) {
            c->present = HONU_HAS_COLLECTION;
            st = decode_collection_body(&r, base + 1, c, &L);
        }
    }
    if (st != HONU_OK) {
        memset(c, 0, sizeof *c);
        return st;
    }
    counts[0] = L.acl_n;
    counts[1] = L.reg_n;
    counts[2] = L.idx_n;
    return HONU_OK;
}

int oracle_system_decode(const uint8_t *o, uint64_t len, uint64_t base, honu_collection *c,
                         honu_acl *acl_out, uint64_t acl_cap, uint32_t *regions_out,
                         uint64_t regions_cap, honu_index *idx_out, uint64_t idx_cap,
                         uint64_t counts[3]) {
    return collection_decode(o, len, base, 0, c, acl_out, acl_cap, regions_out, regions_cap,
                             idx_out, idx_cap, counts);
}

int oracle_system_marshal_batch(const honu_collection *rows, const uint8_t *var, uint64_t var_len,
                                const honu_acl *acl, uint64_t acl_len, const uint32_t *regions,
                                uint64_t regions_len, const honu_index *idx, uint64_t idx_len,
                                uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                                int32_t *status) {
    uint64_t pos = 0;
    int any_cap = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t sz = 0;
        int st = oracle_system_marshal(&rows[i], var, var_len, acl, acl_len, regions, regions_len,
                                       idx, idx_len, NULL, 0, &sz);
        out_off[i] = pos;
        pos += sz;
        if (status) status[i] = st;
    }
    out_off[n] = pos;
    for (uint64_t i = 0; i < n; i++) {
        if (status && status[i] != HONU_OK) continue;
        uint64_t beg = out_off[i], end = out_off[i + 1];
        if (end > out_cap) {
            if (status) status[i] = HONU_ERR_CAPACITY;
            any_cap = 1;
            continue;
        }
        uint64_t sz;
        int st = oracle_system_marshal(&rows[i], var, var_len, acl, acl_len, regions, regions_len,
                                       idx, idx_len, out + beg, end - beg, &sz);
        if (status) status[i] = st;
    }
    return any_cap ? HONU_ERR_CAPACITY : HONU_OK;
}

static int collection_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   int headless, honu_collection *rows, int32_t *status,
                                   honu_acl *acl, uint64_t acl_cap, uint32_t *regions,
                                   uint64_t regions_cap, honu_index *idx, uint64_t idx_cap,
                                   uint64_t totals[3]) {
    uint64_t pos[3] = {0, 0, 0};
    int any_cap = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t beg = rec_off[i], len = rec_off[i + 1] - rec_off[i];
        uint64_t cnt[3];
        honu_acl *ao = acl ? acl + (pos[0] < acl_cap ? pos[0] : acl_cap) : NULL;
        uint32_t *ro = regions ? regions + (pos[1] < regions_cap ? pos[1] : regions_cap) : NULL;
        honu_index *xo = idx ? idx + (pos[2] < idx_cap ? pos[2] : idx_cap) : NULL;
        uint64_t ac = acl && pos[0] < acl_cap ? acl_cap - pos[0] : 0;
        uint64_t rc = regions && pos[1] < regions_cap ? regions_cap - pos[1] : 0;
        uint64_t xc = idx && pos[2] < idx_cap ? idx_cap - pos[2] : 0;
        int st = collection_decode(rec + beg, len, beg, headless, &rows[i], ao, ac, ro, rc, xo, xc,
                                   cnt);
        if (st == HONU_OK) {
            if (rows[i].acl_count) rows[i].acl_off = pos[0];
            if (rows[i].regions_count) rows[i].regions_off = pos[1];
            if (rows[i].index_count) rows[i].index_off = pos[2];
            if (pos[0] + cnt[0] > acl_cap || pos[1] + cnt[1] > regions_cap ||
                pos[2] + cnt[2] > idx_cap) {
                st = HONU_ERR_CAPACITY;
                any_cap = 1;
            }
            for (int k = 0; k < 3; k++) pos[k] += cnt[k];
        }
        status[i] = st;
    }
    if (totals)
        for (int k = 0; k < 3; k++) totals[k] = pos[k];
    return any_cap ? HONU_ERR_CAPACITY : HONU_OK;
}

int oracle_system_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               honu_collection *rows, int32_t *status, honu_acl *acl,
                               uint64_t acl_cap, uint32_t *regions, uint64_t regions_cap,
                               honu_index *idx, uint64_t idx_cap, uint64_t totals[3]) {
    return collection_decode_batch(rec, rec_off, n, 0, rows, status, acl, acl_cap, regions,
                                   regions_cap, idx, idx_cap, totals);
}

int oracle_collection_decode_batch(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                   honu_collection *rows, int32_t *status, honu_acl *acl,
                                   uint64_t acl_cap, uint32_t *regions, uint64_t regions_cap,
                                   honu_index *idx, uint64_t idx_cap, uint64_t totals[3]) {
    return collection_decode_batch(rec, rec_off, n, 1, rows, status, acl, acl_cap, regions,
                                   regions_cap, idx, idx_cap, totals);
}
