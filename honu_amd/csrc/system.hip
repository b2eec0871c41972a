// system.hip — system objects on the GPU: object.MarshalSystem /
// UnmarshalSystem (object/system.go:10-45) of metadata.Collection
// (collection.go:137-356) with its Index / Field lists (index.go:58-120,
// field.go:42-80).
//
// A store holds few collections, so these kernels favour simplicity: one
// record per lane, the same lani primitives as the object codec (lane.h), a
// size pass + exclusive scan + writer for encode, and a parse + count scans +
// table fill for decode (ACL entries, regions and Index rows land in CSR
// tables like the object decoder's).
#include "kernels.h"
#include "lane.h"

namespace honu {

#define GO_MAX_ALLOC (1ull << 48)  // runtime maxAlloc, linux/amd64
#define COFF(f) ((int)offsetof(honu_collection, f))

using CRow = RowT<92>;

HONU_DEV bool sys_span_in(honu_span s, uint64_t var_len) {
    return s.len == 0 || (s.off <= var_len && s.len <= var_len - s.off);
}
HONU_DEV uint64_t sys_frame_len(uint64_t len) { return uvarint_len(len) + len; }

// Field.Encode (field.go:42-60) length
HONU_DEV uint64_t field_len(honu_span name) { return sys_frame_len(name.len) + 1 + 16; }

// ------------------------------------------------------------------------
// encode size pass: 1 + EncodeStruct(collection) + 1
// ------------------------------------------------------------------------
HONU_DEV void system_size_one(uint64_t i, const honu_collection *__restrict__ rows,
                              uint64_t var_len, const honu_acl *__restrict__ acl,
                              uint64_t acl_len, const uint32_t *__restrict__ reg,
                              uint64_t reg_len, const honu_index *__restrict__ idx,
                              uint64_t idx_len, uint64_t *__restrict__ sizes,
                              int32_t *__restrict__ status) {
    const honu_collection &c = rows[i];
    const uint32_t pr = c.present;
    if (!(pr & HONU_HAS_COLLECTION)) {  // MarshalSystem(nil): 01 00 00
        sizes[i] = 3;
        if (status) status[i] = HONU_OK;
        return;
    }
    bool ok = sys_span_in(c.name, var_len);
    if (pr & HONU_HAS_SCHEMA) ok = ok && sys_span_in(c.schema_name, var_len);
    if (pr & HONU_HAS_PUBLISHER)
        ok = ok && sys_span_in(c.ip_address, var_len) && sys_span_in(c.user_agent, var_len);
    if (pr & HONU_HAS_ENCRYPTION)
        ok = ok && sys_span_in(c.public_key_id, var_len) &&
             sys_span_in(c.encryption_key, var_len) && sys_span_in(c.hmac_secret, var_len) &&
             sys_span_in(c.signature, var_len);
    const uint64_t na = c.acl_count, nr = c.regions_count, nx = c.index_count;
    if (na) ok = ok && c.acl_off <= acl_len && na <= acl_len - c.acl_off;
    if (nr) ok = ok && c.regions_off <= reg_len && nr <= reg_len - c.regions_off;
    if (nx) ok = ok && c.index_off <= idx_len && nx <= idx_len - c.index_off;
    uint64_t t = 0;
    for (uint64_t k = 0; ok && k < nx; k++) {  // :220-225, index.go:58-86
        const honu_index &x = idx[c.index_off + k];
        t += 1;
        if (!x.present) continue;
        ok = sys_span_in(x.name, var_len) && (!x.has_field || sys_span_in(x.field_name, var_len)) &&
             (!x.has_ref || sys_span_in(x.ref_name, var_len));
        t += 16 + sys_frame_len(x.name.len) + 1 + 2;
        if (x.has_field) t += field_len(x.field_name);
        if (x.has_ref) t += field_len(x.ref_name);
    }
    if (!ok) {
        sizes[i] = 0;
        if (status) status[i] = HONU_ERR_INPUT;
        return;
    }
    t += 1 + 16 + sys_frame_len(c.name.len);  // struct flag, ID, Name
    t += 1;                                   // Version flag
    if (pr & HONU_HAS_VERSION)
        t += uvarint_len(c.pid) + uvarint_len(c.vid) + uvarint_len(c.region) + 1 +
             ((pr & HONU_HAS_PARENT) ? uvarint_len(c.parent_pid) + uvarint_len(c.parent_vid) : 0) +
             1 + uvarint_len(zigzag(c.version_created));
    t += 33;  // Owner, Group, Permissions
    t += uvarint_len(na);
    for (uint64_t k = 0; k < na; k++) t += acl[c.acl_off + k].present ? 18 : 1;
    t += uvarint_len(nr);
    for (uint64_t k = 0; k < nr; k++) t += uvarint_len(reg[c.regions_off + k]);
    t += 4;  // Publisher, Schema, Encryption, Compression flags
    if (pr & HONU_HAS_PUBLISHER)
        t += 32 + sys_frame_len(c.ip_address.len) + sys_frame_len(c.user_agent.len);
    if (pr & HONU_HAS_SCHEMA)
        t += sys_frame_len(c.schema_name.len) + uvarint_len(c.schema_major) +
             uvarint_len(c.schema_minor) + uvarint_len(c.schema_patch);
    if (pr & HONU_HAS_ENCRYPTION)
        t += sys_frame_len(c.public_key_id.len) + sys_frame_len(c.encryption_key.len) +
             sys_frame_len(c.hmac_secret.len) + sys_frame_len(c.signature.len) + 3;
    if (pr & HONU_HAS_COMPRESSION) t += 1 + uvarint_len(zigzag(c.compression_level));
    t += 1 + uvarint_len(nx);  // Flags, len(Indexes)
    t += uvarint_len(zigzag(c.created)) + uvarint_len(zigzag(c.modified));
    sizes[i] = 1 + t + 1;  // version byte, collection, nil metadata
    if (status) status[i] = HONU_OK;
}

__global__ __launch_bounds__(HONU_BLOCK) void k_system_sizes(
    const honu_collection *__restrict__ rows, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const honu_index *__restrict__ idx, uint64_t idx_len, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        system_size_one(i, rows, var_len, acl, acl_len, reg, reg_len, idx, idx_len, sizes, status);
}

// ------------------------------------------------------------------------
// encode writer
// ------------------------------------------------------------------------
HONU_DEV void put_ulid(LaneWriter &W, const uint8_t *p) {
    W.put16(*reinterpret_cast<const uint64_t *>(p), *reinterpret_cast<const uint64_t *>(p + 8));
}

HONU_DEV void system_encode_one(uint64_t i, const honu_collection *__restrict__ rows,
                                const uint8_t *__restrict__ var,
                                const honu_acl *__restrict__ acl,
                                const uint32_t *__restrict__ reg,
                                const honu_index *__restrict__ idx, uint8_t *__restrict__ out,
                                uint64_t out_cap, const uint64_t *__restrict__ out_off,
                                int32_t *__restrict__ status) {
    if (status[i] != HONU_OK) return;
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    if (end > out_cap) {
        status[i] = HONU_ERR_CAPACITY;
        return;
    }
    const honu_collection &c = rows[i];
    const uint32_t pr = c.present;
    LaneWriter W;
    W.init(out, beg);
    W.byte(HONU_STORAGE_VERSION);                                   // system.go:17
    if (!(pr & HONU_HAS_COLLECTION)) {
        W.byte(0);                                                  // EncodeStruct(nil obj)
        W.byte(0);                                                  // :27 nil metadata
        W.finish();
        return;
    }
    W.byte(1);                                                      // :22 EncodeStruct(obj)
    put_ulid(W, c.id);                                              // collection.go:139
    W.frame(var, c.name);                                           // :144
    if (pr & HONU_HAS_VERSION) {                                    // :149, version.go:44-70
        W.byte(1);
        W.uv(c.pid);
        W.uv(c.vid);
        W.uv(c.region);
        if (pr & HONU_HAS_PARENT) {
            W.byte(1);
            W.uv(c.parent_pid);
            W.uv(c.parent_vid);
        } else {
            W.byte(0);
        }
        W.byte(c.tombstone ? 1 : 0);
        W.uv(zigzag(c.version_created));
    } else {
        W.byte(0);
    }
    put_ulid(W, c.owner);                                           // :154
    put_ulid(W, c.group);                                           // :159
    W.byte(c.permissions);                                          // :164
    W.uv(c.acl_count);                                              // :170
    for (uint64_t k = 0; k < c.acl_count; k++) {                    // :176-181, acls.go:26-39
        const honu_acl &a = acl[c.acl_off + k];
        if (a.present) {
            W.byte(1);
            put_ulid(W, a.client_id);
            W.byte(a.permissions);
        } else {
            W.byte(0);
        }
    }
    W.uv(c.regions_count);                                          // :183, region.go:137-152
    for (uint64_t k = 0; k < c.regions_count; k++) W.uv(reg[c.regions_off + k]);
    if (pr & HONU_HAS_PUBLISHER) {                                  // :188, provenance.go:34-57
        W.byte(1);
        put_ulid(W, c.publisher_id);
        put_ulid(W, c.client_id);
        W.frame(var, c.ip_address);
        W.frame(var, c.user_agent);
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_SCHEMA) {                                     // :193, schema.go:30-53
        W.byte(1);
        W.frame(var, c.schema_name);
        W.uv(c.schema_major);
        W.uv(c.schema_minor);
        W.uv(c.schema_patch);
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_ENCRYPTION) {                                 // :198, encryption.go:51-89
        W.byte(1);
        W.frame(var, c.public_key_id);
        W.frame(var, c.encryption_key);
        W.frame(var, c.hmac_secret);
        W.frame(var, c.signature);
        W.byte(c.sealing_alg);
        W.byte(c.encryption_alg);
        W.byte(c.signature_alg);
    } else {
        W.byte(0);
    }
    if (pr & HONU_HAS_COMPRESSION) {                                // :203, compression.go:40-53
        W.byte(1);
        W.byte(c.compression_alg);
        W.uv(zigzag(c.compression_level));
    } else {
        W.byte(0);
    }
    W.byte(c.flags);                                                // :208
    W.uv(c.index_count);                                            // :214
    for (uint64_t k = 0; k < c.index_count; k++) {                  // :220-225
        const honu_index &x = idx[c.index_off + k];
        if (!x.present) {
            W.byte(0);
            continue;
        }
        W.byte(1);                                                  // index.go:58-86
        put_ulid(W, x.id);
        W.frame(var, x.name);
        W.byte(x.type);
        if (x.has_field) {                                          // field.go:42-60
            W.byte(1);
            W.frame(var, x.field_name);
            W.byte(x.field_type);
            put_ulid(W, x.field_collection);
        } else {
            W.byte(0);
        }
        if (x.has_ref) {
            W.byte(1);
            W.frame(var, x.ref_name);
            W.byte(x.ref_type);
            put_ulid(W, x.ref_collection);
        } else {
            W.byte(0);
        }
    }
    W.uv(zigzag(c.created));                                        // :227
    W.uv(zigzag(c.modified));                                       // :232
    W.byte(0);                                                      // system.go:27 nil metadata
    W.finish();
}

__global__ __launch_bounds__(HONU_BLOCK) void k_system_encode(
    const honu_collection *__restrict__ rows, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const honu_index *__restrict__ idx, uint64_t n, uint8_t *__restrict__ out, uint64_t out_cap,
    const uint64_t *__restrict__ out_off, int32_t *__restrict__ status) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        system_encode_one(i, rows, var, acl, reg, idx, out, out_cap, out_off, status);
}

// ------------------------------------------------------------------------
// decode: UnmarshalSystem(obj, &Collection{}) over obj[1 : len-1]
// ------------------------------------------------------------------------
#define TRY(x)              \
    do {                    \
        st = (x);           \
        if (st) goto done;  \
    } while (0)

// Field.Decode (field.go:62-80): walk only (the fill writes the row)
HONU_DEV int skip_field(LaneDec &D) {
    uint64_t o, l, lo, hi;
    uint32_t u;
    int st = D.frame(o, l);
    if (st) return st;
    st = D.u8(u);
    if (st) return st;
    return D.ulid(lo, hi);
}

// Index.Decode (index.go:88-120) of a non-nil entry, walk only
HONU_DEV int skip_index(LaneDec &D) {
    uint64_t o, l, lo, hi;
    uint32_t u, f;
    int st;
    if ((st = D.ulid(lo, hi))) return st;
    if ((st = D.frame(o, l))) return st;
    if ((st = D.u8(u))) return st;
    if ((st = D.boolean(f))) return st;
    if (f && (st = skip_field(D))) return st;
    if ((st = D.boolean(f))) return st;
    if (f && (st = skip_field(D))) return st;
    return HONU_OK;
}

// headless = false: object.UnmarshalSystem(obj, &Collection{}) (system.go:36-45):
// obj[1 : len-1], struct flag first. headless = true: lani.Unmarshal(obj,
// &Collection{}) (lani.go:29-33) as store.go:367 calls it on a raw bbolt
// value: Collection.Decode from byte 0 to the end, no flag.
HONU_DEV void system_parse_one(uint64_t i, const uint8_t *__restrict__ rec,
                               const uint64_t *__restrict__ rec_off, bool headless,
                               honu_collection *__restrict__ rows,
                               int32_t *__restrict__ status, DecodeScratch *__restrict__ scratch,
                               uint64_t *__restrict__ counts) {
    const uint64_t beg = rec_off[i], end = rec_off[i + 1];
    const uint64_t t0 = headless ? beg : beg + 1, t1 = headless ? end : end - 1;
    CRow R;
    R.clear();
    uint64_t nacl = 0, nreg = 0, nidx = 0, acl_pos = 0, reg_pos = 0, idx_pos = 0;
    int st = HONU_OK;
    if (!headless && end - beg < 2) {
        st = HONU_ERR_PANIC;  // obj[1 : len(obj)-1] out of range (system.go:40)
    } else {
        LaneDec D;
        D.base = rec;
        D.tstart = t0;
        D.p = t0;
        D.end = t1;
        uint32_t f = 1, u;
        uint64_t v, o, l, lo, hi;
        int64_t t;
        uint32_t pr = 0;
        if (!headless) TRY(D.boolean(f));                   // DecodeStruct(v) system.go:41
        if (f) {
            pr = HONU_HAS_COLLECTION;
            TRY(D.ulid(lo, hi)); R.bytes16(COFF(id), lo, hi);          // collection.go:248
            TRY(D.frame(o, l)); R.span(COFF(name), o, l);              // :252
            TRY(D.boolean(f));                              // :257 Version
            if (f) {
                pr |= HONU_HAS_VERSION;
                TRY(D.u32(u)); R.u32(COFF(pid), u);
                TRY(D.u64(v)); R.u64(COFF(vid), v);
                TRY(D.u32(u)); R.u32(COFF(region), u);
                TRY(D.boolean(f));
                if (f) {
                    pr |= HONU_HAS_PARENT;
                    TRY(D.u32(u)); R.u32(COFF(parent_pid), u);
                    TRY(D.u64(v)); R.u64(COFF(parent_vid), v);
                }
                TRY(D.boolean(f)); R.u8(COFF(tombstone), f);
                TRY(D.i64(t)); R.u64(COFF(version_created), (uint64_t)t);
            }
            TRY(D.ulid(lo, hi)); R.bytes16(COFF(owner), lo, hi);       // :263
            TRY(D.ulid(lo, hi)); R.bytes16(COFF(group), lo, hi);       // :267
            TRY(D.u8(u)); R.u8(COFF(permissions), u);       // :271
            TRY(D.u64(nacl));                               // :277
            if (nacl > 0) {                                 // :282-293
                if (nacl > GO_MAX_ALLOC / 8) TRY(HONU_ERR_PANIC);
                acl_pos = D.p;
                for (uint64_t k = 0; k < nacl; k++) {       // acls.go:41-51
                    TRY(D.boolean(f));
                    if (f) {
                        TRY(D.ulid(lo, hi));
                        TRY(D.u8(u));
                    }
                }
                R.u64(COFF(acl_count), nacl);
            }
            TRY(D.u64(nreg));                               // :295, region.go:154-169
            if (nreg > GO_MAX_ALLOC / 4) TRY(HONU_ERR_PANIC);
            pr |= HONU_REGIONS_NONNIL;
            reg_pos = D.p;
            for (uint64_t k = 0; k < nreg; k++) TRY(D.u32(u));
            R.u64(COFF(regions_count), nreg);
            TRY(D.boolean(f));                              // :299 Publisher
            if (f) {
                pr |= HONU_HAS_PUBLISHER;
                TRY(D.ulid(lo, hi)); R.bytes16(COFF(publisher_id), lo, hi);
                TRY(D.ulid(lo, hi)); R.bytes16(COFF(client_id), lo, hi);
                TRY(D.frame(o, l)); R.span(COFF(ip_address), o, l);
                TRY(D.frame(o, l)); R.span(COFF(user_agent), o, l);
            }
            TRY(D.boolean(f));                              // :305 Schema
            if (f) {
                pr |= HONU_HAS_SCHEMA;
                TRY(D.frame(o, l)); R.span(COFF(schema_name), o, l);
                TRY(D.u32(u)); R.u32(COFF(schema_major), u);
                TRY(D.u32(u)); R.u32(COFF(schema_minor), u);
                TRY(D.u32(u)); R.u32(COFF(schema_patch), u);
            }
            TRY(D.boolean(f));                              // :311 Encryption
            if (f) {
                pr |= HONU_HAS_ENCRYPTION;
                TRY(D.frame(o, l)); R.span(COFF(public_key_id), o, l);
                TRY(D.frame(o, l)); R.span(COFF(encryption_key), o, l);
                TRY(D.frame(o, l)); R.span(COFF(hmac_secret), o, l);
                TRY(D.frame(o, l)); R.span(COFF(signature), o, l);
                TRY(D.u8(u)); R.u8(COFF(sealing_alg), u);
                TRY(D.u8(u)); R.u8(COFF(encryption_alg), u);
                TRY(D.u8(u)); R.u8(COFF(signature_alg), u);
            }
            TRY(D.boolean(f));                              // :317 Compression
            if (f) {
                pr |= HONU_HAS_COMPRESSION;
                TRY(D.u8(u)); R.u8(COFF(compression_alg), u);
                TRY(D.i64(t)); R.u64(COFF(compression_level), (uint64_t)t);
            }
            TRY(D.u8(u)); R.u8(COFF(flags), u);             // :323
            TRY(D.u64(nidx));                               // :329
            if (nidx > 0) {                                 // :334-345
                if (nidx > GO_MAX_ALLOC / 8) TRY(HONU_ERR_PANIC);  // make([]*Index, n)
                idx_pos = D.p;
                for (uint64_t k = 0; k < nidx; k++) {
                    TRY(D.boolean(f));                      // DecodeStruct(c.Indexes[i])
                    if (f) TRY(skip_index(D));
                }
                R.u64(COFF(index_count), nidx);
            }
            TRY(D.i64(t)); R.u64(COFF(created), (uint64_t)t);   // :347
            TRY(D.i64(t)); R.u64(COFF(modified), (uint64_t)t);  // :351
        }
        R.u32(COFF(present), pr);
    }
done:
    if (st != HONU_OK) {  // UnmarshalSystem returns err; the row is cleared
        R.clear();
        nacl = nreg = nidx = 0;
    }
    R.store(rows + i);
    status[i] = st;
    scratch[i] = DecodeScratch{acl_pos, reg_pos, idx_pos, t1};
    counts[3 * i + 0] = nacl;
    counts[3 * i + 1] = nreg;
    counts[3 * i + 2] = nidx;
}
#undef TRY

__global__ __launch_bounds__(HONU_BLOCK) void k_system_parse(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    bool headless, honu_collection *__restrict__ rows, int32_t *__restrict__ status,
    DecodeScratch *__restrict__ scratch, uint64_t *__restrict__ counts) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        system_parse_one(i, rec, rec_off, headless, rows, status, scratch, counts);
}

// Field.Decode into an index row (walk validated by the parse)
HONU_DEV void fill_field(LaneDec &D, honu_span &name, uint8_t &type, uint8_t col[16]) {
    uint64_t o = 0, l = 0, lo = 0, hi = 0;
    uint32_t u = 0;
    D.frame(o, l);
    name = honu_span{o, l};
    D.u8(u);
    type = (uint8_t)u;
    D.ulid(lo, hi);
    reinterpret_cast<uint64_t *>(col)[0] = lo;
    reinterpret_cast<uint64_t *>(col)[1] = hi;
}

HONU_DEV void system_fill_one(uint64_t i, const uint8_t *__restrict__ rec,
                              honu_collection *__restrict__ rows, int32_t *__restrict__ status,
                              const DecodeScratch *__restrict__ scratch,
                              const uint64_t *__restrict__ counts,
                              const uint64_t *__restrict__ offs, honu_acl *__restrict__ acl,
                              uint64_t acl_cap, uint32_t *__restrict__ reg, uint64_t reg_cap,
                              honu_index *__restrict__ idx, uint64_t idx_cap) {
    if (status[i] != HONU_OK) return;
    const uint64_t na = counts[3 * i], nr = counts[3 * i + 1], nx = counts[3 * i + 2];
    const uint64_t ao = offs[3 * i], ro = offs[3 * i + 1], xo = offs[3 * i + 2];
    if (na) rows[i].acl_off = ao;
    if (nr) rows[i].regions_off = ro;
    if (nx) rows[i].index_off = xo;
    if (ao + na > acl_cap || ro + nr > reg_cap || xo + nx > idx_cap) {
        status[i] = HONU_ERR_CAPACITY;
        return;
    }
    const DecodeScratch sc = scratch[i];
    LaneDec D;
    D.base = rec;
    D.end = sc.rec_end;
    D.tstart = 0;
    uint32_t f = 0, u = 0;
    uint64_t lo = 0, hi = 0, o = 0, l = 0;
    D.p = sc.acl_pos;
    for (uint64_t k = 0; k < na; k++) {
        honu_acl a;
        uint32_t *e = reinterpret_cast<uint32_t *>(&a);
        e[0] = e[1] = e[2] = e[3] = e[4] = 0;
        D.boolean(f);
        if (f) {
            D.ulid(lo, hi);
            D.u8(u);
            e[0] = (uint32_t)lo;
            e[1] = (uint32_t)(lo >> 32);
            e[2] = (uint32_t)hi;
            e[3] = (uint32_t)(hi >> 32);
            e[4] = u | (1u << 8);
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(acl + ao + k);
#pragma unroll
        for (int j = 0; j < 5; j++) dst[j] = e[j];
    }
    D.p = sc.regions_pos;
    for (uint64_t k = 0; k < nr; k++) {
        D.u32(u);
        reg[ro + k] = u;
    }
    D.p = sc.data_src;  // first Index flag
    for (uint64_t k = 0; k < nx; k++) {
        honu_index x;
        uint32_t *w = reinterpret_cast<uint32_t *>(&x);
#pragma unroll
        for (int j = 0; j < (int)(sizeof(honu_index) / 4); j++) w[j] = 0;
        D.boolean(f);
        if (f) {  // index.go:88-120
            x.present = 1;
            D.ulid(lo, hi);
            reinterpret_cast<uint64_t *>(x.id)[0] = lo;
            reinterpret_cast<uint64_t *>(x.id)[1] = hi;
            D.frame(o, l);
            x.name = honu_span{o, l};
            D.u8(u);
            x.type = (uint8_t)u;
            D.boolean(f);
            if (f) {
                x.has_field = 1;
                fill_field(D, x.field_name, x.field_type, x.field_collection);
            }
            D.boolean(f);
            if (f) {
                x.has_ref = 1;
                fill_field(D, x.ref_name, x.ref_type, x.ref_collection);
            }
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(idx + xo + k);
#pragma unroll
        for (int j = 0; j < (int)(sizeof(honu_index) / 4); j++) dst[j] = w[j];
    }
}

__global__ __launch_bounds__(HONU_BLOCK) void k_system_fill(
    const uint8_t *__restrict__ rec, uint64_t n, honu_collection *__restrict__ rows,
    int32_t *__restrict__ status, const DecodeScratch *__restrict__ scratch,
    const uint64_t *__restrict__ counts, const uint64_t *__restrict__ offs,
    honu_acl *__restrict__ acl, uint64_t acl_cap, uint32_t *__restrict__ reg, uint64_t reg_cap,
    honu_index *__restrict__ idx, uint64_t idx_cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        system_fill_one(i, rec, rows, status, scratch, counts, offs, acl, acl_cap, reg, reg_cap,
                        idx, idx_cap);
}

#undef COFF

static dim3 sys_grid(uint64_t n) {
    const uint64_t b = (n + HONU_BLOCK - 1) / HONU_BLOCK;
    return dim3((unsigned)(b > 65536 ? 65536 : b));
}

hipError_t launch_system_sizes(const honu_collection *rows, uint64_t var_len, const honu_acl *acl,
                               uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                               const honu_index *idx, uint64_t idx_len, uint64_t n,
                               uint64_t *sizes, int32_t *status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_system_sizes, sys_grid(n), dim3(HONU_BLOCK), 0, s, rows, var_len, acl,
                       acl_len, reg, reg_len, idx, idx_len, n, sizes, status);
    return hipGetLastError();
}

hipError_t launch_system_encode(const honu_collection *rows, const uint8_t *var,
                                const honu_acl *acl, const uint32_t *reg, const honu_index *idx,
                                uint64_t n, uint8_t *out, uint64_t out_cap,
                                const uint64_t *out_off, int32_t *status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_system_encode, sys_grid(n), dim3(HONU_BLOCK), 0, s, rows, var, acl, reg,
                       idx, n, out, out_cap, out_off, status);
    return hipGetLastError();
}

hipError_t launch_system_parse(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                               bool headless, honu_collection *rows, int32_t *status,
                               DecodeScratch *scratch, uint64_t *counts, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_system_parse, sys_grid(n), dim3(HONU_BLOCK), 0, s, rec, rec_off, n,
                       headless, rows, status, scratch, counts);
    return hipGetLastError();
}

hipError_t launch_system_fill(const uint8_t *rec, uint64_t n, honu_collection *rows,
                              int32_t *status, const DecodeScratch *scratch,
                              const uint64_t *counts, const uint64_t *offs, honu_acl *acl,
                              uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, honu_index *idx,
                              uint64_t idx_cap, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_system_fill, sys_grid(n), dim3(HONU_BLOCK), 0, s, rec, n, rows, status,
                       scratch, counts, offs, acl, acl_cap, reg, reg_cap, idx, idx_cap);
    return hipGetLastError();
}

}  // namespace honu
