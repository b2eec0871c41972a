// lane.hip — the per-record metadata kernels with one record per LANE
// (see lane.h for why): decode parse, decode fill and the encode size pass.
#include "kernels.h"
#include "lane.h"

namespace honu {

#define GO_MAX_ALLOC (1ull << 48)  // runtime maxAlloc, linux/amd64
#define OFF(f) ((int)offsetof(honu_meta, f))

#define TRY(x)              \
    do {                    \
        st = (x);           \
        if (st) goto done;  \
    } while (0)

// ------------------------------------------------------------------------
// decode parse: Object.Metadata() + Data() + Tombstone() + StorageVersion()
// (object.go:47-134) with the lani walk of metadata.go:202-302.
// ------------------------------------------------------------------------
HONU_DEV void k_decode_parse_lane_one(uint64_t i, const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint32_t *__restrict__ reg_inline,
    uint64_t *__restrict__ counts) {
    const uint64_t beg = rec_off[i], end = rec_off[i + 1];
    const uint64_t len = end - beg;
    uint32_t ver = 0;
    int64_t d = -1, b = -1;
    if (len) {
        uint64_t lo, hi;
        lane_fetch16(rec, beg, end, lo, hi);
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
    int32_t data_status;
    uint64_t data_off = 0, data_len = 0;
    if (!v1) data_status = HONU_ERR_BAD_VERSION;
    else if (d < 0) data_status = HONU_ERR_MALFORMED;
    else if (d == 0) data_status = HONU_OK;
    else if (!in_range) data_status = HONU_ERR_PANIC;  // o[1+b:1+b+d]
    else {
        data_status = HONU_OK;
        data_off = beg + 1 + (uint64_t)b;
        data_len = (uint64_t)d;
    }

    Row R;
    R.clear();
    uint64_t nacl = 0, nreg = 0, acl_pos = 0, reg_pos = 0;
    int st = HONU_OK;
    if (!v1) st = HONU_ERR_BAD_VERSION;
    else if (d < 0) st = HONU_ERR_MALFORMED;
    else if (!in_range) st = HONU_ERR_PANIC;  // o[1+d+b:]
    else {
        LaneDec D;
        D.base = rec;
        D.end = end;
        D.tstart = beg + 1 + (uint64_t)b + (uint64_t)d;
        D.p = D.tstart;
        uint32_t f, u;
        uint64_t v, o, l, lo, hi;
        int64_t t;
        uint32_t pr = 0;
        TRY(D.boolean(f));                                      // DecodeStruct(meta) object.go:78
        if (f) {
            pr = HONU_HAS_META;
            TRY(D.ulid(lo, hi)); R.bytes16(OFF(object_id), lo, hi);        // metadata.go:210
            TRY(D.ulid(lo, hi)); R.bytes16(OFF(collection_id), lo, hi);    // :214
            TRY(D.boolean(f));                                  // :219 Version
            if (f) {
                pr |= HONU_HAS_VERSION;
                TRY(D.u32(u)); R.u32(OFF(pid), u);              // scalar.go:121-131
                TRY(D.u64(v)); R.u64(OFF(vid), v);
                TRY(D.u32(u)); R.u32(OFF(region), u);           // version.go:80
                TRY(D.boolean(f));                              // :88 Parent
                if (f) {
                    pr |= HONU_HAS_PARENT;
                    TRY(D.u32(u)); R.u32(OFF(parent_pid), u);
                    TRY(D.u64(v)); R.u64(OFF(parent_vid), v);
                }
                TRY(D.boolean(f)); R.u8(OFF(tombstone), f);     // :96
                TRY(D.i64(t)); R.u64(OFF(version_created), (uint64_t)t);  // :100
            }
            TRY(D.boolean(f));                                  // :225 Schema
            if (f) {
                pr |= HONU_HAS_SCHEMA;
                TRY(D.frame(o, l)); R.span(OFF(schema_name), o, l);        // schema.go:55-73
                TRY(D.u32(u)); R.u32(OFF(schema_major), u);
                TRY(D.u32(u)); R.u32(OFF(schema_minor), u);
                TRY(D.u32(u)); R.u32(OFF(schema_patch), u);
            }
            TRY(D.frame(o, l)); R.span(OFF(mime), o, l);        // :231
            TRY(D.ulid(lo, hi)); R.bytes16(OFF(owner), lo, hi); // :235
            TRY(D.ulid(lo, hi)); R.bytes16(OFF(group), lo, hi); // :239
            TRY(D.u8(u)); R.u8(OFF(permissions), u);            // :243
            TRY(D.u64(nacl));                                   // :249
            if (nacl > 0) {                                     // :254-265
                if (nacl > GO_MAX_ALLOC / 8) TRY(HONU_ERR_PANIC);  // make([]*AccessControl)
                acl_pos = D.p;
                // acls.go:41-51. Speculate that entries are present: the next
                // 8 flags then sit at p + 18j and load independently; the walk
                // checks them in order and re-speculates after a nil entry.
                bool all_present = true;
                for (uint64_t k = 0; k < nacl;) {
                    uint32_t fl[8];
                    const uint64_t p0 = D.p;
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const uint64_t q = p0 + 18 * j;
                        fl[j] = (k + j < nacl && q < D.end) ? rec[q] : 0;
                    }
                    bool stop = false;
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        if (k < nacl && !stop) {
                            if (D.p >= D.end) TRY(HONU_ERR_EOF);     // DecodeBool
                            if (fl[j] > 1) TRY(HONU_ERR_PARSE_BOOLEAN);
                            if (fl[j]) {
                                if (D.p + 1 >= D.end) TRY(HONU_ERR_EOF);             // DecodeULID
                                if (D.p + 17 > D.end) TRY(HONU_ERR_UNEXPECTED_EOF);
                                if (D.p + 17 >= D.end) TRY(HONU_ERR_EOF);            // DecodeUint8
                                D.p += 18;
                            } else {
                                D.p += 1;
                                stop = true;
                                all_present = false;
                            }
                            k++;
                        }
                    }
                }
                R.u64(OFF(acl_count), nacl);
                if (all_present) acl_pos |= GRP_ACL_FAST;  // for the group fill
            }
            TRY(D.u64(nreg));                                   // region.go:154-169
            if (nreg > GO_MAX_ALLOC / 4) TRY(HONU_ERR_PANIC);   // make(Regions, length)
            pr |= HONU_REGIONS_NONNIL;
            reg_pos = D.p;
            for (uint64_t k = 0; k < nreg; k++) {
                TRY(D.u32(u));
                if (k < 8) reg_inline[8 * i + k] = u;
            }
            if (nreg <= 8) reg_pos |= GRP_REG_INLINE;
            R.u64(OFF(regions_count), nreg);
            TRY(D.boolean(f));                                  // :271 Publisher
            if (f) {
                pr |= HONU_HAS_PUBLISHER;
                TRY(D.ulid(lo, hi)); R.bytes16(OFF(publisher_id), lo, hi);  // provenance.go:59-79
                TRY(D.ulid(lo, hi)); R.bytes16(OFF(client_id), lo, hi);
                TRY(D.frame(o, l)); R.span(OFF(ip_address), o, l);
                TRY(D.frame(o, l)); R.span(OFF(user_agent), o, l);
            }
            TRY(D.boolean(f));                                  // :277 Encryption
            if (f) {
                pr |= HONU_HAS_ENCRYPTION;
                TRY(D.frame(o, l)); R.span(OFF(public_key_id), o, l);      // encryption.go:91-125
                TRY(D.frame(o, l)); R.span(OFF(encryption_key), o, l);
                TRY(D.frame(o, l)); R.span(OFF(hmac_secret), o, l);
                TRY(D.frame(o, l)); R.span(OFF(signature), o, l);
                TRY(D.u8(u)); R.u8(OFF(sealing_alg), u);
                TRY(D.u8(u)); R.u8(OFF(encryption_alg), u);
                TRY(D.u8(u)); R.u8(OFF(signature_alg), u);
            }
            TRY(D.boolean(f));                                  // :283 Compression
            if (f) {
                pr |= HONU_HAS_COMPRESSION;
                TRY(D.u8(u)); R.u8(OFF(compression_alg), u);    // compression.go:55-67
                TRY(D.i64(t)); R.u64(OFF(compression_level), (uint64_t)t);
            }
            TRY(D.u8(u)); R.u8(OFF(flags), u);                  // :289
            TRY(D.i64(t)); R.u64(OFF(created), (uint64_t)t);    // :293
            TRY(D.i64(t)); R.u64(OFF(modified), (uint64_t)t);   // :297
        }
        R.u32(OFF(present), pr);
    }
done:
    if (st != HONU_OK) {  // Go returns nil, err
        R.clear();
        nacl = nreg = 0;
    }
    R.store(meta + i);
    honu_record_info inf;
    inf.data_off = data_off;
    inf.data_len = data_len;
    inf.data_status = data_status;
    inf.meta_status = st;
    inf.storage_version = (uint8_t)ver;
    inf.tombstone = (v1 && d == 0) ? 1 : 0;  // Tombstone :103-112
#pragma unroll
    for (int k = 0; k < 6; k++) inf._pad[k] = 0;
    store_info(info + i, inf);
    scratch[i] = DecodeScratch{acl_pos, reg_pos, data_off, end};
    counts[3 * i + 0] = nacl;
    counts[3 * i + 1] = nreg;
    counts[3 * i + 2] = (data_len + 15) & ~15ull;
}

__global__ __launch_bounds__(HONU_BLOCK) void k_decode_parse_lane(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint32_t *__restrict__ reg_inline,
    uint64_t *__restrict__ counts) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        k_decode_parse_lane_one(i, rec, rec_off, n, meta, info, scratch, reg_inline, counts);
}

// ------------------------------------------------------------------------
// decode fill: ACL/region tables and offsets (after the count scans)
// ------------------------------------------------------------------------
HONU_DEV void k_decode_fill_lane_one(uint64_t i, const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint64_t *__restrict__ counts, const uint64_t *__restrict__ offs,
    honu_acl *__restrict__ acl, uint64_t acl_cap, uint32_t *__restrict__ reg, uint64_t reg_cap,
    uint8_t *__restrict__ data, uint64_t data_cap) {
    honu_record_info *inf = info + i;
    if (inf->meta_status == HONU_OK) {
        const uint64_t na = counts[3 * i], nr = counts[3 * i + 1];
        const uint64_t ao = offs[3 * i], ro = offs[3 * i + 1];
        if (na) meta[i].acl_off = ao;
        if (nr) meta[i].regions_off = ro;
        if (ao + na > acl_cap || ro + nr > reg_cap) {
            inf->meta_status = HONU_ERR_CAPACITY;
        } else if (na + nr) {
            const DecodeScratch sc = scratch[i];
            const uint64_t end = sc.rec_end;
            uint64_t p = sc.acl_pos & GRP_POS_MASK;
            // entries validated by the parse; speculate 8 present entries at a
            // time (flags at p + 18j) so their loads issue together
            for (uint64_t k = 0; k < na;) {
                uint32_t fl[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint64_t q = p + 18 * j;
                    fl[j] = (k + j < na && q < end) ? rec[q] : 0;
                }
                uint32_t run = 0;  // leading present entries
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (run == (uint32_t)j && fl[j] == 1 && k + j < na) run = j + 1;
                uint64_t lo[8], hi[8];
                uint32_t pm[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    if ((uint32_t)j < run) {
                        lane_fetch16(rec, p + 18 * j + 1, end, lo[j], hi[j]);
                        pm[j] = rec[p + 18 * j + 17];
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    if ((uint32_t)j < run) {
                        uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + k + j);
                        e[0] = (uint32_t)lo[j];
                        e[1] = (uint32_t)(lo[j] >> 32);
                        e[2] = (uint32_t)hi[j];
                        e[3] = (uint32_t)(hi[j] >> 32);
                        e[4] = pm[j] | (1u << 8);
                    }
                }
                k += run;
                p += 18 * (uint64_t)run;
                if (run < 8 && k < na) {  // a nil entry: one 0x00 flag byte
                    uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + k);
                    e[0] = e[1] = e[2] = e[3] = e[4] = 0;
                    k += 1;
                    p += 1;
                }
            }
            p = sc.regions_pos & GRP_POS_MASK;
            for (uint64_t k = 0; k < nr; k++) {
                const uint64_t avail = end - p;
                uint64_t lo, hi, v = 0;
                lane_fetch16(rec, p, end, lo, hi);
                const uint32_t kk = uvarint_window(lo, hi, avail < 5 ? (uint32_t)avail : 5, v);
                reg[ro + k] = (uint32_t)v;
                p += kk;
            }
        }
    }
    if (data && inf->data_status == HONU_OK && inf->data_len) {
        const uint64_t doff = offs[3 * i + 2];
        if (doff + inf->data_len > data_cap) {
            inf->data_status = HONU_ERR_CAPACITY;
            inf->data_off = 0;
            inf->data_len = 0;
        } else {
            inf->data_off = doff;
        }
    }
}

__global__ __launch_bounds__(HONU_BLOCK) void k_decode_fill_lane(
    const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint64_t *__restrict__ counts, const uint64_t *__restrict__ offs,
    honu_acl *__restrict__ acl, uint64_t acl_cap, uint32_t *__restrict__ reg, uint64_t reg_cap,
    uint8_t *__restrict__ data, uint64_t data_cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        k_decode_fill_lane_one(i, rec, n, meta, info, scratch, counts, offs, acl, acl_cap, reg, reg_cap, data, data_cap);
}

// ------------------------------------------------------------------------
// encode size pass: exact record length (object.go:24-45 / App. A)
// ------------------------------------------------------------------------
HONU_DEV void k_encode_sizes_lane_one(uint64_t i, const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    const honu_meta &m = meta[i];
    uint64_t size = 0;
    const int32_t st = encode_check(m, var_len, acl_len, reg_len);
    if (st == HONU_OK) {
        const uint64_t na = m.acl_count, ao = m.acl_off;
        uint64_t t = encode_tail_bytes_noacl(m, reg);
        for (uint64_t k0 = 0; k0 < na; k0 += 8) {  // 8 independent loads per round
            uint32_t pz[8];
#pragma unroll
            for (int j = 0; j < 8; j++) pz[j] = k0 + j < na ? acl[ao + k0 + j].present : 2;
#pragma unroll
            for (int j = 0; j < 8; j++) t += pz[j] == 2 ? 0 : (pz[j] ? 18 : 1);
        }
        const uint64_t dlen = payload_off[i + 1] - payload_off[i];
        size = 1 + uvarint_len(dlen) + dlen + t;  // object.go:30,35,40
    }
    sizes[i] = size;
    if (status) status[i] = st;
}

__global__ __launch_bounds__(HONU_BLOCK) void k_encode_sizes_lane(
    const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        k_encode_sizes_lane_one(i, meta, var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
}

// ------------------------------------------------------------------------
// encode: header + Metadata tail (object.go:24-45, metadata.go:108-200)
// ------------------------------------------------------------------------
template <bool SKIP_ACL>
HONU_DEV void k_encode_meta_lane_one(uint64_t i, const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    uint64_t *__restrict__ acl_out) {
    if (status[i] != HONU_OK) return;
    const uint64_t beg = out_off[i], end = out_off[i + 1];
    if (end > out_cap) {
        status[i] = HONU_ERR_CAPACITY;
        return;
    }
    // the whole row in registers first (loads cannot pass the output stores)
    honu_meta m;
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(meta + i);
        u32x4 *dstr = reinterpret_cast<u32x4 *>(&m);
#pragma unroll
        for (int k = 0; k < 22; k++) dstr[k] = src[k];
    }
    const uint64_t dlen = payload_off[i + 1] - payload_off[i];
    const uint64_t pos = encode_record_lane<SKIP_ACL>(m, var, acl, reg, dlen, beg, end, out);
    if constexpr (SKIP_ACL) acl_out[i] = pos;
}

template <bool SKIP_ACL>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_meta_lane(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status,
    uint64_t *__restrict__ acl_out) {
    for (uint64_t i = (uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * HONU_BLOCK)
        k_encode_meta_lane_one<SKIP_ACL>(i, meta, var, acl, reg, payload_off, n, out, out_cap, out_off, status, acl_out);
}

#undef TRY
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

hipError_t launch_decode_parse_lane(const uint8_t *rec, const uint64_t *rec_off, uint64_t n,
                                    honu_meta *meta, honu_record_info *info,
                                    DecodeScratch *scratch, uint32_t *reg_inline,
                                    uint64_t *counts, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_parse_lane, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, rec, rec_off, n,
                       meta, info, scratch, reg_inline, counts);
    return hipGetLastError();
}

hipError_t launch_decode_fill_lane(const uint8_t *rec, uint64_t n, honu_meta *meta,
                                   honu_record_info *info, const DecodeScratch *scratch,
                                   const uint64_t *counts, const uint64_t *offs, honu_acl *acl,
                                   uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap,
                                   uint8_t *data, uint64_t data_cap, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_fill_lane, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, rec, n, meta, info,
                       scratch, counts, offs, acl, acl_cap, reg, reg_cap, data, data_cap);
    return hipGetLastError();
}

hipError_t launch_encode_sizes_lane(const honu_meta *meta, uint64_t var_len, const honu_acl *acl,
                                    uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                                    const uint64_t *payload_off, uint64_t n, uint64_t *sizes,
                                    int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_sizes_lane, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, var_len,
                       acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
    return hipGetLastError();
}

}  // namespace honu

namespace honu {
hipError_t launch_encode_meta_lane(const honu_meta *meta, const uint8_t *var, const honu_acl *acl,
                                   const uint32_t *reg, const uint64_t *payload_off, uint64_t n,
                                   uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                   int32_t *status, uint64_t *acl_out, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (acl_out)
        hipLaunchKernelGGL(k_encode_meta_lane<true>, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta,
                           var, acl, reg, payload_off, n, out, out_cap, out_off, status, acl_out);
    else
        hipLaunchKernelGGL(k_encode_meta_lane<false>, lane_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta,
                           var, acl, reg, payload_off, n, out, out_cap, out_off, status, acl_out);
    return hipGetLastError();
}
}  // namespace honu
