// decode.hip — Object.Metadata() + Object.Data() over a batch on gfx950
// (object/object.go:66-99, lani/decode.go, metadata/*.go Decode methods).
//
//   k_decode_parse: one wave per record. The header and dataLength window
//       (object.go:114-134) are read with one lane per byte; the Metadata tail
//       (which starts right after the payload, so the payload itself is never
//       read) is staged into a per-wave LDS window with 16-byte loads and
//       walked field by field with Go's exact varint/frame/error semantics.
//       The walk is inherently serial (every field position depends on the
//       previous varint), so all 64 lanes execute it in lockstep on
//       wave-uniform values; LDS reads at a uniform address broadcast.
//       The decoded row is assembled in LDS and leaves with coalesced
//       16-byte stores. Frames come out as zero-copy spans into the input
//       (like lani.DecodeFixed / Object.Data()).
//   k_decode_fill: one wave per record, after the exclusive scans of the
//       per-record list counts: writes ACL/region table entries and offsets,
//       and the materialised-payload offsets (payload bytes: copy.hip).
#include "kernels.h"

namespace honu {

#define GO_MAX_ALLOC (1ull << 48)  // runtime maxAlloc, linux/amd64

// ------------------------------------------------------------------------
// LDS window over one record's bytes
// ------------------------------------------------------------------------
struct Win {
    uint8_t *L;           // per-wave LDS buffer, DEC_WIN bytes, 16-aligned
    const uint8_t *rec;   // arena base (16-aligned)
    uint64_t lo, hi, end; // window [lo, hi) absolute; record end

    HONU_DEV void load(uint64_t p) {
        wave_sync();  // earlier LDS reads of this wave have retired
        lo = p & ~15ull;
        uint64_t h = lo + DEC_WIN;
        hi = h < end ? h : end;
        const uint64_t nch = (hi - lo + 15) >> 4;
        const u32x4 *s = reinterpret_cast<const u32x4 *>(rec + lo);
        u32x4 *d = reinterpret_cast<u32x4 *>(L);
        for (uint64_t c = lane_id(); c < nch; c += HONU_WAVE) d[c] = s[c];
        wave_sync();
    }
    // make [p, min(p+n, end)) readable
    HONU_DEV void ensure(uint64_t p, uint64_t n) {
        uint64_t need = p + n;
        if (need > end) need = end;
        if (p < lo || need > hi) load(p);
    }
    HONU_DEV uint8_t at(uint64_t p) const { return L[p - lo]; }
};

// lani.Decoder over [tstart, end) with the cursor as an absolute offset.
struct Dec {
    Win w;
    uint64_t p;       // cursor (absolute)
    uint64_t tstart;  // decoder buffer start: o[1+d+b:] (object.go:77)

    // binary.Uvarint over the window [p, min(p+maxw, end)); err on k <= 0.
    HONU_DEV int uvarint(uint32_t maxw, int err, uint64_t &v) {
        if (p >= w.end) return HONU_ERR_EOF;
        uint64_t j = p + maxw;
        if (j > w.end) j = w.end;
        const uint32_t n = (uint32_t)(j - p);
        w.ensure(p, n);
        uint64_t x = 0;
        uint32_t s = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t b = w.at(p + i);
            if (b < 0x80) {
                if (i == 9 && b > 1) return err;  // overflow
                v = x | ((uint64_t)b << s);
                p += i + 1;
                return HONU_OK;
            }
            x |= (uint64_t)(b & 0x7f) << s;
            s += 7;
        }
        return err;  // buffer too small
    }
    HONU_DEV int u8(uint8_t &v) {  // DecodeByte decode.go:94-103
        if (p >= w.end) return HONU_ERR_EOF;
        w.ensure(p, 1);
        v = w.at(p);
        p += 1;
        return HONU_OK;
    }
    HONU_DEV int boolean(bool &v) {  // DecodeBool :105-120
        uint8_t c;
        int st = u8(c);
        if (st) return st;
        if (c > 1) return HONU_ERR_PARSE_BOOLEAN;
        v = c == 1;
        return HONU_OK;
    }
    HONU_DEV int u32(uint32_t &v) {  // DecodeUint32 :127-146 (5-byte window)
        uint64_t x;
        int st = uvarint(5, HONU_ERR_PARSE_VARINT, x);
        v = (uint32_t)x;
        return st;
    }
    HONU_DEV int u64(uint64_t &v) { return uvarint(10, HONU_ERR_PARSE_VARINT, v); }  // :149-168
    HONU_DEV int i64(int64_t &v) {                                                  // :171-190
        uint64_t x;
        int st = uvarint(10, HONU_ERR_PARSE_VARINT, x);
        v = unzigzag(x);
        return st;
    }
    // DecodeULID :209-221, copied into the LDS row image at R[off..off+16).
    HONU_DEV int ulid(uint8_t *R, uint32_t off) {
        if (p >= w.end) return HONU_ERR_EOF;
        if (p + 16 > w.end) return HONU_ERR_UNEXPECTED_EOF;
        w.ensure(p, 16);
        const uint32_t l = lane_id();
        if (l < 16) R[off + l] = w.at(p + l);
        p += 16;
        return HONU_OK;
    }
    HONU_DEV int skip_ulid() {
        if (p >= w.end) return HONU_ERR_EOF;
        if (p + 16 > w.end) return HONU_ERR_UNEXPECTED_EOF;
        p += 16;
        return HONU_OK;
    }
    // Decode :30-56 with readLength :261-282, as a zero-copy span.
    HONU_DEV int frame(honu_span &sp) {
        uint64_t rl;
        int st = uvarint(10, HONU_ERR_NO_LENGTH, rl);
        if (st) return st;
        if (rl >= (1ull << 63)) return HONU_ERR_PANIC;  // int(rl) < 0 -> makeslice
        if (rl == 0) {
            sp.off = 0;
            sp.len = 0;
            return HONU_OK;
        }
        const uint64_t di = p - tstart;  // d.i
        if (rl > (uint64_t)INT64_MAX - di) return HONU_ERR_PANIC;  // j overflows
        if (p + rl > w.end) return HONU_ERR_UNEXPECTED_EOF;
        sp.off = p;
        sp.len = rl;
        p += rl;
        return HONU_OK;
    }
};

#define TRY(x)              \
    do {                    \
        st = (x);           \
        if (st) goto done;  \
    } while (0)

#define ROWF(field) (reinterpret_cast<honu_meta *>(R)->field)
#define SET(field, v)                    \
    do {                                 \
        if (lane == 0) ROWF(field) = (v); \
    } while (0)

__global__ __launch_bounds__(HONU_BLOCK) void k_decode_parse(
    const uint8_t *__restrict__ rec, const uint64_t *__restrict__ rec_off, uint64_t n,
    honu_meta *__restrict__ meta, honu_record_info *__restrict__ info,
    DecodeScratch *__restrict__ scratch, uint64_t *__restrict__ counts) {
    __shared__ __attribute__((aligned(16))) uint8_t win_lds[HONU_WAVES_PER_BLOCK][DEC_WIN];
    __shared__ __attribute__((aligned(16))) uint8_t row_lds[HONU_WAVES_PER_BLOCK][sizeof(honu_meta)];
    const uint32_t wib = wave_in_block();
    const uint32_t lane = lane_id();
    uint8_t *R = row_lds[wib];
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;

    for (uint64_t r = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wib; r < n; r += nwaves) {
        const uint64_t beg = rec_off[r], end = rec_off[r + 1];
        const uint64_t len = end - beg;
        // Header bytes o[0..11): one lane per byte.
        uint32_t hb = 0;
        if (lane < 11 && lane < len) hb = rec[beg + lane];
        const uint8_t ver = len ? (uint8_t)readlane32(hb, 0) : 0;  // StorageVersion :47-52
        // dataLength :114-134: Uvarint(o[1 : min(11, len-1)])
        int64_t d = -1, b = -1;
        if (len >= 2) {
            const uint32_t wl = (uint32_t)((len - 1 < 11 ? len - 1 : 11) - 1);
            // continuation bits of o[1..1+wl)
            const uint64_t cont = __ballot(lane >= 1 && lane <= wl && (hb & 0x80));
            const uint64_t inwin = wl ? ((wl >= 63 ? ~0ull : ((1ull << (wl + 1)) - 1)) & ~1ull) : 0ull;
            const uint64_t term = inwin & ~cont;  // terminal bytes in the window
            if (term) {
                const uint32_t t = __builtin_ctzll(term);  // lane of the last byte
                const uint32_t k = t;                     // bytes consumed (1-based lanes)
                // Go: overflow if the 10th byte (i == 9) is > 1
                const uint32_t last = readlane32(hb, t);
                if (!(k == 10 && last > 1)) {
                    uint64_t x = 0;
                    for (uint32_t i = 1; i <= t; i++)
                        x |= (uint64_t)(readlane32(hb, i) & 0x7f) << (7 * (i - 1));
                    d = (int64_t)x;
                    b = k;
                }
            }
        }
        const bool v1 = ver == HONU_STORAGE_VERSION;
        int32_t data_status, meta_status;
        uint64_t data_off = 0, data_len = 0;
        const bool in_range = d >= 0 && (uint64_t)d <= len - 1 - (uint64_t)b;
        if (!v1) data_status = HONU_ERR_BAD_VERSION;
        else if (d < 0) data_status = HONU_ERR_MALFORMED;
        else if (d == 0) data_status = HONU_OK;
        else if (!in_range) data_status = HONU_ERR_PANIC;  // o[1+b:1+b+d] out of range
        else {
            data_status = HONU_OK;
            data_off = beg + 1 + (uint64_t)b;
            data_len = (uint64_t)d;
        }

        // zero the row image
        if (lane < sizeof(honu_meta) / 16) reinterpret_cast<u32x4 *>(R)[lane] = u32x4{0, 0, 0, 0};
        wave_sync();
        uint64_t nacl = 0, nreg = 0, acl_pos = 0, reg_pos = 0;
        int st = HONU_OK;
        if (!v1) st = HONU_ERR_BAD_VERSION;
        else if (d < 0) st = HONU_ERR_MALFORMED;
        else if (!in_range) st = HONU_ERR_PANIC;  // o[1+d+b:]
        else {
            Dec D;
            D.w.L = win_lds[wib];
            D.w.rec = rec;
            D.w.end = end;
            D.tstart = beg + 1 + (uint64_t)b + (uint64_t)d;
            D.p = D.tstart;
            D.w.lo = 1;  // empty window: forces the first load
            D.w.hi = 0;
            bool present;
            uint32_t pr = 0;
            TRY(D.boolean(present));  // DecodeStruct(meta) object.go:78
            if (present) {
                pr = HONU_HAS_META;
                TRY(D.ulid(R, offsetof(honu_meta, object_id)));      // metadata.go:210
                TRY(D.ulid(R, offsetof(honu_meta, collection_id)));  // :214
                TRY(D.boolean(present));                             // :219 Version
                if (present) {
                    pr |= HONU_HAS_VERSION;
                    uint32_t u;
                    uint64_t v;
                    int64_t t;
                    TRY(D.u32(u)); SET(pid, u);                       // scalar.go:121-131
                    TRY(D.u64(v)); SET(vid, v);
                    TRY(D.u32(u)); SET(region, u);                    // version.go:80
                    TRY(D.boolean(present));                          // :88 Parent
                    if (present) {
                        pr |= HONU_HAS_PARENT;
                        TRY(D.u32(u)); SET(parent_pid, u);
                        TRY(D.u64(v)); SET(parent_vid, v);
                    }
                    TRY(D.boolean(present)); SET(tombstone, (uint8_t)present);  // :96
                    TRY(D.i64(t)); SET(version_created, t);           // :100
                }
                TRY(D.boolean(present));                             // :225 Schema
                if (present) {
                    pr |= HONU_HAS_SCHEMA;
                    honu_span sp;
                    uint32_t u;
                    TRY(D.frame(sp)); SET(schema_name, sp);           // schema.go:55-73
                    TRY(D.u32(u)); SET(schema_major, u);
                    TRY(D.u32(u)); SET(schema_minor, u);
                    TRY(D.u32(u)); SET(schema_patch, u);
                }
                {
                    honu_span sp;
                    TRY(D.frame(sp)); SET(mime, sp);                  // :231
                }
                TRY(D.ulid(R, offsetof(honu_meta, owner)));          // :235
                TRY(D.ulid(R, offsetof(honu_meta, group)));          // :239
                {
                    uint8_t c;
                    TRY(D.u8(c)); SET(permissions, c);                // :243
                }
                TRY(D.u64(nacl));                                    // :249
                if (nacl > 0) {                                      // :254-265
                    if (nacl > GO_MAX_ALLOC / 8) TRY(HONU_ERR_PANIC);  // make([]*AccessControl)
                    acl_pos = D.p;
                    for (uint64_t i = 0; i < nacl; i++) {
                        TRY(D.boolean(present));
                        if (present) {
                            uint8_t c;
                            TRY(D.skip_ulid());                       // acls.go:41-51
                            TRY(D.u8(c));
                        }
                    }
                    SET(acl_count, nacl);
                }
                TRY(D.u64(nreg));                                    // region.go:154-169
                if (nreg > GO_MAX_ALLOC / 4) TRY(HONU_ERR_PANIC);     // make(Regions, length)
                pr |= HONU_REGIONS_NONNIL;
                reg_pos = D.p;
                for (uint64_t i = 0; i < nreg; i++) {
                    uint32_t u;
                    TRY(D.u32(u));
                }
                SET(regions_count, nreg);
                TRY(D.boolean(present));                             // :271 Publisher
                if (present) {
                    pr |= HONU_HAS_PUBLISHER;
                    honu_span sp;
                    TRY(D.ulid(R, offsetof(honu_meta, publisher_id)));  // provenance.go:59-79
                    TRY(D.ulid(R, offsetof(honu_meta, client_id)));
                    TRY(D.frame(sp)); SET(ip_address, sp);
                    TRY(D.frame(sp)); SET(user_agent, sp);
                }
                TRY(D.boolean(present));                             // :277 Encryption
                if (present) {
                    pr |= HONU_HAS_ENCRYPTION;
                    honu_span sp;
                    uint8_t c;
                    TRY(D.frame(sp)); SET(public_key_id, sp);         // encryption.go:91-125
                    TRY(D.frame(sp)); SET(encryption_key, sp);
                    TRY(D.frame(sp)); SET(hmac_secret, sp);
                    TRY(D.frame(sp)); SET(signature, sp);
                    TRY(D.u8(c)); SET(sealing_alg, c);
                    TRY(D.u8(c)); SET(encryption_alg, c);
                    TRY(D.u8(c)); SET(signature_alg, c);
                }
                TRY(D.boolean(present));                             // :283 Compression
                if (present) {
                    pr |= HONU_HAS_COMPRESSION;
                    uint8_t c;
                    int64_t t;
                    TRY(D.u8(c)); SET(compression_alg, c);            // compression.go:55-67
                    TRY(D.i64(t)); SET(compression_level, t);
                }
                {
                    uint8_t c;
                    int64_t t;
                    TRY(D.u8(c)); SET(flags, c);                      // :289
                    TRY(D.i64(t)); SET(created, t);                   // :293
                    TRY(D.i64(t)); SET(modified, t);                  // :297
                }
            }
            SET(present, pr);
        }
    done:
        meta_status = st;
        wave_sync();
        {
            u32x4 *dst = reinterpret_cast<u32x4 *>(meta + r);
            if (lane < sizeof(honu_meta) / 16)
                dst[lane] = st == HONU_OK ? reinterpret_cast<const u32x4 *>(R)[lane]
                                          : u32x4{0, 0, 0, 0};  // Go: nil, err
        }
        if (st != HONU_OK) nacl = nreg = 0;
        if (lane == 0) {
            honu_record_info inf;
            inf.data_off = data_off;
            inf.data_len = data_len;
            inf.data_status = data_status;
            inf.meta_status = meta_status;
            inf.storage_version = ver;
            inf.tombstone = (v1 && d == 0) ? 1 : 0;  // Tombstone :103-112
#pragma unroll
            for (int i = 0; i < 6; i++) inf._pad[i] = 0;
            store_info(info + r, inf);
            scratch[r] = DecodeScratch{acl_pos, reg_pos, data_off, end};
            counts[3 * r + 0] = nacl;
            counts[3 * r + 1] = nreg;
            counts[3 * r + 2] = (data_len + 15) & ~15ull;
        }
        wave_sync();  // row image and window are reused by the next record
    }
}
#undef TRY
#undef SET
#undef ROWF

// ------------------------------------------------------------------------
// fill: list tables, list offsets and materialised-payload offsets
// ------------------------------------------------------------------------
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_fill(
    const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint64_t *__restrict__ counts, const uint64_t *__restrict__ offs,
    honu_acl *__restrict__ acl, uint64_t acl_cap, uint32_t *__restrict__ reg, uint64_t reg_cap,
    uint8_t *__restrict__ data, uint64_t data_cap) {
    __shared__ __attribute__((aligned(16))) uint8_t win_lds[HONU_WAVES_PER_BLOCK][DEC_WIN];
    const uint32_t wib = wave_in_block();
    const uint32_t lane = lane_id();
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    for (uint64_t r = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wib; r < n; r += nwaves) {
        honu_record_info *inf = info + r;
        if (inf->meta_status == HONU_OK) {
            const uint64_t na = counts[3 * r], nr = counts[3 * r + 1];
            const uint64_t ao = offs[3 * r], ro = offs[3 * r + 1];
            if (lane == 0) {
                if (na) meta[r].acl_off = ao;
                if (nr) meta[r].regions_off = ro;
            }
            if (ao + na > acl_cap || ro + nr > reg_cap) {
                if (lane == 0) inf->meta_status = HONU_ERR_CAPACITY;
            } else if (na + nr) {
                const DecodeScratch sc = scratch[r];
                Win w;
                w.L = win_lds[wib];
                w.rec = rec;
                const uint64_t lists_end = (sc.regions_pos & GRP_POS_MASK) + 5 * nr;  // never past the lists
                w.end = lists_end < sc.rec_end ? lists_end : sc.rec_end;
                w.lo = 1;
                w.hi = 0;
                uint64_t p = sc.acl_pos & GRP_POS_MASK;
                for (uint64_t i = 0; i < na; i++) {  // entries validated by the parse
                    w.ensure(p, 18);
                    const uint8_t flag = w.at(p);
                    uint8_t *e = reinterpret_cast<uint8_t *>(acl + ao + i);
                    if (lane < 20) {
                        uint8_t v = 0;
                        if (flag) {
                            if (lane < 16) v = w.at(p + 1 + lane);
                            else if (lane == 16) v = w.at(p + 17);
                            else if (lane == 17) v = 1;
                        }
                        e[lane] = v;
                    }
                    p += flag ? 18 : 1;
                }
                p = sc.regions_pos & GRP_POS_MASK;
                for (uint64_t i = 0; i < nr; i++) {
                    w.ensure(p, 5);
                    uint64_t x = 0;
                    uint32_t s = 0, k = 0;
                    for (; k < 5; k++) {
                        const uint32_t bb = (p + k < w.end) ? w.at(p + k) : 0;
                        x |= (uint64_t)(bb & 0x7f) << s;
                        s += 7;
                        if (bb < 0x80) break;
                    }
                    if (lane == 0) reg[ro + i] = (uint32_t)x;
                    p += k + 1;
                }
                wave_sync();
            }
        }
        if (data && inf->data_status == HONU_OK && inf->data_len) {
            const uint64_t doff = offs[3 * r + 2];
            if (lane == 0) {
                if (doff + inf->data_len > data_cap) {
                    inf->data_status = HONU_ERR_CAPACITY;
                    inf->data_off = 0;
                    inf->data_len = 0;
                } else {
                    inf->data_off = doff;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------
// keys: Object.Key() -> keys.New(ObjectID, &Version.Scalar) (keys.go:42-51)
// ------------------------------------------------------------------------
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_keys(const honu_meta *__restrict__ meta,
                                                            const honu_record_info *__restrict__ info,
                                                            uint64_t n, uint8_t *__restrict__ keys,
                                                            int32_t *__restrict__ key_status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const honu_meta &m = meta[i];
    int32_t st = info[i].meta_status;
    if (st == HONU_OK && !(m.present & HONU_HAS_VERSION)) st = HONU_ERR_PANIC;  // metadata.go:54
    uint8_t *k = keys + HONU_KEY_LEN * i;
    if (st == HONU_OK) {
        k[0] = 0x01;  // keyVersion keys.go:18
        for (int j = 0; j < 16; j++) k[1 + j] = m.object_id[j];
        for (int j = 0; j < 8; j++) k[17 + j] = (uint8_t)(m.vid >> (56 - 8 * j));  // BE64(VID)
        for (int j = 0; j < 4; j++) k[25 + j] = (uint8_t)(m.pid >> (24 - 8 * j));  // BE32(PID)
    } else {
        for (int j = 0; j < HONU_KEY_LEN; j++) k[j] = 0;
    }
    if (key_status) key_status[i] = st;
}

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
static int record_blocks(const LaunchGeom &g, uint64_t n) {
    uint64_t b = (n + HONU_WAVES_PER_BLOCK - 1) / HONU_WAVES_PER_BLOCK;
    if (b > (uint64_t)g.per_record_blocks) b = g.per_record_blocks;
    return b ? (int)b : 1;
}

hipError_t launch_decode_parse(const LaunchGeom &g, const uint8_t *rec, const uint64_t *rec_off,
                               uint64_t n, honu_meta *meta, honu_record_info *info,
                               DecodeScratch *scratch, uint64_t *counts, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_parse, dim3(record_blocks(g, n)), dim3(HONU_BLOCK), 0, s, rec,
                       rec_off, n, meta, info, scratch, counts);
    return hipGetLastError();
}

hipError_t launch_decode_fill(const LaunchGeom &g, const uint8_t *rec, uint64_t n,
                              honu_meta *meta, honu_record_info *info,
                              const DecodeScratch *scratch, const uint64_t *counts,
                              const uint64_t *offs, const uint64_t *totals, honu_acl *acl,
                              uint64_t acl_cap, uint32_t *reg, uint64_t reg_cap, uint8_t *data,
                              uint64_t data_cap, hipStream_t s) {
    (void)totals;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_fill, dim3(record_blocks(g, n)), dim3(HONU_BLOCK), 0, s, rec, n,
                       meta, info, scratch, counts, offs, acl, acl_cap, reg, reg_cap, data,
                       data_cap);
    return hipGetLastError();
}

hipError_t launch_decode_keys(const LaunchGeom &g, const honu_meta *meta,
                              const honu_record_info *info, uint64_t n, uint8_t *keys,
                              int32_t *key_status, hipStream_t s) {
    (void)g;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_decode_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, meta,
                       info, n, keys, key_status);
    return hipGetLastError();
}

}  // namespace honu
