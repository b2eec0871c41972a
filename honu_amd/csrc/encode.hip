// encode.hip — object.Marshal over a batch on gfx950 (object/object.go:24-45).
//
// A record is  01 | uvarint(len data) | data | 01 | Metadata   (SURVEY App. A).
// The work splits by what bounds it:
//   k_encode_sizes : one wave per record, exact encoded length (no bytes moved
//                    but the ~1 KB row + list entries it reads).
//   k_encode_meta  : one wave per record, writes the header and builds the
//                    Metadata tail (metadata.go:108-200) in LDS at the phase of
//                    its global destination, then flushes it with aligned
//                    16-byte stores. Lists (ACL, regions) are laid out with a
//                    wave prefix scan over per-entry sizes, one entry per lane.
//   k_copy_segments: (copy.hip) the payload bytes, split evenly by bytes over
//                    all waves — the HBM-bound part.
#include "kernels.h"

namespace honu {

// ------------------------------------------------------------------------
// Tail layout: byte sizes of the Metadata encoding, computed identically by
// the size pass and the writer (all values wave-uniform).
// ------------------------------------------------------------------------
struct TailSizes {
    uint64_t version;     // EncodeStruct(Version)        metadata.go:120
    uint64_t schema;      // EncodeStruct(Schema)         :125
    uint64_t acl;         // uvarint(len) + entries       :151-162
    uint64_t regions;     // Regions.Encode               :164
    uint64_t total;       // whole EncodeStruct(meta) incl. its nil flag
};

HONU_DEV bool span_ok(honu_span s, uint64_t var_len) {
    return s.len == 0 || (s.off <= var_len && s.len <= var_len - s.off);
}
HONU_DEV uint64_t frame_size(uint64_t len) { return uvarint_len(len) + len; }

// ACL entry sizes: 1 (nil flag) or 18 (flag + ULID + permissions), acls.go:26-39.
HONU_DEV uint64_t acl_list_size(const honu_acl *__restrict__ acl, uint64_t off, uint64_t count) {
    uint64_t s = 0;
    for (uint64_t base = 0; base < count; base += HONU_WAVE) {
        const uint64_t k = base + lane_id();
        uint32_t sz = 0;
        if (k < count) sz = acl[off + k].present ? 18u : 1u;
        s += wave_sum(sz);
    }
    return uvarint_len(count) + s;
}

// Regions.Encode: uvarint(count) + uvarint32 per region (region.go:137-152).
HONU_DEV uint64_t region_list_size(const uint32_t *__restrict__ reg, uint64_t off, uint64_t count) {
    uint64_t s = 0;
    for (uint64_t base = 0; base < count; base += HONU_WAVE) {
        const uint64_t k = base + lane_id();
        uint32_t sz = 0;
        if (k < count) sz = uvarint_len(reg[off + k]);
        s += wave_sum(sz);
    }
    return uvarint_len(count) + s;
}

// Returns false when a span or list lies outside its arena (HONU_ERR_INPUT).
HONU_DEV bool tail_sizes(const honu_meta *__restrict__ m, uint64_t var_len,
                         const honu_acl *__restrict__ acl, uint64_t acl_len,
                         const uint32_t *__restrict__ reg, uint64_t reg_len, TailSizes &t) {
    const uint32_t pr = m->present;
    bool ok = span_ok(m->mime, var_len);
    if (pr & HONU_HAS_SCHEMA) ok = ok && span_ok(m->schema_name, var_len);
    if (pr & HONU_HAS_PUBLISHER)
        ok = ok && span_ok(m->ip_address, var_len) && span_ok(m->user_agent, var_len);
    if (pr & HONU_HAS_ENCRYPTION)
        ok = ok && span_ok(m->public_key_id, var_len) && span_ok(m->encryption_key, var_len) &&
             span_ok(m->hmac_secret, var_len) && span_ok(m->signature, var_len);
    const uint64_t na = m->acl_count, nr = m->regions_count;
    if (na) ok = ok && m->acl_off <= acl_len && na <= acl_len - m->acl_off;
    if (nr) ok = ok && m->regions_off <= reg_len && nr <= reg_len - m->regions_off;
    if (!ok) return false;

    t.version = 1;
    if (pr & HONU_HAS_VERSION) {
        // Scalar (scalar.go:106-119), Region (version.go:51), Parent, Tombstone, Created
        t.version += uvarint_len(m->pid) + uvarint_len(m->vid) + uvarint_len(m->region) + 1 +
                     ((pr & HONU_HAS_PARENT) ? uvarint_len(m->parent_pid) + uvarint_len(m->parent_vid) : 0) +
                     1 + uvarint_len(zigzag(m->version_created));
    }
    t.schema = 1;
    if (pr & HONU_HAS_SCHEMA)  // schema.go:30-53
        t.schema += frame_size(m->schema_name.len) + uvarint_len(m->schema_major) +
                    uvarint_len(m->schema_minor) + uvarint_len(m->schema_patch);
    t.acl = acl_list_size(acl, m->acl_off, na);
    t.regions = region_list_size(reg, m->regions_off, nr);
    uint64_t publisher = 1, encryption = 1, compression = 1;
    if (pr & HONU_HAS_PUBLISHER)  // provenance.go:34-57
        publisher += 32 + frame_size(m->ip_address.len) + frame_size(m->user_agent.len);
    if (pr & HONU_HAS_ENCRYPTION)  // encryption.go:51-89
        encryption += frame_size(m->public_key_id.len) + frame_size(m->encryption_key.len) +
                      frame_size(m->hmac_secret.len) + frame_size(m->signature.len) + 3;
    if (pr & HONU_HAS_COMPRESSION)  // compression.go:40-53
        compression += 1 + uvarint_len(zigzag(m->compression_level));
    t.total = 1 /*meta flag*/ + 32 /*oid, collection*/ + t.version + t.schema +
              frame_size(m->mime.len) + 33 /*owner, group, permissions*/ + t.acl + t.regions +
              publisher + encryption + compression + 1 /*flags*/ +
              uvarint_len(zigzag(m->created)) + uvarint_len(zigzag(m->modified));
    return true;
}

// ------------------------------------------------------------------------
// size pass
// ------------------------------------------------------------------------
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_sizes(
    const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    for (uint64_t r = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wave_in_block(); r < n;
         r += nwaves) {
        const honu_meta *m = meta + r;
        uint64_t size = 0;
        int32_t st = HONU_OK;
        if (!(m->present & HONU_HAS_META)) {
            st = HONU_ERR_PANIC;  // Marshal(nil, ...) -> nil deref in Size(), metadata.go:66
        } else {
            TailSizes t;
            if (!tail_sizes(m, var_len, acl, acl_len, reg, reg_len, t)) {
                st = HONU_ERR_INPUT;
            } else {
                const uint64_t dlen = payload_off[r + 1] - payload_off[r];
                size = 1 + uvarint_len(dlen) + dlen + t.total;  // object.go:30,35,40
            }
        }
        if (lane_id() == 0) {
            sizes[r] = size;
            if (status) status[r] = st;
        }
    }
}

// ------------------------------------------------------------------------
// tail writer
// ------------------------------------------------------------------------
// Writes the Metadata encoding through T (LDS in the fast path, the global
// destination in the fallback). Scalars are written by lane 0; byte runs
// (ULIDs, frames) and list entries by all lanes. `o` stays wave-uniform.
struct TailWriter {
    uint8_t *T;
    uint64_t o;

    HONU_DEV void byte(uint8_t v) {
        if (lane_id() == 0) T[o] = v;
        o += 1;
    }
    HONU_DEV void uv(uint64_t v) {
        if (lane_id() == 0) put_uvarint(T + o, v);
        o += uvarint_len(v);
    }
    HONU_DEV void bytes(const uint8_t *__restrict__ src, uint64_t n) {
        wave_copy_bytes(T + o, src, n);
        o += n;
    }
    HONU_DEV void frame(const uint8_t *__restrict__ var, honu_span s) {  // lani Encode :62-77
        uv(s.len);
        bytes(var + s.off, s.len);
    }
};

HONU_DEV void write_tail(TailWriter &w, const honu_meta *__restrict__ m,
                         const uint8_t *__restrict__ var, const honu_acl *__restrict__ acl,
                         const uint32_t *__restrict__ reg) {
    const uint32_t pr = m->present;
    const uint32_t lane = lane_id();
    w.byte(1);                                   // EncodeStruct(meta) flag
    w.bytes(m->object_id, 16);                   // metadata.go:110
    w.bytes(m->collection_id, 16);               // :115
    if (pr & HONU_HAS_VERSION) {                 // :120, version.go:44-70
        w.byte(1);
        w.uv(m->pid);
        w.uv(m->vid);
        w.uv(m->region);
        if (pr & HONU_HAS_PARENT) {
            w.byte(1);
            w.uv(m->parent_pid);
            w.uv(m->parent_vid);
        } else {
            w.byte(0);
        }
        w.byte(m->tombstone ? 1 : 0);
        w.uv(zigzag(m->version_created));
    } else {
        w.byte(0);
    }
    if (pr & HONU_HAS_SCHEMA) {                  // :125, schema.go:30-53
        w.byte(1);
        w.frame(var, m->schema_name);
        w.uv(m->schema_major);
        w.uv(m->schema_minor);
        w.uv(m->schema_patch);
    } else {
        w.byte(0);
    }
    w.frame(var, m->mime);                       // :130
    w.bytes(m->owner, 16);                       // :135
    w.bytes(m->group, 16);                       // :140
    w.byte(m->permissions);                      // :145
    // ACL (:151-162): one entry per lane, offsets by a wave prefix scan.
    const uint64_t na = m->acl_count;
    w.uv(na);
    for (uint64_t base = 0; base < na; base += HONU_WAVE) {
        const uint64_t k = base + lane;
        uint32_t sz = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0;
        if (k < na) {
            const uint32_t *a = reinterpret_cast<const uint32_t *>(acl + m->acl_off + k);
            w0 = a[0]; w1 = a[1]; w2 = a[2]; w3 = a[3]; w4 = a[4];
            sz = ((w4 >> 8) & 0xff) ? 18u : 1u;
        }
        const uint32_t incl = wave_inclusive_scan32(sz);
        if (k < na) {
            uint8_t *e = w.T + w.o + (incl - sz);
            if (sz == 1) {
                e[0] = 0;
            } else {
                e[0] = 1;
                const uint32_t ws[4] = {w0, w1, w2, w3};
#pragma unroll
                for (int j = 0; j < 16; j++) e[1 + j] = (uint8_t)(ws[j >> 2] >> (8 * (j & 3)));
                e[17] = (uint8_t)w4;
            }
        }
        w.o += readlane32(incl, 63);
    }
    // Regions (region.go:137-152): one region per lane.
    const uint64_t nr = m->regions_count;
    w.uv(nr);
    for (uint64_t base = 0; base < nr; base += HONU_WAVE) {
        const uint64_t k = base + lane;
        uint32_t v = 0, sz = 0;
        if (k < nr) {
            v = reg[m->regions_off + k];
            sz = uvarint_len(v);
        }
        const uint32_t incl = wave_inclusive_scan32(sz);
        if (k < nr) put_uvarint(w.T + w.o + (incl - sz), v);
        w.o += readlane32(incl, 63);
    }
    if (pr & HONU_HAS_PUBLISHER) {               // :169, provenance.go:34-57
        w.byte(1);
        w.bytes(m->publisher_id, 16);
        w.bytes(m->client_id, 16);
        w.frame(var, m->ip_address);
        w.frame(var, m->user_agent);
    } else {
        w.byte(0);
    }
    if (pr & HONU_HAS_ENCRYPTION) {              // :174, encryption.go:51-89
        w.byte(1);
        w.frame(var, m->public_key_id);
        w.frame(var, m->encryption_key);
        w.frame(var, m->hmac_secret);
        w.frame(var, m->signature);
        w.byte(m->sealing_alg);
        w.byte(m->encryption_alg);
        w.byte(m->signature_alg);
    } else {
        w.byte(0);
    }
    if (pr & HONU_HAS_COMPRESSION) {             // :179, compression.go:40-53
        w.byte(1);
        w.byte(m->compression_alg);
        w.uv(zigzag(m->compression_level));
    } else {
        w.byte(0);
    }
    w.byte(m->flags);                            // :184
    w.uv(zigzag(m->created));                    // :189 EncodeTime
    w.uv(zigzag(m->modified));                   // :194
}

// Flush T[phase, phase+len) (LDS, 16-aligned base) to dst (global, dst % 16 ==
// phase): edge chunks byte-wise, interior chunks as aligned 16-byte stores.
HONU_DEV void flush_lds(uint8_t *__restrict__ dst, const uint8_t *T, uint32_t phase,
                        uint64_t len) {
    const uint32_t lane = lane_id();
    uint64_t head = (16u - phase) & 15u;
    if (head > len) head = len;
    if (lane < head) dst[lane] = T[phase + lane];
    const uint64_t rest = len - head;
    const uint64_t chunks = rest >> 4;
    const u32x4 *T4 = reinterpret_cast<const u32x4 *>(T + phase + head);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst + head);
    for (uint64_t c = lane; c < chunks; c += HONU_WAVE) d4[c] = T4[c];
    const uint64_t tail = rest & 15u;
    const uint64_t t0 = head + (chunks << 4);
    if (lane < tail) dst[t0 + lane] = T[phase + t0 + lane];
}

__global__ __launch_bounds__(HONU_BLOCK) void k_encode_meta(
    const honu_meta *__restrict__ meta, const uint8_t *__restrict__ var,
    const honu_acl *__restrict__ acl, const uint32_t *__restrict__ reg,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint8_t *__restrict__ out,
    uint64_t out_cap, const uint64_t *__restrict__ out_off, int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[HONU_WAVES_PER_BLOCK][ENC_TAIL_LDS];
    const uint32_t wib = wave_in_block();
    uint8_t *T = lds[wib];
    const uint64_t nwaves = (uint64_t)gridDim.x * HONU_WAVES_PER_BLOCK;
    for (uint64_t r = (uint64_t)blockIdx.x * HONU_WAVES_PER_BLOCK + wib; r < n; r += nwaves) {
        if (status[r] != HONU_OK) continue;
        const uint64_t beg = out_off[r], end = out_off[r + 1];
        if (end > out_cap) {
            if (lane_id() == 0) status[r] = HONU_ERR_CAPACITY;
            continue;
        }
        const honu_meta *m = meta + r;
        const uint64_t dlen = payload_off[r + 1] - payload_off[r];
        const uint32_t hlen = 1 + uvarint_len(dlen);
        if (lane_id() == 0) {                    // object.go:30,35 (frame length)
            out[beg] = HONU_STORAGE_VERSION;
            put_uvarint(out + beg + 1, dlen);
        }
        const uint64_t tstart = beg + hlen + dlen;
        const uint64_t tlen = end - tstart;
        const uint32_t phase = (uint32_t)(((uint64_t)out + tstart) & 15u);
        if (tlen + phase <= ENC_TAIL_LDS) {
            TailWriter w{T + phase, 0};
            write_tail(w, m, var, acl, reg);
            wave_sync();
            flush_lds(out + tstart, T, phase, tlen);
            wave_sync();                         // T is reused by the next record
        } else {
            TailWriter w{out + tstart, 0};       // oversized tail: write in place
            write_tail(w, m, var, acl, reg);
        }
    }
}

}  // namespace honu

// ------------------------------------------------------------------------
// launch wrappers
// ------------------------------------------------------------------------
namespace honu {

static int record_blocks(const LaunchGeom &g, uint64_t n) {
    uint64_t b = (n + HONU_WAVES_PER_BLOCK - 1) / HONU_WAVES_PER_BLOCK;
    if (b > (uint64_t)g.per_record_blocks) b = g.per_record_blocks;
    return b ? (int)b : 1;
}

hipError_t launch_encode_sizes(const LaunchGeom &g, const honu_meta *meta, uint64_t var_len,
                               const honu_acl *acl, uint64_t acl_len, const uint32_t *reg,
                               uint64_t reg_len, const uint64_t *payload_off, uint64_t n,
                               uint64_t *sizes, int32_t *status, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_sizes, dim3(record_blocks(g, n)), dim3(HONU_BLOCK), 0, s, meta,
                       var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
    return hipGetLastError();
}

hipError_t launch_encode_meta(const LaunchGeom &g, const honu_meta *meta, const uint8_t *var,
                              const honu_acl *acl, const uint32_t *reg,
                              const uint64_t *payload_off, uint64_t n, uint8_t *out,
                              uint64_t out_cap, const uint64_t *out_off, int32_t *status,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_meta, dim3(record_blocks(g, n)), dim3(HONU_BLOCK), 0, s, meta,
                       var, acl, reg, payload_off, n, out, out_cap, out_off, status);
    return hipGetLastError();
}

}  // namespace honu
