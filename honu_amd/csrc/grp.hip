// grp.hip — the list kernels of the default path with one record per GROUP
// of 16 lanes: the encode size pass, the encoder's ACL entries and the split
// decode's table fill (the group walk and group encoder of record_variant 2
// are A/B-only: ab/grp_walk.hip).
//
// Why groups for lists: with one record per lane each load instruction
// touches 64 different cache lines, one per record; with 16 lanes per record
// the entries of a record's ACL list (20-byte rows in, 18-byte encodings out)
// and its regions spread over the group's lanes, so loads and stores of one
// instruction cover a few contiguous lines, and positions come from group
// ballots and prefix sums. The row image is staged in LDS by the group as
// aligned 16-byte loads.
#include "grp.h"

namespace honu {

#define OFF(f) ((int)offsetof(honu_meta, f))

// ------------------------------------------------------------------------
// encode size pass (object.go:24-45 / App. A), row image staged in LDS
// ------------------------------------------------------------------------
HONU_DEV bool gspan_in(uint64_t off, uint64_t len, uint64_t var_len) {
    return len == 0 || (off <= var_len && len <= var_len - off);
}
HONU_DEV uint64_t gframe_len(uint64_t len) { return uvarint_len(len) + len; }

template <int G>
HONU_DEV void k_encode_sizes_grp_one(uint64_t i, uint8_t *smem, const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    const uint32_t r = threadIdx.x & (G - 1);
    uint8_t *row = smem + (threadIdx.x / G) * (GROW + 16);
    grp_stage_row<G>(row, meta + i, r);
    wave_sync();
    const honu_meta &m = *reinterpret_cast<const honu_meta *>(row);
    const uint32_t pr = m.present;
    uint64_t size = 0;
    int32_t stc = HONU_OK;
    if (!(pr & HONU_HAS_META)) {
        stc = HONU_ERR_PANIC;  // Marshal(nil, ...): nil deref in Size(), metadata.go:66
    } else {
        bool ok = gspan_in(m.mime.off, m.mime.len, var_len);
        if (pr & HONU_HAS_SCHEMA) ok = ok && gspan_in(m.schema_name.off, m.schema_name.len, var_len);
        if (pr & HONU_HAS_PUBLISHER)
            ok = ok && gspan_in(m.ip_address.off, m.ip_address.len, var_len) &&
                 gspan_in(m.user_agent.off, m.user_agent.len, var_len);
        if (pr & HONU_HAS_ENCRYPTION)
            ok = ok && gspan_in(m.public_key_id.off, m.public_key_id.len, var_len) &&
                 gspan_in(m.encryption_key.off, m.encryption_key.len, var_len) &&
                 gspan_in(m.hmac_secret.off, m.hmac_secret.len, var_len) &&
                 gspan_in(m.signature.off, m.signature.len, var_len);
        const uint64_t na = m.acl_count, nr = m.regions_count;
        const uint64_t ao = m.acl_off, ro = m.regions_off;
        if (na) ok = ok && ao <= acl_len && na <= acl_len - ao;
        if (nr) ok = ok && ro <= reg_len && nr <= reg_len - ro;
        ok = ok && !(pr & (HONU_ACL_INPLACE | HONU_REGIONS_INPLACE));  // a decode output row: lists not in the tables
        // a carried list length (HONU_ACL_SIZED): 1..18 bytes per entry (the
        // list kernel checks it exactly against the entries)
        const bool sized = (pr & HONU_ACL_SIZED) != 0;
        if (sized) ok = ok && m.acl_bytes >= na && m.acl_bytes <= 18 * na;
        if (!ok) {
            stc = HONU_ERR_INPUT;
        } else {
            uint64_t t = 1 + 32;  // meta flag, ObjectID, CollectionID
            t += 1;               // Version flag
            if (pr & HONU_HAS_VERSION)
                t += uvarint_len(m.pid) + uvarint_len(m.vid) + uvarint_len(m.region) + 1 +
                     ((pr & HONU_HAS_PARENT) ? uvarint_len(m.parent_pid) + uvarint_len(m.parent_vid) : 0) +
                     1 + uvarint_len(zigzag(m.version_created));
            t += 1;  // Schema flag
            if (pr & HONU_HAS_SCHEMA)
                t += gframe_len(m.schema_name.len) + uvarint_len(m.schema_major) +
                     uvarint_len(m.schema_minor) + uvarint_len(m.schema_patch);
            t += gframe_len(m.mime.len) + 33;  // MIME, Owner, Group, Permissions
            t += uvarint_len(na) + uvarint_len(nr);
            uint64_t part = 0;  // this lane's share of the lists
            if (sized) t += m.acl_bytes;  // no ACL entry read
            else
                for (uint64_t k = r; k < na; k += G) part += acl[ao + k].present ? 18 : 1;
            for (uint64_t k = r; k < nr; k += G) part += uvarint_len(reg[ro + k]);
            t += 3;  // Publisher, Encryption, Compression flags
            if (pr & HONU_HAS_PUBLISHER) t += 32 + gframe_len(m.ip_address.len) + gframe_len(m.user_agent.len);
            if (pr & HONU_HAS_ENCRYPTION)
                t += gframe_len(m.public_key_id.len) + gframe_len(m.encryption_key.len) +
                     gframe_len(m.hmac_secret.len) + gframe_len(m.signature.len) + 3;
            if (pr & HONU_HAS_COMPRESSION) t += 1 + uvarint_len(zigzag(m.compression_level));
            t += 1 + uvarint_len(zigzag(m.created)) + uvarint_len(zigzag(m.modified));
            t += grp_sum64<G>(part);
            const uint64_t dlen = payload_off[i + 1] - payload_off[i];
            size = 1 + uvarint_len(dlen) + dlen + t;  // object.go:30,35,40
        }
    }
    if (r == 0) {
        sizes[i] = size;
        if (status) status[i] = stc;
    }
}

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_sizes_grp(
    const honu_meta *__restrict__ meta, uint64_t var_len, const honu_acl *__restrict__ acl,
    uint64_t acl_len, const uint32_t *__restrict__ reg, uint64_t reg_len,
    const uint64_t *__restrict__ payload_off, uint64_t n, uint64_t *__restrict__ sizes,
    int32_t *__restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t smem[GRECS * (GROW + 16)];
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_encode_sizes_grp_one<G>(i, smem, meta, var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
}

// ------------------------------------------------------------------------
// decode fill: ACL/region tables and offsets (after the count scans)
// ------------------------------------------------------------------------
template <int G>
HONU_DEV void k_decode_fill_grp_one(uint64_t i, const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint32_t *__restrict__ reg_inline, const uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ offs, honu_acl *__restrict__ acl, uint64_t acl_cap,
    uint32_t *__restrict__ reg, uint64_t reg_cap, uint8_t *__restrict__ data, uint64_t data_cap) {
    const uint32_t r = threadIdx.x & (G - 1);
    honu_record_info *inf = info + i;
    // independent loads first (one round trip)
    const int32_t mst = inf->meta_status;
    const uint64_t na = counts[3 * i], nr = counts[3 * i + 1];
    const uint64_t ao = offs[3 * i], ro = offs[3 * i + 1];
    const DecodeScratch sc = scratch[i];
    if (mst == HONU_OK) {
        if (r == 0) {
            if (na) meta[i].acl_off = ao;
            if (nr) meta[i].regions_off = ro;
        }
        if (ao + na > acl_cap || ro + nr > reg_cap) {
            if (r == 0) inf->meta_status = HONU_ERR_CAPACITY;
        } else if (na + nr) {
            const uint64_t end = sc.rec_end;
            const uint64_t ap = sc.acl_pos & GRP_POS_MASK;
            if (na && (sc.acl_pos & GRP_ACL_FAST)) {
                constexpr int K = FILL_K;  // entries per lane loaded before any store
                for (uint64_t j0 = r; j0 < na; j0 += (uint64_t)G * K) {
                    uint64_t lo[K], hi[K];
                    uint32_t pm[K];
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const uint64_t j = j0 + (uint64_t)G * k;
                        if (j < na) {
                            const uint64_t q = ap + 18 * j;
                            lane_fetch16(rec, q + 1, end, lo[k], hi[k]);
                            pm[k] = rec[q + 17];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < K; k++) {
                        const uint64_t j = j0 + (uint64_t)G * k;
                        if (j < na) {
                            uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + j);
                            e[0] = (uint32_t)lo[k];
                            e[1] = (uint32_t)(lo[k] >> 32);
                            e[2] = (uint32_t)hi[k];
                            e[3] = (uint32_t)(hi[k] >> 32);
                            e[4] = pm[k] | (1u << 8);
                        }
                    }
                }
            } else if (na && r == 0) {  // nil entries: walk (validated by the parse)
                uint64_t p = ap;
                for (uint64_t k = 0; k < na; k++) {
                    uint32_t *e = reinterpret_cast<uint32_t *>(acl + ao + k);
                    if (rec[p]) {
                        uint64_t lo, hi;
                        lane_fetch16(rec, p + 1, end, lo, hi);
                        e[0] = (uint32_t)lo;
                        e[1] = (uint32_t)(lo >> 32);
                        e[2] = (uint32_t)hi;
                        e[3] = (uint32_t)(hi >> 32);
                        e[4] = rec[p + 17] | (1u << 8);
                        p += 18;
                    } else {
                        e[0] = e[1] = e[2] = e[3] = e[4] = 0;
                        p += 1;
                    }
                }
            }
            if (nr && (sc.regions_pos & GRP_REG_INLINE)) {
                if (r < nr) reg[ro + r] = reg_inline[8 * i + r];
            } else if (nr && r == 0) {
                uint64_t p = sc.regions_pos & GRP_POS_MASK;
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
    }
    if (r == 0 && data && inf->data_status == HONU_OK && inf->data_len) {
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

template <int G>
__global__ __launch_bounds__(HONU_BLOCK) void k_decode_fill_grp(
    const uint8_t *__restrict__ rec, uint64_t n, honu_meta *__restrict__ meta,
    honu_record_info *__restrict__ info, const DecodeScratch *__restrict__ scratch,
    const uint32_t *__restrict__ reg_inline, const uint64_t *__restrict__ counts,
    const uint64_t *__restrict__ offs, honu_acl *__restrict__ acl, uint64_t acl_cap,
    uint32_t *__restrict__ reg, uint64_t reg_cap, uint8_t *__restrict__ data, uint64_t data_cap) {
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_decode_fill_grp_one<G>(i, rec, n, meta, info, scratch, reg_inline, counts, offs, acl, acl_cap, reg, reg_cap, data, data_cap);
}


// ------------------------------------------------------------------------
// encode ACL entries (metadata.go:157-162, acls.go:26-39) into the gap the
// lane encoder left at acl_pos[i]. With every entry present, output byte x of
// the list is byte (x - P) % 18 of entry (x - P) / 18 encoded as
// 01 | ClientID | Permissions, so each lane builds whole aligned 16-byte
// output chunks from the (at most) two entries they straddle: coalesced entry
// loads, one aligned store per chunk, byte stores only at the list's ends.
// A list with nil entries is written serially by the group's lead lane.
// ------------------------------------------------------------------------
// SELF: the kernel places the list itself (no acl_pos from the lane
// encoder), so it can run beside the lane encoder: the list starts after the
// header, the payload and the tail fields up to the ACL count (the size
// pass's prefix, k_encode_sizes_grp_one), and is written whole-chunk when
// every entry is present (the lane encoder's own test, lane.h).
template <int G, bool SELF>
HONU_DEV void k_encode_acl_grp_one(uint64_t i, const honu_meta *__restrict__ meta, const honu_acl *__restrict__ acl, uint64_t n,
    uint8_t *__restrict__ out, int32_t *__restrict__ status,
    const EncAclPos *__restrict__ acl_pos, const uint64_t *__restrict__ payload_off,
    const uint64_t *__restrict__ out_off, uint64_t out_cap) {
    const uint32_t r = threadIdx.x & (G - 1);
    // independent loads first: one round trip before the entries. After the
    // lane encoder (!SELF) its 32-byte hand-over holds the row fields needed
    // here, so the row itself is not read again.
    const int32_t sti = status[i];
    uint64_t na, ao, carried;
    bool sized;
    if constexpr (SELF) {
        const honu_meta &m = meta[i];
        na = m.acl_count;
        ao = m.acl_off;
        sized = (m.present & HONU_ACL_SIZED) != 0;
        carried = m.acl_bytes;
    } else {
        const EncAclPos h = acl_pos[i];
        na = h.acl_count;
        ao = h.acl_off;
        sized = (h.carried & ENC_ACL_SIZED) != 0;
        carried = h.carried & ~ENC_ACL_SIZED;
    }
    // a carried list length (HONU_ACL_SIZED) sized the record: every entry is
    // read below anyway, so the length is checked here (a row that lies gets
    // HONU_ERR_INPUT; its range of the output is then unspecified)
    uint64_t pos;
    if constexpr (SELF) {
        const honu_meta &m = meta[i];
        const uint64_t beg = out_off[i], end = out_off[i + 1];
        if (sti != HONU_OK || !na || end > out_cap) return;  // (the lane encoder flags the capacity)
        const uint32_t pr = m.present;
        uint64_t t = 1 + 32 + 1;  // meta flag, ObjectID, CollectionID, Version flag
        if (pr & HONU_HAS_VERSION)
            t += uvarint_len(m.pid) + uvarint_len(m.vid) + uvarint_len(m.region) + 1 +
                 ((pr & HONU_HAS_PARENT) ? uvarint_len(m.parent_pid) + uvarint_len(m.parent_vid) : 0) + 1 +
                 uvarint_len(zigzag(m.version_created));
        t += 1;  // Schema flag
        if (pr & HONU_HAS_SCHEMA)
            t += gframe_len(m.schema_name.len) + uvarint_len(m.schema_major) + uvarint_len(m.schema_minor) +
                 uvarint_len(m.schema_patch);
        t += gframe_len(m.mime.len) + 33 + uvarint_len(na);  // MIME, Owner, Group, Permissions, count
        const uint64_t dlen = payload_off[i + 1] - payload_off[i];
        uint64_t miss = 0;  // nil entries
        for (uint64_t k = r; k < na; k += G) miss += acl[ao + k].present ? 0 : 1;
        miss = grp_sum64<G>(miss);
        if (sized && carried != 18 * (na - miss) + miss) {
            if (r == 0) status[i] = HONU_ERR_INPUT;
            return;
        }
        pos = (beg + 1 + uvarint_len(dlen) + dlen + t) | (miss == 0 ? ACL_ALL_PRESENT : 0);
    } else {
        if (sti != HONU_OK || !na) return;
        pos = acl_pos[i].pos;
    }
    const honu_acl *A = acl + ao;
    const uint64_t P = pos & ~ACL_ALL_PRESENT;
    if (!SELF && sized) {  // the lane encoder laid the list out by the carried length
        uint64_t miss = 0;  // (the lines the chunks below read anyway)
        for (uint64_t k = r; k < na; k += G) miss += A[k].present ? 0 : 1;
        miss = grp_sum64<G>(miss);
        if (carried != 18 * (na - miss) + miss) {
            if (r == 0) status[i] = HONU_ERR_INPUT;
            return;
        }
    }
    if (pos & ACL_ALL_PRESENT) {  // whole chunks [ceil16(P), floor16(E))
        // whole ACL_UNIT units on absolute addresses (lane.h writes the ends)
        const uint64_t ab = (uint64_t)out;
        const uint64_t X0 = ((ab + P + ACL_UNIT - 1) & ~(ACL_UNIT - 1)) - ab,
                       X1 = ((ab + P + 18 * na) & ~(ACL_UNIT - 1)) - ab;
        if constexpr (HONU_ACL_ENDS && ACL_UNIT == 16) {
            // the partial chunks at both ends ([P, X0) and [X1, E): fewer than
            // 16 bytes each; a list is >= 18 bytes, so X0 <= X1), byte stores by
            // two lanes of the group
            const uint64_t E = P + 18 * na;
            const uint64_t x = r == 0 ? P : X1;
            const uint32_t cnt = (uint32_t)(r == 0 ? X0 - P : E - X1);
            if (r < 2 && cnt) {
                const u32x4 v = acl_chunk(A, na, P, x);
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (uint32_t b = 0; b < 15; b++)
                    if (b < cnt) out[x + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
            }
        }
        if (X1 <= X0) return;
        const uint64_t nch = (X1 - X0) >> 4;
        constexpr int K = 2;  // chunks per lane computed before any store
        for (uint64_t c0 = r; c0 < nch; c0 += (uint64_t)G * K) {
            u32x4 v[K];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint64_t c = c0 + (uint64_t)G * k;
                if (c < nch) v[k] = acl_chunk(A, na, P, X0 + 16 * c);
            }
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint64_t c = c0 + (uint64_t)G * k;
                if (c < nch) *reinterpret_cast<u32x4 *>(out + X0 + 16 * c) = v[k];
            }
        }
        return;
    }
    if (r == 0) {  // nil entries: 00 for a nil entry, else 01 | ClientID | Permissions
        uint64_t p = P;
        for (uint64_t j = 0; j < na; j++) {
            if (A[j].present) {
                uint32_t d[5];
                acl_enc_words(A + j, d);
                for (int b = 0; b < 18; b++) out[p + b] = (uint8_t)(d[b >> 2] >> (8 * (b & 3)));
                p += 18;
            } else {
                out[p++] = 0;
            }
        }
    }
}

template <int G, bool SELF>
__global__ __launch_bounds__(HONU_BLOCK) void k_encode_acl_grp(
    const honu_meta *__restrict__ meta, const honu_acl *__restrict__ acl, uint64_t n,
    uint8_t *__restrict__ out, int32_t *__restrict__ status,
    const EncAclPos *__restrict__ acl_pos, const uint64_t *__restrict__ payload_off,
    const uint64_t *__restrict__ out_off, uint64_t out_cap) {
    for (uint64_t i = ((uint64_t)blockIdx.x * HONU_BLOCK + threadIdx.x) / G; i < n;
         i += (uint64_t)gridDim.x * (HONU_BLOCK / G))
        k_encode_acl_grp_one<G, SELF>(i, meta, acl, n, out, status, acl_pos, payload_off, out_off, out_cap);
}

#undef OFF

hipError_t launch_encode_sizes_grp(const honu_meta *meta, uint64_t var_len, const honu_acl *acl,
                                   uint64_t acl_len, const uint32_t *reg, uint64_t reg_len,
                                   const uint64_t *payload_off, uint64_t n, uint64_t *sizes,
                                   int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_encode_sizes_grp<GRP>, grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta,
                       var_len, acl, acl_len, reg, reg_len, payload_off, n, sizes, status);
    return hipGetLastError();
}

hipError_t launch_encode_acl_grp(const honu_meta *meta, const honu_acl *acl, uint64_t n,
                                 uint8_t *out, int32_t *status, const EncAclPos *acl_pos,
                                 int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((k_encode_acl_grp<GRP, false>), grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, acl,
                       n, out, status, acl_pos, nullptr, nullptr, 0);
    return hipGetLastError();
}

hipError_t launch_encode_acl_grp_self(const honu_meta *meta, const honu_acl *acl, const uint64_t *payload_off,
                                      uint64_t n, uint8_t *out, uint64_t out_cap, const uint64_t *out_off,
                                      int32_t *status, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL((k_encode_acl_grp<GRP, true>), grp_grid(n, max_blocks), dim3(HONU_BLOCK), 0, s, meta, acl,
                       n, out, status, nullptr, payload_off, out_off, out_cap);
    return hipGetLastError();
}

hipError_t launch_decode_fill_grp(const uint8_t *rec, uint64_t n, honu_meta *meta,
                                  honu_record_info *info, const DecodeScratch *scratch,
                                  const uint32_t *reg_inline, const uint64_t *counts,
                                  const uint64_t *offs, honu_acl *acl, uint64_t acl_cap,
                                  uint32_t *reg, uint64_t reg_cap, uint8_t *data,
                                  uint64_t data_cap, int max_blocks, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t b = (n * FILL_G + HONU_BLOCK - 1) / HONU_BLOCK;
    const dim3 grid((unsigned)(max_blocks > 0 && b > (uint64_t)max_blocks ? (uint64_t)max_blocks : b));
    hipLaunchKernelGGL(k_decode_fill_grp<FILL_G>, grid, dim3(HONU_BLOCK), 0, s, rec, n, meta,
                       info, scratch, reg_inline, counts, offs, acl, acl_cap, reg, reg_cap, data,
                       data_cap);
    return hipGetLastError();
}

}  // namespace honu
