// put_feed.cpp — the write feed (include/honu_codec.h, "Write feed"): the
// batching a store's Put path needs in front of the GPU encoder. In the
// reference every Put marshals one record on the calling goroutine
// (object.Marshal, object.go:24-45, called from store.go:226,530 and the
// tests); here records are appended into pinned memory (row + the bytes its
// spans and lists reference, compacted, + payload) and each submitted batch
// is copied to the device, marshalled (sizes, scan, header + Metadata tails,
// payload copy) and copied back on its own stream while the next batch fills.
//
// Two slots, as the read feed (feed.cpp). The encoded records come back by a
// D2H copy sized by an upper bound of the batch's encoded bytes that append()
// keeps (kFixedBound below), so submit() never has to wait for the size pass.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/honu_codec.h"
#include "host_copy.h"

namespace {

enum SlotState { FREE = 0, INFLIGHT = 1, DONE = 2 };

// Upper bound of the Metadata tail + object header beyond the bytes that
// append() counts separately (span bytes, payload, 18 per ACL entry, 5 per
// region): 1+10 header, 1 nil flag, 32 ObjectID/CollectionID, Version 48
// (flag, PID 5, VID 10, Region 5, Parent flag+15, Tombstone 1, time 10),
// Schema 26 (flag, frame length 10, 3 x 5), MIME length 10, Owner/Group/
// Permissions 33, ACL count 10, Regions count 10, Publisher 53 (flag, 2
// ULIDs, 2 frame lengths), Encryption 44 (flag, 4 frame lengths, 3 enums),
// Compression 12, Flags 1, Created/Modified 20 (metadata.go:108-200).
constexpr uint64_t kFixedBound = 12 + 32 + 48 + 26 + 10 + 33 + 10 + 10 + 53 + 44 + 12 + 1 + 20;

struct Slot {
    honu_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    // pinned host inputs
    honu_meta *h_meta = nullptr;
    uint8_t *h_var = nullptr;
    honu_acl *h_acl = nullptr;
    uint32_t *h_reg = nullptr;
    uint8_t *h_pay = nullptr;
    uint64_t *h_poff = nullptr;
    // pinned host outputs
    uint8_t *h_out = nullptr;
    uint64_t *h_ooff = nullptr;
    int32_t *h_st = nullptr;
    // device
    honu_meta *d_meta = nullptr;
    uint8_t *d_var = nullptr;
    honu_acl *d_acl = nullptr;
    uint32_t *d_reg = nullptr;
    uint8_t *d_pay = nullptr;
    uint64_t *d_poff = nullptr;
    uint8_t *d_out = nullptr;
    uint64_t *d_ooff = nullptr;
    int32_t *d_st = nullptr;
    // fill
    uint64_t n = 0, var = 0, acl = 0, reg = 0, pay = 0, budget = 0, bound = 0;
    uint64_t ticket = 0;
    SlotState state = FREE;
};

}  // namespace

struct honu_put_feed {
    int device = 0;
    uint64_t cap_n = 0, cap_bytes = 0, acl_cap = 0, reg_cap = 0, out_cap = 0;
    Slot slot[2];
    int cur = 0;
    uint64_t next_ticket = 1;
};

#define PCHK(x)                                   \
    do {                                          \
        if ((x) != hipSuccess) return HONU_E_HIP; \
    } while (0)

static void put_slot_free(Slot &s) {
    if (s.ctx) honu_ctx_destroy(s.ctx);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    void *host[] = {s.h_meta, s.h_var, s.h_acl, s.h_reg, s.h_pay, s.h_poff, s.h_out, s.h_ooff, s.h_st};
    for (void *p : host)
        if (p) (void)hipHostFree(p);
    void *dev[] = {s.d_meta, s.d_var, s.d_acl, s.d_reg, s.d_pay, s.d_poff, s.d_out, s.d_ooff, s.d_st};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    s = Slot();
}

static int32_t put_slot_alloc(honu_put_feed *f, Slot &s) {
    int32_t err = HONU_OK;
    s.ctx = honu_ctx_create(f->device, f->cap_n, &err);
    if (!s.ctx) return err ? err : HONU_E_HIP;
    PCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    const uint64_t n = f->cap_n, b = f->cap_bytes + 16;
    const uint64_t sz_meta = sizeof(honu_meta) * n, sz_acl = sizeof(honu_acl) * f->acl_cap + 16;
    const uint64_t sz_reg = 4 * f->reg_cap + 16, sz_off = 8 * (n + 1), sz_out = f->out_cap + 16;
    PCHK(hipHostMalloc((void **)&s.h_meta, sz_meta, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_var, b, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_acl, sz_acl, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_reg, sz_reg, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_pay, b, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_poff, sz_off, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_out, sz_out, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_ooff, sz_off, hipHostMallocDefault));
    PCHK(hipHostMalloc((void **)&s.h_st, 4 * n + 16, hipHostMallocDefault));
    PCHK(hipMalloc((void **)&s.d_meta, sz_meta));
    PCHK(hipMalloc((void **)&s.d_var, b));
    PCHK(hipMalloc((void **)&s.d_acl, sz_acl));
    PCHK(hipMalloc((void **)&s.d_reg, sz_reg));
    PCHK(hipMalloc((void **)&s.d_pay, b));
    PCHK(hipMalloc((void **)&s.d_poff, sz_off));
    PCHK(hipMalloc((void **)&s.d_out, sz_out));
    PCHK(hipMalloc((void **)&s.d_ooff, sz_off));
    PCHK(hipMalloc((void **)&s.d_st, 4 * n + 16));
    s.h_poff[0] = 0;
    return HONU_OK;
}

honu_put_feed *honu_put_feed_create(int device, uint64_t batch_records, uint64_t batch_bytes,
                                    int32_t *err) {
    int32_t dummy;
    if (!err) err = &dummy;
    *err = HONU_OK;
    if (!batch_records || !batch_bytes) {
        *err = HONU_E_ARG;
        return nullptr;
    }
    honu_put_feed *f = new honu_put_feed();
    f->device = device;
    f->cap_n = batch_records;
    f->cap_bytes = batch_bytes;
    // every input byte (span bytes, payload, 20 per ACL entry, 4 per region)
    // counts against batch_bytes, so these tables can never overflow
    f->acl_cap = batch_bytes / sizeof(honu_acl) + 1;
    f->reg_cap = batch_bytes / 4 + 1;
    // Σ put_bound: input bytes + 1 per region (5-byte varints for 4 counted
    // bytes) + kFixedBound per record
    f->out_cap = batch_bytes + batch_bytes / 4 + kFixedBound * batch_records;
    if (hipSetDevice(device) != hipSuccess) {
        *err = HONU_E_NO_DEVICE;
        delete f;
        return nullptr;
    }
    for (Slot &s : f->slot) {
        const int32_t st = put_slot_alloc(f, s);
        if (st != HONU_OK) {
            *err = st;
            honu_put_feed_destroy(f);
            return nullptr;
        }
    }
    return f;
}

void honu_put_feed_destroy(honu_put_feed *f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    for (Slot &s : f->slot) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        put_slot_free(s);
    }
    delete f;
}

static Slot *put_filling(honu_put_feed *f, int32_t *err) {
    Slot &s = f->slot[f->cur];
    if (s.state == INFLIGHT) {
        *err = HONU_E_ARG;  // its batch was submitted and not waited for
        return nullptr;
    }
    if (s.state == DONE) {
        s.state = FREE;
        s.n = s.var = s.acl = s.reg = s.pay = s.budget = s.bound = 0;
        s.h_poff[0] = 0;
    }
    return &s;
}

// The spans a row's present sub-structs reference (absent ones are ignored by
// the encoder, metadata.go:120-179, and zeroed here).
static void live_spans(const honu_meta &r, honu_span *out[8], bool live[8], honu_meta &w) {
    out[0] = &w.schema_name;
    out[1] = &w.mime;
    out[2] = &w.ip_address;
    out[3] = &w.user_agent;
    out[4] = &w.public_key_id;
    out[5] = &w.encryption_key;
    out[6] = &w.hmac_secret;
    out[7] = &w.signature;
    const uint32_t p = r.present;
    live[0] = p & HONU_HAS_SCHEMA;
    live[1] = true;
    live[2] = live[3] = p & HONU_HAS_PUBLISHER;
    live[4] = live[5] = live[6] = live[7] = p & HONU_HAS_ENCRYPTION;
}

// A record's placement: what append() checks and counts before any byte
// moves (phase 1), then where its bytes go in the slot (phase 2).
struct PutPlan {
    honu_meta w;  // the row, absent sub-structs' spans zeroed
    uint64_t span_bytes = 0, nacl = 0, nreg = 0, need = 0, bound = 0;
    uint64_t var_at = 0, acl_at = 0, reg_at = 0, pay_at = 0;  // slot positions
};

// Phase 1: validate the row's spans and lists against the caller's arrays
// and size the record (HONU_ERR_INPUT: nothing may be appended).
static int32_t put_plan(const honu_put_feed *f, const honu_meta *row, const uint8_t *var,
                        uint64_t var_len, const honu_acl *acl, uint64_t acl_len,
                        const uint32_t *regions, uint64_t regions_len, uint64_t data_len,
                        PutPlan &p) {
    p.w = *row;
    honu_span *spans[8];
    bool live[8];
    live_spans(*row, spans, live, p.w);
    p.span_bytes = p.nacl = p.nreg = 0;
    if (row->present & HONU_HAS_META) {
        for (int k = 0; k < 8; k++) {
            if (!live[k]) {
                *spans[k] = honu_span{0, 0};
                continue;
            }
            const honu_span sv = *spans[k];
            if (sv.len && (!var || sv.off > var_len || sv.len > var_len - sv.off)) return HONU_ERR_INPUT;
            p.span_bytes += sv.len;
        }
        if (row->present & (HONU_ACL_INPLACE | HONU_REGIONS_INPLACE))
            return HONU_ERR_INPUT;  // a decode output row (table forms only)
        p.nacl = row->acl_count;
        p.nreg = row->regions_count;
        if (p.nacl && (!acl || row->acl_off > acl_len || p.nacl > acl_len - row->acl_off))
            return HONU_ERR_INPUT;
        if (p.nreg && (!regions || row->regions_off > regions_len || p.nreg > regions_len - row->regions_off))
            return HONU_ERR_INPUT;
    } else {  // Marshal(nil, data): the encoder reports HONU_ERR_PANIC
        for (int k = 0; k < 8; k++) *spans[k] = honu_span{0, 0};
        p.w.acl_count = p.w.regions_count = 0;
    }
    if (p.nacl > f->cap_bytes / sizeof(honu_acl) || p.nreg > f->cap_bytes / 4) return HONU_ERR_CAPACITY;
    p.need = p.span_bytes + data_len + sizeof(honu_acl) * p.nacl + 4 * p.nreg;
    p.bound = kFixedBound + p.span_bytes + data_len + 18 * p.nacl + 5 * p.nreg;
    return HONU_OK;
}

// Phase 2: copy the referenced bytes to the plan's slot positions, compacted,
// and store the rebased row as record `idx` of the slot.
static void put_fill(Slot &s, uint64_t idx, const PutPlan &p, const honu_meta *row,
                     const uint8_t *var, const honu_acl *acl, const uint32_t *regions,
                     const uint8_t *data, uint64_t data_len) {
    honu_meta w = p.w;
    honu_span *spans[8];
    bool live[8];
    live_spans(w, spans, live, w);
    uint64_t at = p.var_at;
    for (int k = 0; k < 8; k++) {
        honu_span &sv = *spans[k];
        if (!sv.len) {
            sv.off = 0;
            continue;
        }
        std::memcpy(s.h_var + at, var + sv.off, sv.len);
        sv.off = at;
        at += sv.len;
    }
    if (p.nacl) std::memcpy(s.h_acl + p.acl_at, acl + row->acl_off, sizeof(honu_acl) * p.nacl);
    if (p.nreg) std::memcpy(s.h_reg + p.reg_at, regions + row->regions_off, 4 * p.nreg);
    if (p.nacl && !(w.present & HONU_ACL_SIZED)) {
        // the list's encoded length, from the entries just copied (HONU_ACL_SIZED:
        // the size pass then reads no ACL entry; a row that carries one keeps it)
        uint64_t nb = 0;
        for (uint64_t j = 0; j < p.nacl; j++) nb += acl[row->acl_off + j].present ? 18 : 1;
        w.acl_bytes = nb;
        w.present |= HONU_ACL_SIZED;
    }
    w.acl_off = p.nacl ? p.acl_at : 0;
    w.regions_off = p.nreg ? p.reg_at : 0;
    if (data_len) std::memcpy(s.h_pay + p.pay_at, data, data_len);
    s.h_meta[idx] = w;
    s.h_poff[idx + 1] = p.pay_at + data_len;
}

// Reserve the plan's positions at the slot's fill point.
static void put_place(Slot &s, PutPlan &p, uint64_t data_len) {
    p.var_at = s.var;
    p.acl_at = s.acl;
    p.reg_at = s.reg;
    p.pay_at = s.pay;
    s.var += p.span_bytes;
    s.acl += p.nacl;
    s.reg += p.nreg;
    s.pay += data_len;
    s.budget += p.need;
    s.bound += p.bound;
    s.n += 1;
}

int32_t honu_put_feed_append(honu_put_feed *f, const honu_meta *row, const uint8_t *var,
                             uint64_t var_len, const honu_acl *acl, uint64_t acl_len,
                             const uint32_t *regions, uint64_t regions_len, const uint8_t *data,
                             uint64_t data_len) {
    if (!f || !row || (data_len && !data)) return HONU_E_ARG;
    int32_t err = HONU_OK;
    Slot *sp = put_filling(f, &err);
    if (!sp) return err;
    Slot &s = *sp;
    PutPlan p;
    err = put_plan(f, row, var, var_len, acl, acl_len, regions, regions_len, data_len, p);
    if (err) return err;
    if (s.n == f->cap_n || p.need > f->cap_bytes - s.budget) return HONU_ERR_CAPACITY;
    const uint64_t idx = s.n;
    put_place(s, p, data_len);
    put_fill(s, idx, p, row, var, acl, regions, data, data_len);
    return HONU_OK;
}

int32_t honu_put_feed_append_batch(honu_put_feed *f, const honu_meta *rows, uint64_t n,
                                   const uint8_t *var, uint64_t var_len, const honu_acl *acl,
                                   uint64_t acl_len, const uint32_t *regions, uint64_t regions_len,
                                   const uint8_t *payload, const uint64_t *payload_off,
                                   uint64_t *appended) {
    if (!f || (n && (!rows || !payload_off)) || !appended) return HONU_E_ARG;
    *appended = 0;
    int32_t st = HONU_OK;
    Slot *sp = put_filling(f, &st);
    if (!sp) return st;
    Slot &s = *sp;
    // phase 1, serial: check and place every record that goes in
    std::vector<PutPlan> plans;
    plans.reserve(n < f->cap_n - s.n ? n : f->cap_n - s.n);
    const uint64_t first = s.n;
    uint64_t bytes = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t a = payload_off[i], b = payload_off[i + 1];
        if (b < a || (b > a && !payload)) {
            st = b < a ? HONU_ERR_INPUT : HONU_E_ARG;
            break;
        }
        PutPlan p;
        st = put_plan(f, rows + i, var, var_len, acl, acl_len, regions, regions_len, b - a, p);
        if (st) break;
        if (s.n == f->cap_n || p.need > f->cap_bytes - s.budget) {
            st = HONU_ERR_CAPACITY;
            break;
        }
        put_place(s, p, b - a);
        plans.push_back(p);
        bytes += p.need;
    }
    // phase 2: the copies, record ranges over a few threads for big batches
    const uint64_t k = plans.size();
    auto fill = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; i++) {
            const uint64_t a = payload_off[i], b = payload_off[i + 1];
            put_fill(s, first + i, plans[i], rows + i, var, acl, regions,
                     payload ? payload + a : nullptr, b - a);
        }
    };
    const unsigned T = bytes >= honu::kParallelCopyMin && k > 1 ? honu::host_copy_threads() : 1;
    if (T == 1) {
        fill(0, k);
    } else {  // equal-byte record ranges
        std::vector<uint64_t> cuts{0};
        uint64_t acc = 0, t = 1;
        for (uint64_t i = 0; i < k && t < T; i++) {
            acc += plans[i].need;
            if (acc >= bytes * t / T) {
                cuts.push_back(i + 1);
                t++;
            }
        }
        cuts.push_back(k);
        std::vector<std::thread> pool;
        for (size_t c = 1; c + 1 < cuts.size(); c++) pool.emplace_back(fill, cuts[c], cuts[c + 1]);
        fill(cuts[0], cuts[1]);
        for (std::thread &th : pool) th.join();
    }
    *appended = k;
    return st;
}

uint64_t honu_put_feed_pending(const honu_put_feed *f) {
    if (!f) return 0;
    const Slot &s = f->slot[f->cur];
    return s.state == FREE ? s.n : 0;
}

int32_t honu_put_feed_submit(honu_put_feed *f, uint64_t *ticket) {
    if (!f) return HONU_E_ARG;
    int32_t err = HONU_OK;
    Slot *sp = put_filling(f, &err);
    if (!sp) return err;
    Slot &s = *sp;
    PCHK(hipSetDevice(f->device));
    const uint64_t n = s.n;
    hipStream_t q = s.stream;
    PCHK(hipMemcpyAsync(s.d_poff, s.h_poff, 8 * (n + 1), hipMemcpyHostToDevice, q));
    if (n) PCHK(hipMemcpyAsync(s.d_meta, s.h_meta, sizeof(honu_meta) * n, hipMemcpyHostToDevice, q));
    if (s.var) PCHK(hipMemcpyAsync(s.d_var, s.h_var, s.var, hipMemcpyHostToDevice, q));
    if (s.acl) PCHK(hipMemcpyAsync(s.d_acl, s.h_acl, sizeof(honu_acl) * s.acl, hipMemcpyHostToDevice, q));
    if (s.reg) PCHK(hipMemcpyAsync(s.d_reg, s.h_reg, 4 * s.reg, hipMemcpyHostToDevice, q));
    if (s.pay) PCHK(hipMemcpyAsync(s.d_pay, s.h_pay, s.pay, hipMemcpyHostToDevice, q));
    err = honu_marshal_batch(s.ctx, s.d_meta, s.d_var, s.var, s.d_acl, s.acl, s.d_reg, s.reg,
                             s.d_pay, s.d_poff, n, s.d_out, f->out_cap, s.d_ooff, s.d_st, q);
    if (err) return err;
    PCHK(hipMemcpyAsync(s.h_ooff, s.d_ooff, 8 * (n + 1), hipMemcpyDeviceToHost, q));
    if (n) PCHK(hipMemcpyAsync(s.h_st, s.d_st, 4 * n, hipMemcpyDeviceToHost, q));
    // the bound, not the exact total: known now, so nothing waits here
    if (s.bound) PCHK(hipMemcpyAsync(s.h_out, s.d_out, s.bound, hipMemcpyDeviceToHost, q));
    s.state = INFLIGHT;
    s.ticket = f->next_ticket++;
    if (ticket) *ticket = s.ticket;
    f->cur ^= 1;
    return HONU_OK;
}

int32_t honu_put_feed_wait(honu_put_feed *f, uint64_t ticket, honu_put_result *out) {
    if (!f || !out) return HONU_E_ARG;
    Slot *sp = nullptr;
    for (Slot &s : f->slot)
        if (s.state != FREE && s.ticket == ticket) sp = &s;
    if (!sp) return HONU_E_ARG;
    Slot &s = *sp;
    PCHK(hipSetDevice(f->device));
    if (s.state == INFLIGHT) {
        PCHK(hipStreamSynchronize(s.stream));
        s.state = DONE;
    }
    out->n = s.n;
    out->records = s.h_out;
    out->rec_off = s.h_ooff;
    out->status = s.h_st;
    return HONU_OK;
}
