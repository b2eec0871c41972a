// feed.cpp — the read feed (include/honu_codec.h, "Read feed"): the batching
// a bbolt cursor scan needs in front of the GPU codec (iterator/cursor.go:
// 31-38 copies each value out of the mmap; here the copy lands in pinned
// memory, and a batch is decoded while the next one fills).
//
// Two slots. Each owns pinned host buffers (records, offsets, results), device
// buffers, a HIP stream and a codec context (contexts hold per-stream
// scratch). submit() enqueues on the slot's stream: H2D of the records and
// offsets, honu_decode_batch (zero copy) or honu_decode_headers, keys, and the
// D2H of rows, info, keys and table totals; wait() synchronises and copies the
// ACL / region tables by their totals.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "../../include/honu_codec.h"
#include "host_copy.h"

using honu::host_copy;

namespace {

enum SlotState { FREE = 0, INFLIGHT = 1, DONE = 2 };

struct Slot {
    honu_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    // pinned host
    uint8_t *h_rec = nullptr;
    uint64_t *h_off = nullptr;
    honu_meta *h_meta = nullptr;
    honu_record_info *h_info = nullptr;
    honu_acl *h_acl = nullptr;
    uint32_t *h_reg = nullptr;
    uint8_t *h_keys = nullptr;
    int32_t *h_kst = nullptr;
    uint64_t *h_tot = nullptr;
    // device
    uint8_t *d_rec = nullptr;
    uint64_t *d_off = nullptr;
    honu_meta *d_meta = nullptr;
    honu_record_info *d_info = nullptr;
    honu_acl *d_acl = nullptr;
    uint32_t *d_reg = nullptr;
    uint8_t *d_keys = nullptr;
    int32_t *d_kst = nullptr;
    uint64_t *d_tot = nullptr;
    uint64_t n = 0, bytes = 0, ticket = 0;
    SlotState state = FREE;
};

}  // namespace

struct honu_feed {
    int device = 0;
    uint32_t flags = 0;
    uint64_t cap_n = 0, cap_bytes = 0;
    uint64_t acl_cap = 0, reg_cap = 0;  // entries: every entry takes >= 1 record byte
    Slot slot[2];
    int cur = 0;
    uint64_t next_ticket = 1;
};

#define FCHK(x)                                  \
    do {                                         \
        if ((x) != hipSuccess) return HONU_E_HIP; \
    } while (0)

static void slot_free(Slot &s) {
    if (s.ctx) honu_ctx_destroy(s.ctx);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    void *host[] = {s.h_rec, s.h_off, s.h_meta, s.h_info, s.h_acl, s.h_reg, s.h_keys, s.h_kst,
                    s.h_tot};
    for (void *p : host)
        if (p) (void)hipHostFree(p);
    void *dev[] = {s.d_rec, s.d_off, s.d_meta, s.d_info, s.d_acl, s.d_reg, s.d_keys, s.d_kst,
                   s.d_tot};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    s = Slot();
}

static int32_t slot_alloc(honu_feed *f, Slot &s) {
    int32_t err = HONU_OK;
    s.ctx = honu_ctx_create(f->device, f->cap_n, &err);
    if (!s.ctx) return err ? err : HONU_E_HIP;
    FCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    const uint64_t n = f->cap_n, b = f->cap_bytes + 16;
    FCHK(hipHostMalloc((void **)&s.h_rec, b, hipHostMallocDefault));
    FCHK(hipHostMalloc((void **)&s.h_off, 8 * (n + 1), hipHostMallocDefault));
    FCHK(hipHostMalloc((void **)&s.h_info, sizeof(honu_record_info) * n, hipHostMallocDefault));
    FCHK(hipHostMalloc((void **)&s.h_tot, 32, hipHostMallocDefault));
    FCHK(hipMalloc((void **)&s.d_rec, b));
    FCHK(hipMalloc((void **)&s.d_off, 8 * (n + 1)));
    FCHK(hipMalloc((void **)&s.d_info, sizeof(honu_record_info) * n));
    FCHK(hipMalloc((void **)&s.d_tot, 32));
    if (!(f->flags & HONU_FEED_HEADERS)) {
        FCHK(hipHostMalloc((void **)&s.h_meta, sizeof(honu_meta) * n, hipHostMallocDefault));
        FCHK(hipHostMalloc((void **)&s.h_acl, sizeof(honu_acl) * f->acl_cap, hipHostMallocDefault));
        FCHK(hipHostMalloc((void **)&s.h_reg, 4 * f->reg_cap, hipHostMallocDefault));
        FCHK(hipHostMalloc((void **)&s.h_keys, (uint64_t)HONU_KEY_LEN * n, hipHostMallocDefault));
        FCHK(hipHostMalloc((void **)&s.h_kst, 4 * n, hipHostMallocDefault));
        FCHK(hipMalloc((void **)&s.d_meta, sizeof(honu_meta) * n));
        FCHK(hipMalloc((void **)&s.d_acl, sizeof(honu_acl) * f->acl_cap));
        FCHK(hipMalloc((void **)&s.d_reg, 4 * f->reg_cap));
        FCHK(hipMalloc((void **)&s.d_keys, (uint64_t)HONU_KEY_LEN * n));
        FCHK(hipMalloc((void **)&s.d_kst, 4 * n));
    }
    s.h_off[0] = 0;
    return HONU_OK;
}

honu_feed *honu_feed_create(int device, uint64_t batch_records, uint64_t batch_bytes,
                            uint32_t flags, int32_t *err) {
    int32_t dummy;
    if (!err) err = &dummy;
    *err = HONU_OK;
    if (!batch_records || !batch_bytes) {
        *err = HONU_E_ARG;
        return nullptr;
    }
    honu_feed *f = new honu_feed();
    f->device = device;
    f->flags = flags;
    f->cap_n = batch_records;
    f->cap_bytes = batch_bytes;
    // table capacities (entries): a present ACL entry takes 18 record bytes, a
    // region 1-5; batches of nil-entry floods report HONU_ERR_CAPACITY per
    // record rather than overflow
    f->acl_cap = batch_bytes / 8 + 1024;
    f->reg_cap = batch_bytes / 4 + 1024;
    if (hipSetDevice(device) != hipSuccess) {
        *err = HONU_E_NO_DEVICE;
        delete f;
        return nullptr;
    }
    for (Slot &s : f->slot) {
        const int32_t st = slot_alloc(f, s);
        if (st != HONU_OK) {
            *err = st;
            honu_feed_destroy(f);
            return nullptr;
        }
    }
    return f;
}

void honu_feed_destroy(honu_feed *f) {
    if (!f) return;
    (void)hipSetDevice(f->device);
    for (Slot &s : f->slot) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        slot_free(s);
    }
    delete f;
}

// the filling slot, made writable (a waited-for batch is released here)
static Slot *filling(honu_feed *f, int32_t *err) {
    Slot &s = f->slot[f->cur];
    if (s.state == INFLIGHT) {
        *err = HONU_E_ARG;  // its batch was submitted and not waited for
        return nullptr;
    }
    if (s.state == DONE) {
        s.state = FREE;
        s.n = s.bytes = 0;
        s.h_off[0] = 0;
    }
    return &s;
}

uint8_t *honu_feed_reserve(honu_feed *f, uint64_t len, int32_t *err) {
    int32_t dummy;
    if (!err) err = &dummy;
    *err = HONU_OK;
    if (!f) {
        *err = HONU_E_ARG;
        return nullptr;
    }
    Slot *s = filling(f, err);
    if (!s) return nullptr;
    if (s->n == f->cap_n || len > f->cap_bytes - s->bytes) {
        *err = HONU_ERR_CAPACITY;
        return nullptr;
    }
    uint8_t *p = s->h_rec + s->bytes;
    s->bytes += len;
    s->n += 1;
    s->h_off[s->n] = s->bytes;
    return p;
}

int32_t honu_feed_append(honu_feed *f, const uint8_t *rec, uint64_t len) {
    int32_t err;
    uint8_t *p = honu_feed_reserve(f, len, &err);
    if (!p) return err;
    if (len) std::memcpy(p, rec, len);
    return HONU_OK;
}

int32_t honu_feed_append_batch(honu_feed *f, const uint8_t *arena, const uint64_t *off, uint64_t n,
                               uint64_t *appended) {
    if (!f || (n && (!arena || !off)) || !appended) return HONU_E_ARG;
    *appended = 0;
    int32_t err = HONU_OK;
    Slot *sp = filling(f, &err);
    if (!sp) return err;
    Slot &s = *sp;
    // the run of records that fits: they are contiguous in the arena, so they
    // land as one (multi-threaded) copy
    uint64_t k = 0;
    for (; k < n && s.n + k < f->cap_n; k++) {
        if (off[k + 1] < off[k]) return HONU_E_ARG;
        if (off[k + 1] - off[0] > f->cap_bytes - s.bytes) break;
    }
    const uint64_t bytes = k ? off[k] - off[0] : 0;
    if (bytes) host_copy({honu::HostCopy{s.h_rec + s.bytes, arena + off[0], bytes}}, bytes);
    for (uint64_t j = 0; j < k; j++) s.h_off[s.n + j + 1] = s.bytes + (off[j + 1] - off[0]);
    s.n += k;
    s.bytes += bytes;
    *appended = k;
    return k == n ? HONU_OK : HONU_ERR_CAPACITY;
}

uint64_t honu_feed_pending(const honu_feed *f) {
    if (!f) return 0;
    const Slot &s = f->slot[f->cur];
    return s.state == FREE ? s.n : 0;
}

int32_t honu_feed_submit(honu_feed *f, uint64_t *ticket) {
    if (!f) return HONU_E_ARG;
    int32_t err = HONU_OK;
    Slot *sp = filling(f, &err);
    if (!sp) return err;
    Slot &s = *sp;
    FCHK(hipSetDevice(f->device));
    const uint64_t n = s.n;
    void *st = s.stream;
    FCHK(hipMemcpyAsync(s.d_off, s.h_off, 8 * (n + 1), hipMemcpyHostToDevice, s.stream));
    if (s.bytes)
        FCHK(hipMemcpyAsync(s.d_rec, s.h_rec, s.bytes, hipMemcpyHostToDevice, s.stream));
    if (f->flags & HONU_FEED_HEADERS) {
        err = honu_decode_headers(s.ctx, s.d_rec, s.d_off, n, s.d_info, st);
        if (err) return err;
    } else {
        err = honu_decode_batch(s.ctx, s.d_rec, s.d_off, n, s.d_meta, s.d_info, s.d_acl,
                                f->acl_cap, s.d_reg, f->reg_cap, nullptr, 0, s.d_tot, st);
        if (err) return err;
        err = honu_decode_keys(s.ctx, s.d_meta, s.d_info, n, s.d_keys, s.d_kst, st);
        if (err) return err;
        FCHK(hipMemcpyAsync(s.h_meta, s.d_meta, sizeof(honu_meta) * n, hipMemcpyDeviceToHost,
                            s.stream));
        FCHK(hipMemcpyAsync(s.h_keys, s.d_keys, (uint64_t)HONU_KEY_LEN * n,
                            hipMemcpyDeviceToHost, s.stream));
        FCHK(hipMemcpyAsync(s.h_kst, s.d_kst, 4 * n, hipMemcpyDeviceToHost, s.stream));
        FCHK(hipMemcpyAsync(s.h_tot, s.d_tot, 24, hipMemcpyDeviceToHost, s.stream));
    }
    FCHK(hipMemcpyAsync(s.h_info, s.d_info, sizeof(honu_record_info) * n, hipMemcpyDeviceToHost,
                        s.stream));
    s.state = INFLIGHT;
    s.ticket = f->next_ticket++;
    if (ticket) *ticket = s.ticket;
    f->cur ^= 1;
    return HONU_OK;
}

int32_t honu_feed_wait(honu_feed *f, uint64_t ticket, honu_feed_result *out) {
    if (!f || !out) return HONU_E_ARG;
    Slot *sp = nullptr;
    for (Slot &s : f->slot)
        if (s.state != FREE && s.ticket == ticket) sp = &s;
    if (!sp) return HONU_E_ARG;
    Slot &s = *sp;
    FCHK(hipSetDevice(f->device));
    if (s.state == INFLIGHT) {
        FCHK(hipStreamSynchronize(s.stream));
        if (!(f->flags & HONU_FEED_HEADERS)) {
            const uint64_t na = s.h_tot[0] < f->acl_cap ? s.h_tot[0] : f->acl_cap;
            const uint64_t nr = s.h_tot[1] < f->reg_cap ? s.h_tot[1] : f->reg_cap;
            if (na)
                FCHK(hipMemcpyAsync(s.h_acl, s.d_acl, sizeof(honu_acl) * na,
                                    hipMemcpyDeviceToHost, s.stream));
            if (nr)
                FCHK(hipMemcpyAsync(s.h_reg, s.d_reg, 4 * nr, hipMemcpyDeviceToHost, s.stream));
            FCHK(hipStreamSynchronize(s.stream));
        }
        s.state = DONE;
    }
    const bool hdr = f->flags & HONU_FEED_HEADERS;
    out->n = s.n;
    out->records = s.h_rec;
    out->rec_off = s.h_off;
    out->meta = hdr ? nullptr : s.h_meta;
    out->info = s.h_info;
    out->acl = hdr ? nullptr : s.h_acl;
    // the tables hold at most acl_cap / reg_cap entries; a batch that needs
    // more (nil-entry floods) reports its need separately, so a binding that
    // slices acl[0:acl_n] never reads past the pinned allocation
    out->acl_n = hdr ? 0 : (s.h_tot[0] < f->acl_cap ? s.h_tot[0] : f->acl_cap);
    out->regions = hdr ? nullptr : s.h_reg;
    out->regions_n = hdr ? 0 : (s.h_tot[1] < f->reg_cap ? s.h_tot[1] : f->reg_cap);
    out->acl_needed = hdr ? 0 : s.h_tot[0];
    out->regions_needed = hdr ? 0 : s.h_tot[1];
    out->keys = hdr ? nullptr : s.h_keys;
    out->key_status = hdr ? nullptr : s.h_kst;
    return HONU_OK;
}
