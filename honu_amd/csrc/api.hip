// api.hip — the C ABI (include/honu_codec.h) over the gfx950 kernels.
//
// One context per device: it owns the only allocations the library makes
// (per-record decode scratch, count/offset columns and scan partials), sized
// once for a maximum batch so that every codec call is allocation- and
// sync-free and can be captured into a hipGraph.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kernels.h"

using namespace honu;

struct honu_ctx {
    int device;
    uint64_t max_n;
    LaunchGeom geom;
    void *ws;
    uint64_t *counts;        // 3 * max_n
    uint64_t *offs;          // 3 * max_n
    uint64_t *totals;        // 4 (3: decode totals; word 3: the HBM probe's sink)
    DecodeScratch *scratch;  // max_n
    uint32_t *reg_inline;    // 8 * max_n: region ids handed from the group parse to fill
    EncAclPos *enc_acl;      // max_n: ACL list hand-over, lane encoder -> group ACL encoder
    // decoupled look-back state of the fused decode (fused.hip): a
    // ticket/epoch block and 3 status words per 64-record tile
    LbState *lb_dec;
    uint64_t *lb_dec_status;
    uint64_t *lb_dec_gstatus;  // the group words, after the tile words (same epoch scheme)
    uint64_t lb_dec_words;     // tile + group words
    uint64_t lb_bytes;       // the look-back blocks + status words, from lb_dec
    ScanState scan;          // look-back state of the one-launch scans (scan.hip)
    // speculation back-off (fused.hip): a guarded recovery launch that ran sets
    // *spec_seen (pinned host word, written by the device); the next call sees
    // it and decodes SPEC_BACKOFF_CALLS calls without speculation, so a stream
    // of batches with malformed records pays ~1.1x instead of ~2x per batch
    uint32_t *spec_seen;     // pinned: [0] the back-off flag, [1] recovery launches run (a count)
    uint32_t spec_off;       // calls left without speculation
    int speculate;           // honu_ctx_set_param("speculate"): 0 off, 1 on, 2 where it hides a wait
    // honu_encode_records: the ACL lists' kernel on a stream of the context's
    // own, beside the header/tail encoder (forked from and joined back into
    // the caller's stream by events)
    hipStream_t aux;
    hipEvent_t ev_fork, ev_join;
    int enc_fork;            // honu_ctx_set_param("encode_fork", 0 off / 1 on / 2 auto: when lane_blocks caps the grid)
    bool acl_inplace;        // honu_ctx_set_param("acl_inplace"): decode returns all-present ACL lists in place
    bool reg_inplace;        // honu_ctx_set_param("regions_inplace"): decode returns region lists in place
    bool inline_recovery;    // honu_ctx_set_param("inline_recovery"): ticket-form launches recover in-launch
    int guard_blocks;        // honu_ctx_set_param("guard_blocks"): one-wave workgroups of the guarded launch
                             // (0: as many as the speculative launch has waves)
    uint32_t copy_seq;       // copy calls issued: call k takes counter line k % COPY_TICKET_LINES
    int enc_form;            // the last honu_encode_records* call: 0 none, 1 plain, 2 units
};

// The launch geometry of one payload-copy call: the context's, with the
// range-tail counters of the next line of the ring (kernels.h), so copy calls
// in flight at once on different streams each count on a line of their own
// (one shared line let a launch skip tails another one took).
static LaunchGeom copy_geom(honu_ctx *ctx) {
    LaunchGeom g = ctx->geom;
    const uint32_t k = __atomic_fetch_add(&ctx->copy_seq, 1u, __ATOMIC_RELAXED) % COPY_TICKET_LINES;
    g.copy_tickets = ctx->geom.copy_tickets + (uint64_t)k * COPY_TICKET_STRIDE;
    return g;
}
static constexpr uint32_t SPEC_BACKOFF_CALLS = 16;
// Speculation only where it hides a look-back wait (materialising decodes,
// table forms): a zero-copy in-place launch skips those waits already, and
// there the flag gather and guard cost more than the walk's own flag check
// (round 6: 0.392 vs 0.427 ms for 1M Large records, profiles/r06).
#ifndef SPECULATE_DEFAULT
#define SPECULATE_DEFAULT 2
#endif

static thread_local char g_last_error[256];

static int32_t hip_fail(hipError_t e, const char *what) {
    snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
    return HONU_E_HIP;
}
#define HIPCHK(x)                                  \
    do {                                           \
        hipError_t e_ = (x);                       \
        if (e_ != hipSuccess) return hip_fail(e_, #x); \
    } while (0)

static int32_t arg_fail(const char *what) {
    snprintf(g_last_error, sizeof g_last_error, "invalid argument: %s", what);
    return HONU_E_ARG;
}

static bool aligned(const void *p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; }

// record_variant 5 runs the batch entries through the split kernels of
// variant 0, 6 through the fused decode at every size; variant 0 picks by size
#define FUSED_DECODE_MIN_RECORDS (48ull << 10)
// the A/B build (make ab: -DHONU_AB) adds the measurement-only copy variants and
// the fused decode's measurement knobs
#ifdef HONU_AB
#define HONU_AB_BUILD 1
#else
#define HONU_AB_BUILD 0
#endif

// Fused kernels: persistent waves (2 workgroups of 4 waves per CU fit the LDS
// and registers), fewer under a lane_blocks cap.
static int fused_blocks(const LaunchGeom &g) {
    const int resident = 2 * g.num_cu;
    return g.lane_blocks > 0 && g.lane_blocks < resident ? g.lane_blocks : resident;
}

// A stream with a CU mask or a non-default priority: honu_encode_records then
// does not fork the ACL lists onto the context's own (unmasked, default
// priority) stream, so the work stays where the caller put it.
static bool stream_is_restricted(hipStream_t s, int num_cu) {
    int prio = 0;
    if (hipStreamGetPriority(s, &prio) == hipSuccess && prio != 0) return true;
    uint32_t mask[32] = {0};
    const uint32_t words = (uint32_t)((num_cu + 31) / 32);
    if (words > 32 || hipExtStreamGetCUMask(s, words, mask) != hipSuccess) return false;
    bool any = false, all = true;  // (an all-zero answer: no mask)
    for (int i = 0; i < num_cu; i++) {
        const bool on = mask[i / 32] >> (i % 32) & 1u;
        any |= on;
        all &= on;
    }
    return any && !all;
}

// The product library takes its configuration from honu_ctx_set_param only:
// it behaves the same whatever the caller's process environment holds. The
// A/B build (make ab) also reads HONU_* variables at context creation, for
// tools/*.sh sweeps that cannot set params.
static int env_int(const char *name, int dflt) {
#ifdef HONU_AB
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
#else
    (void)name;
    return dflt;
#endif
}

extern "C" {

uint32_t honu_abi_version(void) { return HONU_ABI_VERSION; }
uint64_t honu_sizeof_meta(void) { return sizeof(honu_meta); }
uint64_t honu_sizeof_acl(void) { return sizeof(honu_acl); }
uint64_t honu_sizeof_collection(void) { return sizeof(honu_collection); }
uint64_t honu_sizeof_index(void) { return sizeof(honu_index); }
uint64_t honu_sizeof_record_info(void) { return sizeof(honu_record_info); }
const char *honu_last_error(void) { return g_last_error; }

const char *honu_status_string(int32_t st) {
    switch (st) {
    case HONU_OK: return "ok";
    case HONU_ERR_BAD_VERSION: return "object is malformed: cannot decode specified version";
    case HONU_ERR_MALFORMED: return "object is malformed: cannot parse data or metadata";
    case HONU_ERR_EOF: return "EOF";
    case HONU_ERR_UNEXPECTED_EOF: return "unexpected EOF";
    case HONU_ERR_NO_LENGTH: return "field not written with length value";
    case HONU_ERR_PARSE_BOOLEAN: return "could not parse boolean value";
    case HONU_ERR_PARSE_VARINT: return "could not parse varint";
    case HONU_ERR_PANIC: return "input on which the Go reference panics";
    case HONU_ERR_CAPACITY: return "output capacity exceeded";
    case HONU_ERR_INPUT: return "input span or list outside its arena";
    case HONU_UNPARSED: return "metadata not decoded (headers only)";
    case HONU_E_ARG: return "invalid argument";
    case HONU_E_WORKSPACE: return "batch larger than the context's reserved records";
    case HONU_E_HIP: return "HIP runtime error";
    case HONU_E_NO_DEVICE: return "no gfx950 device";
    default: return "unknown status";
    }
}

honu_ctx *honu_ctx_create(int device, uint64_t max_records, int32_t *err) {
    int32_t dummy;
    if (!err) err = &dummy;
    *err = HONU_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
        snprintf(g_last_error, sizeof g_last_error, "no HIP device %d (count %d)", device, count);
        *err = HONU_E_NO_DEVICE;
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
        strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        snprintf(g_last_error, sizeof g_last_error, "device %d is %s, this build targets gfx950",
                 device, prop.gcnArchName);
        *err = HONU_E_NO_DEVICE;
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        *err = HONU_E_HIP;
        return nullptr;
    }
    honu_ctx *c = (honu_ctx *)calloc(1, sizeof(honu_ctx));
    if (!c) {
        *err = HONU_E_HIP;
        return nullptr;
    }
    // every failure below ends here: whatever was created is destroyed
    auto fail = [&](int32_t e, const char *what) -> honu_ctx * {
        if (what) snprintf(g_last_error, sizeof g_last_error, "%s", what);
        if (c->ev_join) (void)hipEventDestroy(c->ev_join);
        if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
        if (c->aux) (void)hipStreamDestroy(c->aux);
        if (c->spec_seen) (void)hipHostFree(c->spec_seen);
        if (c->ws) (void)hipFree(c->ws);
        free(c);
        *err = e;
        return nullptr;
    };
    c->device = device;
    c->max_n = max_records ? max_records : 1;
    c->geom.num_cu = prop.multiProcessorCount;
    c->geom.per_record_blocks = env_int("HONU_RECORD_BLOCKS", prop.multiProcessorCount * 8);
    c->geom.lane_blocks = env_int("HONU_LANE_BLOCKS", 0);
    c->geom.copy_blocks = env_int("HONU_COPY_BLOCKS", prop.multiProcessorCount * 2);
    c->geom.copy_variant = HONU_AB_BUILD ? env_int("HONU_COPY_VARIANT", 0) : 0;
    c->geom.record_variant = env_int("HONU_RECORD_VARIANT", 0);
    c->geom.encode_variant = HONU_AB_BUILD && env_int("HONU_ENCODE_VARIANT", 0) == 1 ? 1 : 0;  // 0 default
    if (c->geom.record_variant != 5 && c->geom.record_variant != 6)
        c->geom.record_variant = 0;
    c->acl_inplace = env_int("HONU_ACL_INPLACE", 1) != 0;
    c->reg_inplace = env_int("HONU_REGIONS_INPLACE", 1) != 0;
    // measured slower than the guarded launch (1M Small zero copy 0.56 ->
    // 0.67-0.70 ms, the Small step 4.17-4.21 -> 4.26-4.42 ms; DESIGN §3
    // "Round 5"): off by default
    c->inline_recovery = env_int("HONU_INLINE_RECOVERY", 0) != 0;
    c->guard_blocks = env_int("HONU_GUARD_BLOCKS", 0);
    if (c->guard_blocks < 0) c->guard_blocks = 0;
    const uint64_t n = c->max_n;
    const uint64_t np = 0;
    const uint64_t map_cap = HONU_AB_BUILD ? 1ull << 22 : 0;  // tile map (A/B sweep copy)
    const uint64_t tiles = (n + HONU_WAVE - 1) / HONU_WAVE;
    const uint64_t scan_words = scan_status_words(n);
    // 3 status words per tile, then 3 per 64-tile group (lookback.h
    // lb_resolve_grouped*)
    const uint64_t groups = (tiles / HONU_WAVE + 1) > LB_GROUPS ? tiles / HONU_WAVE + 1 : LB_GROUPS;
    const uint64_t lb_dec_words = 3 * tiles + 3 * groups;
    // (+ the copies' range-tail counters: a ring of 128-byte lines)
    const uint64_t lb_bytes =
        2 * sizeof(LbState) + 8 * (lb_dec_words + scan_words) + COPY_TICKET_LINES * 4 * COPY_TICKET_STRIDE;
    const uint64_t bytes = 8 * (3 * n + 3 * n + 4 + np) + sizeof(DecodeScratch) * n + 32 * n +
                           sizeof(EncAclPos) * n + 4 * map_cap + lb_bytes + 256;
    if (hipMalloc(&c->ws, bytes) != hipSuccess) {
        c->ws = nullptr;
        char msg[96];
        snprintf(msg, sizeof msg, "hipMalloc(%llu) failed", (unsigned long long)bytes);
        return fail(HONU_E_HIP, msg);
    }
    if (hipHostMalloc((void **)&c->spec_seen, 2 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
        hipSuccess) {
        c->spec_seen = nullptr;
        return fail(HONU_E_HIP, "hipHostMalloc(spec_seen) failed");
    }
    c->spec_seen[0] = 0;
    c->spec_seen[1] = 0;
    c->speculate = SPECULATE_DEFAULT;
    c->enc_fork = env_int("HONU_ENCODE_FORK", 2);
    if (c->enc_fork < 0 || c->enc_fork > 2) c->enc_fork = 2;
    if (hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess) {
        c->aux = nullptr;
        return fail(HONU_E_HIP, "stream creation failed");
    }
    if (hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess) {
        c->ev_fork = nullptr;
        return fail(HONU_E_HIP, "event creation failed");
    }
    if (hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess) {
        c->ev_join = nullptr;
        return fail(HONU_E_HIP, "event creation failed");
    }
    uint64_t *w = (uint64_t *)c->ws;
    c->counts = w;
    w += 3 * n;
    c->offs = w;
    w += 3 * n;
    c->totals = w;
    w += 4;
    c->scratch = (DecodeScratch *)w;
    c->reg_inline = (uint32_t *)(c->scratch + n);
    c->enc_acl = (EncAclPos *)(c->reg_inline + 8 * n);
    c->geom.tile_map = (uint32_t *)(c->enc_acl + n);
    c->geom.tile_map_cap = map_cap;
    c->lb_dec = (LbState *)(c->geom.tile_map + map_cap);
    c->scan.lb = c->lb_dec + 1;
    c->lb_dec_status = (uint64_t *)(c->scan.lb + 1);
    c->lb_dec_words = lb_dec_words;
    c->lb_dec_gstatus = c->lb_dec_status + 3 * tiles;
    c->scan.status = c->lb_dec_status + c->lb_dec_words;
    c->scan.words = scan_words;
    c->geom.copy_tickets = (uint32_t *)(c->scan.status + scan_words);
    c->geom.copy_steal = 1;
    c->scan.max_blocks = 4 * prop.multiProcessorCount;
    c->lb_bytes = lb_bytes;
    // clean look-back state: epoch 0 with no published tile. On a stream of
    // the call's own, so work other contexts have in flight keeps running.
    hipStream_t s = nullptr;
    bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMemsetAsync(c->lb_dec, 0, lb_bytes, s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    if (s) (void)hipStreamDestroy(s);
    if (!ok) return fail(HONU_E_HIP, "look-back state initialisation failed");
    return c;
}

int32_t honu_ctx_reset(honu_ctx *ctx, void *stream) {
    if (!ctx) return arg_fail("ctx");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipMemsetAsync(ctx->lb_dec, 0, ctx->lb_bytes, (hipStream_t)stream));
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return HONU_OK;
}

void honu_ctx_destroy(honu_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->aux);
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_join);
    (void)hipStreamDestroy(ctx->aux);
    (void)hipFree(ctx->ws);
    (void)hipHostFree(ctx->spec_seen);
    free(ctx);
}

uint64_t honu_ctx_max_records(const honu_ctx *ctx) { return ctx ? ctx->max_n : 0; }

int32_t honu_ctx_set_param(honu_ctx *ctx, const char *name, int64_t value) {
    if (!ctx || !name) return arg_fail("ctx/name");
    if (!strcmp(name, "copy_blocks") && value > 0) ctx->geom.copy_blocks = (int)value;
    else if (!strcmp(name, "record_blocks") && value > 0) ctx->geom.per_record_blocks = (int)value;
    else if (!strcmp(name, "lane_blocks") && value >= 0) ctx->geom.lane_blocks = (int)value;
    else if (!strcmp(name, "speculate") && value >= 0 && value <= 2) ctx->speculate = (int)value;
    else if (!strcmp(name, "encode_fork") && value >= 0 && value <= 2) ctx->enc_fork = (int)value;
    else if (!strcmp(name, "acl_inplace") && (value == 0 || value == 1)) ctx->acl_inplace = value != 0;
    else if (!strcmp(name, "regions_inplace") && (value == 0 || value == 1)) ctx->reg_inplace = value != 0;
    else if (!strcmp(name, "inline_recovery") && (value == 0 || value == 1)) ctx->inline_recovery = value != 0;
    else if (!strcmp(name, "guard_blocks") && value >= 0 && value <= 65536) ctx->guard_blocks = (int)value;
    else if (!strcmp(name, "speculate_backoff") && value >= 0 && value <= (int64_t)SPEC_BACKOFF_CALLS) {
        __atomic_store_n(ctx->spec_seen, 0u, __ATOMIC_RELAXED);
        ctx->spec_off = (uint32_t)value;
    }
    else if (!strcmp(name, "copy_steal") && (value == 0 || value == 1)) ctx->geom.copy_steal = (int)value;
    else if (!strcmp(name, "copy_variant") && value >= 0 && (value == 0 || HONU_AB_BUILD))
        ctx->geom.copy_variant = (int)value;
    else if (!strcmp(name, "encode_variant") && (value == 0 || (value == 1 && HONU_AB_BUILD)))
        ctx->geom.encode_variant = (int)value;
    else if (!strcmp(name, "record_variant") &&
             (value == 0 || value == 5 || value == 6))
        ctx->geom.record_variant = (int)value;
    else return arg_fail(name);
    return HONU_OK;
}

int32_t honu_ctx_get_param(const honu_ctx *ctx, const char *name, int64_t *value) {
    if (!ctx || !name || !value) return arg_fail("ctx/name/value");
    if (!strcmp(name, "copy_blocks")) *value = ctx->geom.copy_blocks;
    else if (!strcmp(name, "record_blocks")) *value = ctx->geom.per_record_blocks;
    else if (!strcmp(name, "lane_blocks")) *value = ctx->geom.lane_blocks;
    else if (!strcmp(name, "speculate")) *value = ctx->speculate;
    else if (!strcmp(name, "encode_fork")) *value = ctx->enc_fork;
    else if (!strcmp(name, "acl_inplace")) *value = ctx->acl_inplace ? 1 : 0;
    else if (!strcmp(name, "regions_inplace")) *value = ctx->reg_inplace ? 1 : 0;
    else if (!strcmp(name, "inline_recovery")) *value = ctx->inline_recovery ? 1 : 0;
    else if (!strcmp(name, "guard_blocks")) *value = ctx->guard_blocks;
    else if (!strcmp(name, "recoveries"))  // recovery launches that ran, since the context was created
        *value = __atomic_load_n(ctx->spec_seen + 1, __ATOMIC_RELAXED);
    else if (!strcmp(name, "speculate_backoff"))  // calls the next call starts without speculation
        *value = __atomic_load_n(ctx->spec_seen, __ATOMIC_RELAXED) ? SPEC_BACKOFF_CALLS : ctx->spec_off;
    else if (!strcmp(name, "copy_steal")) *value = ctx->geom.copy_steal;
    else if (!strcmp(name, "copy_variant")) *value = ctx->geom.copy_variant;
    else if (!strcmp(name, "encode_variant")) *value = ctx->geom.encode_variant;
    else if (!strcmp(name, "record_variant")) *value = ctx->geom.record_variant;
    else if (!strcmp(name, "walk_flag_checks")) *value = decode_walk_flag_checks();  // read only: the build's
    else return arg_fail(name);
    return HONU_OK;
}

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
int32_t honu_encode_sizes(honu_ctx *ctx, const honu_meta *d_meta, uint64_t var_len,
                          const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                          uint64_t regions_len, const uint64_t *d_payload_off, uint64_t n,
                          uint64_t *d_sizes, int32_t *d_status, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_meta || !d_payload_off || !d_sizes)) return arg_fail("null pointer");
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4)) return arg_fail("tables must be 4-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_encode_sizes_grp(d_meta, var_len, d_acl, acl_len, d_regions, regions_len,
                                   d_payload_off, n, d_sizes, d_status, ctx->geom.lane_blocks,
                                   (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_exclusive_scan(honu_ctx *ctx, const uint64_t *d_in, uint64_t n, uint64_t *d_out,
                            void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_scan(d_in, n, 1, d_out, d_out + n, ctx->scan, (hipStream_t)stream));
    return HONU_OK;
}

// units: the payload arena (honu_encode_records_units), or null
static int32_t encode_records(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                              const honu_acl *d_acl, const uint32_t *d_regions, const uint8_t *units,
                              const uint64_t *d_payload_off, uint64_t n, uint8_t *d_out,
                              uint64_t out_cap, const uint64_t *d_out_off, int32_t *d_status,
                              void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_meta || !d_payload_off || !d_out || !d_out_off || !d_status))
        return arg_fail("null pointer");
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4)) return arg_fail("tables must be 4-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    ctx->enc_form = units ? 2 : 1;  // (the payload call checks it: never mix the two forms)
#ifdef HONU_AB
    if (ctx->geom.encode_variant == 1 && !units) {  // one launch, 16 lanes per record (enc.hip, A/B build only)
        HIPCHK(launch_encode_tail_grp(d_meta, d_var, d_acl, d_regions, d_payload_off, n, d_out,
                                      out_cap, d_out_off, d_status, ctx->geom.lane_blocks,
                                      (hipStream_t)stream));
        return HONU_OK;
    }
#endif
    // encode_variant 0 (default, measured faster: DESIGN §3): header + tail
    // with the ACL lists' partial end chunks (one record per lane), then the
    // lists' whole chunks (16 lanes per record)
    hipStream_t s = (hipStream_t)stream;
    // (auto: not on a CU-masked or prioritised caller stream, whose placement
    // the fork would escape)
    const bool fork = ctx->enc_fork == 1 ||
                      (ctx->enc_fork == 2 && ctx->geom.lane_blocks > 0 && n &&
                       !stream_is_restricted(s, ctx->geom.num_cu));
    if (fork && n) {
        // the lists' whole chunks on the context's own stream, beside the
        // header/tail encoder (disjoint bytes: the lane encoder writes the
        // lists' partial end chunks, or skips a list with nil entries whole)
        HIPCHK(hipEventRecord(ctx->ev_fork, s));
        HIPCHK(hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0));
        HIPCHK(launch_encode_acl_grp_self(d_meta, d_acl, d_payload_off, n, d_out, out_cap, d_out_off, d_status,
                                          ctx->geom.lane_blocks, ctx->aux));
        HIPCHK(hipEventRecord(ctx->ev_join, ctx->aux));
        HIPCHK(launch_encode_meta_lane(d_meta, d_var, d_acl, d_regions, d_payload_off, n, d_out,
                                       out_cap, d_out_off, d_status, ctx->enc_acl,
                                       ctx->geom.lane_blocks, ctx->geom.num_cu, units, s));
        HIPCHK(hipStreamWaitEvent(s, ctx->ev_join, 0));
        return HONU_OK;
    }
    HIPCHK(launch_encode_meta_lane(d_meta, d_var, d_acl, d_regions, d_payload_off, n, d_out,
                                   out_cap, d_out_off, d_status, ctx->enc_acl,
                                   ctx->geom.lane_blocks, ctx->geom.num_cu, units, s));
    HIPCHK(launch_encode_acl_grp(d_meta, d_acl, n, d_out, d_status, ctx->enc_acl,
                                 ctx->geom.lane_blocks, s));
    return HONU_OK;
}

int32_t honu_encode_records(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                            const honu_acl *d_acl, const uint32_t *d_regions,
                            const uint64_t *d_payload_off, uint64_t n, uint8_t *d_out,
                            uint64_t out_cap, const uint64_t *d_out_off, int32_t *d_status,
                            void *stream) {
    return encode_records(ctx, d_meta, d_var, d_acl, d_regions, nullptr, d_payload_off, n, d_out, out_cap,
                          d_out_off, d_status, stream);
}

int32_t honu_encode_records_units(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                                  const honu_acl *d_acl, const uint32_t *d_regions,
                                  const uint8_t *d_payload, const uint64_t *d_payload_off, uint64_t n,
                                  uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                                  int32_t *d_status, void *stream) {
    if (n && !d_payload) return arg_fail("null pointer");
    return encode_records(ctx, d_meta, d_var, d_acl, d_regions, d_payload, d_payload_off, n, d_out, out_cap,
                          d_out_off, d_status, stream);
}

static int32_t encode_payloads(honu_ctx *ctx, const uint8_t *d_payload, const uint64_t *d_payload_off,
                               uint64_t n, uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                               const int32_t *d_status, bool units, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_payload_off || !d_out || !d_out_off || !d_status)) return arg_fail("null pointer");
    // the units pair completes only what its own records call left out: a
    // payload call of the other form than the context's last records call
    // would leave bytes unwritten (or write them twice) with every status OK
    if (ctx->enc_form && ctx->enc_form != (units ? 2 : 1))
        return arg_fail(units ? "honu_encode_payloads_units after honu_encode_records (mixed forms)"
                              : "honu_encode_payloads after honu_encode_records_units (mixed forms)");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_encode_copy(copy_geom(ctx), d_payload, d_payload_off, n, d_out, out_cap, d_out_off,
                              d_status, units, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_encode_payloads(honu_ctx *ctx, const uint8_t *d_payload, const uint64_t *d_payload_off,
                             uint64_t n, uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                             const int32_t *d_status, void *stream) {
    return encode_payloads(ctx, d_payload, d_payload_off, n, d_out, out_cap, d_out_off, d_status, false, stream);
}

int32_t honu_encode_payloads_units(honu_ctx *ctx, const uint8_t *d_payload, const uint64_t *d_payload_off,
                                   uint64_t n, uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                                   const int32_t *d_status, void *stream) {
    return encode_payloads(ctx, d_payload, d_payload_off, n, d_out, out_cap, d_out_off, d_status, true, stream);
}

int32_t honu_encode(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var, uint64_t var_len,
                    const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                    uint64_t regions_len, const uint8_t *d_payload, const uint64_t *d_payload_off,
                    uint64_t n, uint8_t *d_out, uint64_t out_cap, const uint64_t *d_out_off,
                    int32_t *d_status, void *stream) {
    (void)var_len;
    (void)acl_len;
    (void)regions_len;
    if (!d_payload) {  // a batch of empty payloads only (nothing to copy): the plain pair,
                       // which reads the arena only for a non-empty payload
        int32_t st = honu_encode_records(ctx, d_meta, d_var, d_acl, d_regions, d_payload_off, n, d_out,
                                         out_cap, d_out_off, d_status, stream);
        if (st) return st;
        return honu_encode_payloads(ctx, d_payload, d_payload_off, n, d_out, out_cap, d_out_off, d_status,
                                    stream);
    }
    // the payload-unit pair (one kernel per 64-byte unit of the output)
    int32_t st = honu_encode_records_units(ctx, d_meta, d_var, d_acl, d_regions, d_payload, d_payload_off, n,
                                           d_out, out_cap, d_out_off, d_status, stream);
    if (st) return st;
    return honu_encode_payloads_units(ctx, d_payload, d_payload_off, n, d_out, out_cap, d_out_off,
                                      d_status, stream);
}

int32_t honu_marshal_batch(honu_ctx *ctx, const honu_meta *d_meta, const uint8_t *d_var,
                           uint64_t var_len, const honu_acl *d_acl, uint64_t acl_len,
                           const uint32_t *d_regions, uint64_t regions_len,
                           const uint8_t *d_payload, const uint64_t *d_payload_off, uint64_t n,
                           uint8_t *d_out, uint64_t out_cap, uint64_t *d_out_off,
                           int32_t *d_status, void *stream) {
    int32_t st = honu_encode_sizes(ctx, d_meta, var_len, d_acl, acl_len, d_regions, regions_len,
                                   d_payload_off, n, d_out_off, d_status, stream);
    if (st) return st;
    st = honu_exclusive_scan(ctx, d_out_off, n, d_out_off, stream);
    if (st) return st;
    return honu_encode(ctx, d_meta, d_var, var_len, d_acl, acl_len, d_regions, regions_len,
                       d_payload, d_payload_off, n, d_out, out_cap, d_out_off, d_status, stream);
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
int32_t honu_decode_parse(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                          uint64_t n, honu_meta *d_meta, honu_record_info *d_info, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (n && (!d_rec || !d_rec_off || !d_meta || !d_info)) return arg_fail("null pointer");
    if (!aligned(d_rec, 16) || !aligned(d_meta, 16) || !aligned(d_info, 8))
        return arg_fail("records arena and rows must be 16-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_decode_parse_win(d_rec, d_rec_off, n, d_meta, d_info, ctx->scratch,
                                   ctx->reg_inline, ctx->counts, ctx->geom.lane_blocks,
                                   ctx->acl_inplace, ctx->reg_inplace, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_decode_tables(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n, honu_meta *d_meta,
                           honu_record_info *d_info, honu_acl *d_acl, uint64_t acl_cap,
                           uint32_t *d_regions, uint64_t regions_cap, uint8_t *d_data,
                           uint64_t data_cap, uint64_t *d_totals, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4) || !aligned(d_data, 16))
        return arg_fail("tables 4-byte / data arena 16-byte aligned");
    if (acl_cap && !d_acl) return arg_fail("acl table");
    if (regions_cap && !d_regions) return arg_fail("region table");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    uint64_t *tot = d_totals ? d_totals : ctx->totals;
    HIPCHK(launch_scan(ctx->counts, n, 3, ctx->offs, tot, ctx->scan, s));
    HIPCHK(launch_decode_fill_grp(d_rec, n, d_meta, d_info, ctx->scratch, ctx->reg_inline,
                                  ctx->counts, ctx->offs, d_acl, acl_cap, d_regions, regions_cap,
                                  d_data, data_cap, ctx->geom.lane_blocks, s));
    return HONU_OK;
}

int32_t honu_decode_payloads(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n,
                             const honu_record_info *d_info, uint8_t *d_data,
                             const uint64_t *d_totals, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (!d_data || !aligned(d_data, 16)) return arg_fail("data arena");
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t *tot = d_totals ? d_totals : ctx->totals;
    HIPCHK(launch_decode_copy(copy_geom(ctx), d_rec, n, d_info, ctx->scratch, ctx->offs, tot, d_data,
                              (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_decode_fill(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                         uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                         honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                         uint64_t regions_cap, uint8_t *d_data, uint64_t data_cap,
                         uint64_t *d_totals, void *stream) {
    (void)d_rec_off;
    int32_t st = honu_decode_tables(ctx, d_rec, n, d_meta, d_info, d_acl, acl_cap, d_regions,
                                    regions_cap, d_data, data_cap, d_totals, stream);
    if (st || !d_data) return st;
    return honu_decode_payloads(ctx, d_rec, n, d_info, d_data, d_totals, stream);
}

int32_t honu_decode_records(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                            uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                            honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                            uint64_t regions_cap, int32_t materialize, uint64_t data_cap,
                            uint64_t *d_totals, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (n && (!d_rec || !d_rec_off || !d_meta || !d_info)) return arg_fail("null pointer");
    if (!aligned(d_rec, 16) || !aligned(d_meta, 16) || !aligned(d_info, 8))
        return arg_fail("records arena and rows must be 16-byte aligned");
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4)) return arg_fail("tables must be 4-byte aligned");
    if (acl_cap && !d_acl) return arg_fail("acl table");
    if (regions_cap && !d_regions) return arg_fail("region table");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    uint64_t *tot = d_totals ? d_totals : ctx->totals;
    if (n == 0) {
        HIPCHK(hipMemsetAsync(tot, 0, 3 * sizeof(uint64_t), s));
        return HONU_OK;
    }
    // speculation back-off: a recovery of an earlier call has finished (the
    // word is read without waiting: a recovery still in flight is seen later)
    if (__atomic_load_n(ctx->spec_seen, __ATOMIC_RELAXED)) {
        __atomic_store_n(ctx->spec_seen, 0u, __ATOMIC_RELAXED);
        ctx->spec_off = SPEC_BACKOFF_CALLS;
    }
    // speculation hides the look-back wait; a zero-copy call with both list
    // forms in place has none to hide (fused.hip: tiles without table entries
    // do not wait), so "speculate" 2 (auto) decodes it without speculation:
    // no ACL flag burst after the walk re-reading the list's lines, no guarded
    // second launch
    const bool hides = materialize || !ctx->acl_inplace || !ctx->reg_inplace;
    const bool spec = (ctx->speculate == 1 || (ctx->speculate == 2 && hides)) && ctx->spec_off == 0;
    if (ctx->spec_off) ctx->spec_off--;
    HIPCHK(launch_decode_fused(d_rec, d_rec_off, n, d_meta, d_info, d_acl, acl_cap, d_regions,
                               regions_cap, materialize != 0, data_cap, ctx->scratch, ctx->offs,
                               tot, ctx->lb_dec, ctx->lb_dec_status, ctx->lb_dec_gstatus,
                               ctx->lb_dec_words, fused_blocks(ctx->geom), ctx->spec_seen,
                               ctx->spec_seen + 1, spec, ctx->acl_inplace, ctx->reg_inplace, ctx->inline_recovery,
                               ctx->guard_blocks, s));
    return HONU_OK;
}

int32_t honu_decode_batch(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                          uint64_t n, honu_meta *d_meta, honu_record_info *d_info,
                          honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                          uint64_t regions_cap, uint8_t *d_data, uint64_t data_cap,
                          uint64_t *d_totals, void *stream) {
    // fused from 48 K records (measured: even with split at ~48 K, 3-5 % ahead
    // at 62-65 K, and the 1M Large bench's 62 K-record chunks 4 % faster with
    // one metadata launch per chunk beside the copies; below, the split
    // kernels' extra waves hide the walk's latency better), always with
    // record_variant 6
    const int rv = ctx ? ctx->geom.record_variant : 0;
    if (rv == 6 || (rv == 0 && n >= FUSED_DECODE_MIN_RECORDS)) {
        if (d_data && !aligned(d_data, 16)) return arg_fail("data arena must be 16-byte aligned");
        int32_t st = honu_decode_records(ctx, d_rec, d_rec_off, n, d_meta, d_info, d_acl, acl_cap,
                                         d_regions, regions_cap, d_data != nullptr, data_cap,
                                         d_totals, stream);
        if (st || !d_data) return st;
        return honu_decode_payloads(ctx, d_rec, n, d_info, d_data, d_totals, stream);
    }
    int32_t st = honu_decode_parse(ctx, d_rec, d_rec_off, n, d_meta, d_info, stream);
    if (st) return st;
    return honu_decode_fill(ctx, d_rec, d_rec_off, n, d_meta, d_info, d_acl, acl_cap, d_regions,
                            regions_cap, d_data, data_cap, d_totals, stream);
}

int32_t honu_decode_headers(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                            uint64_t n, honu_record_info *d_info, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_rec || !d_rec_off || !d_info)) return arg_fail("null pointer");
    if (!aligned(d_info, 8)) return arg_fail("record info must be 8-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_decode_headers(d_rec, d_rec_off, n, d_info, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_decode_data_place(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                               uint64_t n, honu_record_info *d_info, uint64_t data_cap,
                               uint64_t *d_totals, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (n && (!d_rec || !d_rec_off || !d_info)) return arg_fail("null pointer");
    if (!aligned(d_info, 8)) return arg_fail("record info must be 8-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (d_totals) HIPCHK(hipMemsetAsync(d_totals, 0, 8, s));
        return HONU_OK;
    }
    // spans -> exclusive scan of the aligned sizes (offs[n] = total) -> place
    HIPCHK(launch_decode_spans(d_rec, d_rec_off, n, d_info, ctx->scratch, ctx->counts, s));
    HIPCHK(launch_scan(ctx->counts, n, 1, ctx->offs, ctx->offs + n, ctx->scan, s));
    HIPCHK(launch_decode_data_place(n, d_info, ctx->offs, data_cap, s));
    if (d_totals)
        HIPCHK(hipMemcpyAsync(d_totals, ctx->offs + n, 8, hipMemcpyDeviceToDevice, s));
    return HONU_OK;
}

int32_t honu_decode_data_copy(honu_ctx *ctx, const uint8_t *d_rec, uint64_t n,
                              const honu_record_info *d_info, uint8_t *d_data, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (n && (!d_rec || !d_info || !d_data)) return arg_fail("null pointer");
    if (!aligned(d_data, 16)) return arg_fail("data arena must be 16-byte aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_span_copy(copy_geom(ctx), d_rec, n, d_info, ctx->scratch, ctx->offs, d_data,
                            (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_decode_data(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                         uint64_t n, honu_record_info *d_info, uint8_t *d_data, uint64_t data_cap,
                         uint64_t *d_totals, void *stream) {
    if (n && !d_data) return arg_fail("data arena");
    int32_t st = honu_decode_data_place(ctx, d_rec, d_rec_off, n, d_info, data_cap, d_totals, stream);
    if (st) return st;
    return honu_decode_data_copy(ctx, d_rec, n, d_info, d_data, stream);
}

int32_t honu_decode_keys(honu_ctx *ctx, const honu_meta *d_meta, const honu_record_info *d_info,
                         uint64_t n, uint8_t *d_keys, int32_t *d_key_status, void *stream) {
    if (!ctx) return arg_fail("ctx");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_decode_keys(ctx->geom, d_meta, d_info, n, d_keys, d_key_status,
                              (hipStream_t)stream));
    return HONU_OK;
}

// ---------------------------------------------------------------------------
// system objects (object/system.go)
// ---------------------------------------------------------------------------
int32_t honu_system_sizes(honu_ctx *ctx, const honu_collection *d_rows, uint64_t var_len,
                          const honu_acl *d_acl, uint64_t acl_len, const uint32_t *d_regions,
                          uint64_t regions_len, const honu_index *d_index, uint64_t index_len,
                          uint64_t n, uint64_t *d_sizes, int32_t *d_status, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_rows || !d_sizes)) return arg_fail("null pointer");
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4) || !aligned(d_index, 8))
        return arg_fail("tables must be aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_system_sizes(d_rows, var_len, d_acl, acl_len, d_regions, regions_len, d_index,
                               index_len, n, d_sizes, d_status, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_system_encode(honu_ctx *ctx, const honu_collection *d_rows, const uint8_t *d_var,
                           const honu_acl *d_acl, const uint32_t *d_regions,
                           const honu_index *d_index, uint64_t n, uint8_t *d_out,
                           uint64_t out_cap, const uint64_t *d_out_off, int32_t *d_status,
                           void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_rows || !d_out || !d_out_off || !d_status)) return arg_fail("null pointer");
    if (!aligned(d_acl, 4) || !aligned(d_regions, 4) || !aligned(d_index, 8))
        return arg_fail("tables must be aligned");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_system_encode(d_rows, d_var, d_acl, d_regions, d_index, n, d_out, out_cap,
                                d_out_off, d_status, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_system_marshal_batch(honu_ctx *ctx, const honu_collection *d_rows,
                                  const uint8_t *d_var, uint64_t var_len, const honu_acl *d_acl,
                                  uint64_t acl_len, const uint32_t *d_regions,
                                  uint64_t regions_len, const honu_index *d_index,
                                  uint64_t index_len, uint64_t n, uint8_t *d_out,
                                  uint64_t out_cap, uint64_t *d_out_off, int32_t *d_status,
                                  void *stream) {
    int32_t st = honu_system_sizes(ctx, d_rows, var_len, d_acl, acl_len, d_regions, regions_len,
                                   d_index, index_len, n, d_out_off, d_status, stream);
    if (st) return st;
    st = honu_exclusive_scan(ctx, d_out_off, n, d_out_off, stream);
    if (st) return st;
    return honu_system_encode(ctx, d_rows, d_var, d_acl, d_regions, d_index, n, d_out, out_cap,
                              d_out_off, d_status, stream);
}

static int32_t collection_decode(honu_ctx *ctx, bool headless, const uint8_t *d_rec,
                                 const uint64_t *d_rec_off, uint64_t n, honu_collection *d_rows,
                                 int32_t *d_status, honu_acl *d_acl, uint64_t acl_cap,
                                 uint32_t *d_regions, uint64_t regions_cap, honu_index *d_index,
                                 uint64_t index_cap, uint64_t *d_totals, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n > ctx->max_n) return HONU_E_WORKSPACE;
    if (n && (!d_rec || !d_rec_off || !d_rows || !d_status)) return arg_fail("null pointer");
    if (!aligned(d_rows, 16) || !aligned(d_acl, 4) || !aligned(d_regions, 4) ||
        !aligned(d_index, 8))
        return arg_fail("rows 16-byte / tables 4- and 8-byte aligned");
    if ((acl_cap && !d_acl) || (regions_cap && !d_regions) || (index_cap && !d_index))
        return arg_fail("table");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    uint64_t *tot = d_totals ? d_totals : ctx->totals;
    HIPCHK(launch_system_parse(d_rec, d_rec_off, n, headless, d_rows, d_status, ctx->scratch,
                               ctx->counts, s));
    HIPCHK(launch_scan(ctx->counts, n, 3, ctx->offs, tot, ctx->scan, s));
    HIPCHK(launch_system_fill(d_rec, n, d_rows, d_status, ctx->scratch, ctx->counts, ctx->offs,
                              d_acl, acl_cap, d_regions, regions_cap, d_index, index_cap, s));
    return HONU_OK;
}

int32_t honu_system_decode_batch(honu_ctx *ctx, const uint8_t *d_rec, const uint64_t *d_rec_off,
                                 uint64_t n, honu_collection *d_rows, int32_t *d_status,
                                 honu_acl *d_acl, uint64_t acl_cap, uint32_t *d_regions,
                                 uint64_t regions_cap, honu_index *d_index, uint64_t index_cap,
                                 uint64_t *d_totals, void *stream) {
    return collection_decode(ctx, false, d_rec, d_rec_off, n, d_rows, d_status, d_acl, acl_cap,
                             d_regions, regions_cap, d_index, index_cap, d_totals, stream);
}

int32_t honu_collection_decode_batch(honu_ctx *ctx, const uint8_t *d_rec,
                                     const uint64_t *d_rec_off, uint64_t n,
                                     honu_collection *d_rows, int32_t *d_status, honu_acl *d_acl,
                                     uint64_t acl_cap, uint32_t *d_regions, uint64_t regions_cap,
                                     honu_index *d_index, uint64_t index_cap, uint64_t *d_totals,
                                     void *stream) {
    return collection_decode(ctx, true, d_rec, d_rec_off, n, d_rows, d_status, d_acl, acl_cap,
                             d_regions, regions_cap, d_index, index_cap, d_totals, stream);
}

// ---------------------------------------------------------------------------
// synthetic payload, digests, memory helpers
// ---------------------------------------------------------------------------
int32_t honu_gen_payload(honu_ctx *ctx, uint64_t seed, uint64_t first, uint64_t n,
                         const uint64_t *d_payload_off, uint8_t *d_payload, void *stream) {
    if (!ctx) return arg_fail("ctx");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_gen_payload(ctx->geom, seed, first, n, d_payload_off, d_payload,
                              (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_hbm_probe(honu_ctx *ctx, int32_t mode, const void *d_src, void *d_dst, uint64_t bytes,
                       uint32_t blocks_per_cu, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (mode < 0 || mode > 4) return arg_fail("mode");
    if (!aligned(d_src, 16) || !aligned(d_dst, 16) || (mode != 1 && !d_src) || (mode != 0 && !d_dst))
        return arg_fail("buffers must be non-null and 16-byte aligned");
    if (!blocks_per_cu) blocks_per_cu = 2;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_hbm_probe(mode, d_src, d_dst, bytes, blocks_per_cu * (uint32_t)ctx->geom.num_cu,
                            reinterpret_cast<uint32_t *>(ctx->totals + 3), (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_digest_records(honu_ctx *ctx, const uint8_t *d_arena, const uint64_t *d_off,
                            const uint64_t *d_len, uint64_t n, uint64_t *d_digest, void *stream) {
    if (!ctx) return arg_fail("ctx");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_digest(ctx->geom, d_arena, d_off, d_len, n, d_digest, (hipStream_t)stream));
    return HONU_OK;
}

int32_t honu_verify_decoded(honu_ctx *ctx, const honu_meta *d_src, const uint8_t *d_var,
                            const honu_acl *d_src_acl, const uint32_t *d_src_regions,
                            const uint64_t *d_payload_off, const uint8_t *d_rec,
                            const honu_meta *d_dec, const honu_record_info *d_info,
                            const honu_acl *d_dec_acl, const uint32_t *d_dec_regions, uint64_t n,
                            uint32_t *d_mismatch, void *stream) {
    if (!ctx) return arg_fail("ctx");
    if (n && (!d_src || !d_payload_off || !d_rec || !d_dec || !d_info || !d_mismatch))
        return arg_fail("null pointer");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_verify_decoded(ctx->geom, d_src, d_var, d_src_acl, d_src_regions, d_payload_off,
                                 d_rec, d_dec, d_info, d_dec_acl, d_dec_regions, n, d_mismatch,
                                 (hipStream_t)stream));
    return HONU_OK;
}

void *honu_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}
void honu_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}
void *honu_device_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    return p;
}
void honu_device_free(void *p) {
    if (p) (void)hipFree(p);
}
int32_t honu_memcpy_h2d(void *d_dst, const void *h_src, uint64_t bytes, void *stream) {
    HIPCHK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return HONU_OK;
}
int32_t honu_memcpy_d2h(void *h_dst, const void *d_src, uint64_t bytes, void *stream) {
    HIPCHK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return HONU_OK;
}
int32_t honu_stream_sync(void *stream) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return HONU_OK;
}

}  // extern "C"
