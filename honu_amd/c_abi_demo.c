/*
 * c_abi_demo.c — the batch flow a cgo shim runs (INTEGRATION.md MarshalBatch /
 * DecodeBatch), written against include/honu_codec.h in plain C: no Python, no
 * torch, only the library's own pinned/device allocation helpers, plain
 * pointers, sizes and the null stream. Built by honu_amd/Makefile; run by
 * tests/test_c_abi.py on a GPU box.
 *
 *   c_abi_demo [shape] [n] [dump_dir]   shape: 0 Small, 1 Medium, 2 Large, 4 Mixed
 *
 * Steps: generate a synthetic host batch (rows, var arena, ACL and region
 * tables, payloads) -> H2D -> honu_marshal_batch -> D2H of offsets/records ->
 * honu_decode_batch (zero copy) with ACL / region tables sized from COUNTS,
 * not record bytes: a first call with small caps, the totals it reports
 * (d_totals: the entries the batch needs), tables re-allocated to exactly
 * those and a second call -> D2H of rows/info/tables -> honu_decode_batch
 * materialising -> D2H of payloads; checks every status, the decoded rows'
 * scalar fields against the input rows, every ACL list as the binding builds
 * its []*AccessControl (acl_entry: from the records arena for a list returned
 * in place, HONU_ACL_INPLACE, else from the ACL table) against the input
 * entries, and every payload's digest. With
 * dump_dir, the records arena, offsets and the zero-copy outputs are written
 * there (rec.bin, off.bin, meta.bin, info.bin, acl.bin, reg.bin, tot.bin) for
 * tests/test_c_abi.py to compare with the oracle. Exit 0 and one "ok" line on
 * success.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/honu_codec.h"
#include "../include/honu_bench.h" /* the synthetic batch and the digest */

#define CHECK(x)                                                                          \
    do {                                                                                  \
        int32_t st_ = (x);                                                                \
        if (st_ != HONU_OK) {                                                             \
            fprintf(stderr, "%s:%d %s -> %d (%s: %s)\n", __FILE__, __LINE__, #x, st_,     \
                    honu_status_string(st_), honu_last_error());                          \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)
#define NEED(p)                                                          \
    do {                                                                 \
        if (!(p)) {                                                      \
            fprintf(stderr, "%s:%d allocation failed: %s\n", __FILE__, __LINE__, #p); \
            return 1;                                                    \
        }                                                                \
    } while (0)

static int dump(const char *dir, const char *name, const void *p, uint64_t bytes) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "wb");
    if (!f) return 1;
    const int bad = bytes && fwrite(p, 1, bytes, f) != bytes;
    return fclose(f) != 0 || bad;
}

/* Entry j of a decoded row's ACL list, as the binding's Go code builds
 * &AccessControl{ClientID, Permissions} (nil when *present == 0): in place,
 * the 18 bytes 01 | ClientID | Permissions at acl_off + 18 j of the records
 * arena; otherwise row j of the list in the ACL table. */
static void acl_entry(const honu_meta *m, const uint8_t *rec, const honu_acl *table, uint64_t j,
                      uint8_t client_id[16], uint8_t *perm, uint8_t *present) {
    if (m->present & HONU_ACL_INPLACE) {
        const uint8_t *e = rec + m->acl_off + 18 * j;
        *present = e[0];
        memcpy(client_id, e + 1, 16);
        *perm = e[17];
        return;
    }
    const honu_acl *a = table + m->acl_off + j;
    *present = a->present;
    memcpy(client_id, a->client_id, 16);
    *perm = a->permissions;
}

/* The regions of a decoded row, as the binding's Regions.Decode loop builds
 * them (region.go:154-169): in place (HONU_REGIONS_INPLACE), the uvarints
 * from regions_off of the records arena, each read as lani.DecodeUint32 does
 * (<= 5 bytes, truncated to uint32; the GPU decode validated them); otherwise
 * row j of the list in the region table. */
static void region_values(const honu_meta *m, const uint8_t *rec, const uint32_t *table, uint32_t *out) {
    if (!(m->present & HONU_REGIONS_INPLACE)) {
        memcpy(out, table + m->regions_off, 4 * m->regions_count);
        return;
    }
    const uint8_t *p = rec + m->regions_off;
    for (uint64_t j = 0; j < m->regions_count; j++) {
        uint64_t v = 0;
        for (int k = 0, sh = 0; k < 5; k++, sh += 7) {
            v |= (uint64_t)(p[0] & 0x7F) << sh;
            if (!(*p++ & 0x80)) break;
        }
        out[j] = (uint32_t)v;
    }
}

static void *h2d(const void *h, uint64_t bytes) {
    void *d = honu_device_alloc(bytes + 16);
    if (d && bytes && honu_memcpy_h2d(d, h, bytes, NULL) != HONU_OK) return NULL;
    return d;
}

int main(int argc, char **argv) {
    const int32_t shape = argc > 1 ? atoi(argv[1]) : HONU_SHAPE_SMALL;
    const uint64_t n = argc > 2 ? strtoull(argv[2], NULL, 10) : 4096;
    const char *dump_dir = argc > 3 && strcmp(argv[3], "-") ? argv[3] : NULL;
    /* "table": every ACL and region list in its table (context params
     * acl_inplace 0, regions_inplace 0); default: the library's in-place forms */
    const int table_form = argc > 4 && !strcmp(argv[4], "table");
    const uint64_t seed = 12345;
    int32_t err = 0;
    honu_ctx *ctx = honu_ctx_create(0, n, &err);
    if (!ctx) {
        fprintf(stderr, "honu_ctx_create: %s (%s)\n", honu_status_string(err), honu_last_error());
        return 2;
    }
    if (table_form) {
        CHECK(honu_ctx_set_param(ctx, "acl_inplace", 0));
        CHECK(honu_ctx_set_param(ctx, "regions_inplace", 0));
    }
    /* 1. the host batch, as the Go side's flatten() would build it */
    uint64_t tot[4];
    honu_gen_totals(seed, shape, 0, n, tot); /* var bytes, ACL entries, regions, payload bytes */
    honu_meta *rows = (honu_meta *)honu_host_alloc(sizeof(honu_meta) * n);
    uint8_t *var = (uint8_t *)honu_host_alloc(tot[0] + 16);
    honu_acl *acl = (honu_acl *)honu_host_alloc(sizeof(honu_acl) * tot[1] + 16);
    uint32_t *reg = (uint32_t *)honu_host_alloc(4 * tot[2] + 16);
    uint64_t *poff = (uint64_t *)honu_host_alloc(8 * (n + 1));
    uint8_t *pay = (uint8_t *)honu_host_alloc(tot[3] + 16);
    NEED(rows && var && acl && reg && poff && pay);
    honu_gen_meta(seed, shape, 0, n, rows, var, acl, reg, poff);
    honu_gen_payload_host(seed, 0, n, poff, pay);
    /* 2. H2D */
    void *d_rows = h2d(rows, sizeof(honu_meta) * n), *d_var = h2d(var, tot[0]);
    void *d_acl = h2d(acl, sizeof(honu_acl) * tot[1]), *d_reg = h2d(reg, 4 * tot[2]);
    void *d_poff = h2d(poff, 8 * (n + 1)), *d_pay = h2d(pay, tot[3]);
    NEED(d_rows && d_var && d_acl && d_reg && d_poff && d_pay);
    /* 3. Marshal: an upper bound for the output arena (payload + 4 KiB/record) */
    const uint64_t cap = tot[3] + 4096 * n;
    uint64_t *d_off = (uint64_t *)honu_device_alloc(8 * (n + 1));
    int32_t *d_st = (int32_t *)honu_device_alloc(4 * n + 16);
    uint8_t *d_out = (uint8_t *)honu_device_alloc(cap);
    NEED(d_off && d_st && d_out);
    CHECK(honu_marshal_batch(ctx, (const honu_meta *)d_rows, (const uint8_t *)d_var, tot[0],
                             (const honu_acl *)d_acl, tot[1], (const uint32_t *)d_reg, tot[2],
                             (const uint8_t *)d_pay, (const uint64_t *)d_poff, n, d_out, cap,
                             d_off, d_st, NULL));
    uint64_t *off = (uint64_t *)honu_host_alloc(8 * (n + 1));
    int32_t *st = (int32_t *)honu_host_alloc(4 * n + 16);
    NEED(off && st);
    CHECK(honu_memcpy_d2h(off, d_off, 8 * (n + 1), NULL));
    CHECK(honu_memcpy_d2h(st, d_st, 4 * n, NULL));
    CHECK(honu_stream_sync(NULL));
    for (uint64_t i = 0; i < n; i++)
        if (st[i] != HONU_OK) {
            fprintf(stderr, "record %llu: marshal status %d\n", (unsigned long long)i, st[i]);
            return 1;
        }
    const uint64_t rec_bytes = off[n];
    /* 4. Metadata() + zero-copy Data(), then a materialising decode. The ACL
     * and region tables are sized by the batch's entry counts: a first call
     * with small caps (a binding starts from its typical counts: none with
     * the in-place forms, whose tables take only ACL lists with a nil entry;
     * one entry per record with the table forms, so the retry always runs
     * there) reports the totals in d_totals (records past the caps get
     * HONU_ERR_CAPACITY), the tables are re-allocated to exactly the totals
     * and the call is repeated. Sizing them by record bytes instead (an entry
     * takes >= 1 byte) would allocate 20 + 4 bytes per RECORD BYTE: 24x the
     * records arena. */
    honu_meta *d_meta = (honu_meta *)honu_device_alloc(sizeof(honu_meta) * n);
    honu_record_info *d_info = (honu_record_info *)honu_device_alloc(sizeof(honu_record_info) * n);
    uint64_t *d_tot = (uint64_t *)honu_device_alloc(32);
    NEED(d_meta && d_info && d_tot);
    uint64_t acl_cap = table_form ? n : 0, reg_cap = table_form ? n : 0, totals[4] = {0, 0, 0, 0};
    honu_acl *d_tacl = NULL;
    uint32_t *d_treg = NULL;
    int calls = 0;
    for (;;) {
        d_tacl = (honu_acl *)honu_device_alloc(sizeof(honu_acl) * acl_cap + 16);
        d_treg = (uint32_t *)honu_device_alloc(4 * reg_cap + 16);
        NEED(d_tacl && d_treg);
        CHECK(honu_decode_batch(ctx, d_out, d_off, n, d_meta, d_info, d_tacl, acl_cap, d_treg, reg_cap,
                                NULL, 0, d_tot, NULL));
        calls++;
        CHECK(honu_memcpy_d2h(totals, d_tot, 24, NULL));
        CHECK(honu_stream_sync(NULL));
        if (totals[0] <= acl_cap && totals[1] <= reg_cap) break;
        if (calls == 2) {
            fprintf(stderr, "totals grew between two decodes of one batch\n");
            return 1;
        }
        honu_device_free(d_tacl);
        honu_device_free(d_treg);
        acl_cap = totals[0];
        reg_cap = totals[1];
    }
    const uint64_t table_bytes = sizeof(honu_acl) * acl_cap + 4 * reg_cap;
    const uint64_t data_cap = rec_bytes + 16 * n;
    uint8_t *d_data = (uint8_t *)honu_device_alloc(data_cap);
    NEED(d_data);
    honu_meta *meta = (honu_meta *)honu_host_alloc(sizeof(honu_meta) * n);
    honu_record_info *info = (honu_record_info *)honu_host_alloc(sizeof(honu_record_info) * n);
    honu_acl *tacl = (honu_acl *)honu_host_alloc(sizeof(honu_acl) * acl_cap + 16);
    uint32_t *treg = (uint32_t *)honu_host_alloc(4 * reg_cap + 16);
    NEED(meta && info && tacl && treg);
    CHECK(honu_memcpy_d2h(meta, d_meta, sizeof(honu_meta) * n, NULL));
    CHECK(honu_memcpy_d2h(info, d_info, sizeof(honu_record_info) * n, NULL));
    CHECK(honu_memcpy_d2h(tacl, d_tacl, sizeof(honu_acl) * totals[0], NULL));
    CHECK(honu_memcpy_d2h(treg, d_treg, 4 * totals[1], NULL));
    CHECK(honu_stream_sync(NULL));
    /* the records arena: Data(), the spans and in-place ACL lists point into it */
    uint8_t *rec = (uint8_t *)honu_host_alloc(rec_bytes + 16);
    NEED(rec);
    CHECK(honu_memcpy_d2h(rec, d_out, rec_bytes, NULL));
    CHECK(honu_stream_sync(NULL));
    if (dump_dir) {
        if (dump(dump_dir, "rec.bin", rec, rec_bytes) || dump(dump_dir, "off.bin", off, 8 * (n + 1)) ||
            dump(dump_dir, "meta.bin", meta, sizeof(honu_meta) * n) ||
            dump(dump_dir, "info.bin", info, sizeof(honu_record_info) * n) ||
            dump(dump_dir, "acl.bin", tacl, sizeof(honu_acl) * totals[0]) ||
            dump(dump_dir, "reg.bin", treg, 4 * totals[1]) || dump(dump_dir, "tot.bin", totals, 24)) {
            fprintf(stderr, "cannot write %s\n", dump_dir);
            return 1;
        }
    }
    uint64_t lists_inplace = 0, lists_table = 0, regions_inplace = 0;
    uint32_t *rv = (uint32_t *)honu_host_alloc(4 * 4096);
    NEED(rv);
    for (uint64_t i = 0; i < n; i++) {
        const honu_meta *a = rows + i, *b = meta + i;
        if (info[i].meta_status != HONU_OK || info[i].data_status != HONU_OK ||
            info[i].data_len != poff[i + 1] - poff[i] || a->pid != b->pid || a->vid != b->vid ||
            a->created != b->created || a->modified != b->modified || a->acl_count != b->acl_count ||
            a->regions_count != b->regions_count || memcmp(a->owner, b->owner, 16) != 0) {
            fprintf(stderr, "record %llu: decoded fields differ (meta %d data %d)\n",
                    (unsigned long long)i, info[i].meta_status, info[i].data_status);
            return 1;
        }
        for (uint64_t j = 0; j < b->acl_count; j++) {
            uint8_t cid[16], perm, present;
            acl_entry(b, rec, tacl, j, cid, &perm, &present);
            const honu_acl *src = acl + a->acl_off + j;
            if (present != src->present || (present && (perm != src->permissions ||
                                                        memcmp(cid, src->client_id, 16) != 0))) {
                fprintf(stderr, "record %llu: ACL entry %llu differs\n", (unsigned long long)i,
                        (unsigned long long)j);
                return 1;
            }
        }
        if (b->acl_count) (b->present & HONU_ACL_INPLACE) ? lists_inplace++ : lists_table++;
        if (b->regions_count > 4096) return 1;  /* (the generator writes at most 9) */
        region_values(b, rec, treg, rv);
        if (memcmp(rv, reg + a->regions_off, 4 * a->regions_count) != 0) {
            fprintf(stderr, "record %llu: regions differ\n", (unsigned long long)i);
            return 1;
        }
        if (b->regions_count && (b->present & HONU_REGIONS_INPLACE)) regions_inplace++;
    }
    CHECK(honu_decode_batch(ctx, d_out, d_off, n, d_meta, d_info, d_tacl, acl_cap, d_treg,
                            reg_cap, d_data, data_cap, d_tot, NULL));
    uint8_t *data = (uint8_t *)honu_host_alloc(data_cap);
    NEED(data);
    CHECK(honu_memcpy_d2h(info, d_info, sizeof(honu_record_info) * n, NULL));
    CHECK(honu_memcpy_d2h(data, d_data, data_cap, NULL));
    CHECK(honu_stream_sync(NULL));
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t len = poff[i + 1] - poff[i];
        if (info[i].data_len != len ||
            honu_digest_host(data + info[i].data_off, len) != honu_digest_host(pay + poff[i], len)) {
            fprintf(stderr, "record %llu: payload differs\n", (unsigned long long)i);
            return 1;
        }
    }
    printf("ok: %llu records, %llu encoded bytes, marshal + decode + materialise through the C ABI; "
           "decode calls %d, table bytes %llu (ACL entries %llu, regions %llu); ACL lists in place "
           "%llu, in the table %llu; region lists in place %llu\n",
           (unsigned long long)n, (unsigned long long)rec_bytes, calls, (unsigned long long)table_bytes,
           (unsigned long long)totals[0], (unsigned long long)totals[1],
           (unsigned long long)lists_inplace, (unsigned long long)lists_table,
           (unsigned long long)regions_inplace);
    honu_ctx_destroy(ctx);
    return 0;
}
