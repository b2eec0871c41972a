// copy_sweep.hip — the forms of a streaming HBM copy on this part (round-4
// verdict item 3: can a copy reach the guide's 6.29 TB/s float4-copy figure,
// MI355X_MICROARCH.md "Chip-level parameters", and which form does).
// Standalone measurement tool, not product code:
//   hipcc -O3 --offload-arch=gfx950 -o copy_sweep tools/copy_sweep.hip
//   ./copy_sweep [GiB per buffer, default 8] [reps, default 5] [read|write|copy]
// (the third argument: that one form only, for rocprofv3 --pmc passes)
// Swept: 16/32/64 B per lane, 1-16 chunks per lane in flight, each wave on a
// contiguous range (the codec copy engine's layout, copy.hip) or grid-stride
// (the guide's float4 copy), global_load/store or buffer_load/store with the
// sc0 / sc1 / nt cache-policy bits, 1-8 workgroups of 256 threads per CU, and
// the source/destination offset inside a 2 MiB page. Rates count read + write
// bytes (2 x the copied bytes), as bench.py's roofline does.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                       \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

enum { L_RANGE = 0, L_GS = 1 };
enum { M_GLOBAL = 0, M_NT = 1, M_BUF = 2 };

// V: 16-byte vectors per lane per chunk (1, 2, 4 = 16/32/64 B per lane);
// U: chunks per lane in flight; LAYOUT; MEM: global, global non-temporal, or
// buffer instructions with cache-policy aux LP (loads) / SP (stores).
template <int V, int U, int LAYOUT, int MEM, int LP, int SP>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ a, u32x4 *__restrict__ b,
                                             uint64_t n) {
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint64_t STEP = 64ull * V;  // vectors per wave per chunk
    uint64_t lo, hi, stride, first;
    if constexpr (LAYOUT == L_RANGE) {
        const uint64_t W = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
        const uint64_t chunks = n / STEP;
        lo = chunks * w / W * STEP;
        hi = chunks * (w + 1) / W * STEP;
        first = lo;
        stride = STEP * U;
    } else {
        lo = 0;
        hi = n / STEP * STEP;
        first = ((uint64_t)blockIdx.x * 4 + threadIdx.x / 64) * STEP * U;
        stride = (uint64_t)gridDim.x * 4 * STEP * U;
    }
    if constexpr (MEM == M_BUF) {
        // one resource per wave range (32-bit offsets); the grid-stride form
        // rebases per iteration
        for (uint64_t i = first; i < hi; i += stride) {
            const uint64_t base = i;
            __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)(a + base), 0, 0x7fffffff, 0x00020000);
            __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void *)(b + base), 0, 0x7fffffff, 0x00020000);
            u32x4 v[U][V];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int k = 0; k < V; k++) {
                    const uint64_t j = (uint64_t)u * STEP + (uint64_t)lane * V + k;
                    if (base + j < hi) v[u][k] = __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(16 * j), 0, LP);
                }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int k = 0; k < V; k++) {
                    const uint64_t j = (uint64_t)u * STEP + (uint64_t)lane * V + k;
                    if (base + j < hi) __builtin_amdgcn_raw_buffer_store_b128(v[u][k], rb, (uint32_t)(16 * j), 0, SP);
                }
        }
        return;
    }
    for (uint64_t i = first; i < hi; i += stride) {
        u32x4 v[U][V];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int k = 0; k < V; k++) {
                const uint64_t j = i + (uint64_t)u * STEP + (uint64_t)lane * V + k;
                if (j < hi) {
                    if constexpr (MEM == M_NT && (LP & 2)) v[u][k] = __builtin_nontemporal_load(a + j);
                    else v[u][k] = a[j];
                }
            }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int k = 0; k < V; k++) {
                const uint64_t j = i + (uint64_t)u * STEP + (uint64_t)lane * V + k;
                if (j < hi) {
                    if constexpr (MEM == M_NT && (SP & 2)) __builtin_nontemporal_store(v[u][k], b + j);
                    else b[j] = v[u][k];
                }
            }
    }
}

__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ a, uint64_t n, unsigned *out) {
    const uint64_t W = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t lo = n * w / W, hi = n * (w + 1) / W;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = lo + (threadIdx.x & 63); i < hi; i += 64 * 8) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = i + 64 * u < hi ? a[i + 64 * u] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_write(u32x4 *__restrict__ b, uint64_t n) {
    const uint64_t W = (uint64_t)gridDim.x * 4, w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t lo = n * w / W, hi = n * (w + 1) / W;
    for (uint64_t i = lo + (threadIdx.x & 63); i < hi; i += 64 * 8) {
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (i + 64 * u < hi) b[i + 64 * u] = u32x4{(unsigned)i, (unsigned)u, 1, 2};
    }
}

struct Variant {
    const char *name;
    void (*launch)(dim3, const u32x4 *, u32x4 *, uint64_t);
};
template <int V, int U, int LAYOUT, int MEM, int LP, int SP>
void launch_copy(dim3 g, const u32x4 *a, u32x4 *b, uint64_t n) {
    hipLaunchKernelGGL((k_copy<V, U, LAYOUT, MEM, LP, SP>), g, dim3(256), 0, 0, a, b, n);
}
#define VAR(name, V, U, L, M, LP, SP) Variant{name, launch_copy<V, U, L, M, LP, SP>}

int main(int argc, char **argv) {
    const uint64_t gib = argc > 1 ? strtoull(argv[1], 0, 10) : 8;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t bytes = gib << 30;
    const uint64_t page = 2ull << 20;
    int dev = 0, cus = 0;
    CHK(hipGetDevice(&dev));
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    uint8_t *A, *B;
    unsigned *o;
    CHK(hipMalloc(&A, bytes + 2 * page));
    CHK(hipMalloc(&B, bytes + 2 * page));
    CHK(hipMalloc(&o, 64));
    CHK(hipMemset(A, 1, bytes + 2 * page));
    CHK(hipMemset(B, 2, bytes + 2 * page));
    printf("{\"cus\": %d, \"gib\": %llu, \"A\": \"%p\", \"B\": \"%p\"}\n", cus, (unsigned long long)gib, A, B);
    // 2 MiB-aligned bases inside the allocations
    const u32x4 *a = (const u32x4 *)(((uintptr_t)A + page - 1) & ~(uintptr_t)(page - 1));
    u32x4 *b = (u32x4 *)(((uintptr_t)B + page - 1) & ~(uintptr_t)(page - 1));
    const uint64_t n = bytes / 16;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto time = [&](auto launch) {
        launch();
        CHK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) launch();
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipGetLastError());
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    auto line = [&](const char *kind, const char *name, int bpc, double traffic, float ms, const char *extra) {
        printf("{\"kind\": \"%s\", \"form\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"tbs\": %.4f%s}\n", kind,
               name, bpc, ms, traffic / (ms * 1e-3) / 1e12, extra);
        fflush(stdout);
    };
    // "only": one form, reps launches, for counter passes (rocprofv3 --pmc)
    const char *only = argc > 3 ? argv[3] : nullptr;
    if (only) {
        const dim3 g(cus * 2);
        float ms = 0;
        if (!strcmp(only, "read"))
            ms = time([&] { hipLaunchKernelGGL(k_read, g, dim3(256), 0, 0, a, n, o); });
        else if (!strcmp(only, "write"))
            ms = time([&] { hipLaunchKernelGGL(k_write, g, dim3(256), 0, 0, b, n); });
        else
            ms = time([&] { launch_copy<1, 8, L_RANGE, M_GLOBAL, 0, 0>(g, a, b, n); });
        line(only, "range_16B_u8", 2, (strcmp(only, "copy") ? 1.0 : 2.0) * bytes, ms, "");
        return 0;
    }
    const int bpcs[] = {1, 2, 3, 4, 6, 8};
    for (int bpc : bpcs) {
        const dim3 g(cus * bpc);
        line("read", "range_u8_16B", bpc, (double)bytes,
             time([&] { hipLaunchKernelGGL(k_read, g, dim3(256), 0, 0, a, n, o); }), "");
        line("write", "range_u8_16B", bpc, (double)bytes,
             time([&] { hipLaunchKernelGGL(k_write, g, dim3(256), 0, 0, b, n); }), "");
    }
    std::vector<Variant> vars = {
        VAR("range_16B_u1", 1, 1, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_16B_u2", 1, 2, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_16B_u4", 1, 4, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_16B_u8", 1, 8, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_16B_u16", 1, 16, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_32B_u2", 2, 2, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_32B_u4", 2, 4, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_64B_u1", 4, 1, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_64B_u2", 4, 2, L_RANGE, M_GLOBAL, 0, 0),
        VAR("range_64B_u4", 4, 4, L_RANGE, M_GLOBAL, 0, 0),
        VAR("gs_16B_u1", 1, 1, L_GS, M_GLOBAL, 0, 0),
        VAR("gs_16B_u2", 1, 2, L_GS, M_GLOBAL, 0, 0),
        VAR("gs_16B_u4", 1, 4, L_GS, M_GLOBAL, 0, 0),
        VAR("gs_16B_u8", 1, 8, L_GS, M_GLOBAL, 0, 0),
        VAR("gs_32B_u2", 2, 2, L_GS, M_GLOBAL, 0, 0),
        VAR("gs_64B_u1", 4, 1, L_GS, M_GLOBAL, 0, 0),
        VAR("range_16B_u8_ntload", 1, 8, L_RANGE, M_NT, 2, 0),
        VAR("range_16B_u8_ntstore", 1, 8, L_RANGE, M_NT, 0, 2),
        VAR("range_16B_u8_ntboth", 1, 8, L_RANGE, M_NT, 2, 2),
        VAR("range_16B_u8_buf", 1, 8, L_RANGE, M_BUF, 0, 0),
        VAR("range_16B_u8_buf_sc0", 1, 8, L_RANGE, M_BUF, 1, 1),
        VAR("range_16B_u8_buf_sc1", 1, 8, L_RANGE, M_BUF, 16, 16),
        VAR("range_16B_u8_buf_sc0sc1", 1, 8, L_RANGE, M_BUF, 17, 17),
        VAR("range_16B_u8_buf_nt", 1, 8, L_RANGE, M_BUF, 2, 2),
        VAR("range_16B_u8_buf_ntsc1", 1, 8, L_RANGE, M_BUF, 18, 18),
        VAR("range_16B_u8_buf_ldsc1_stnt", 1, 8, L_RANGE, M_BUF, 16, 2),
        VAR("range_16B_u8_buf_ldnt_st0", 1, 8, L_RANGE, M_BUF, 2, 0),
        VAR("gs_16B_u4_buf_nt", 1, 4, L_GS, M_BUF, 2, 2),
    };
    for (const Variant &v : vars)
        for (int bpc : bpcs) {
            const dim3 g(cus * bpc);
            line("copy", v.name, bpc, 2.0 * bytes, time([&] { v.launch(g, a, b, n); }), "");
        }
    // placement: the best-known form at 2 WG/CU with the bases moved inside
    // the 2 MiB page (4 KiB, 64 KiB, 1 MiB) and the buffers' roles swapped
    const uint64_t shifts[] = {0, 4096, 65536, 1u << 20};
    for (uint64_t sa : shifts)
        for (uint64_t sb : shifts) {
            if (sa != sb && sa != 0 && sb != 0) continue;
            const u32x4 *a2 = (const u32x4 *)((const uint8_t *)a + sa);
            u32x4 *b2 = (u32x4 *)((uint8_t *)b + sb);
            char extra[96];
            snprintf(extra, sizeof extra, ", \"src_shift\": %llu, \"dst_shift\": %llu", (unsigned long long)sa,
                     (unsigned long long)sb);
            const dim3 g(cus * 2);
            line("copy_shift", "range_16B_u8", 2, 2.0 * bytes,
                 time([&] { launch_copy<1, 8, L_RANGE, M_GLOBAL, 0, 0>(g, a2, b2, n); }), extra);
        }
    {
        const dim3 g(cus * 2);
        line("copy_swapped", "range_16B_u8", 2, 2.0 * bytes,
             time([&] { launch_copy<1, 8, L_RANGE, M_GLOBAL, 0, 0>(g, (const u32x4 *)b, (u32x4 *)a, n); }), "");
        line("memcpy", "hipMemcpyAsync_d2d", 0, 2.0 * bytes,
             time([&] { CHK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); }), "");
    }
    CHK(hipFree(A));
    CHK(hipFree(B));
    CHK(hipFree(o));
    return 0;
}
