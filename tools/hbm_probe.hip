// hbm_probe.hip — achievable HBM rates on this device (read-only, write-only,
// copy) for grid-stride and per-wave-range access, 16 B per lane. Standalone:
//   hipcc -O3 --offload-arch=gfx950 -o hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U>
__global__ __launch_bounds__(256) void k_copy_gs(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = a[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; u++) b[i + u * 256] = v[u];
    }
}
template <int U>
__global__ __launch_bounds__(256) void k_copy_range(const u32x4 *__restrict__ a, u32x4 *__restrict__ b, size_t n) {
    size_t W = (size_t)gridDim.x * 4, w = (size_t)blockIdx.x * 4 + threadIdx.x / 64;
    size_t lo = n * w / W, hi = n * (w + 1) / W;
    for (size_t i = lo + (threadIdx.x & 63); i < hi; i += 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * 64 < hi) v[u] = a[i + u * 64];
#pragma unroll
        for (int u = 0; u < U; u++) if (i + u * 64 < hi) b[i + u * 64] = v[u];
    }
}
__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ a, size_t n, unsigned *out) {
    size_t stride = (size_t)gridDim.x * 256 * 4;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        u32x4 v0 = a[i], v1 = a[i + 256], v2 = a[i + 512], v3 = a[i + 768];
        acc ^= v0 ^ v1 ^ v2 ^ v3;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
}
__global__ __launch_bounds__(256) void k_write(u32x4 *__restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * 256 * 4;
    for (size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        u32x4 v = {(unsigned)i, 1, 2, 3};
        b[i] = v; b[i + 256] = v; b[i + 512] = v; b[i + 768] = v;
    }
}

int main(int argc, char **argv) {
    size_t bytes = (argc > 1 ? atoll(argv[1]) : 16) << 30;
    size_t n = bytes / 16;
    u32x4 *a, *b;
    unsigned *o;
    CHK(hipMalloc(&a, bytes));
    CHK(hipMalloc(&b, bytes));
    CHK(hipMalloc(&o, 64));
    CHK(hipMemset(a, 1, bytes));
    CHK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    int blocks[] = {256, 512, 1024, 2048, 4096};
    for (int rep = 0; rep < 2; rep++)
    for (int bi = 0; bi < 5; bi++) {
        int g = blocks[bi];
        float ms;
        auto run = [&](const char *name, double traffic, auto launch) {
            launch();
            CHK(hipEventRecord(e0));
            for (int r = 0; r < 5; r++) launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) printf("%-14s blocks %5d  %8.1f GB/s\n", name, g, traffic * 5 / (ms / 1e3) / 1e9);
        };
        run("read", bytes, [&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, n - 1024, o); });
        run("write", bytes, [&] { hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, 0, b, n - 1024); });
        run("copy_gs_u4", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy_gs<4>, dim3(g), dim3(256), 0, 0, a, b, n - 1024); });
        run("copy_gs_u1", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy_gs<1>, dim3(g), dim3(256), 0, 0, a, b, n - 1024); });
        run("copy_range_u4", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy_range<4>, dim3(g), dim3(256), 0, 0, a, b, n); });
        run("copy_range_u8", 2.0 * bytes, [&] { hipLaunchKernelGGL(k_copy_range<8>, dim3(g), dim3(256), 0, 0, a, b, n); });
    }
    float ms;
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) CHK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0));
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-14s %8.1f GB/s\n", "hipMemcpyD2D", 2.0 * bytes * 5 / (ms / 1e3) / 1e9);
    return 0;
}
