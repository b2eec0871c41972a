// Does a partially written 128-byte line cost an HBM read on gfx950? Two
// store-only kernels over the same buffer, run under rocprofv3 --pmc
// FETCH_SIZE / WRITE_SIZE (tools/tmp scripts): k_full writes every byte of
// every line (16 B per lane), k_partial writes 7 of every line's 8 16-byte
// chunks (the line's last chunk untouched, as at a record's payload end), and
// k_partial_pair writes the same line's two halves from two different waves
// far apart in time (a line shared by two records' copies). Nothing is read
// by any kernel, so any FETCH_SIZE is the memory side filling lines.
//   hipcc --offload-arch=gfx950 -O3 -o tools/partial_write_probe tools/partial_write_probe.hip
//   rocprofv3 --pmc FETCH_SIZE -- tools/partial_write_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_full(u32x4 *p, uint64_t chunks) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * blockDim.x)
        p[c] = u32x4{(uint32_t)c, 1u, 2u, 3u};
}

__global__ void k_partial(u32x4 *p, uint64_t chunks) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * blockDim.x)
        if ((c & 7) != 7) p[c] = u32x4{(uint32_t)c, 1u, 2u, 3u};
}

// chunks of every line whose bit is set in mask (8 chunks of 16 B per line)
__global__ void k_mask(u32x4 *p, uint64_t chunks, uint32_t mask) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * blockDim.x)
        if ((mask >> (c & 7)) & 1) p[c] = u32x4{(uint32_t)c, 1u, 2u, 3u};
}

// first half of every line, then (second launch) the second half
__global__ void k_half(u32x4 *p, uint64_t chunks, uint32_t second) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < chunks; c += (uint64_t)gridDim.x * blockDim.x)
        if (((c >> 2) & 1) == second) p[c] = u32x4{(uint32_t)c, 1u, 2u, 3u};
}

int main() {
    const uint64_t bytes = 8ull << 30, chunks = bytes / 16;
    u32x4 *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return 1;
    const dim3 grid(256 * 8), block(256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int rep = 0; rep < 2; rep++) {
        float ms[4];
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_full, grid, block, 0, 0, p, chunks);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[0], a, b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_partial, grid, block, 0, 0, p, chunks);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[1], a, b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_half, grid, block, 0, 0, p, chunks, 0u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[2], a, b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_half, grid, block, 0, 0, p, chunks, 1u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms[3], a, b);
        printf("{\"bytes\": %llu, \"full_ms\": %.3f, \"partial_7of8_ms\": %.3f, \"half1_ms\": %.3f, \"half2_ms\": %.3f",
               (unsigned long long)bytes, ms[0], ms[1], ms[2], ms[3]);
        // masks: 0x3F 96 B (32-B sectors 0-2 whole, 3 untouched), 0x7F 112 B
        // (sector 3 half), 0xFE (sector 0 half), 0x33 (sectors 0 and 2
        // whole, 64-B halves each half written), 0x0F / 0xF0 64-B halves
        const uint32_t masks[] = {0x3F, 0x7F, 0xFE, 0x33, 0x0F, 0xF0, 0x55};
        for (uint32_t m : masks) {
            float t;
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_mask, grid, block, 0, 0, p, chunks, m);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&t, a, b);
            printf(", \"mask_%02x_ms\": %.3f", m, t);
        }
        printf("}\n");
    }
    (void)hipFree(p);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
