// host_copy.h — multi-threaded host memcpy for the storage feeds.
//
// Filling a pinned batch is the host side of both feeds (the copy that
// iterator/cursor.go:31-38 makes of each bbolt value; the payloads a Put
// hands over). One thread copies 10-20 GB/s; PCIe Gen5 x16 moves ~50 GB/s,
// so large batches split their copies by bytes over a few threads.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace honu {

struct HostCopy {
    uint8_t *dst;
    const uint8_t *src;
    uint64_t len;
};

// Below this many bytes a batch is copied on the calling thread.
constexpr uint64_t kParallelCopyMin = 8ull << 20;

inline unsigned host_copy_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min(8u, hw ? hw / 2 : 1u));
}

// Copies every job; with total >= kParallelCopyMin the byte space of the
// jobs (in order) is cut into equal ranges, one per thread.
inline void host_copy(const std::vector<HostCopy> &jobs, uint64_t total) {
    const unsigned T = total >= kParallelCopyMin ? host_copy_threads() : 1;
    if (T == 1) {
        for (const HostCopy &j : jobs)
            if (j.len) std::memcpy(j.dst, j.src, j.len);
        return;
    }
    auto run = [&](uint64_t lo, uint64_t hi) {  // bytes [lo, hi) of the job sequence
        uint64_t at = 0;
        for (const HostCopy &j : jobs) {
            const uint64_t a = std::max(lo, at), b = std::min(hi, at + j.len);
            if (a < b) std::memcpy(j.dst + (a - at), j.src + (a - at), b - a);
            at += j.len;
            if (at >= hi) break;
        }
    };
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    for (unsigned t = 1; t < T; t++) pool.emplace_back(run, total * t / T, total * (t + 1) / T);
    run(0, total / T);
    for (std::thread &th : pool) th.join();
}

}  // namespace honu
