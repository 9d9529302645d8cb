// Stress test of mr::HostPool (marshrutka_amd/csrc/mr_pool.hpp), built by
// tests/test_host_pool.py with -fsanitize=thread: many short jobs back to back, each
// item must run exactly once per job and run() must not return before every item of
// its job has finished (a worker holding a stale ticket could claim an item
// of the next job against the old job's count).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../marshrutka_amd/csrc/mr_pool.hpp"

int main(int argc, char **argv) {
    const int jobs = argc > 1 ? std::atoi(argv[1]) : 20000;
    mr::HostPool &pool = mr::HostPool::get();
    std::vector<std::atomic<uint32_t>> hits(64);
    uint64_t bad = 0;
    for (int j = 0; j < jobs; ++j) {
        const uint32_t n = 2 + uint32_t(j % 31);  // short jobs of varying size
        for (uint32_t i = 0; i < n; ++i) hits[i].store(0, std::memory_order_relaxed);
        std::vector<uint32_t> local(n, 0);  // written by the items, read after run(): TSan sees a missing join
        pool.run(n, [&](uint32_t i) {
            hits[i].fetch_add(1, std::memory_order_relaxed);
            local[i] = uint32_t(j) + 1;
        });
        for (uint32_t i = 0; i < n; ++i)
            if (hits[i].load(std::memory_order_relaxed) != 1 || local[i] != uint32_t(j) + 1) ++bad;
    }
    // a job larger than one ticket's item field (split into consecutive jobs)
    const uint32_t big = (1u << 20) + 5;
    std::vector<uint8_t> once(big, 0);
    pool.run(big, [&](uint32_t i) { once[i] += 1; });
    for (uint32_t i = 0; i < big; ++i) bad += once[i] != 1;
    std::printf("threads=%u jobs=%d bad=%llu\n", pool.size(), jobs, (unsigned long long)bad);
    return bad ? 1 : 0;
}
