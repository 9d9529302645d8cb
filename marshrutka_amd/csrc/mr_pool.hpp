// mr_pool.hpp — the host thread pool of libmarshrutka_pf.so (plain C++, no HIP), in a
// header of its own so that tests/cpp/pool_stress.cpp can run it under ThreadSanitizer.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>

namespace mr {
// A persistent pool for the per-batch host work (grouping a batch by source, the fetch's
// copies): run(n, fn) calls fn(i) for every i in [0, n) on the pool's workers and the
// calling thread, and returns when every call has finished.  One job at a time (callers
// are serialised); min(16, hardware threads) threads (MR_HOST_THREADS overrides: a GPU
// box's share of its host is 16 CPUs, more threads would only time-slice).
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();  // never destroyed: workers wait on it at exit
        return *p;
    }
    uint32_t size() const { return nthreads_; }
    void run(uint32_t n, const std::function<void(uint32_t)> &fn) {
        if (n == 0) return;
        if (nthreads_ <= 1 || n == 1) {
            for (uint32_t i = 0; i < n; ++i) fn(i);
            return;
        }
        if (n > kItemMask) {  // more items than a ticket holds: consecutive jobs
            for (uint32_t lo = 0; lo < n; lo += kItemMask) {
                const uint32_t cnt = std::min<uint32_t>(kItemMask, n - lo);
                run(cnt, [&](uint32_t i) { fn(lo + i); });
            }
            return;
        }
        std::lock_guard<std::mutex> job(job_mu_);
        fn_ = &fn;
        done_.store(0, std::memory_order_relaxed);
        const uint64_t g = ((ticket_.load(std::memory_order_relaxed) >> kJobShift) + 1) & kJobMask;
        // the job's item count travels in the ticket word itself: a worker that read the
        // previous job's ticket can only fail its compare-and-swap, never claim an item of
        // this job against a stale count
        ticket_.store(g << kJobShift | uint64_t(n) << kItemBits, std::memory_order_release);  // publishes fn_
        if (sleepers_.load(std::memory_order_acquire) > 0) {
            std::lock_guard<std::mutex> lk(mu_);
            cv_.notify_all();
        }
        work(g);
        while (done_.load(std::memory_order_acquire) < n) __builtin_ia32_pause();
    }

  private:
    static constexpr uint32_t kItemBits = 20, kJobShift = 2 * kItemBits;
    static constexpr uint32_t kItemMask = (1u << kItemBits) - 1;
    static constexpr uint64_t kJobMask = (uint64_t(1) << (64 - kJobShift)) - 1;
    HostPool() {
        nthreads_ = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
        if (const char *e = std::getenv("MR_HOST_THREADS")) nthreads_ = uint32_t(std::max(1, std::min(64, std::atoi(e))));
        for (uint32_t t = 1; t < nthreads_; ++t) std::thread([this] { loop(); }).detach();
    }
    // Items are claimed by compare-and-swap on {job, item count, next item}: a worker still
    // in an old job can never take (and lose) an item of the next one.  fn_ is read only
    // after a successful claim, while run() of that job waits for the item to finish.
    void work(uint64_t g) {
        for (;;) {
            uint64_t v = ticket_.load(std::memory_order_acquire);
            if ((v >> kJobShift) != g) return;
            const uint32_t next = uint32_t(v) & kItemMask, n = uint32_t(v >> kItemBits) & kItemMask;
            if (next >= n) return;
            if (!ticket_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
            (*fn_)(next);
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g = ticket_.load(std::memory_order_acquire) >> kJobShift;
            // spin briefly for the next job (a batch's phases come back to back), then sleep: a
            // longer spin burns the CPU quota a GPU box gives the process (cgroup cpu.max)
            for (int k = 0; g == seen && k < 2000; ++k) {
                __builtin_ia32_pause();
                g = ticket_.load(std::memory_order_acquire) >> kJobShift;
            }
            if (g == seen) {
                std::unique_lock<std::mutex> lk(mu_);
                sleepers_.fetch_add(1, std::memory_order_acq_rel);
                cv_.wait(lk, [&] { return (ticket_.load(std::memory_order_acquire) >> kJobShift) != seen; });
                sleepers_.fetch_sub(1, std::memory_order_acq_rel);
                g = ticket_.load(std::memory_order_acquire) >> kJobShift;
            }
            seen = g;
            work(g);
        }
    }
    uint32_t nthreads_ = 1;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_;
    const std::function<void(uint32_t)> *fn_ = nullptr;
    std::atomic<uint64_t> ticket_{0};  // job << 40 | item count << 20 | next item
    std::atomic<uint32_t> done_{0};
    std::atomic<int> sleepers_{0};
};
}  // namespace mr
