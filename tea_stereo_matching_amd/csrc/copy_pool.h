// copy_pool.h -- host-only row-band copies over a small persistent worker pool (engine.cpp
// uses it to move images between callers' pageable buffers and the pinned staging).
// Header-only and free of HIP so the same code is built by tests/cpp/test_copy_pool.cpp
// under ThreadSanitizer and AddressSanitizer (tests/test_sanitizers.py).
#pragma once
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace tsm {

// Host copies between the caller's pageable buffers and the pinned staging: one core
// moves ~15-20 GB/s, so a config-B frame's 4.7 MB of copies cost ~0.3 ms on one thread,
// the largest part of the host call's overhead over the device pipeline.  A small pool
// of persistent workers (woken per job) splits each copy by row bands.
class CopyPool {
  public:
    static CopyPool& get() {
        static CopyPool pool;
        return pool;
    }
    // fn(i) for i in [0, n) on the workers and the calling thread; returns when all ran
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 1 || th_.empty() || getpid() != pid_) {  // a forked child has no workers
            for (int i = 0; i < n; ++i) fn(i);
            return;
        }
        std::lock_guard<std::mutex> job(job_mu_);  // one job at a time (handles on several threads)
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            active_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return active_ == 0; });
        fn_ = nullptr;
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }

  private:
    CopyPool() : pid_(getpid()) {
        const unsigned hw = std::thread::hardware_concurrency();
        const int nt = (int)std::min(7u, hw > 1 ? hw - 1 : 0u);
        for (int i = 0; i < nt; ++i) th_.emplace_back([this] { loop(); });
    }
    void work() {
        for (int i = next_.fetch_add(1); i < n_; i = next_.fetch_add(1)) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            work();
            std::lock_guard<std::mutex> lk(mu_);
            if (--active_ == 0) done_.notify_one();
        }
    }
    const pid_t pid_;
    std::vector<std::thread> th_;
    std::mutex job_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0;
    std::atomic<int> next_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// rows x rowb bytes from src (row step sstep) to dst (row step dstep), in row bands of
// >= 128 KB over the copy pool
inline void copy_rows(void* dst, size_t dstep, const void* src, size_t sstep, size_t rowb, int rows) {
    const size_t total = rowb * (size_t)rows;
    const int bands = (int)std::max<size_t>(1, std::min<size_t>(8, total / (128 * 1024)));
    const int per = (rows + bands - 1) / bands;
    CopyPool::get().run(bands, [&](int b) {
        const int y0 = b * per, y1 = std::min(rows, y0 + per);
        if (y0 >= y1) return;
        char* d = static_cast<char*>(dst) + (size_t)y0 * dstep;
        const char* s = static_cast<const char*>(src) + (size_t)y0 * sstep;
        if (dstep == rowb && sstep == rowb) std::memcpy(d, s, rowb * (size_t)(y1 - y0));
        else for (int y = y0; y < y1; ++y) std::memcpy(d + (size_t)(y - y0) * dstep, s + (size_t)(y - y0) * sstep, rowb);
    });
}

}  // namespace tsm
