// The host walk's worker threads (ipxg_engine.cpp plugin_walk).  Host C++ only -- no HIP -- so
// tests/test_walkpool.py compiles it alone with g++ under ThreadSanitizer / AddressSanitizer.
//
// run(f, n) calls f(t) for every t in [0, n) -- t = 0 on the calling thread -- and returns when all
// have returned; threads n .. size()-1 sit the job out.  The pool may hold more threads than one
// walk uses (a small batch walks on fewer), and the round-3 fault came from exactly that: run(f)
// then called f on EVERY pool thread, and a job indexing per-walk arrays sized n by t wrote past
// them.  The bound now lives here, where a job cannot forget it.
//
// Persistent across batches: a configs[2] batch walks ~10^5 flows, and spawning threads per batch
// would cost more than a small walk.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ipxg {

class WalkPool {
public:
    explicit WalkPool(unsigned n) {
        for (unsigned t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
    }
    ~WalkPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    WalkPool(const WalkPool&) = delete;
    WalkPool& operator=(const WalkPool&) = delete;

    unsigned size() const { return (unsigned)th_.size() + 1; }
    // true when a job raised out of a thread since the last call (then: an engine bug or a plugin
    // that throws past the C ABI; plugin_walk fails the batch with IPXG_EPLUGIN)
    bool take_escaped() { return escaped_.exchange(false); }

    // f(t) for t in [0, min(n, size())); returns the number of calls made
    unsigned run(const std::function<void(unsigned)>& f, unsigned n) {
        if (n > size()) n = size();
        if (n == 0) return 0;
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            n_ = n;
            left_ = (unsigned)th_.size();  // every thread wakes and reports, used or not
            ++gen_;
        }
        cv_.notify_all();
        // the caller's share: whatever it raises is held until the other threads are done with f
        // (f may live in the caller's frame, which an unwind would leave while they still run it)
        try {
            f(0);
        } catch (...) {
            escaped_.store(true);
        }
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        job_ = nullptr;
        return n;
    }

private:
    void loop(unsigned t) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* f;
            unsigned n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                f = job_;
                n = n_;
            }
            // nothing may unwind out of a worker thread (std::terminate): recorded and reported
            // by the caller like a failed range
            if (t < n) {
                try {
                    (*f)(t);
                } catch (...) {
                    escaped_.store(true);
                }
            }
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    unsigned n_ = 0;
    unsigned left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
    std::atomic<bool> escaped_{false};
};

}  // namespace ipxg
