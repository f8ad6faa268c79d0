// host_pool.cpp -- see host_pool.hpp.
#include "host_pool.hpp"

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>

namespace zfec_hip {

unsigned HostPool::usable_cpus() {
    unsigned n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = static_cast<unsigned>(CPU_COUNT(&set));
    if (n == 0) {
        const long v = sysconf(_SC_NPROCESSORS_ONLN);
        n = v > 0 ? static_cast<unsigned>(v) : 1;
    }
    // cgroup v2 quota: "max 100000" or "<quota> <period>"
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const unsigned long long quota = strtoull(q, nullptr, 10);
            const unsigned cap = static_cast<unsigned>(std::max<unsigned long long>(1, quota / period));
            n = std::min(n, cap);
        }
        fclose(f);
    }
    return std::max(1u, n);
}

HostPool& HostPool::get() {
    // One pool per process.  A forked child has none of its parent's threads,
    // so it builds its own (the parent's object is left alone, never freed).
    static std::mutex m;
    static HostPool* pool = nullptr;
    static pid_t owner = 0;
    std::lock_guard<std::mutex> g(m);
    if (!pool || owner != getpid()) {
        unsigned n = usable_cpus();
        if (const char* e = getenv("ZFEC_HIP_HOST_THREADS")) {
            const long v = strtol(e, nullptr, 10);
            if (v >= 1) n = static_cast<unsigned>(v);
        }
        n = std::min(32u, std::max(1u, n));
        pool = new HostPool(n);  // lives for the process: workers may be parked at exit
        owner = getpid();
    }
    return *pool;
}

HostPool::HostPool(unsigned nthreads) {
    // the caller of wait() is one of the copying threads; if the system cannot
    // create them all, the pool keeps the ones it got (at least the caller)
    for (unsigned i = 1; i < nthreads; ++i) {
        try {
            workers_.emplace_back([this] { worker(); });
        } catch (const std::exception&) {
            break;
        }
    }
}

HostPool::~HostPool() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    work_cv_.notify_all();
    for (auto& t : workers_) t.join();
}

void HostPool::copy_async(void* dst, const void* src, size_t len, CopyLatch* latch, size_t piece) {
    if (len == 0) return;
    piece = std::max<size_t>(piece, 64u << 10);
    const size_t n = (len + piece - 1) / piece;
    {
        // counted one by one, so a failed push (bad_alloc) leaves the latch
        // counting exactly the pieces that will run
        std::lock_guard<std::mutex> g(mu_);
        for (size_t i = 0; i < n; ++i) {
            const size_t off = i * piece;
            queue_.push_back({static_cast<char*>(dst) + off, static_cast<const char*>(src) + off,
                              std::min(piece, len - off), latch, nullptr});
            latch->pending += 1;
        }
    }
    if (n == 1)
        work_cv_.notify_one();
    else
        work_cv_.notify_all();
}

void HostPool::run_async(std::function<void()> fn, CopyLatch* latch) {
    {
        std::lock_guard<std::mutex> g(mu_);
        queue_.push_back({nullptr, nullptr, 0, latch, std::move(fn)});
        latch->pending += 1;
    }
    work_cv_.notify_one();
}

// Pops one piece and runs it with the lock released; false if the queue is empty.
bool HostPool::run_one(std::unique_lock<std::mutex>& lk) {
    if (queue_.empty()) return false;
    CopyPiece p = std::move(queue_.front());
    queue_.pop_front();
    lk.unlock();
    if (p.fn)
        p.fn();
    else
        std::memcpy(p.dst, p.src, p.len);
    lk.lock();
    if (--p.latch->pending == 0) done_cv_.notify_all();
    return true;
}

void HostPool::worker() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
        work_cv_.wait(lk, [this] { return stop_ || !queue_.empty(); });
        if (stop_) return;
        run_one(lk);
    }
}

void HostPool::wait(CopyLatch* latch) {
    std::unique_lock<std::mutex> lk(mu_);
    while (latch->pending) {
        if (!run_one(lk)) done_cv_.wait(lk, [&] { return latch->pending == 0 || !queue_.empty(); });
    }
}

}  // namespace zfec_hip
