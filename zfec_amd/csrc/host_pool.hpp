// host_pool.hpp -- persistent host worker threads for the staged host path.
//
// The drop-in `bytes` API hands the library pageable host buffers
// (/root/reference/zfec/_fecmodule.c:206-242 allocates fresh output `bytes`
// objects per call).  The staged path (fec_abi.cpp, run_staged) moves them
// through pinned staging slots with memcpy on these threads: the inputs are
// copied in, the kernel reads and writes the pinned slots over PCIe, and the
// outputs are copied out into the callers' (fresh, unmapped) pages, faulting
// them in on many cores at once.  One pool per process, created on first use.
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace zfec_hip {

// Counts outstanding copy pieces of one batch; wait() returns when all ran.
struct CopyLatch {
    size_t pending = 0;  // guarded by the pool's mutex
};

struct CopyPiece {
    void* dst;
    const void* src;
    size_t len;
    CopyLatch* latch;
    std::function<void()> fn;  // a task instead of a memcpy when set
};

class HostPool {
public:
    // Threads: ZFEC_HIP_HOST_THREADS, else the CPUs this process may use
    // (affinity mask, capped by the cgroup's cpu.max quota), at most 32.
    static HostPool& get();
    static unsigned usable_cpus();

    unsigned threads() const { return static_cast<unsigned>(workers_.size()) + 1; }

    // Queue memcpy(dst, src, len) cut into pieces of about `piece` bytes;
    // the latch counts them.  Returns immediately.
    void copy_async(void* dst, const void* src, size_t len, CopyLatch* latch, size_t piece = size_t(1) << 20);

    // Queue a task (e.g. a group of row copies); the latch counts it.
    void run_async(std::function<void()> fn, CopyLatch* latch);

    // Wait for every piece counted by `latch`; the calling thread runs queued
    // pieces (of any latch) while it waits.
    void wait(CopyLatch* latch);

    ~HostPool();

private:
    explicit HostPool(unsigned nthreads);
    void worker();
    bool run_one(std::unique_lock<std::mutex>& lk);

    std::mutex mu_;
    std::condition_variable work_cv_, done_cv_;
    std::deque<CopyPiece> queue_;
    std::vector<std::thread> workers_;
    bool stop_ = false;
};

}  // namespace zfec_hip
