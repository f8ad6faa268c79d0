// fec_abi.cpp -- the C-ABI of libzfec_hip.so (include/zfec_hip.h).
//
// Part 1 replaces /root/reference/zfec/fec.h:33-57 (fec_init, fec_new,
// fec_free, fec_encode, fec_decode) and the two helpers fec.c also exports.
// Host-side work here is O(k^3) matrix algebra and argument checking; every
// output byte is produced by the HIP kernels in kernels.hip.  Host buffers are
// staged through per-thread device buffers; device buffers are used in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <thread>
#include <unistd.h>

#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/zfec_hip.h"
#include "bitslice.hpp"
#include "config.hpp"
#include "gf256.hpp"
#include "host_pool.hpp"
#include "kernels.hpp"

#define FEC_API extern "C" __attribute__((visibility("default")))

namespace zfec_hip {
namespace {

constexpr unsigned long kFecMagic = 0xFECC0DECUL;  // zfec/fec.c:421

thread_local int t_status = FEC_OK;
thread_local char t_msg[256] = "";

int set_status(int st, const char* fmt = nullptr, ...) {
    t_status = st;
    if (fmt) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(t_msg, sizeof t_msg, fmt, ap);
        va_end(ap);
    } else {
        t_msg[0] = '\0';
    }
    return st;
}

int hip_fail(hipError_t e, const char* what) {
    return set_status(FEC_EHIP, "%s: %s", what, hipGetErrorString(e));
}

// No C++ exception crosses the C-ABI: a failed allocation (or a thread the
// system cannot create) inside a call becomes its status.
template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_status(FEC_ENOMEM, "out of host memory");
    } catch (const std::exception& x) {
        return set_status(FEC_ENOMEM, "host resources exhausted: %s", x.what());
    }
}

unsigned long magic_of(const fec_t* p) {
    return ((kFecMagic ^ p->k) ^ p->n) ^ reinterpret_cast<unsigned long>(p->enc_matrix);
}

bool valid_code(const fec_t* c) { return c && c->enc_matrix && c->magic == magic_of(c); }

// ---- per-thread, per-device staging -----------------------------------------

constexpr int kStageSlots = 3;  // staged host path: copy-in | kernel | copy-out

struct DevCtx {
    hipStream_t stream = nullptr;  // library stream: kernels of the host path, sync calls
    void* dbuf = nullptr;
    size_t dcap = 0;
    void* hbuf = nullptr;  // pinned
    void* hbuf_dev = nullptr;  // its address in the device's view (kernels read / write it over PCIe)
    size_t hcap = 0;
    void* sbuf = nullptr;  // pinned staging slots of the staged host path
    void* sbuf_dev = nullptr;
    size_t scap = 0;
    hipEvent_t ev_stg[kStageSlots] = {};
    uint32_t* flag = nullptr;      // pinned completion word of small synchronous calls
    uint32_t* flag_dev = nullptr;  // its address in the device's view
    uint32_t seq = 0;
};

struct ThreadCtx {
    std::unordered_map<int, DevCtx> dev;
    ~ThreadCtx() {
        for (auto& kv : dev) {
            int cur = 0;
            if (hipGetDevice(&cur) != hipSuccess) continue;
            if (hipSetDevice(kv.first) != hipSuccess) continue;
            DevCtx& d = kv.second;
            if (d.stream) (void)hipStreamDestroy(d.stream);
            for (int i = 0; i < kStageSlots; ++i)
                if (d.ev_stg[i]) (void)hipEventDestroy(d.ev_stg[i]);
            if (d.dbuf) (void)hipFree(d.dbuf);
            if (d.hbuf) (void)hipHostFree(d.hbuf);
            if (d.sbuf) (void)hipHostFree(d.sbuf);
            if (d.flag) (void)hipHostFree(d.flag);
            (void)hipSetDevice(cur);
        }
    }
};

thread_local ThreadCtx t_ctx;

int dev_ctx(int device, DevCtx** out) {
    DevCtx& d = t_ctx.dev[device];
    if (!d.stream) {
        hipError_t e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking);
        if (e != hipSuccess) return hip_fail(e, "hipStreamCreateWithFlags");
    }
    *out = &d;
    return FEC_OK;
}

int ensure_dbuf(DevCtx& d, size_t bytes) {
    if (bytes <= d.dcap) return FEC_OK;
    if (d.dbuf) {
        (void)hipStreamSynchronize(d.stream);
        (void)hipFree(d.dbuf);
        d.dbuf = nullptr;
        d.dcap = 0;
    }
    const size_t cap = std::max<size_t>(bytes, 1u << 20);
    hipError_t e = hipMalloc(&d.dbuf, cap);
    if (e != hipSuccess) return set_status(FEC_ENOMEM, "hipMalloc(%zu): %s", cap, hipGetErrorString(e));
    d.dcap = cap;
    return FEC_OK;
}

int ensure_hbuf(DevCtx& d, size_t bytes) {
    if (bytes <= d.hcap) return FEC_OK;
    if (d.hbuf) {
        (void)hipStreamSynchronize(d.stream);
        (void)hipHostFree(d.hbuf);
        d.hbuf = nullptr;
        d.hbuf_dev = nullptr;
        d.hcap = 0;
    }
    const size_t cap = std::max<size_t>(bytes, 1u << 20);
    hipError_t e = hipHostMalloc(&d.hbuf, cap, hipHostMallocDefault);
    if (e != hipSuccess) return set_status(FEC_ENOMEM, "hipHostMalloc(%zu): %s", cap, hipGetErrorString(e));
    if ((e = hipHostGetDevicePointer(&d.hbuf_dev, d.hbuf, 0)) != hipSuccess || !d.hbuf_dev) {
        (void)hipGetLastError();
        d.hbuf_dev = d.hbuf;  // unified addressing: the host address is valid on the device
    }
    d.hcap = cap;
    return FEC_OK;
}

// Device holding p, or -1 for host memory.  For page-locked host memory
// (hipHostMalloc / hipHostRegister, torch pin_memory) *pinned is set and
// *dev_ptr is the address a kernel uses to read / write it over PCIe.
int pointer_device(const void* p, bool* pinned = nullptr, void** dev_ptr = nullptr) {
    hipPointerAttribute_t a;
    if (pinned) *pinned = false;
    if (dev_ptr) *dev_ptr = nullptr;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return a.device;
    if (a.type == hipMemoryTypeHost) {
        if (pinned) *pinned = true;
        if (dev_ptr) *dev_ptr = a.devicePointer ? a.devicePointer : const_cast<void*>(p);
    }
    return -1;
}

int gpu_available() {
    // the device count of a process does not change: cached once positive
    static std::atomic<int> cached{0};
    const int c = cached.load(std::memory_order_relaxed);
    if (c > 0) return c;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (n > 0) cached.store(n, std::memory_order_relaxed);
    return n;
}

// Small synchronous calls (one-workgroup register-kernel launches): the
// kernel publishes completion in pinned host memory and the calling thread
// spins on it -- launch to return 6.4-6.9 us against 12.2 us through
// hipStreamSynchronize (tools/mb_sync.hip, profiles/r02_sync_probe.log).
// The stream is queried every 1024 spins, so an error ends the wait; past
// 200 us it blocks in hipStreamSynchronize.  ZFEC_HIP_WAIT=sync turns it off.
uint32_t* signal_slot(DevCtx& d) {
    if (!config().wait_signal) return nullptr;
    if (!d.flag) {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        void* pd = nullptr;
        if (hipHostGetDevicePointer(&pd, p, 0) != hipSuccess || !pd) {
            (void)hipGetLastError();
            pd = p;
        }
        d.flag = static_cast<uint32_t*>(p);
        d.flag_dev = static_cast<uint32_t*>(pd);
        __atomic_store_n(d.flag, 0u, __ATOMIC_RELEASE);
    }
    if (++d.seq == 0) d.seq = 1;
    return d.flag_dev;
}

hipError_t wait_signal(DevCtx& d, hipStream_t st) {
    const uint32_t seq = d.seq;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t n = 1;; ++n) {
        if (__atomic_load_n(d.flag, __ATOMIC_ACQUIRE) == seq) return hipSuccess;
        if ((n & 1023u) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) return hipSuccess;  // the stream is idle: the kernel has finished
            if (q != hipErrorNotReady) return q;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
        }
    }
    return hipStreamSynchronize(st);
}

// RAII: restore the caller's current device.
struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) {
            (void)hipSetDevice(dev);
            changed = true;
        }
    }
    ~DeviceGuard() {
        if (changed && prev >= 0) (void)hipSetDevice(prev);
    }
};

// ---- the engine: apply an r x k matrix to k blocks -----------------------------

constexpr size_t align_up_4k(size_t x) { return (x + 4095) / 4096 * 4096; }

// in[j] / out[i] are device pointers (block bases of stripe 0); stripes are
// in_sstride / out_sstride apart; coef is r x k with rows coef_stride apart.
// Splits into launches that respect the kernels' limits: <= kMaxOut outputs
// per launch; all k inputs in one pass where a bit-sliced kernel takes them
// (wide_launch_ok), otherwise groups of <= kMaxIn inputs, later groups
// XOR-accumulating, and <= kMaxCoef coefficients per launch; at most
// Config::launch_units kMinChunk-byte units per launch.  Blocks longer than
// that are cut into byte ranges of their own launches: output byte x depends
// only on byte x of the inputs (zfec/fec.c:494-503, :547-556).
thread_local unsigned t_launches = 0;  // launches made by this thread (the signal path checks it made one)
thread_local int t_last_wait = 0;      // 1: the last synchronous small call waited on its kernel's signal (fec_last_wait)

int apply_matrix_range(const uint8_t* coef, unsigned coef_stride, unsigned k, unsigned r, const uint8_t* const* in,
                       uint8_t* const* out, size_t sz, size_t nstripes, size_t in_sstride, size_t out_sstride,
                       hipStream_t stream);

int apply_matrix(const uint8_t* coef /* r x k */, unsigned k, unsigned r, const uint8_t* const* in,
                 uint8_t* const* out, size_t sz, size_t nstripes, size_t in_sstride, size_t out_sstride,
                 hipStream_t stream, unsigned coef_stride = 0) {
    if (r == 0 || sz == 0 || nstripes == 0) return FEC_OK;
    if (!coef_stride) coef_stride = k;
    const size_t cps = (sz + kMinChunk - 1) / kMinChunk;
    const size_t max_units = config().launch_units;
    if (cps <= max_units)
        return apply_matrix_range(coef, coef_stride, k, r, in, out, sz, nstripes, in_sstride, out_sstride, stream);
    // near-equal byte ranges on 4 KiB boundaries, each within the unit limit
    const size_t pieces = (cps + max_units - 1) / max_units;
    const size_t piece = align_up_4k((sz + pieces - 1) / pieces);
    const uint8_t* pin[kMaxWideIn];
    uint8_t* pout[kMaxWideIn];
    for (size_t b0 = 0; b0 < sz; b0 += piece) {
        const size_t len = std::min(piece, sz - b0);
        for (unsigned j = 0; j < k; ++j) pin[j] = in[j] + b0;
        for (unsigned i = 0; i < r; ++i) pout[i] = out[i] + b0;
        if (apply_matrix_range(coef, coef_stride, k, r, pin, pout, len, nstripes, in_sstride, out_sstride, stream))
            return t_status;
    }
    return FEC_OK;
}

int apply_matrix_range(const uint8_t* coef, unsigned coef_stride, unsigned k, unsigned r, const uint8_t* const* in,
                       uint8_t* const* out, size_t sz, size_t nstripes, size_t in_sstride, size_t out_sstride,
                       hipStream_t stream) {
    const size_t cps = (sz + kMinChunk - 1) / kMinChunk;
    const size_t stripes_per_launch = std::max<size_t>(1, config().launch_units / cps);
    // wide codes: every input in one bit-sliced pass per row group
    // (not under graph capture: the one-pass wide kernels read device-side
    // tables filled at enqueue time; the passes' kernels take their arguments)
    const bool wide = k > static_cast<unsigned>(kMaxIn) &&
                      wide_launch_ok(k, r, sz, std::min(stripes_per_launch, nstripes)) && !stream_capturing(stream);
    const unsigned kstep = wide ? k : static_cast<unsigned>(kMaxIn);
    const uint8_t* pin[kMaxWideIn];
    uint8_t* pout[kMaxWideIn];
    for (unsigned j0 = 0; j0 < k; j0 += kstep) {
        const unsigned kg = std::min<unsigned>(kstep, k - j0);
        // wide: every row in one launch (matapply_bsg walks row groups itself,
        // the JIT takes k * r <= kJitMaxCoef)
        const unsigned rmax = wide ? r : std::max<unsigned>(1, std::min<unsigned>(kMaxOut, kMaxCoef / kg));
        const unsigned ngroups = (r + rmax - 1) / rmax;
        for (unsigned g = 0; g < ngroups; ++g) {
            // near-equal row groups
            const unsigned i0 = g * r / ngroups, rg = (g + 1) * r / ngroups - i0;
            for (size_t s0 = 0; s0 < nstripes; s0 += stripes_per_launch) {
                const size_t ns = std::min(stripes_per_launch, nstripes - s0);
                for (unsigned j = 0; j < kg; ++j) pin[j] = in[j0 + j] + s0 * in_sstride;
                for (unsigned i = 0; i < rg; ++i) pout[i] = out[i0 + i] + s0 * out_sstride;
                ApplySpec a;
                a.coef = coef + size_t(i0) * coef_stride + j0;
                a.coef_stride = coef_stride;
                a.k = kg;
                a.r = rg;
                a.in = pin;
                a.out = pout;
                a.sz = sz;
                a.nstripes = ns;
                a.in_sstride = in_sstride;
                a.out_sstride = out_sstride;
                a.accumulate = j0 > 0;
                ++t_launches;
                const hipError_t e = launch_apply(a, stream);
                if (e != hipSuccess) return hip_fail(e, "launch_apply");
            }
        }
    }
    return FEC_OK;
}

// ---- host/device pointer marshalling for the fec.h-shaped entry points -------

struct Marshal {
    int device = -1;
    std::vector<const uint8_t*> din;
    std::vector<uint8_t*> dout;
    std::vector<int> in_host, out_host;  // indices of host-memory blocks
    bool all_pinned = true;              // every host block is page-locked
    std::vector<const uint8_t*> zin;     // kernel-visible address of every block (zero-copy), when all_pinned
    std::vector<uint8_t*> zout;
};

// Classify pointers and pick the device.  All device pointers must live on one device.
int classify(const gf* const* in, size_t nin, gf* const* out, size_t nout, Marshal& m) {
    m.in_host.clear();
    m.out_host.clear();
    m.all_pinned = true;
    m.zin.assign(in, in + nin);
    m.zout.assign(out, out + nout);
    int dev = -1;
    auto visit = [&](const void* p, bool is_in, size_t idx) -> int {
        if (!p) return set_status(FEC_EINVAL, "%s block %zu is NULL", is_in ? "input" : "output", idx);
        bool pinned = false;
        void* dp = nullptr;
        const int d = pointer_device(p, &pinned, &dp);
        if (d < 0) {
            (is_in ? m.in_host : m.out_host).push_back(static_cast<int>(idx));
            m.all_pinned = m.all_pinned && pinned;
            if (pinned) {
                if (is_in)
                    m.zin[idx] = static_cast<const uint8_t*>(dp);
                else
                    m.zout[idx] = static_cast<uint8_t*>(dp);
            }
        } else if (dev < 0) {
            dev = d;
        } else if (d != dev) {
            return set_status(FEC_EINVAL, "blocks live on different devices (%d, %d)", dev, d);
        }
        return FEC_OK;
    };
    for (size_t i = 0; i < nin; ++i)
        if (visit(in[i], true, i)) return t_status;
    for (size_t i = 0; i < nout; ++i)
        if (visit(out[i], false, i)) return t_status;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return set_status(FEC_ENODEV, "no current HIP device");
    m.device = dev;
    return FEC_OK;
}

// Host blocks of up to Config::pack_limit bytes in total (4 MiB) go through
// one pinned bounce buffer (one H2D / D2H each way); larger ones take the
// staged path.  From Config::stage_min bytes (512 KiB), blocks of at least
// kStageMinBlock bytes take the staged path too: its overlapped copy-in / kernel / copy-out beats the bounce
// buffer's serial memcpy / DMA / kernel / DMA / memcpy (K=3/M=10 from bytes,
// 1 MiB stripe: 137 vs 209 us per encode; 256 KiB stripe: 69 vs 77 us), but
// not for many small blocks (K=20/M=60, 256 KiB stripe of 13 KB blocks: 260
// vs 122 us; tools/archive/host_lat_ab.py, profiles/r02_host_lat_ab.log).
constexpr size_t kStageMinBlock = size_t(64) << 10;
// Up to Config::zc_limit bytes (1.5 MiB; calls of k <= 4, r <= 8 up to that
// size stay on the bounce buffer, run_single) the kernel accesses the bounce
// buffer in place.  Round 2 stopped at 256 KiB; an interleaved A/B of 100-150
// KB K=3/M=10 stripes from bytes (tools/archive/small_ab_inproc.py --set zc,
// profiles/r03_zc_ab.log): encode 44.5-51.3 -> 25.1-33.0 us, decode
// 17.0-38.3 -> 16.9-19.8 us against one H2D and one D2H copy.

constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Kernel-visible address of the host block [p, p + n), or nullptr unless the
// whole block is page-locked (first and last byte mapped at the same offset).
const uint8_t* mapped_block(const void* p, size_t n) {
    bool pa = false, pb = false;
    void *da = nullptr, *db = nullptr;
    const char* last = static_cast<const char*>(p) + (n ? n - 1 : 0);
    if (pointer_device(p, &pa, &da) >= 0 || !pa) return nullptr;
    if (pointer_device(last, &pb, &db) >= 0 || !pb) return nullptr;
    if (static_cast<char*>(db) - static_cast<char*>(da) != last - static_cast<const char*>(p)) return nullptr;
    return static_cast<const uint8_t*>(da);
}

// Bytes of every host block per staged chunk: ZFEC_HIP_STAGE_CHUNK, else
// at most a quarter of the block (so that copy-in, kernel and copy-out of
// consecutive chunks overlap) and at most about 16 MiB of staging per chunk
// over all host blocks, in whole 64 KiB
// (K=3/M=10, 64 MiB from bytes: 8 MiB chunks 8.7 GB/s encode, 16-20 MiB 9.3;
// 2.5 MiB 6.4; profiles/r02_host_stage_ab.log).
size_t staged_chunk(size_t nblocks, size_t sz) {
    if (const size_t v = config().stage_chunk) return v;
    const size_t total = size_t(16) << 20, g = size_t(64) << 10;
    const size_t by_total = total / std::max<size_t>(1, nblocks) / g * g;
    const size_t quarter = (sz + 4 * g - 1) / (4 * g) * g;  // at least 4 chunks, so the stages overlap
    return std::max<size_t>(256u << 10, std::min(by_total, quarter));
}

int ensure_sbuf(DevCtx& d, size_t bytes) {
    if (!d.ev_stg[0])
        for (int i = 0; i < kStageSlots; ++i) {
            hipError_t e = hipEventCreateWithFlags(&d.ev_stg[i], hipEventDisableTiming);
            if (e != hipSuccess) return hip_fail(e, "staging events");
        }
    if (bytes <= d.scap) return FEC_OK;
    if (d.sbuf) {
        (void)hipDeviceSynchronize();  // no kernel of an earlier call may still use the old slots
        (void)hipHostFree(d.sbuf);
        d.sbuf = d.sbuf_dev = nullptr;
        d.scap = 0;
    }
    hipError_t e = hipHostMalloc(&d.sbuf, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return set_status(FEC_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    if ((e = hipHostGetDevicePointer(&d.sbuf_dev, d.sbuf, 0)) != hipSuccess || !d.sbuf_dev) {
        (void)hipGetLastError();
        d.sbuf_dev = d.sbuf;
    }
    d.scap = bytes;
    return FEC_OK;
}

// Large pageable host blocks, staged: nothing of the caller's is page-locked.
// The byte range is cut into chunks; for chunk c the host threads (HostPool)
// copy the input blocks' bytes into a pinned staging slot, the kernel reads
// that slot and writes the outputs into the slot over PCIe (zero-copy), and
// the threads copy the outputs out into the caller's blocks -- faulting in
// fresh output pages (new `bytes` objects, zfec/_fecmodule.c:206-242) on every
// pool thread at once.  kStageSlots slots rotate, so copy-in of chunk c + 1 and
// copy-out of chunk c - 1 run while chunk c's kernel does.  Replaces
// hipHostRegister of every block (run_pageable), whose cost is the kernel
// mapping each fresh page one by one.  Device-resident and
// caller-locked blocks are read / written in place.
int run_staged(DevCtx& d, const uint8_t* coef, unsigned k, unsigned r, const gf* const* in, gf* const* out,
               size_t sz, Marshal& m, hipStream_t st) {
    std::vector<char> host_in(k, 0), host_out(r, 0);
    std::vector<const uint8_t*> base_in(m.zin);  // kernel-visible bases of device / caller-locked blocks
    std::vector<uint8_t*> base_out(m.zout);
    std::vector<unsigned> sin, sout;  // staged blocks
    for (int i : m.in_host) {
        const uint8_t* z = mapped_block(in[i], sz);
        if (z) base_in[i] = z;
        else {
            host_in[i] = 1;
            sin.push_back(static_cast<unsigned>(i));
        }
    }
    for (int i : m.out_host) {
        const uint8_t* z = mapped_block(out[i], sz);
        if (z) base_out[i] = const_cast<uint8_t*>(z);
        else {
            host_out[i] = 1;
            sout.push_back(static_cast<unsigned>(i));
        }
    }
    const size_t nin = sin.size(), nout = sout.size();
    const size_t C = staged_chunk(nin + nout, sz);
    const size_t slot_bytes = C * (nin + nout);
    if (ensure_sbuf(d, slot_bytes * kStageSlots)) return t_status;
    uint8_t* const hs = static_cast<uint8_t*>(d.sbuf);
    uint8_t* const ds = static_cast<uint8_t*>(d.sbuf_dev);
    HostPool& pool = HostPool::get();
    CopyLatch lin[kStageSlots], lout[kStageSlots];
    const size_t nchunks = (sz + C - 1) / C;

    auto stage_in = [&](size_t c) {
        const int s = static_cast<int>(c % kStageSlots);
        const size_t off = c * C, len = std::min(C, sz - off);
        for (size_t q = 0; q < nin; ++q)
            pool.copy_async(hs + s * slot_bytes + q * C, in[sin[q]] + off, len, &lin[s], len);
    };
    auto copy_out = [&](size_t c) {
        const int s = static_cast<int>(c % kStageSlots);
        const size_t off = c * C, len = std::min(C, sz - off);
        const size_t piece = std::max<size_t>(256u << 10, len / 4);
        for (size_t q = 0; q < nout; ++q)
            pool.copy_async(out[sout[q]] + off, hs + s * slot_bytes + (nin + q) * C, len, &lout[s], piece);
    };
    // every queued copy references the caller's buffers and the slots: all of
    // them finish before this returns, whatever the outcome
    auto drain = [&](int status) {
        (void)hipStreamSynchronize(st);
        for (int s = 0; s < kStageSlots; ++s) {
            pool.wait(&lin[s]);
            pool.wait(&lout[s]);
        }
        return status;
    };
    std::vector<const uint8_t*> zin(k);
    std::vector<uint8_t*> zout(r);
    hipError_t e;
    try {  // a failed allocation while queueing copies: drain what was queued
    stage_in(0);
    for (size_t c = 0; c < nchunks; ++c) {
        const int s = static_cast<int>(c % kStageSlots);
        const size_t off = c * C, len = std::min(C, sz - off);
        pool.wait(&lin[s]);  // this chunk's inputs are in the slot
        pool.wait(&lout[s]);  // the slot's previous outputs have been copied out
        for (unsigned j = 0; j < k; ++j) zin[j] = base_in[j] + off;
        for (unsigned i = 0; i < r; ++i) zout[i] = base_out[i] + off;
        for (size_t q = 0; q < nin; ++q) zin[sin[q]] = ds + s * slot_bytes + q * C;
        for (size_t q = 0; q < nout; ++q) zout[sout[q]] = ds + s * slot_bytes + (nin + q) * C;
        if (apply_matrix(coef, k, r, zin.data(), zout.data(), len, 1, 0, 0, st)) return drain(t_status);
        if ((e = hipEventRecord(d.ev_stg[s], st)) != hipSuccess) return drain(hip_fail(e, "hipEventRecord"));
        if (c + 1 < nchunks) {
            // the next slot's inputs were last read by chunk c + 1 - kStageSlots,
            // synchronised below in an earlier iteration (kStageSlots >= 2)
            stage_in(c + 1);
        }
        if (c >= 1) {
            const int sp = static_cast<int>((c - 1) % kStageSlots);
            e = hipEventSynchronize(d.ev_stg[sp]);
            if (e != hipSuccess)
                return drain(hip_fail(e, "hipEventSynchronize"));
            copy_out(c - 1);
        }
    }
    if ((e = hipEventSynchronize(d.ev_stg[(nchunks - 1) % kStageSlots])) != hipSuccess)
        return drain(hip_fail(e, "hipEventSynchronize"));
    copy_out(nchunks - 1);
    } catch (const std::exception& x) {
        return drain(set_status(FEC_ENOMEM, "staged host path: %s", x.what()));
    }
    drain(FEC_OK);
    return set_status(FEC_OK);
}

// Batched calls on pageable host memory (fec_encode_batch / fec_decode_batch
// with a src or dst the GPU cannot address), staged like run_staged but cut
// into groups of whole stripes: the host pool copies a group's input rows
// into a pinned slot, one batched launch runs the group on the slot, and the
// pool copies the output rows out -- only the rows, so bytes between rows
// and past sz in the caller's arrays are never written.  In the slot a
// group's rows are packed [stripe][block][sz], or [block][stripe][sz] when the
// caller's side is block-major (stripe stride == sz), which keeps the
// block-major launch shape.  A side in device or page-locked memory is used
// in place (`src` / `dst` are then kernel-visible addresses).
int run_batch_staged(DevCtx& d, const uint8_t* coef, unsigned k, unsigned r, const gf* src, size_t sbs, size_t sss,
                     bool src_host, gf* dst, size_t dbs, size_t dss, bool dst_host, size_t sz, size_t ns,
                     hipStream_t st) {
    const bool in_bm = sss == sz, out_bm = dss == sz;
    const size_t per = (src_host ? size_t(k) * sz : 0) + (dst_host ? size_t(r) * sz : 0);
    size_t gs = std::max<size_t>(1, (size_t(16) << 20) / std::max<size_t>(1, per));
    if (ns >= 4) gs = std::min(gs, (ns + 3) / 4);  // at least 4 groups, so the stages overlap
    gs = std::min(gs, ns);
    const size_t in_bytes = align_up(src_host ? gs * k * sz : 0, 256);
    const size_t out_bytes = align_up(dst_host ? gs * r * sz : 0, 256);
    const size_t slot_bytes = in_bytes + out_bytes;
    if (ensure_sbuf(d, slot_bytes * kStageSlots)) return t_status;
    uint8_t* const hs = static_cast<uint8_t*>(d.sbuf);
    uint8_t* const ds = static_cast<uint8_t*>(d.sbuf_dev);
    HostPool& pool = HostPool::get();
    CopyLatch lin[kStageSlots], lout[kStageSlots];
    const size_t ngroups = (ns + gs - 1) / gs;
    // stripes per copy task when rows are copied one stripe at a time
    const size_t task_stripes = std::max<size_t>(1, (size_t(1) << 20) / std::max<size_t>(1, per));

    // rows of stripes [s0, s0 + n) between the caller's array (block stride
    // bs, stripe stride ss) and a slot; `to_slot` picks the direction
    auto move_rows = [&](uint8_t* slot, gf* user, size_t bs, size_t ss, unsigned nb, bool bm, size_t s0, size_t n,
                         bool to_slot, CopyLatch* latch) {
        if (bm) {  // block b of the group: n*sz contiguous bytes on both sides
            for (unsigned b = 0; b < nb; ++b) {
                uint8_t* sp = slot + size_t(b) * n * sz;
                uint8_t* up = user + b * bs + s0 * sz;
                if (to_slot)
                    pool.copy_async(sp, up, n * sz, latch);
                else
                    pool.copy_async(up, sp, n * sz, latch);
            }
            return;
        }
        for (size_t t0 = 0; t0 < n; t0 += task_stripes) {
            const size_t t1 = std::min(n, t0 + task_stripes);
            pool.run_async(
                [=]() {
                    for (size_t s = t0; s < t1; ++s) {
                        uint8_t* sp = slot + s * nb * sz;
                        uint8_t* up = user + (s0 + s) * ss;
                        if (bs == sz) {  // the stripe's rows are contiguous
                            if (to_slot)
                                std::memcpy(sp, up, nb * sz);
                            else
                                std::memcpy(up, sp, nb * sz);
                            continue;
                        }
                        for (unsigned b = 0; b < nb; ++b) {
                            if (to_slot)
                                std::memcpy(sp + b * sz, up + b * bs, sz);
                            else
                                std::memcpy(up + b * bs, sp + b * sz, sz);
                        }
                    }
                },
                latch);
        }
    };
    auto group = [&](size_t g, size_t* s0, size_t* n) {
        *s0 = g * gs;
        *n = std::min(gs, ns - *s0);
    };
    auto stage_in = [&](size_t g) {
        if (!src_host) return;
        size_t s0, n;
        group(g, &s0, &n);
        const int s = static_cast<int>(g % kStageSlots);
        move_rows(hs + s * slot_bytes, const_cast<gf*>(src), sbs, sss, k, in_bm, s0, n, true, &lin[s]);
    };
    auto copy_out = [&](size_t g) {
        if (!dst_host) return;
        size_t s0, n;
        group(g, &s0, &n);
        const int s = static_cast<int>(g % kStageSlots);
        move_rows(hs + s * slot_bytes + in_bytes, dst, dbs, dss, r, out_bm, s0, n, false, &lout[s]);
    };
    auto drain = [&](int status) {
        (void)hipStreamSynchronize(st);
        for (int s = 0; s < kStageSlots; ++s) {
            pool.wait(&lin[s]);
            pool.wait(&lout[s]);
        }
        return status;
    };
    std::vector<const uint8_t*> zin(k);
    std::vector<uint8_t*> zout(r);
    hipError_t e;
    try {  // a failed allocation while queueing copies: drain what was queued
    stage_in(0);
    for (size_t g = 0; g < ngroups; ++g) {
        const int s = static_cast<int>(g % kStageSlots);
        size_t s0, n;
        group(g, &s0, &n);
        pool.wait(&lin[s]);
        pool.wait(&lout[s]);
        size_t iss = sss, oss = dss;
        for (unsigned j = 0; j < k; ++j) zin[j] = src + j * sbs + s0 * sss;
        for (unsigned i = 0; i < r; ++i) zout[i] = dst + i * dbs + s0 * dss;
        if (src_host) {
            uint8_t* b = ds + s * slot_bytes;
            for (unsigned j = 0; j < k; ++j) zin[j] = b + (in_bm ? size_t(j) * n * sz : size_t(j) * sz);
            iss = in_bm ? sz : size_t(k) * sz;
        }
        if (dst_host) {
            uint8_t* b = ds + s * slot_bytes + in_bytes;
            for (unsigned i = 0; i < r; ++i) zout[i] = b + (out_bm ? size_t(i) * n * sz : size_t(i) * sz);
            oss = out_bm ? sz : size_t(r) * sz;
        }
        if (apply_matrix(coef, k, r, zin.data(), zout.data(), sz, n, iss, oss, st)) return drain(t_status);
        if ((e = hipEventRecord(d.ev_stg[s], st)) != hipSuccess) return drain(hip_fail(e, "hipEventRecord"));
        if (g + 1 < ngroups) stage_in(g + 1);
        if (g >= 1) {
            if ((e = hipEventSynchronize(d.ev_stg[(g - 1) % kStageSlots])) != hipSuccess)
                return drain(hip_fail(e, "hipEventSynchronize"));
            copy_out(g - 1);
        }
    }
    if ((e = hipEventSynchronize(d.ev_stg[(ngroups - 1) % kStageSlots])) != hipSuccess)
        return drain(hip_fail(e, "hipEventSynchronize"));
    copy_out(ngroups - 1);
    } catch (const std::exception& x) {
        return drain(set_status(FEC_ENOMEM, "staged batch path: %s", x.what()));
    }
    drain(FEC_OK);
    return set_status(FEC_OK);
}

// Run `coef` (r x k) over in -> out.  Device blocks are used in place; host
// blocks are staged (small calls: one pinned bounce buffer each way; large
// calls: the staged path).  Synchronous unless FEC_FLAG_ASYNC and every
// block is device memory.
int run_single(const uint8_t* coef, unsigned k, unsigned r, const gf* const* in, gf* const* out, size_t sz,
               void* stream_arg, unsigned flags) {
    if (!gpu_available()) return set_status(FEC_ENODEV, "no GPU visible to HIP (the engine has no CPU path)");
    thread_local Marshal t_m;  // reused: no allocation per call once its vectors have grown
    Marshal& m = t_m;
    if (flags & FEC_FLAG_HOST_MEMORY) {  // the caller vouches: every block is host memory
        for (unsigned j = 0; j < k; ++j)
            if (!in[j]) return set_status(FEC_EINVAL, "input block %u is NULL", j);
        for (unsigned i = 0; i < r; ++i)
            if (!out[i]) return set_status(FEC_EINVAL, "output block %u is NULL", i);
        m.zin.assign(in, in + k);
        m.zout.assign(out, out + r);
        m.in_host.clear();
        m.out_host.clear();
        for (unsigned j = 0; j < k; ++j) m.in_host.push_back(static_cast<int>(j));
        for (unsigned i = 0; i < r; ++i) m.out_host.push_back(static_cast<int>(i));
        m.all_pinned = false;
        if (hipGetDevice(&m.device) != hipSuccess) return set_status(FEC_ENODEV, "no current HIP device");
    } else if (classify(in, k, out, r, m)) {
        return t_status;
    }
    DeviceGuard guard(m.device);
    DevCtx* d = nullptr;
    if (dev_ctx(m.device, &d)) return t_status;
    hipStream_t st = (flags & FEC_FLAG_LIBRARY_STREAM) ? d->stream : static_cast<hipStream_t>(stream_arg);
    if (sz == 0 || r == 0) return set_status(FEC_OK);
    const size_t nhost = m.in_host.size() + m.out_host.size();
    const Config& cfg = config();
    hipError_t e;
    if (nhost == 0) {
        if (apply_matrix(coef, k, r, in, out, sz, 1, 0, 0, st)) return t_status;
        if (!(flags & FEC_FLAG_ASYNC) && (e = hipStreamSynchronize(st)) != hipSuccess)
            return hip_fail(e, "hipStreamSynchronize");
        return set_status(FEC_OK);
    }
    // Page-locked host blocks are read and written by the kernel itself over
    // PCIe (zero-copy): both link directions run at once with no staging
    // copies (K=3/M=10, 64 MiB: 21 GB/s of input vs 16.6 through a chunked
    // copy pipeline; tools/mb_host.hip).
    auto map_all = [&]() {
        bool ok = true;
        for (int i : m.in_host) ok = ok && (m.zin[i] = mapped_block(in[i], sz)) != nullptr;
        for (int i : m.out_host) ok = ok && (m.zout[i] = const_cast<uint8_t*>(mapped_block(out[i], sz))) != nullptr;
        return ok;
    };
    if (m.all_pinned && map_all()) {
        if (apply_matrix(coef, k, r, m.zin.data(), m.zout.data(), sz, 1, 0, 0, st)) return t_status;
        if (!(flags & FEC_FLAG_ASYNC) && (e = hipStreamSynchronize(st)) != hipSuccess)
            return hip_fail(e, "hipStreamSynchronize");
        return set_status(FEC_OK);
    }
    // large pageable blocks: staged through pinned slots by the host threads.
    // Calls whose kernel can use the bounce buffer in place (k <= 4, r <= 8)
    // stay on it up to Config::zc_limit: K=3/M=10 from bytes, 256 KiB stripes
    // (874 KB of host blocks) encode in 47-57 us there against 62-71 us staged
    // and decode in 30-35 against 45-52; 512 KiB stripes (1.75 MB) encode
    // 78-97 against 84-86 us (box-dependent: staged from 1.5 MiB) and decode
    // (1.05 MB) 49-56 against 61 us; 1 MiB stripes 186 against 159 us
    // (tools/archive/small_ab_inproc.py --set stage, profiles/r03_stage_ab.log).
    const bool zc_shape = k <= 4 && r <= 8;
    const size_t stage_from = zc_shape ? std::max(cfg.stage_min, cfg.zc_limit) : cfg.stage_min;
    if (sz * nhost > cfg.pack_limit || (sz * nhost > stage_from && sz >= kStageMinBlock))
        return run_staged(*d, coef, k, r, in, out, sz, m, st);

    // small call: pack the host inputs into the thread's pinned buffer.  Up to
    // Config::zc_limit bytes the kernel reads them and writes the host outputs
    // there in place over PCIe (no copy calls: 4 KiB K=3/M=10 encode 21.9 ->
    // 16.6 us per call, 128 KiB 46.8 -> 26.6 us); wide codes (and calls past
    // the limit) move the packed blocks with one H2D and one D2H copy.
    // Device-resident blocks are used in place.  Then unpack.
    m.din.assign(in, in + k);
    m.dout.assign(out, out + r);
    const size_t slot = align_up(sz, 256);
    const size_t nin = m.in_host.size(), nout = m.out_host.size();
    if (ensure_hbuf(*d, slot * (nin + nout))) return t_status;
    uint8_t* hb = static_cast<uint8_t*>(d->hbuf);  // free: the previous call on this thread synchronised
    // the copies run on this thread (on the host pool they measured slower at
    // every size this path serves: profiles/r02_host_lat_ab.log, r03_pool_ab.log)
    auto copy_blocks = [&](bool to_slot) {
        const size_t n = to_slot ? nin : nout;
        for (size_t q = 0; q < n; ++q) {
            uint8_t* sl = hb + slot * (to_slot ? q : nin + q);
            if (to_slot)
                std::memcpy(sl, in[m.in_host[q]], sz);
            else
                std::memcpy(out[m.out_host[q]], sl, sz);
        }
    };
    // Every block in the bounce buffer: its slots are 256-byte multiples, so
    // the kernel may run each row out to its next 128-byte line (whole 16-byte
    // units, no byte-wise tail: over PCIe each tail byte load is a round trip
    // of its own); the bytes past sz are never copied out.
    const size_t ksz = nhost == size_t(k) + r ? std::min(slot, align_up(sz, 128)) : sz;
    // The compact one-workgroup kernel takes the inputs inside its argument
    // block where they fit (kernels.hip OneJobInline): no copy into the bounce
    // buffer, no PCIe reads in the kernel.
    const bool one_shape = k <= 4 && r <= 8 && ksz % 16 == 0 && ksz <= 4096 && sz * nhost <= cfg.zc_limit;
    const bool inline_in = one_shape && nin == k && nhost == size_t(k) + r && one_inline_fits(k, ksz, sz);
    if (!inline_in) copy_blocks(true);
    // Zero-copy only for the register kernels (k <= 4, r <= 8), which issue
    // all their input loads at once: the wide-code kernels read inputs in
    // groups, each group a PCIe round trip of its own (K=20/M=60, 4 KiB stripe:
    // 40 us in the kernel over PCIe; tools/small_call_probe.py under
    // rocprofv3, profiles/r02_small_calls.log) -- except small packs, up to
    // kZcWideLimit: K=20/M=60 from bytes, 4 KiB stripes encode in 20.5 us in
    // place against 25.3 us with the copies, 64 KiB (197 KB of host blocks)
    // 44.7 against 47.9 us, but 128 KiB (393 KB) 63.8 against 57.9 us
    // (round-3 A/B, profiles/r03_zcwide_ab.log).  Fixed since round 4; the
    // GPU test test_medium_call_wait_modes runs K=10/M=16 on both sides of it.
    constexpr size_t kZcWideLimit = size_t(256) << 10;
    const bool zc_kernel = (k <= 4 && r <= 8) || sz * nhost <= kZcWideLimit;
    bool signalled = false;
    const bool zero_copy = sz * nhost <= cfg.zc_limit && zc_kernel;
    if (zero_copy) {
        uint8_t* hbd = static_cast<uint8_t*>(d->hbuf_dev);
        for (size_t q = 0; q < nin; ++q) m.din[m.in_host[q]] = hbd + slot * q;
        for (size_t q = 0; q < nout; ++q) m.dout[m.out_host[q]] = hbd + slot * (nin + q);
        if (one_shape) {
            // whole 16-byte units in one workgroup: the compact kernel
            // (kernels.hip matapply_one), which signals its own completion
            uint32_t* f = signal_slot(*d);
            ApplySpec a;
            a.coef = coef;
            a.coef_stride = k;
            a.k = k;
            a.r = r;
            a.in = m.din.data();
            a.out = m.dout.data();
            a.sz = ksz;
            a.nstripes = 1;
            a.in_sstride = a.out_sstride = 0;
            a.accumulate = false;
            ++t_launches;
            const hipError_t le = launch_one(a, st, f, f ? d->seq : 0, inline_in ? in : nullptr, sz);
            if (le != hipSuccess) return hip_fail(le, "launch_one");
            signalled = f != nullptr;
        } else {
            // one launch of at most one workgroup (k <= 4, r <= 8, sz <= 4 KiB): it
            // signals its own completion
            if (k <= 4 && r <= 8 && sz <= 4096)
                if (uint32_t* f = signal_slot(*d)) matapply_request_signal(f, d->seq);
            const unsigned launches0 = t_launches;
            const int st0 = apply_matrix(coef, k, r, m.din.data(), m.dout.data(), ksz, 1, 0, 0, st);
            // the kernel's signal covers the call only if it was its one launch
            signalled = st0 == FEC_OK && matapply_signal_used() && t_launches - launches0 == 1;
            matapply_request_signal(nullptr, 0);  // an unconsumed request must not reach a later launch
            if (st0) return t_status;
        }
    } else {
        if (ensure_dbuf(*d, slot * nhost)) return t_status;
        uint8_t* base = static_cast<uint8_t*>(d->dbuf);
        for (size_t q = 0; q < nin; ++q) m.din[m.in_host[q]] = base + slot * q;
        for (size_t q = 0; q < nout; ++q) m.dout[m.out_host[q]] = base + slot * (nin + q);
        if (nin && (e = hipMemcpyAsync(base, hb, slot * nin, hipMemcpyHostToDevice, st)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync H2D");
        if (apply_matrix(coef, k, r, m.din.data(), m.dout.data(), ksz, 1, 0, 0, st)) return t_status;
        if (nout && (e = hipMemcpyAsync(hb + slot * nin, base + slot * nin, slot * nout, hipMemcpyDeviceToHost,
                                        st)) != hipSuccess)
            return hip_fail(e, "hipMemcpyAsync D2H");
    }
    if (!signalled && zero_copy) {
        // a zero-copy launch of several workgroups: the stream itself writes
        // the call's sequence number into the pinned completion word after the
        // kernel, and the thread spins on that (64 KiB K=3/M=10 encode 23.8 ->
        // 21.2 us, decode 19.1 -> 16.4 us in an interleaved A/B,
        // profiles/r03_wait_ab.log).  Not behind the copy path's D2H copy:
        // there it measured 6-7 us slower than hipStreamSynchronize.
        if (uint32_t* f = signal_slot(*d)) {
            if (hipStreamWriteValue32(st, f, d->seq, 0) == hipSuccess)
                signalled = true;
            else
                (void)hipGetLastError();
        }
    }
    t_last_wait = signalled ? 1 : 0;
    if ((e = signalled ? wait_signal(*d, st) : hipStreamSynchronize(st)) != hipSuccess)
        return hip_fail(e, "hipStreamSynchronize");
    copy_blocks(false);
    return set_status(FEC_OK);
}

int check_block_nums(const fec_t* code, const unsigned* nums, size_t num) {
    if (num && !nums) return set_status(FEC_EINVAL, "block_nums is NULL");
    for (size_t i = 0; i < num; ++i)
        if (nums[i] >= code->n)
            return set_status(FEC_EINVAL, "block number %u out of range (n = %u)", nums[i], unsigned(code->n));
    return FEC_OK;
}

// The decode matrix rows to apply (r x k, into `rows`): the missing
// primaries' (ascending), or with all_primaries every primary's (a present
// primary's row is a unit vector: the output is a copy, so the k outputs are
// the stripe in order).
int decode_rows(const fec_t* code, const unsigned* index, std::vector<uint8_t>& rows, unsigned& r,
                bool all_primaries = false) {
    const unsigned k = code->k;
    if (!index) return set_status(FEC_EINVAL, "index is NULL");
    unsigned char seen[256] = {};
    for (unsigned i = 0; i < k; ++i) {
        if (index[i] >= code->n)
            return set_status(FEC_EINVAL, "block number %u out of range (n = %u)", index[i], unsigned(code->n));
        if (seen[index[i]]) return set_status(FEC_EINVAL, "duplicate block number %u", index[i]);
        seen[index[i]] = 1;
        if (index[i] < k && index[i] != i)
            return set_status(FEC_EINVAL, "primary block %u must be at slot %u, found at slot %u", index[i], index[i], i);
    }
    // The inverse is O(k^3) on the host (255 x 255 with 128 secondaries:
    // ~0.8 ms, more than the kernel), and batches of stripes are decoded from
    // the same blocks call after call, so each thread keeps its last few
    // decode matrices.  The key is (k, index): the encoding matrix's row b
    // depends on k and b only, not on n (zfec/fec.c:456-469; checked against
    // the reference).
    struct Cached {
        unsigned k = 0;
        bool all = false;
        std::vector<unsigned> idx;
        std::vector<uint8_t> rows;
        unsigned r = 0;
    };
    constexpr int kCache = 8;
    thread_local Cached cache[kCache];
    thread_local unsigned next = 0;
    for (const Cached& c : cache)
        if (c.k == k && c.all == all_primaries && std::equal(index, index + k, c.idx.begin(), c.idx.end())) {
            rows.assign(c.rows.begin(), c.rows.end());
            r = c.r;
            return FEC_OK;
        }
    thread_local std::vector<uint8_t> dec;
    dec.resize(size_t(k) * k);
    if (!build_decode_matrix(code->enc_matrix, k, index, dec.data()))
        return set_status(FEC_ESINGULAR, "decode matrix is singular");
    rows.clear();
    r = 0;
    for (unsigned i = 0; i < k; ++i) {
        if (index[i] < k && !all_primaries) continue;
        rows.insert(rows.end(), dec.begin() + size_t(i) * k, dec.begin() + size_t(i + 1) * k);
        ++r;
    }
    Cached& c = cache[next++ % kCache];
    c.k = k;
    c.all = all_primaries;
    c.idx.assign(index, index + k);
    c.rows.assign(rows.begin(), rows.end());
    c.r = r;
    return FEC_OK;
}

// The encoding matrix rows of block_nums (num x k): consecutive ascending
// numbers are one contiguous run of enc_matrix (used in place), others are
// gathered into the thread's buffer.
const uint8_t* encode_rows(const fec_t* code, const unsigned* nums, size_t num) {
    const unsigned k = code->k;
    bool run = true;
    for (size_t i = 1; i < num && run; ++i) run = nums[i] == nums[0] + i;
    if (run) return code->enc_matrix + size_t(nums[0]) * k;
    thread_local std::vector<uint8_t> rows;
    rows.resize(num * k);
    for (size_t i = 0; i < num; ++i) std::memcpy(&rows[i * k], code->enc_matrix + size_t(nums[i]) * k, k);
    return rows.data();
}

}  // namespace
}  // namespace zfec_hip

using namespace zfec_hip;

// ============================================================================
// Part 1: zfec/fec.h drop-in
// ============================================================================

FEC_API void fec_init(void) {
    field_init();
    set_status(FEC_OK);
}

namespace {
void prefetch_rows(const uint8_t* coef, unsigned k, unsigned r);  // below, with prepare_rows
}

FEC_API fec_t* fec_new(unsigned short k, unsigned short m) {
    if (!field_ready()) {  // zfec/fec.c:442-444
        set_status(FEC_EUNINIT, "fec_init() has not been called");
        return nullptr;
    }
    if (k < 1 || m < 1 || m > 256 || k > m) {  // zfec/fec.c:437-440 (asserts there)
        set_status(FEC_EINVAL, "invalid code parameters k=%u m=%u", unsigned(k), unsigned(m));
        return nullptr;
    }
    fec_t* p = static_cast<fec_t*>(std::calloc(1, sizeof(fec_t)));
    gf* enc = static_cast<gf*>(std::malloc(size_t(k) * m));
    if (!p || !enc) {
        std::free(p);
        std::free(enc);
        set_status(FEC_ENOMEM, "out of host memory");
        return nullptr;
    }
    build_encoding_matrix(k, m, enc);
    p->k = k;
    p->n = m;
    p->enc_matrix = enc;
    p->priv = nullptr;
    p->magic = magic_of(p);
    // the full encode's compiled kernels, where an earlier process left them in
    // the JIT disk cache: loaded in the background, so this code's first large
    // encode can run them (bitslice.hpp jit_prefetch; no compile, no wait)
    prefetch_rows(enc + size_t(k) * k, k, static_cast<unsigned>(m - k));
    set_status(FEC_OK);
    return p;
}

FEC_API void fec_free(fec_t* p) {
    if (!p) return;
    if (!valid_code(p)) {  // zfec/fec.c:425 asserts; we refuse and report
        set_status(FEC_EINVAL, "fec_free: bad magic");
        return;
    }
    p->magic = 0;
    std::free(p->enc_matrix);
    std::free(p);
    set_status(FEC_OK);
}

FEC_API int fec_encode_ex(const fec_t* code, const gf* const* src, gf* const* fecs, const unsigned* block_nums,
                          size_t num_block_nums, size_t sz, void* stream, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    if (check_block_nums(code, block_nums, num_block_nums)) return t_status;
    if (num_block_nums == 0) return set_status(FEC_OK);
    if (!src || !fecs) return set_status(FEC_EINVAL, "NULL block array");
    return guarded([&] {
        const uint8_t* rows = encode_rows(code, block_nums, num_block_nums);
        return run_single(rows, code->k, static_cast<unsigned>(num_block_nums), src, fecs, sz, stream, flags);
    });
}

namespace {
// fec.h's fec_encode / fec_decode return void and their callers (the
// reference's _fecmodule.c, the Haskell binding) never ask for a status, so a
// failure there would hand back unwritten output buffers in silence.  The
// first failure of each entry point is reported on stderr (once per process;
// ZFEC_HIP_QUIET=1 silences it); fec_last_status() still holds every one.
void report_void_failure(const char* fn, int st) {
    static std::atomic<int> reported[2] = {{0}, {0}};
    std::atomic<int>& once = reported[fn[4] == 'd' ? 1 : 0];
    if (config().quiet || once.exchange(1) != 0) return;
    fprintf(stderr,
            "zfec_hip: %s failed (status %d: %s); its output blocks are not valid.  Further failures of %s are "
            "not reported here; fec_last_status() / fec_last_error_message() give each call's status.\n",
            fn, st, t_msg, fn);
    fflush(stderr);
}
}  // namespace

FEC_API void fec_encode(const fec_t* code, const gf* const* src, gf* const* fecs, const unsigned* block_nums,
                        size_t num_block_nums, size_t sz) {
    const int st = fec_encode_ex(code, src, fecs, block_nums, num_block_nums, sz, nullptr, FEC_FLAG_LIBRARY_STREAM);
    if (st != FEC_OK) report_void_failure("fec_encode", st);
}

FEC_API int fec_decode_ex(const fec_t* code, const gf* const* inpkts, gf* const* outpkts, const unsigned* index,
                          size_t sz, void* stream, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    thread_local std::vector<uint8_t> rows;
    unsigned r = 0;
    if (decode_rows(code, index, rows, r, (flags & FEC_FLAG_ALL_PRIMARIES) != 0)) return t_status;
    if (r == 0) return set_status(FEC_OK);
    if (!inpkts || !outpkts) return set_status(FEC_EINVAL, "NULL block array");
    return guarded([&] { return run_single(rows.data(), code->k, r, inpkts, outpkts, sz, stream, flags); });
}

FEC_API void fec_decode(const fec_t* code, const gf* const* inpkts, gf* const* outpkts, const unsigned* index,
                        size_t sz) {
    const int st = fec_decode_ex(code, inpkts, outpkts, index, sz, nullptr, FEC_FLAG_LIBRARY_STREAM);
    if (st != FEC_OK) report_void_failure("fec_decode", st);
}

FEC_API void build_decode_matrix_into_space(const fec_t* code, const unsigned* index, const unsigned k, gf* matrix) {
    if (!valid_code(code) || k != code->k || !index || !matrix) {
        set_status(FEC_EINVAL, "build_decode_matrix_into_space: bad arguments");
        return;
    }
    for (unsigned i = 0; i < k; ++i)
        if (index[i] >= code->n) {
            set_status(FEC_EINVAL, "block number %u out of range", index[i]);
            return;
        }
    if (!build_decode_matrix(code->enc_matrix, k, index, matrix))
        set_status(FEC_ESINGULAR, "decode matrix is singular");
    else
        set_status(FEC_OK);
}

FEC_API void _invert_vdm(gf* src, unsigned k) {
    field_init();
    invert_vandermonde(src, k);
}

// ============================================================================
// Part 2: extensions
// ============================================================================

FEC_API int fec_last_status(void) { return t_status; }
FEC_API const char* fec_last_error_message(void) { return t_msg; }

FEC_API int fec_device_count(void) { return gpu_available(); }

FEC_API void* fec_host_alloc(size_t bytes) {
    if (!gpu_available()) {
        set_status(FEC_ENODEV, "no GPU visible to HIP");
        return nullptr;
    }
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        set_status(FEC_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    set_status(FEC_OK);
    return p;
}

FEC_API void fec_host_free(void* p) {
    if (p) (void)hipHostFree(p);
    set_status(FEC_OK);
}

FEC_API const char* fec_version(void) { return "zfec-hip 0.1.0 (gfx950)"; }

FEC_API const char* fec_kernel_name(unsigned k, unsigned r) {
    if (k == 0 || r == 0 || k > static_cast<unsigned>(kMaxIn) || r > static_cast<unsigned>(kMaxOut)) return "split";
    return matapply_variant_name(k, r, false);
}

FEC_API const char* fec_last_kernel_name(void) { return matapply_last_kernel(); }

FEC_API int fec_jit_mode(int mode) {
    const int prev = static_cast<int>(jit_mode());
    if (mode >= kJitOff && mode <= kJitForce) set_jit_mode(static_cast<JitMode>(mode));
    set_status(FEC_OK);
    return prev;
}

FEC_API int fec_generic_mode(int mode) {
    const int prev = generic_mode();
    if (mode >= 0 && mode <= 2) set_generic_mode(mode);
    set_status(FEC_OK);
    return prev;
}

FEC_API int fec_jit_wait(void) {
    set_status(FEC_OK);
    return jit_wait();
}

FEC_API int fec_reload_config(void) {
    reload_config();
    return set_status(FEC_OK);
}

FEC_API int fec_last_wait(void) { return t_last_wait; }

namespace {
// Compile the specialised kernels apply_matrix_range would launch for this
// r x k matrix in large launches: its row groups of one launch each (the same
// near-equal groups).  Groups past kJitMaxCoef coefficients run on
// matapply_bsg and need no compile.
int prepare_rows(const uint8_t* coef, unsigned k, unsigned r) {
    if (r == 0) return set_status(FEC_OK);
    const bool wide = k > static_cast<unsigned>(kMaxIn);
    const unsigned rmax =
        wide ? static_cast<unsigned>(kMaxOut) : std::max<unsigned>(1, std::min<unsigned>(kMaxOut, kMaxCoef / k));
    const unsigned ngroups = (r + rmax - 1) / rmax;
    for (unsigned g = 0; g < ngroups; ++g) {
        const unsigned i0 = g * r / ngroups, rg = (g + 1) * r / ngroups - i0;
        if (k * rg > kJitMaxCoef) continue;
        if (jit_prepare(coef + size_t(i0) * k, k, rg) != 0)
            return set_status(FEC_EHIP, "JIT compile failed: %s", jit_last_error().c_str());
    }
    return set_status(FEC_OK);
}
}  // namespace

namespace {
// jit_prefetch for the row groups prepare_rows would compile.
void prefetch_rows(const uint8_t* coef, unsigned k, unsigned r) {
    if (r == 0 || jit_mode() != kJitAuto) return;
    const bool wide = k > static_cast<unsigned>(kMaxIn);
    const unsigned rmax =
        wide ? static_cast<unsigned>(kMaxOut) : std::max<unsigned>(1, std::min<unsigned>(kMaxOut, kMaxCoef / k));
    const unsigned ngroups = (r + rmax - 1) / rmax;
    for (unsigned g = 0; g < ngroups; ++g) {
        const unsigned i0 = g * r / ngroups, rg = (g + 1) * r / ngroups - i0;
        if (k * rg <= kJitMaxCoef) jit_prefetch(coef + size_t(i0) * k, k, rg);
    }
}
}  // namespace

FEC_API int fec_jit_prepare_encode(const fec_t* code, const unsigned* block_nums, size_t num_block_nums) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    if (check_block_nums(code, block_nums, num_block_nums)) return t_status;
    if (num_block_nums == 0) return set_status(FEC_OK);
    return prepare_rows(encode_rows(code, block_nums, num_block_nums), code->k, static_cast<unsigned>(num_block_nums));
}

FEC_API int fec_jit_prepare_decode(const fec_t* code, const unsigned* index, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    std::vector<uint8_t> rows;
    unsigned r = 0;
    if (decode_rows(code, index, rows, r, (flags & FEC_FLAG_ALL_PRIMARIES) != 0)) return t_status;
    return prepare_rows(rows.data(), code->k, r);
}

namespace {
// The launch geometry of a batched call on device (or page-locked) memory:
// updates sz and nstripes in place.
void batch_geometry(unsigned k, unsigned r, size_t sbs, size_t sss, size_t dbs, size_t dss, unsigned flags, size_t& sz,
                    size_t& nstripes) {
    // Block-major batches (stripes packed back to back inside each block array,
    // both strides == sz) are one stripe of nstripes * sz bytes: output byte x
    // depends only on byte x of the inputs (zfec/fec.c:494-503, :547-556), so
    // one long-stream launch replaces the walk over short rows.
    // FEC_FLAG_ROW_PADDING: run the rows out to a whole 128-byte line where the
    // strides leave room.  A row ending mid-line leaves a partly written line
    // that HBM completes with a read-modify-write: 10^6 K=3/M=10 stripes of
    // 1366-byte blocks in 1536-byte rows encode in 2.91 ms, of 1408-byte blocks
    // in 2.55 ms (tools/archive/grid_probe.py, profiles/r01_grid_probe_sz.log).
    // `grant`: bytes past a row's start the flag lets us touch (per row).
    size_t grant = sz;
    if (flags & FEC_FLAG_ROW_PADDING) {
        const size_t padded = (sz + 127) / 128 * 128;
        const bool room = sbs >= padded && dbs >= padded && (nstripes == 1 || (sss >= (k - 1) * sbs + padded &&
                                                                                dss >= (r - 1) * dbs + padded));
        if (room) grant = padded;
    }
    if (nstripes > 1 && sss == sz && dss == sz && sz <= SIZE_MAX / nstripes) {
        // the collapsed row may run out to its own next line only inside the
        // last stripe's grant: (nstripes - 1) * sz + grant
        const size_t len = sz * nstripes, padded = (len + 127) / 128 * 128;
        sz = padded <= len - sz + grant ? padded : len;
        nstripes = 1;
    } else {
        sz = grant;
    }
}

int run_batch(const fec_t* code, const uint8_t* coef, unsigned r, const gf* src, size_t sbs, size_t sss, gf* dst,
              size_t dbs, size_t dss, size_t sz, size_t nstripes, void* stream, unsigned flags) {
    const unsigned k = code->k;
    if (!gpu_available()) return set_status(FEC_ENODEV, "no GPU visible to HIP (the engine has no CPU path)");
    if (!src || !dst) return set_status(FEC_EINVAL, "NULL buffer");
    // one pointer query per side: device memory (its device), or host memory
    const int sdev = pointer_device(src), ddev0 = pointer_device(dst);
    // pageable host memory on either side: staged through pinned slots
    // (synchronous whatever the flags; FEC_FLAG_ROW_PADDING does not apply)
    if (sz && nstripes && r && (sdev < 0 || ddev0 < 0)) {
        const size_t src_ext = (nstripes - 1) * sss + (k - 1) * sbs + sz;
        const size_t dst_ext = (nstripes - 1) * dss + (r - 1) * dbs + sz;
        const uint8_t* zs = sdev >= 0 ? src : mapped_block(src, src_ext);
        const uint8_t* zd = ddev0 >= 0 ? dst : mapped_block(dst, dst_ext);
        if (!zs || !zd) {
            if (sdev >= 0 && ddev0 >= 0 && sdev != ddev0)
                return set_status(FEC_EINVAL, "batched entry points take memory on one device");
            int dev = sdev >= 0 ? sdev : ddev0;
            if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return set_status(FEC_ENODEV, "no current HIP device");
            DeviceGuard guard(dev);
            DevCtx* d = nullptr;
            if (dev_ctx(dev, &d)) return t_status;
            hipStream_t st = (flags & FEC_FLAG_LIBRARY_STREAM) ? d->stream : static_cast<hipStream_t>(stream);
            return run_batch_staged(*d, coef, k, r, zs ? zs : src, sbs, sss, !zs, zd ? const_cast<gf*>(zd) : dst, dbs,
                                    dss, !zd, sz, nstripes, st);
        }
    }
    batch_geometry(k, r, sbs, sss, dbs, dss, flags, sz, nstripes);
    // device memory on one device, or page-locked host memory (zero-copy)
    const size_t src_extent = (nstripes - 1) * sss + (k - 1) * sbs + sz;
    const size_t dst_extent = (nstripes - 1) * dss + (r - 1) * dbs + sz;
    int dev = sdev;
    const int ddev = ddev0;
    if (dev < 0) {
        const uint8_t* z = mapped_block(src, src_extent);
        if (!z) return set_status(FEC_EINVAL, "batched entry points take device or page-locked host memory");
        src = z;
    }
    if (ddev < 0) {
        const uint8_t* z = mapped_block(dst, dst_extent);
        if (!z) return set_status(FEC_EINVAL, "batched entry points take device or page-locked host memory");
        dst = const_cast<gf*>(z);
    }
    if (dev < 0) dev = ddev;
    if (dev >= 0 && ddev >= 0 && ddev != dev)
        return set_status(FEC_EINVAL, "batched entry points take memory on one device");
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return set_status(FEC_ENODEV, "no current HIP device");
    DeviceGuard guard(dev);
    DevCtx* d = nullptr;
    if (dev_ctx(dev, &d)) return t_status;
    hipStream_t st = (flags & FEC_FLAG_LIBRARY_STREAM) ? d->stream : static_cast<hipStream_t>(stream);
    const uint8_t* in[kMaxWideIn];
    uint8_t* out[kMaxWideIn];
    for (unsigned j = 0; j < k; ++j) in[j] = src + j * sbs;
    for (unsigned i = 0; i < r; ++i) out[i] = dst + i * dbs;
    if (apply_matrix(coef, k, r, in, out, sz, nstripes, sss, dss, st)) return t_status;
    if (!(flags & FEC_FLAG_ASYNC)) {
        hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    }
    return set_status(FEC_OK);
}
}  // namespace

FEC_API int fec_encode_batch(const fec_t* code, const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                             gf* dst, size_t dst_block_stride, size_t dst_stripe_stride, const unsigned* block_nums,
                             size_t num_block_nums, size_t sz, size_t nstripes, void* stream, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    if (check_block_nums(code, block_nums, num_block_nums)) return t_status;
    if (num_block_nums == 0 || sz == 0 || nstripes == 0) return set_status(FEC_OK);
    return guarded([&] {
        return run_batch(code, encode_rows(code, block_nums, num_block_nums), static_cast<unsigned>(num_block_nums),
                         src, src_block_stride, src_stripe_stride, dst, dst_block_stride, dst_stripe_stride, sz,
                         nstripes, stream, flags);
    });
}

FEC_API int fec_decode_batch(const fec_t* code, const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                             gf* dst, size_t dst_block_stride, size_t dst_stripe_stride, const unsigned* index,
                             size_t sz, size_t nstripes, void* stream, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    thread_local std::vector<uint8_t> rows;
    unsigned r = 0;
    if (decode_rows(code, index, rows, r, (flags & FEC_FLAG_ALL_PRIMARIES) != 0)) return t_status;
    if (r == 0 || sz == 0 || nstripes == 0) return set_status(FEC_OK);
    return guarded([&] {
        return run_batch(code, rows.data(), r, src, src_block_stride, src_stripe_stride, dst, dst_block_stride,
                         dst_stripe_stride, sz, nstripes, stream, flags);
    });
}

namespace zfec_hip {
namespace {
// A fec_run_batch_jobs job resolved for a paired launch (register-kernel
// shapes: k <= 4, r <= 8).
struct PairJobSpec {
    uint8_t coef[4 * 8];
    unsigned k = 0, r = 0;
    const uint8_t* in[4];
    uint8_t* out[8];
    size_t sz = 0, nstripes = 0, sss = 0, dss = 0;
    int dev = -1;
};

// Resolve job j; *ok = false when it cannot share a launch (host memory,
// another shape, an empty job, more units than one launch takes).
int resolve_pair_job(const fec_batch_job& j, PairJobSpec& p, bool* ok) {
    *ok = false;
    const unsigned k = j.code->k;
    if (k > 4 || !j.sz || !j.nstripes || !j.src || !j.dst) return FEC_OK;
    if (j.kind == FEC_JOB_ENCODE) {
        if (j.num_nums == 0 || j.num_nums > 8) return FEC_OK;
        p.r = static_cast<unsigned>(j.num_nums);
        std::memcpy(p.coef, encode_rows(j.code, j.nums, j.num_nums), size_t(p.r) * k);
    } else {
        thread_local std::vector<uint8_t> rows;
        unsigned r = 0;
        if (decode_rows(j.code, j.nums, rows, r, (j.flags & FEC_FLAG_ALL_PRIMARIES) != 0)) return t_status;
        if (r == 0 || r > 8) return FEC_OK;
        p.r = r;
        std::memcpy(p.coef, rows.data(), size_t(r) * k);
    }
    p.k = k;
    const int sdev = pointer_device(j.src), ddev = pointer_device(j.dst);
    if (sdev < 0 || sdev != ddev) return FEC_OK;
    p.dev = sdev;
    p.sz = j.sz;
    p.nstripes = j.nstripes;
    p.sss = j.src_stripe_stride;
    p.dss = j.dst_stripe_stride;
    batch_geometry(k, p.r, j.src_block_stride, p.sss, j.dst_block_stride, p.dss, j.flags, p.sz, p.nstripes);
    // apply_matrix's one-launch condition
    const size_t cps = (p.sz + kMinChunk - 1) / kMinChunk, max_units = config().launch_units;
    if (cps > max_units || std::max<size_t>(1, max_units / cps) < p.nstripes) return FEC_OK;
    for (unsigned i = 0; i < k; ++i) p.in[i] = j.src + i * j.src_block_stride;
    for (unsigned i = 0; i < p.r; ++i) p.out[i] = j.dst + i * j.dst_block_stride;
    *ok = true;
    return FEC_OK;
}

ApplySpec pair_spec(const PairJobSpec& p) {
    ApplySpec a;
    a.coef = p.coef;
    a.coef_stride = p.k;
    a.k = p.k;
    a.r = p.r;
    a.in = p.in;
    a.out = p.out;
    a.sz = p.sz;
    a.nstripes = p.nstripes;
    a.in_sstride = p.sss;
    a.out_sstride = p.dss;
    a.accumulate = false;
    return a;
}

int job_failed(size_t i) {
    char msg[sizeof t_msg];
    snprintf(msg, sizeof msg, "%s", t_msg);
    return set_status(t_status, "job %zu: %s", i, msg);
}
}  // namespace
}  // namespace zfec_hip

FEC_API int fec_run_batch_jobs(const fec_batch_job* jobs, size_t njobs, void* stream, unsigned flags) {
    if (njobs && !jobs) return set_status(FEC_EINVAL, "jobs is NULL");
    for (size_t i = 0; i < njobs; ++i) {
        const fec_batch_job& j = jobs[i];
        if (!valid_code(j.code)) return set_status(FEC_EINVAL, "job %zu: invalid fec_t", i);
        if (j.kind != FEC_JOB_ENCODE && j.kind != FEC_JOB_DECODE)
            return set_status(FEC_EINVAL, "job %zu: kind %u is neither FEC_JOB_ENCODE nor FEC_JOB_DECODE", i, j.kind);
        if (j.kind == FEC_JOB_ENCODE && check_block_nums(j.code, j.nums, j.num_nums)) return job_failed(i);
    }
    if (!gpu_available()) return set_status(FEC_ENODEV, "no GPU visible to HIP (the engine has no CPU path)");
    return guarded([&] {
        const unsigned call = flags & (FEC_FLAG_ASYNC | FEC_FLAG_LIBRARY_STREAM);
        // every device a job ran on, each once (no cap: a synchronous call
        // must wait on all of them before it reports FEC_OK)
        std::vector<int> devs;
        auto note_dev = [&](int dev) {
            for (int d : devs)
                if (d == dev) return;
            devs.push_back(dev);
        };
        size_t i = 0;
        while (i < njobs) {
            if (i + 1 < njobs) {
                PairJobSpec a, b;
                bool oka = false, okb = false;
                if (resolve_pair_job(jobs[i], a, &oka)) return job_failed(i);
                if (oka && resolve_pair_job(jobs[i + 1], b, &okb)) return job_failed(i + 1);
                if (oka && okb && a.dev == b.dev && a.k == b.k) {
                    DeviceGuard guard(a.dev);
                    DevCtx* d = nullptr;
                    if (dev_ctx(a.dev, &d)) return t_status;
                    hipStream_t st = (flags & FEC_FLAG_LIBRARY_STREAM) ? d->stream : static_cast<hipStream_t>(stream);
                    const hipError_t e = launch_apply_pair(pair_spec(a), pair_spec(b), st);
                    if (e == hipSuccess) {
                        ++t_launches;
                        note_dev(a.dev);
                        i += 2;
                        continue;
                    }
                    if (e != hipErrorNotSupported) {
                        hip_fail(e, "launch_apply_pair");
                        return job_failed(i);
                    }
                }
            }
            const fec_batch_job& j = jobs[i];
            const unsigned jf = (j.flags & (FEC_FLAG_ROW_PADDING | FEC_FLAG_ALL_PRIMARIES)) | call | FEC_FLAG_ASYNC;
            const int st = j.kind == FEC_JOB_ENCODE
                               ? fec_encode_batch(j.code, j.src, j.src_block_stride, j.src_stripe_stride, j.dst,
                                                  j.dst_block_stride, j.dst_stripe_stride, j.nums, j.num_nums, j.sz,
                                                  j.nstripes, stream, jf)
                               : fec_decode_batch(j.code, j.src, j.src_block_stride, j.src_stripe_stride, j.dst,
                                                  j.dst_block_stride, j.dst_stripe_stride, j.nums, j.sz, j.nstripes,
                                                  stream, jf);
            if (st) return job_failed(i);
            int dev = pointer_device(j.src);
            if (dev < 0) dev = pointer_device(j.dst);
            if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
            note_dev(dev);
            ++i;
        }
        if (!(flags & FEC_FLAG_ASYNC)) {
            if (!(flags & FEC_FLAG_LIBRARY_STREAM) && stream) {
                const hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
                if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
            } else if (!(flags & FEC_FLAG_LIBRARY_STREAM)) {
                // the null stream: each job ran on its own device's null stream
                for (int dv : devs) {
                    DeviceGuard guard(dv);
                    const hipError_t e = hipStreamSynchronize(nullptr);
                    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
                }
            } else {
                for (int dv : devs) {
                    DeviceGuard guard(dv);
                    DevCtx* d = nullptr;
                    if (dev_ctx(dv, &d)) return t_status;
                    const hipError_t e = hipStreamSynchronize(d->stream);
                    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
                }
            }
        }
        return set_status(FEC_OK);
    });
}

// ============================================================================
// Several GPUs of one process: a batch's stripes are
// independent (zfec/fec.c:494-503 touches one column range of each block), so
// the batch is split into contiguous balanced stripe ranges, one per listed
// device, each run by a persistent host thread bound to that device with its
// own stream and staging slots -- the reference's only parallelism is the
// same thing on CPU threads (the GIL released around fec_encode,
// zfec/_fecmodule.c:221-223).  Host memory only: each GPU reads and writes
// its share over its own PCIe link; device-resident batches stay on their
// device (one fec_encode_batch per device).
// ============================================================================
namespace {

// One persistent thread per (device, position in the call's device list): the
// thread-local contexts (streams, pinned slots) it builds on first use are
// kept for later calls.
class DevWorker {
public:
    explicit DevWorker(int dev) : dev_(dev), th_([this] { loop(); }) {}
    void post(std::function<void()> fn) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(fn));
        }
        cv_.notify_one();
    }

private:
    void loop() {
        (void)hipSetDevice(dev_);
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [this] { return !q_.empty(); });
            std::function<void()> fn = std::move(q_.front());
            q_.pop_front();
            lk.unlock();
            fn();
            lk.lock();
        }
    }
    int dev_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    std::thread th_;
};

DevWorker& dev_worker(int dev, size_t pos) {
    // lives for the process (workers may be parked at exit); a forked child
    // builds its own
    static std::mutex m;
    static std::map<std::pair<int, size_t>, DevWorker*>* workers = nullptr;
    static pid_t owner = 0;
    std::lock_guard<std::mutex> g(m);
    if (!workers || owner != getpid()) {
        workers = new std::map<std::pair<int, size_t>, DevWorker*>;
        owner = getpid();
    }
    DevWorker*& w = (*workers)[{dev, pos}];
    if (!w) w = new DevWorker(dev);
    return *w;
}

struct ShardResult {
    int status = FEC_OK;
    char msg[256] = "";
};

int run_batch_multi(const fec_t* code, const uint8_t* coef, unsigned r, const gf* src, size_t sbs, size_t sss,
                    gf* dst, size_t dbs, size_t dss, size_t sz, size_t nstripes, const int* devices, size_t ndev,
                    unsigned flags) {
    const int ngpu = gpu_available();
    if (!ngpu) return set_status(FEC_ENODEV, "no GPU visible to HIP (the engine has no CPU path)");
    if (!src || !dst) return set_status(FEC_EINVAL, "NULL buffer");
    if (!devices || ndev == 0) return set_status(FEC_EINVAL, "no devices listed");
    for (size_t d = 0; d < ndev; ++d)
        if (devices[d] < 0 || devices[d] >= ngpu)
            return set_status(FEC_EINVAL, "device %d out of range (%d visible)", devices[d], ngpu);
    if (pointer_device(src) >= 0 || pointer_device(dst) >= 0)
        return set_status(FEC_EINVAL,
                          "multi-device calls take host memory (device-resident batches: one call per device)");
    std::vector<ShardResult> res(ndev);
    std::mutex mu;
    std::condition_variable cv;
    // stripes [s0, s1) of shard d: balanced contiguous ranges (zfec_amd/shard.py shard_range)
    const size_t base = nstripes / ndev, extra = nstripes % ndev;
    const size_t shards = std::min(ndev, nstripes);  // the non-empty ones: d < nstripes
    size_t left = shards;  // shards not finished (or never posted); guarded by mu
    // The workers reference this frame (mu, cv, left, res): whatever happens
    // while posting (a thread that cannot be created, bad_alloc), the frame
    // stays until every posted shard has finished.
    int post_status = FEC_OK;
    char post_msg[sizeof t_msg] = "";
    for (size_t d = 0; d < shards; ++d) {
        const size_t s0 = d * base + std::min(d, extra), n = base + (d < extra ? 1 : 0);
        const gf* ps = src + s0 * sss;
        gf* pd = dst + s0 * dss;
        ShardResult* out = &res[d];
        const int dev = devices[d];
        const int pst = guarded([&] {
            dev_worker(dev, d).post([=, &mu, &cv, &left] {
                (void)hipSetDevice(dev);
                const int st = guarded([&] {
                    return run_batch(code, coef, r, ps, sbs, sss, pd, dbs, dss, sz, n, nullptr,
                                     (flags & ~FEC_FLAG_ASYNC) | FEC_FLAG_LIBRARY_STREAM);
                });
                out->status = st;
                if (st != FEC_OK) snprintf(out->msg, sizeof out->msg, "device %d: %s", dev, t_msg);
                std::lock_guard<std::mutex> g(mu);
                if (--left == 0) cv.notify_all();
            });
            return FEC_OK;
        });
        if (pst != FEC_OK) {  // shards d.. were never posted: take them off the count
            post_status = pst;
            snprintf(post_msg, sizeof post_msg, "%s", t_msg);
            std::lock_guard<std::mutex> g(mu);
            left -= shards - d;
            break;
        }
    }
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
    if (post_status != FEC_OK) return set_status(post_status, "%s", post_msg);
    for (const ShardResult& r0 : res)
        if (r0.status != FEC_OK) return set_status(r0.status, "%s", r0.msg);
    return set_status(FEC_OK);
}

}  // namespace

FEC_API int fec_encode_batch_multi(const fec_t* code, const gf* src, size_t src_block_stride,
                                   size_t src_stripe_stride, gf* dst, size_t dst_block_stride,
                                   size_t dst_stripe_stride, const unsigned* block_nums, size_t num_block_nums,
                                   size_t sz, size_t nstripes, const int* devices, size_t ndevices, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    if (check_block_nums(code, block_nums, num_block_nums)) return t_status;
    if (num_block_nums == 0 || sz == 0 || nstripes == 0) return set_status(FEC_OK);
    return guarded([&] {
        return run_batch_multi(code, encode_rows(code, block_nums, num_block_nums),
                               static_cast<unsigned>(num_block_nums), src, src_block_stride, src_stripe_stride, dst,
                               dst_block_stride, dst_stripe_stride, sz, nstripes, devices, ndevices, flags);
    });
}

FEC_API int fec_decode_batch_multi(const fec_t* code, const gf* src, size_t src_block_stride,
                                   size_t src_stripe_stride, gf* dst, size_t dst_block_stride,
                                   size_t dst_stripe_stride, const unsigned* index, size_t sz, size_t nstripes,
                                   const int* devices, size_t ndevices, unsigned flags) {
    if (!valid_code(code)) return set_status(FEC_EINVAL, "invalid fec_t");
    thread_local std::vector<uint8_t> rows;
    unsigned r = 0;
    if (decode_rows(code, index, rows, r, (flags & FEC_FLAG_ALL_PRIMARIES) != 0)) return t_status;
    if (r == 0 || sz == 0 || nstripes == 0) return set_status(FEC_OK);
    return guarded([&] {
        return run_batch_multi(code, rows.data(), r, src, src_block_stride, src_stripe_stride, dst, dst_block_stride,
                               dst_stripe_stride, sz, nstripes, devices, ndevices, flags);
    });
}
