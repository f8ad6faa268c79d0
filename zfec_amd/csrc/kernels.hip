// kernels.hip -- GF(2^8) matrix-apply kernels for gfx950 (MI355X, CDNA4).
//
// The hot loop of zfec is _addmul1 (zfec/fec.c:170-204): dst[i] ^= c*src[i]
// through a 256-byte table row per coefficient, driven by fec_encode
// (fec.c:487-505) and fec_decode (fec.c:527-557).  Here one kernel reads each
// input chunk from HBM once and produces every requested output from it:
//
//   * each lane owns a 16-byte (or 8-byte) column slice of every block, so a
//     wave's loads and stores are 1 KiB (512 B) contiguous;
//   * multiplication by a constant c is GF(2)-linear, so
//       c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
//     with three 8/8/4-entry byte tables; v_perm_b32 looks up four bytes at
//     once in an 8-byte table held in a register pair;
//   * partial products are merged by v_bitop3_b32 (gfx950's 3-input logic
//     op; truth table 0x96 = XOR3).
//
// Kernel families:
//   matapply_reg<K, R>  compile-time k <= 4 and r <= 8 (encode K=3/M=10 is
//                       <3,7>, its decode <3,3>): all K*R tables arrive in a
//                       kernel argument block sized to them (RegJob) and stay
//                       in registers; the per-chunk body is straight-line code.
//   matapply_rows<K, R> the same arithmetic, one wave per stripe of short blocks.
//   matapply_lds        any k <= 32, r <= 48 (longer codes are split by the
//                       caller): each workgroup expands its coefficients into
//                       LDS tables from a compile-time bank of all 256 values;
//                       rows in register tiles, inputs in prefetched groups.
//   matapply_bsr<RT>    bit-sliced, coefficients as run-time data, any
//                       k <= 256, r <= 256: one call per coefficient into
//                       precompiled multiply-by-constant routines
//                       (gf_routines.inc); past 32 inputs or 40 rows its
//                       pointers and coefficients come from a device-side table.
//   matapply_bsg        bit-sliced, coefficients as run-time data, k <= 256
//                       (past 32 inputs its pointers and coefficients come
//                       from a device-side table).
//   matapply_small      launches too small to fill the chip, wide codes.
//
// Measured issue rates on gfx950 (tools/mb_valu.hip): v_perm_b32 and
// v_bitop3_b32 (VOP3) sustain ~37 T lane-ops/s chip-wide, plain VOP2 ops
// ~60 T.  A coefficient costs 3 v_perm + 1.5 v_bitop3 per 4 bytes, so K=3/M=10
// (~9 VOP3 per input byte, ~22 T ops/s at the HBM roofline) is memory-bound,
// while wide codes are bound by VALU issue (K=20/M=60: 45 VOP3 per input
// byte, <= ~0.8 TB/s of input).
#include "kernels.hpp"

#include <hip/hip_runtime.h>

#include "bitslice.hpp"
#include "config.hpp"

#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <unordered_map>
#include <vector>
#include <type_traits>
#include <utility>

namespace zfec_hip {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// v_perm_b32: byte i of the result = byte sel_i of the 8-byte value {hi:lo}
// (selector 0-3 -> lo, 4-7 -> hi).
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// ---- tables -----------------------------------------------------------------
// For a coefficient c, five dwords:
//   w0/w1 = c*{0..7}             (indexed by bits 0-2 of x)
//   w2/w3 = c*{0,8,...,56}       (bits 3-5)
//   w4    = c*{0,64,128,192}     (bits 6-7)
// All 256 values are built at compile time into constant memory (8 dwords
// per value, 8 KiB).

struct TableBank {
    uint32_t w[256 * 8];
};

constexpr uint32_t ct_xtime(uint32_t v) { return ((v << 1) & 0x100u) ? (((v << 1) ^ 0x11Du) & 0xFFu) : (v << 1); }

constexpr TableBank make_bank() {
    TableBank b{};
    for (uint32_t c = 0; c < 256; ++c) {
        uint32_t p[8] = {};
        p[0] = c;  // p[i] = c * alpha^i = c * 2^i
        for (int i = 1; i < 8; ++i) p[i] = ct_xtime(p[i - 1]);
        for (int h = 0; h < 2; ++h) {
            uint32_t lo = 0, hi = 0;
            for (int n = 0; n < 8; ++n) {
                const uint32_t e =
                    ((n & 1) ? p[3 * h] : 0u) ^ ((n & 2) ? p[3 * h + 1] : 0u) ^ ((n & 4) ? p[3 * h + 2] : 0u);
                if (n < 4)
                    lo |= e << (8 * n);
                else
                    hi |= e << (8 * (n - 4));
            }
            b.w[c * 8 + 2 * h] = lo;
            b.w[c * 8 + 2 * h + 1] = hi;
        }
        b.w[c * 8 + 4] = (p[6] << 8) | (p[7] << 16) | ((p[6] ^ p[7]) << 24);
    }
    return b;
}

__constant__ TableBank g_bank = make_bank();

// Host copy of the bank: the register kernels get their coefficients'
// tables in the kernel arguments.
constexpr TableBank kHostBank = make_bank();

struct Tab {
    uint32_t w0, w1, w2, w3, w4;
};

// ---- arithmetic ---------------------------------------------------------------

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
    return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// sum_j c_j*x_j for four bytes of one output row: the 3K partial products are
// merged by a chain of XOR3s, 3K v_perm + ceil((3K-1)/2) v_bitop3.
template <int K>
__device__ __forceinline__ uint32_t gf_dot(const Tab (&T)[K], const Sel (&s)[K]) {
    uint32_t p[3 * K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        p[3 * j + 0] = perm(T[j].w1, T[j].w0, s[j].s0);
        p[3 * j + 1] = perm(T[j].w3, T[j].w2, s[j].s1);
        p[3 * j + 2] = perm(T[j].w4, T[j].w4, s[j].s2);
    }
    uint32_t acc = xor3(p[0], p[1], p[2]);
#pragma unroll
    for (int i = 3; i + 1 < 3 * K; i += 2) acc = xor3(acc, p[i], p[i + 1]);
    if constexpr ((3 * K) % 2 == 0) acc ^= p[3 * K - 1];
    return acc;
}

// ---- memory -------------------------------------------------------------------

__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);  // global_load_dwordx4; unaligned addresses are legal on gfx950
    return v;
}

__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

// Streaming store (global_store_dwordx4 ... nt): outputs are written once and
// not re-read by this kernel.
template <bool NT>
__device__ __forceinline__ void store16_out(uint8_t* p, u32x4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else
        store16(p, v);
}

// Output store of the register kernels: SP = 0 streams it (nt), SP = 3
// streams it and writes it through the L2 at device scope (nt sc1; the
// single-stripe store policy, kernels dispatch below).  The trailing s_nop
// keeps the compiler's next instruction from overwriting the data registers
// before the store has read them.
template <int SP>
__device__ __forceinline__ void store16_pol(uint8_t* p, u32x4 v) {
    if constexpr (SP == 3)
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        store16_out<true>(p, v);
}

// The last (sz % 16) bytes of a block.
__device__ inline u32x4 load_tail(const uint8_t* p, uint32_t nb) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t b = 0; b < nb; ++b) w[b >> 2] |= static_cast<uint32_t>(p[b]) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ inline void store_tail(uint8_t* p, u32x4 v, uint32_t nb) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t b = 0; b < nb; ++b) p[b] = static_cast<uint8_t>(w[b >> 2] >> (8 * (b & 3)));
}

// Walks this lane's (stripe, chunk) units in grid-stride order without a
// division per step.  (An XCD-contiguous workgroup order measured 2 % slower
// on 256 x 1 MiB K=3/M=10 encodes from cold caches, profiles/r02_mb_cold.log.)
struct UnitIter {
    uint32_t s, c;
    template <class J>
    __device__ explicit UnitIter(const J& job) : UnitIter(job, blockIdx.x) {}
    // `block`: the workgroup's index among the job's own workgroups (a paired
    // launch deals its grid across two jobs)
    template <class J>
    __device__ UnitIter(const J& job, uint32_t block) {
        const uint32_t gid = block * kBlock + threadIdx.x;
        s = gid / job.cps;
        c = gid - s * job.cps;
    }
    template <class J>
    __device__ __forceinline__ void next(const J& job) {
        c += job.gs_c;
        s += job.gs_s;
        if (c >= job.cps) {
            c -= job.cps;
            ++s;
        }
    }
};

// ZFEC_TAIL_ORDER (A/B knob, tools/ab_build.sh; 0 = UnitIter, the default):
// where the register kernels' walk puts each stripe's last chunk (the one
// that ends every row, mid-line when sz is not a multiple of 128): 1 = the
// ns row-tail units first in the walk, then the rest in order; 2 = last.
#ifndef ZFEC_TAIL_ORDER
#define ZFEC_TAIL_ORDER 0
#endif
template <int ORDER>
struct TailIter {
    uint32_t s, c, g, step, ns, cpb, bq, br;  // cpb: body chunks per stripe (cps - 1)
    template <class J>
    __device__ TailIter(const J& job, uint32_t block) {
        ns = job.nstripes;
        cpb = job.cps - 1;
        step = job.gs_s * job.cps + job.gs_c;
        g = block * kBlock + threadIdx.x;
        bq = cpb ? step / cpb : 0u;
        br = cpb ? step - bq * cpb : 0u;
        map();
    }
    __device__ void map() {
        if (cpb == 0) {  // one chunk per stripe: no tail of its own
            s = g;
            c = 0;
            return;
        }
        if constexpr (ORDER == 1) {
            if (g < ns) {
                s = g;
                c = cpb;
            } else {
                const uint32_t h = g - ns;
                s = h / cpb;
                c = h - s * cpb;
            }
        } else {
            const uint32_t body = ns * cpb;
            if (g < body) {
                s = g / cpb;
                c = g - s * cpb;
            } else {
                s = g - body;
                c = cpb;
            }
        }
    }
    template <class J>
    __device__ __forceinline__ void next(const J&) {
        const bool tail = cpb && c == cpb;
        g += step;
        if (cpb == 0 || tail || (ORDER == 2 && s + bq + 1 >= ns)) {  // regime change possible: recompute
            map();
            return;
        }
        c += br;
        s += bq;
        if (c >= cpb) {
            c -= cpb;
            ++s;
        }
        if constexpr (ORDER == 1)
            if (s >= ns) s = 0xFFFFFFFFu;  // past the body: done
    }
};
#if ZFEC_TAIL_ORDER
using RegIter = TailIter<ZFEC_TAIL_ORDER>;
#else
using RegIter = UnitIter;
#endif

// Byte span of chunk c of a block of sz bytes.  Chunks are CH bytes; the last
// one, when sz is not a multiple of CH, is shifted back to end at sz and so
// overlaps its neighbour: both lanes compute and store identical bytes there,
// and every lane stays on the full-width load/store path.  Blocks shorter
// than CH, and accumulating launches (XOR into the output is not idempotent),
// take the byte-wise tail instead.
struct Span {
    uint64_t off;
    bool full;
    uint32_t nb;
};

template <uint32_t CH, bool OVERLAP>
__device__ __forceinline__ Span chunk_span(uint32_t c, uint64_t sz, uint32_t nfull) {
    const uint64_t off = static_cast<uint64_t>(c) * CH;
    if (c < nfull) return Span{off, true, CH};
    if (OVERLAP && sz >= CH) return Span{sz - CH, true, CH};
    return Span{off, false, static_cast<uint32_t>(sz - off)};
}

// A kernel's argument block read in place from the kernel-argument segment
// through a pointer the compiler must treat as new at every call (empty asm):
// the loads stay where they are used instead of all being hoisted into the
// prologue, where the table dwords and the block pointers overflow the SGPRs
// and spill to VGPR lanes (v_writelane / v_readlane per wave).
template <class J>
using KPtr = const __attribute__((address_space(4))) J*;

// OFF: the block's byte offset in the argument segment (the second job of a
// paired launch).
template <class J, size_t OFF = 0>
__device__ __forceinline__ KPtr<J> kernarg_job() {
    typedef const __attribute__((address_space(4))) char* KBytes;
    KPtr<J> kj = (KPtr<J>)((KBytes)__builtin_amdgcn_kernarg_segment_ptr() + OFF);
    asm volatile("" : "+s"(kj));
    return kj;
}

// ---------------------------------------------------------------------------
// matapply_reg<K, R>: compile-time k and r.  The kernel argument block holds
// the K + R block pointers and the K*R coefficients' tables (5 dwords each):
// 560 bytes for <3,7>, against 2.2 KiB for the table kernels' MatJob.
// ---------------------------------------------------------------------------
template <int K, int R>
struct alignas(16) RegJob {
    uint64_t sz, in_sstride, out_sstride;
    uint32_t nstripes, cps, gs_c, gs_s;
    uint32_t* done_flag;  // pinned host word a one-workgroup launch stores done_seq into when finished
    uint32_t done_seq, pad_;
    const uint8_t* in[K];
    uint8_t* out[R];
    uint32_t tab[K * R * 5];
};

template <int K, int R>
__device__ __forceinline__ Tab reg_table(const RegJob<K, R>& job, uint32_t i) {
    const uint32_t* t = &job.tab[i * 5];
    return Tab{t[0], t[1], t[2], t[3], t[4]};
}

// One (stripe, chunk) unit: load K x 16 bytes, store R x 16 bytes.  AL: each
// row's tables and output pointer are loaded (scalar loads) right before use.
template <int K, int R, int SP, bool AL, size_t OFF = 0>
__device__ __forceinline__ void reg_compute_store(const RegJob<K, R>& job, const Tab (&T)[R][K], const u32x4 (&x)[K],
                                                  uint64_t ob, bool full, uint32_t nb) {
    Sel sel[4][K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        sel[0][j] = selectors(x[j].x);
        sel[1][j] = selectors(x[j].y);
        sel[2][j] = selectors(x[j].z);
        sel[3][j] = selectors(x[j].w);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        Tab t[K];
        uint8_t* out;
        if constexpr (AL) {
            const KPtr<RegJob<K, R>> kj = kernarg_job<RegJob<K, R>, OFF>();
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t i = (r * K + j) * 5;
                t[j] = Tab{kj->tab[i], kj->tab[i + 1], kj->tab[i + 2], kj->tab[i + 3], kj->tab[i + 4]};
            }
            out = kj->out[r];
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) t[j] = T[r][j];
            out = job.out[r];
        }
        const u32x4 y{gf_dot<K>(t, sel[0]), gf_dot<K>(t, sel[1]), gf_dot<K>(t, sel[2]), gf_dot<K>(t, sel[3])};
        if (full)
            store16_pol<SP>(out + ob, y);
        else
            store_tail(out + ob, y, nb);
    }
}

template <int K, int R>
__device__ __forceinline__ void reg_load(const RegJob<K, R>& job, u32x4 (&x)[K], uint64_t ib, bool full,
                                         uint32_t nb) {
    if (full) {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + ib);
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_tail(job.in[j] + ib, nb);
    }
}

// PF: the next unit's inputs are loaded before the current unit is computed,
// so a lane with several units (grid-stride) keeps loads in flight while it
// computes (tools/mb_encode.hip, variants "PF"; 5-8 rows only: from cold
// caches the 3-row decode is slower with it, profiles/r02_reg_pf_ab.log).
// SP: output store policy (store16_pol).  AL: tables and output pointers read
// where they are used (reg_compute_store).
template <int K, int R, int SP, bool PF, bool AL, size_t OFF>
__device__ __forceinline__ void reg_body(const RegJob<K, R>& job, uint32_t block) {
    Tab T[R][K];
    if constexpr (!AL) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < K; ++j) T[r][j] = reg_table(job, r * K + j);
    }

    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    RegIter u(job, block);
    if constexpr (PF) {
        u32x4 x[K];
        Span sp = chunk_span<kChunk, true>(u.c, sz, nfull);
        uint64_t ob = u.s * job.out_sstride + sp.off;
        if (u.s < job.nstripes) reg_load<K, R>(job, x, u.s * job.in_sstride + sp.off, sp.full, sp.nb);
        while (u.s < job.nstripes) {
            RegIter v = u;
            v.next(job);
            const Span spn = chunk_span<kChunk, true>(v.c, sz, nfull);
            u32x4 xn[K];
            if (v.s < job.nstripes) reg_load<K, R>(job, xn, v.s * job.in_sstride + spn.off, spn.full, spn.nb);
            reg_compute_store<K, R, SP, AL, OFF>(job, T, x, ob, sp.full, sp.nb);
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = xn[j];
            sp = spn;
            ob = v.s * job.out_sstride + spn.off;
            u = v;
        }
    } else {
        while (u.s < job.nstripes) {
            const Span sp = chunk_span<kChunk, true>(u.c, sz, nfull);
            u32x4 x[K];
            reg_load<K, R>(job, x, u.s * job.in_sstride + sp.off, sp.full, sp.nb);
            reg_compute_store<K, R, SP, AL, OFF>(job, T, x, u.s * job.out_sstride + sp.off, sp.full, sp.nb);
            u.next(job);
        }
    }
}

template <int K, int R, int SP, bool PF, bool AL>
__global__ __launch_bounds__(kBlock) void matapply_reg(const RegJob<K, R> job) {
    reg_body<K, R, SP, PF, AL, 0>(job, blockIdx.x);
    // one-workgroup launches of a synchronous small call: publish completion
    // in pinned host memory, so the host need not wait in
    // hipStreamSynchronize (fec_abi.cpp run_single).  Every storing wave waits
    // for its own stores, the workgroup meets at a barrier, and ONE lane
    // releases at system scope and stores the flag (MI355X_MICROARCH.md
    // "Valid forms"): one L2 write-back per call.  (A system fence in every
    // wave before the barrier, round 2's form, cost five write-backs: the
    // kernel took 6.1 us in the trace against 2.6 us for this form,
    // tools/inline_probe.hip, profiles/r03_small_call_kernels.txt.)
    if (job.done_flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(job.done_flag, job.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ---------------------------------------------------------------------------
// matapply_one<K>: the synchronous small call from host memory (fec_abi.cpp
// run_single: every block in the thread's pinned bounce buffer, read and
// written over PCIe).  One workgroup, one whole 16-byte unit per lane (the
// bounce buffer's 256-byte slots let a row run to its 16-byte multiple), and
// the output rows in a loop that is not unrolled, each row's tables and
// pointer read from the argument segment where they are used.  A
// one-workgroup launch lands on any XCD and fetches its instructions cold, so
// code size is latency: matapply_reg<3,7> (7.4 KB of code, the unrolled rows
// and the grid-stride walk with its prefetch and tail paths) took 5.5 us in
// the kernel trace against 2.6 us for a stand-in of the same PCIe traffic
// (profiles/r03_small_call_kernels.txt).
// ---------------------------------------------------------------------------
struct alignas(16) OneJob {
    const uint8_t* in[4];
    uint8_t* out[8];
    uint32_t* done_flag;
    uint32_t units, r, done_seq, pad_;
    alignas(16) uint32_t tab[4 * 8 * 5];  // row-major (r, j) coefficient tables, K per row (16-byte loads)
};
static_assert(offsetof(OneJob, tab) % 16 == 0, "matapply_one loads the tables 16 bytes at a time");

// INL: the k input blocks ride in the argument block itself (k x units x 16
// bytes at most kOneInline), which HIP writes to device memory with the
// launch: the kernel reads them there instead of across PCIe from the bounce
// buffer, and the caller's bytes need no copy into pinned memory first
// (tools/inline_probe.hip: 7.2 against 7.9 us launch to completion seen for
// a 4 KiB K=3/M=10 encode stand-in).
constexpr uint32_t kOneInline = kOneInlineBytes;  // a 4 KiB K=3 stripe: 3 x 88 units of 16 bytes = 4,224
struct alignas(16) OneJobInline {
    OneJob job;
    u32x4 data[kOneInline / 16];  // input j's unit u at data[j * units + u]
};

__device__ __forceinline__ const OneJob& one_job(const OneJob& a) { return a; }
__device__ __forceinline__ const OneJob& one_job(const OneJobInline& a) { return a.job; }

template <int K, bool INL, class J>
__global__ __launch_bounds__(kBlock) void matapply_one(const J arg) {
    const OneJob& job = one_job(arg);
    // the coefficient tables (up to 160 dwords) reach LDS in ONE vector load
    // round trip (a lane per 16 bytes of the argument segment), not in a
    // chain of scalar loads per output row
    __shared__ u32x4 stab[4 * 8 * 5 / 4];
    const uint32_t u = threadIdx.x;
    const uint32_t ntab4 = (job.r * K * 5 + 3) / 4;
    if (u < ntab4) {
        const KPtr<OneJob> kj = kernarg_job<OneJob>();
        stab[u] = reinterpret_cast<const __attribute__((address_space(4))) u32x4*>(kj->tab)[u];
    }
    u32x4 x[K];
    if (u < job.units) {
        if constexpr (INL) {
            const KPtr<OneJobInline> kj = kernarg_job<OneJobInline>();
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = kj->data[j * job.units + u];
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + size_t(u) * 16);
        }
    }
    __syncthreads();
    if (u < job.units) {
        Sel sel[4][K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            sel[0][j] = selectors(x[j].x);
            sel[1][j] = selectors(x[j].y);
            sel[2][j] = selectors(x[j].z);
            sel[3][j] = selectors(x[j].w);
        }
        const uint32_t* st = reinterpret_cast<const uint32_t*>(stab);
#pragma unroll 1
        for (uint32_t r = 0; r < job.r; ++r) {
            Tab t[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                const uint32_t i = (r * K + j) * 5;
                t[j] = Tab{st[i], st[i + 1], st[i + 2], st[i + 3], st[i + 4]};
            }
            const u32x4 y{gf_dot<K>(t, sel[0]), gf_dot<K>(t, sel[1]), gf_dot<K>(t, sel[2]), gf_dot<K>(t, sel[3])};
            store16_pol<3>(job.out[r] + size_t(u) * 16, y);
        }
    }
    // completion as matapply_reg's: every wave waits for its stores, barrier,
    // one lane's system-scope release, then the flag
    if (job.done_flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(job.done_flag, job.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

constexpr bool reg_prefetch(int R) { return R >= 5; }
constexpr bool reg_argload(int K, int R) { return K * R * 5 >= 50; }

// ---------------------------------------------------------------------------
// matapply_pair<K, RA, RB>: two independent matrix applications over the same
// k in one launch (fec_run_batch_jobs: e.g. a stripe's encode and another
// stripe's decode), so the pair pays one launch ramp-up and drain instead of
// two.  The grid is both jobs' grids side by side; each workgroup walks its
// own job exactly as matapply_reg would.  RB <= min(RA, K): the second job
// is the narrower one (a decode recovers at most k blocks).
// ---------------------------------------------------------------------------
template <int K, int RA, int RB>
struct alignas(16) PairJob {
    RegJob<K, RA> a;
    RegJob<K, RB> b;
    uint32_t blocks_a, pad_[3];
};

// Job a's workgroups first, then job b's: the dispatcher starts b's as a's
// retire.  (Alternating the two jobs' workgroups measured 10 % slower on the
// cfg2 step, profiles/r03_pair_ab.json.)
template <int K, int RA, int RB, int SP>
__global__ __launch_bounds__(kBlock) void matapply_pair(const PairJob<K, RA, RB> job) {
    using PJ = PairJob<K, RA, RB>;
    constexpr size_t kOffB = offsetof(PJ, b);
    if (blockIdx.x < job.blocks_a)
        reg_body<K, RA, SP, reg_prefetch(RA), reg_argload(K, RA), 0>(job.a, blockIdx.x);
    else
        reg_body<K, RB, SP, reg_prefetch(RB), reg_argload(K, RB), kOffB>(job.b, blockIdx.x - job.blocks_a);
}

// ---------------------------------------------------------------------------
// matapply_rows<K, R>: many stripes of short blocks (1 KiB < sz <= 4 KiB).
// One wave per stripe: lane l owns bytes 16l + 1024h of every block (the last
// chunk shifted back to end at sz), so each wave instruction reads or writes
// one contiguous piece of one block.  The stripe-major unit walk of
// matapply_reg would let a wave instruction straddle the end of one stripe's
// block and the start of the next one's (two DRAM rows); at K=3/M=10 with
// 1366-byte blocks the row walk is 5 % faster (tools/mb_rows.hip).  Every
// piece of the lane's share of the stripe (at most 4) is loaded before any is
// computed, so all of the wave's loads are in flight at once (cfg5 encode
// 67.7 -> 70.1 % of HBM cold, decode 66.7 -> 69.8 %, profiles/r02_rows_pre_ab.log).
// ---------------------------------------------------------------------------
constexpr uint64_t kRowsMin = 1024, kRowsMax = 4096;

template <int K, int R, bool AL>
__global__ __launch_bounds__(kBlock) void matapply_rows(const RegJob<K, R> job) {
    Tab T[R][K];
    if constexpr (!AL) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < K; ++j) T[r][j] = reg_table(job, r * K + j);
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * (kBlock / 64);
    const uint64_t sz = job.sz;
    for (uint32_t s = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); s < job.nstripes; s += waves) {
        u32x4 x[4][K];
        uint64_t o[4];
        bool live[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint64_t off = lane * 16u + 1024u * h;
            live[h] = off < sz;
            o[h] = off + 16u <= sz ? off : sz - 16u;
            if (live[h]) reg_load<K, R>(job, x[h], s * job.in_sstride + o[h], true, 16u);
        }
#pragma unroll
        for (int h = 0; h < 4; ++h)
            if (live[h]) reg_compute_store<K, R, 0, AL>(job, T, x[h], s * job.out_sstride + o[h], true, 16u);
    }
}

// ---------------------------------------------------------------------------
// matapply_lds<ACC, NT, RT>: runtime k and r like matapply_gen, but each
// workgroup first expands its k*r coefficients into LDS tables (32 bytes per
// coefficient).  In the loop a table is two broadcast LDS reads off one base
// address straight into VGPRs, so v_perm_b32 gets all-VGPR operands (gfx9's
// one-SGPR-per-VALU-op limit forces a v_mov per table word pair on the
// scalar path) and no scalar load -> dependent load chain sits in the loop.
// Inputs go in pairs so six partial products share three XOR3s, and rows
// past r in the last tile are skipped by a wave-uniform branch.
// ---------------------------------------------------------------------------
struct LdsTab {
    u32x4 w03;  // c*{0..7} and c*{0,8,..,56}
    u32x4 w4;   // c*{0,64,128,192}, 3 pad words (keeps both reads on one base address)
};

// Entry (input j, row) at j * rp + row, rp >= r: a tile's rows for one input
// are adjacent; rows r..rp-1 (padding up to whole tiles) get the zero table.
__device__ __forceinline__ void lds_tables_build(const MatJob& job, LdsTab* t, uint32_t rp) {
    const uint32_t n = job.k * rp;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        const uint32_t j = i / rp, row = i - j * rp;
        const uint32_t c = row < job.r ? job.coef[row * job.k + j] : 0u;
        const uint32_t* b = &g_bank.w[c * 8];
        t[i].w03 = u32x4{b[0], b[1], b[2], b[3]};
        t[i].w4 = u32x4{b[4], 0u, 0u, 0u};
    }
    __syncthreads();
}

// acc ^ c0*x0 ^ c1*x1 for four bytes: 6 v_perm_b32 + 3 v_bitop3_b32.
__device__ __forceinline__ uint32_t gf_mac2(uint32_t acc, const u32x4& t0, uint32_t u0, Sel s0, const u32x4& t1,
                                            uint32_t u1, Sel s1) {
    const uint32_t a0 = perm(t0.y, t0.x, s0.s0), b0 = perm(t0.w, t0.z, s0.s1), d0 = perm(u0, u0, s0.s2);
    const uint32_t a1 = perm(t1.y, t1.x, s1.s0), b1 = perm(t1.w, t1.z, s1.s1), d1 = perm(u1, u1, s1.s2);
    return xor3(xor3(xor3(acc, a0, b0), d0, a1), b1, d1);
}

__device__ __forceinline__ uint32_t gf_mac_v(uint32_t acc, const u32x4& t, uint32_t t4, Sel s) {
    const uint32_t a = perm(t.y, t.x, s.s0);
    const uint32_t b = perm(t.w, t.z, s.s1);
    const uint32_t d = perm(t4, t4, s.s2);
    return xor3(xor3(acc, a, b), d, 0u);
}

// D dwords per lane per block (chunk = 4*D bytes): D = 4 is one dwordx4 per
// block, D = 2 halves the accumulator / selector / input registers so more
// waves fit per SIMD.
template <int D>
struct Words {
    uint32_t w[D];
};

template <int D>
__device__ __forceinline__ Words<D> load_words(const uint8_t* p, bool full, uint32_t nb) {
    Words<D> x;
    if (full) {
        __builtin_memcpy(x.w, p, 4 * D);
    } else {
        const u32x4 t = load_tail(p, nb);
        const uint32_t tw[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int v = 0; v < D; ++v) x.w[v] = tw[v];
    }
    return x;
}

template <int D, bool NT>
__device__ __forceinline__ void store_words(uint8_t* p, const Words<D>& y, bool full, uint32_t nb) {
    if (full) {
        if constexpr (D == 4) {
            store16_out<NT>(p, u32x4{y.w[0], y.w[1], y.w[2], y.w[3]});
        } else if constexpr (D == 2) {
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v{y.w[0], y.w[1]};
            if constexpr (NT)
                __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(p));
            else
                __builtin_memcpy(p, &v, 8);
        } else {
            __builtin_memcpy(p, y.w, 4 * D);
        }
    } else {
        u32x4 t{0u, 0u, 0u, 0u};
        t.x = y.w[0];
        if constexpr (D > 1) t.y = y.w[1];
        if constexpr (D > 2) t.z = y.w[2];
        if constexpr (D > 3) t.w = y.w[3];
        store_tail(p, t, nb);
    }
}

// One step of the flattened (unit, row tile, input group) walk.
struct Step {
    UnitIter u;
    uint32_t rb, g;
};

// acc[rr] ^= sum over the group's inputs of table(j, rb + rr) * x_j, for the
// RT_ rows of one tile.  FULL: every row of the tile exists (no per-row
// branch, so no register copies where the two paths of a branch meet).
template <bool FULL, int RT_, int D, int GG>
__device__ __forceinline__ void mac_group(uint32_t (&a)[RT_][D], const Words<D> (&x)[GG], const LdsTab* lds_tab,
                                          uint32_t g, uint32_t rb, uint32_t k, uint32_t r) {
#pragma unroll
    for (int jj = 0; jj < GG; jj += 2) {
        const uint32_t j = g + jj;
        if (j >= k) break;
        Sel s0[D];
#pragma unroll
        for (int v = 0; v < D; ++v) s0[v] = selectors(x[jj].w[v]);
        const LdsTab* t0 = lds_tab + j * r + rb;
        if (jj + 1 < GG && j + 1 < k) {  // two inputs: their six partial products share three XOR3s
            Sel s1[D];
#pragma unroll
            for (int v = 0; v < D; ++v) s1[v] = selectors(x[jj + 1].w[v]);
            const LdsTab* t1 = t0 + r;
#pragma unroll
            for (int rr = 0; rr < RT_; ++rr) {
                if (FULL || rb + rr < r) {  // wave-uniform
                    const u32x4 p = t0[rr].w03, q = t1[rr].w03;
                    const uint32_t pu = t0[rr].w4.x, qu = t1[rr].w4.x;
#pragma unroll
                    for (int v = 0; v < D; ++v) a[rr][v] = gf_mac2(a[rr][v], p, pu, s0[v], q, qu, s1[v]);
                }
            }
        } else {
#pragma unroll
            for (int rr = 0; rr < RT_; ++rr) {
                if (FULL || rb + rr < r) {
                    const u32x4 p = t0[rr].w03;
                    const uint32_t pu = t0[rr].w4.x;
#pragma unroll
                    for (int v = 0; v < D; ++v) a[rr][v] = gf_mac_v(a[rr][v], p, pu, s0[v]);
                }
            }
        }
    }
}

// Row tiling of a launch, fixed by the dispatcher:
enum TileMode {
    kTilesRagged = 0,  // rows past r in the last tile are skipped by a per-row branch
    kTilesPadded = 1,  // the table has zero rows up to whole tiles: no branch in the
                       // multiply-accumulate, only the stores of padding rows are skipped
};

// Rows of the LDS table: r, or r rounded up to whole RT-row tiles.
template <int MODE>
__host__ __device__ constexpr uint32_t table_rows(uint32_t r, uint32_t rt) {
    return MODE == kTilesPadded ? (r + rt - 1) / rt * rt : r;
}

template <bool ACC, bool NT, int RT_, int D, int GG, int MODE>
__device__ __forceinline__ void matapply_lds_body(const MatJob& job) {
    constexpr uint32_t CH = 4 * D;
    extern __shared__ LdsTab lds_tab[];
    const uint32_t k = job.k;
    const uint32_t r = job.r;
    const uint32_t rp = table_rows<MODE>(r, RT_);
    lds_tables_build(job, lds_tab, rp);
    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / CH);
    // The walk visits, for each of this lane's units in grid-stride order, each
    // row tile and, inside it, each group of GG inputs.  The loads of the next
    // step's group (possibly the next tile's first group, or the next unit's)
    // are issued before the current group is computed, so a wave never starts
    // a group waiting on HBM.  (rb, g) are wave-uniform; units differ per lane.
    auto load_step = [&](const Step& st, Words<D> (&x)[GG]) {
        const Span sp = chunk_span<CH, !ACC>(st.u.c, sz, nfull);
        const uint64_t ib = st.u.s * job.in_sstride + sp.off;
#pragma unroll
        for (int jj = 0; jj < GG; ++jj)
            if (st.g + jj < k) x[jj] = load_words<D>(job.in[st.g + jj] + ib, sp.full, sp.nb);
    };
    Step cur{UnitIter(job), 0u, 0u};
    bool live = cur.u.s < job.nstripes;
    uint32_t a[RT_][D];
#pragma unroll
    for (int rr = 0; rr < RT_; ++rr)
#pragma unroll
        for (int v = 0; v < D; ++v) a[rr][v] = 0u;
    // One step: prefetch the next step's group into xb, compute the current
    // group from xa, store the tile when its last group is done.  Every lane
    // walks the same (rb, g) sequence; a lane whose units ran out keeps
    // stepping (without memory traffic) until the whole wave is done.
    Words<D> xa[GG];
    if (live) load_step(cur, xa);
    while (__any(live)) {
        // (g, rb) are wave-uniform; say so, or they live in VGPRs and every
        // block pointer becomes a readfirstlane + dependent scalar load.
        cur.g = __builtin_amdgcn_readfirstlane(cur.g);
        cur.rb = __builtin_amdgcn_readfirstlane(cur.rb);
        Step nxt = cur;
        nxt.g += GG;
        const bool tile_end = nxt.g >= k;
        if (tile_end) {
            nxt.g = 0;
            nxt.rb += RT_;
            if (nxt.rb >= r) {
                nxt.rb = 0;
                nxt.u.next(job);
            }
        }
        const bool nlive = nxt.u.s < job.nstripes;
        Words<D> xb[GG];
        if (nlive) load_step(nxt, xb);
        if (live) {
            mac_group<MODE == kTilesPadded, RT_, D, GG>(a, xa, lds_tab, cur.g, cur.rb, k, rp);
            if (tile_end) {
                const Span sp = chunk_span<CH, !ACC>(cur.u.c, sz, nfull);
                const uint64_t ob = cur.u.s * job.out_sstride + sp.off;
#pragma unroll
                for (int rr = 0; rr < RT_; ++rr) {
                    if (cur.rb + rr >= r) continue;  // ragged tail or padding rows
                    uint8_t* op = job.out[cur.rb + rr] + ob;
                    Words<D> y;
#pragma unroll
                    for (int v = 0; v < D; ++v) y.w[v] = a[rr][v];
                    if constexpr (ACC) {
                        const Words<D> o = load_words<D>(op, sp.full, sp.nb);
#pragma unroll
                        for (int v = 0; v < D; ++v) y.w[v] ^= o.w[v];
                    }
                    store_words<D, NT>(op, y, sp.full, sp.nb);
                }
            }
        }
        if (tile_end) {
#pragma unroll
            for (int rr = 0; rr < RT_; ++rr)
#pragma unroll
                for (int v = 0; v < D; ++v) a[rr][v] = 0u;
        }
#pragma unroll
        for (int jj = 0; jj < GG; ++jj) xa[jj] = xb[jj];
        cur = nxt;
        live = nlive;
    }
}

template <bool ACC, bool NT, int RT_, int D, int GG, int MODE = kTilesRagged>
__global__ __launch_bounds__(kBlock) void matapply_lds(const MatJob job) {
    matapply_lds_body<ACC, NT, RT_, D, GG, MODE>(job);
}

// ---------------------------------------------------------------------------
// matapply_bsg<RT, TBL>: bit-sliced, with the coefficient matrix as run-time
// data (no compile step: every erasure pattern runs at this speed the first
// time).
//
// Multiplication by c is an 8x8 GF(2) matrix on the bits of a byte.  After an
// 8x8 bit transpose a lane's 32 bytes are 8 bit-planes p0..p7, and output
// plane b of c*x is L[ml_b] ^ H[mh_b], where L[m] is the XOR of the planes
// {a < 4 : bit a of m} and H[m] that of {4 + a : bit a of m}; ml_b / mh_b are
// the low / high nibble of the bit-b row of c's matrix (bitslice.cpp's JIT
// bakes the same choice of combinations into the instruction stream).  Here
// each input's 15 + 15 combinations go to LDS, and a wave selects them with
// the nibbles as wave-uniform LDS offsets: per coefficient and output plane two
// ds_read_b64 (both of the lane's 32-byte groups at once) and one v_bitop3
// XOR3 per group, against 4.5 VOP3 per 4 bytes for the table kernels.
//
// One workgroup (4 waves) per unit of 4 KiB of every block of a stripe: lane l
// owns bytes 16l + 1024h (h = 0..3) of each block, two 32-byte groups (h = 0,1
// and h = 2,3).  The r output rows are split over the 4 waves (RT rows each,
// accumulators in registers).  Inputs go in phases of 2: waves 0 and 1 each
// load one input of the phase, transpose it and write its combinations to
// their LDS slot; after a barrier every wave folds the phase's 2 inputs into
// its rows.  LDS per slot: 32 combinations x 64 lanes x 8 B = 16 KiB (entries
// 0 and 16 hold zeros, written once).  (Measured and not kept, DESIGN.md §4:
// 4 inputs per phase, a scheduling barrier per row, the input build balanced
// over all 4 waves.)
//
// TBL = false: block pointers and coefficients in the MatJob kernel arguments
// (k <= 32).  TBL = true: in a device-side table the host fills per launch
// (BsgTblJob::table: k input pointers, r output pointers, then the
// coefficients in walk order), read with scalar loads -- k up to 256 in one
// pass, instead of XOR-accumulating passes of 32 inputs.
// ---------------------------------------------------------------------------
constexpr uint32_t kBsgChunk = 4096;        // bytes of each block per unit
constexpr uint32_t kBsgSlotBytes = 32 * 512;  // one input's combinations
constexpr int kBsgPhase = 2;                // inputs per LDS phase

// g_bsg.off[c]: sixteen dwords, the LDS byte offsets of the combinations
// output plane b of c*x needs: [b] = L[ml_b], [8 + b] = H[mh_b] (b = 0..7).
struct BsgBank {
    uint32_t off[256 * 16];
};

constexpr BsgBank make_bsg_bank() {
    BsgBank t{};
    for (uint32_t c = 0; c < 256; ++c) {
        uint32_t p[8] = {};
        p[0] = c;  // c * 2^a
        for (int a = 1; a < 8; ++a) p[a] = ct_xtime(p[a - 1]);
        for (uint32_t b = 0; b < 8; ++b) {
            uint32_t ml = 0, mh = 0;
            for (uint32_t a = 0; a < 4; ++a) {
                ml |= ((p[a] >> b) & 1u) << a;
                mh |= ((p[a + 4] >> b) & 1u) << a;
            }
            t.off[c * 16 + b] = ml * 512u;
            t.off[c * 16 + 8 + b] = (16u + mh) * 512u;
        }
    }
    return t;
}

__constant__ BsgBank g_bsg = make_bsg_bank();

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(a, b, m, 0xE4);  // m ? a : b, bitwise
}

// one block swap of the 8x8 bit transpose, four byte lanes at once
__device__ __forceinline__ void bswap_blocks(uint32_t& a, uint32_t& b, int s, uint32_t m) {
    const uint32_t t0 = bsel(m, a, b << s);
    const uint32_t t1 = bsel(m, a >> s, b);
    a = t0;
    b = t1;
}

// Two block swaps with the same shift at once: the shifts on 64-bit register
// pairs (v_lshlrev_b64 / v_lshrrev_b64 move two dwords at the issue cost of one
// 32-bit shift, profiles/r02_mb_valu.log); the bits crossing the dword boundary
// land where the swap's mask discards them.  Inline asm, or the compiler splits
// the right shift back into v_alignbit + v_lshrrev.  (a0, a1) and (b0, b1) are
// adjacent registers in the first two stages of transpose8 (the 16-byte loads
// and the accumulator rows are register quads), so forming the pairs costs no
// moves.  Same form as bitslice.cpp's sw2.
__device__ __forceinline__ uint64_t vshl64(uint64_t x, int s) {
    uint64_t r;
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(s), "v"(x));
    return r;
}
__device__ __forceinline__ uint64_t vshr64(uint64_t x, int s) {
    uint64_t r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(s), "v"(x));
    return r;
}
__device__ __forceinline__ void bswap_blocks2(uint32_t& a0, uint32_t& b0, uint32_t& a1, uint32_t& b1, int s,
                                              uint32_t m) {
    const uint64_t bl = vshl64((static_cast<uint64_t>(b1) << 32) | b0, s);
    const uint64_t ar = vshr64((static_cast<uint64_t>(a1) << 32) | a0, s);
    const uint32_t t0 = bsel(m, a0, static_cast<uint32_t>(bl)), t1 = bsel(m, static_cast<uint32_t>(ar), b0);
    const uint32_t t2 = bsel(m, a1, static_cast<uint32_t>(bl >> 32)), t3 = bsel(m, static_cast<uint32_t>(ar >> 32), b1);
    a0 = t0;
    b0 = t1;
    a1 = t2;
    b1 = t3;
}

// 8 dwords (32 bytes) <-> 8 bit-planes; the transpose is its own inverse.
// ZFEC_TR64 (default): the first two stages on 64-bit shift pairs, 40 VOP3
// instructions instead of 48 (tools/ab_bsr.sh, profiles/r06_bsr_ab.json).
#ifndef ZFEC_TR64
#define ZFEC_TR64 1
#endif
__device__ __forceinline__ void transpose8(uint32_t (&v)[8]) {
#if ZFEC_TR64
    bswap_blocks2(v[0], v[4], v[1], v[5], 4, 0x0F0F0F0Fu);
    bswap_blocks2(v[2], v[6], v[3], v[7], 4, 0x0F0F0F0Fu);
    bswap_blocks2(v[0], v[2], v[1], v[3], 2, 0x33333333u);
    bswap_blocks2(v[4], v[6], v[5], v[7], 2, 0x33333333u);
    bswap_blocks(v[0], v[1], 1, 0x55555555u);
    bswap_blocks(v[2], v[3], 1, 0x55555555u);
    bswap_blocks(v[4], v[5], 1, 0x55555555u);
    bswap_blocks(v[6], v[7], 1, 0x55555555u);
    return;
#endif
    bswap_blocks(v[0], v[4], 4, 0x0F0F0F0Fu);
    bswap_blocks(v[1], v[5], 4, 0x0F0F0F0Fu);
    bswap_blocks(v[2], v[6], 4, 0x0F0F0F0Fu);
    bswap_blocks(v[3], v[7], 4, 0x0F0F0F0Fu);
    bswap_blocks(v[0], v[2], 2, 0x33333333u);
    bswap_blocks(v[1], v[3], 2, 0x33333333u);
    bswap_blocks(v[4], v[6], 2, 0x33333333u);
    bswap_blocks(v[5], v[7], 2, 0x33333333u);
    bswap_blocks(v[0], v[1], 1, 0x55555555u);
    bswap_blocks(v[2], v[3], 1, 0x55555555u);
    bswap_blocks(v[4], v[5], 1, 0x55555555u);
    bswap_blocks(v[6], v[7], 1, 0x55555555u);
}

// The 15 nonzero combinations of planes q[0..3] of both groups, to LDS
// entries base + 1..15 (entry e of lane l at e * 512 + l * 8).
__device__ __forceinline__ void write_combos(char* slot, uint32_t lane8, const uint32_t (&q0)[4],
                                             const uint32_t (&q1)[4], uint32_t base) {
    uint32_t c0[16], c1[16];
    c0[0] = 0u;
    c1[0] = 0u;
#pragma unroll
    for (int m = 1; m < 16; ++m) {
        const int top = 31 - __builtin_clz(m);
        c0[m] = c0[m ^ (1 << top)] ^ q0[top];
        c1[m] = c1[m ^ (1 << top)] ^ q1[top];
        *reinterpret_cast<u32x2*>(slot + (base + m) * 512u + lane8) = u32x2{c0[m], c1[m]};
    }
}

// Rows are interleaved over the waves: wave w owns rows w + 4*rr, rr < RT.
// launch_bsg lays the coefficients out for this walk: wave w's bytes of phase
// f are (js, rr) in order, js < 2, rr < RT, at byte (w * nphases + f) *
// bsg_phase_bytes(RT) (rows past r and inputs past k get coefficient 0,
// whose combinations are the zero entries).  A coefficient's eight offset
// dwords come from g_bsg by scalar loads, issued one step (row) ahead: a wait
// for a scalar load also drains the wave's LDS reads, so it must come where
// the wave has none outstanding.
template <int RT>
__host__ __device__ constexpr uint32_t bsg_phase_bytes() {
    return (kBsgPhase * RT + 3) / 4 * 4;
}

struct alignas(16) BsgTblJob {
    uint64_t sz, in_sstride, out_sstride;
    uint32_t nstripes, k, r, cps, gs_c, gs_s;
    uint32_t ngroups;  // row groups of 4 * RT rows: workgroup units are (group, stripe, unit) triples
    uint32_t pad_;
    const uint8_t* table;  // device memory: k input pointers, r output pointers, per group the walk-order coefficients
};

typedef const __attribute__((address_space(4))) uint64_t* CU64;
typedef const __attribute__((address_space(4))) uint32_t* KWords;

// Block pointers and coefficient words of a launch: from the kernel arguments
// (MatJob, one row group) or from the device-side table (scalar loads either way).
struct BsgKarg {
    KPtr<MatJob> kj;
    __device__ const uint8_t* in(uint32_t j) const { return kj->in[j]; }
    __device__ uint8_t* out(uint32_t i) const { return kj->out[i]; }
    __device__ KWords coef() const { return (KWords)kj->coef; }
};

struct BsgTbl {
    CU64 tp;
    uint32_t k, r;
    __device__ const uint8_t* in(uint32_t j) const { return reinterpret_cast<const uint8_t*>(tp[j]); }
    __device__ uint8_t* out(uint32_t i) const { return reinterpret_cast<uint8_t*>(tp[k + i]); }
    __device__ KWords coef() const { return (KWords)(tp + k + r); }
};

template <int RT, bool TBL, class J>
__global__ __launch_bounds__(256) void matapply_bsg(const J job) {
    constexpr int P = kBsgPhase;
    constexpr uint32_t PB = bsg_phase_bytes<RT>();
    constexpr int ND = PB / 4;           // coefficient dwords per wave and phase
    extern __shared__ char bsg_lds[];    // P slots of kBsgSlotBytes
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lane8 = lane * 8u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t k = job.k, r = job.r;
    const uint32_t nph = (k + P - 1) / P;
    // zero entries L[0] and H[0] of every slot (never overwritten)
    for (uint32_t i = threadIdx.x; i < P * 2 * 64; i += 256) {
        const uint32_t sl = i / 128, e = (i / 64) & 1u, l = i & 63u;
        *reinterpret_cast<u32x2*>(bsg_lds + sl * kBsgSlotBytes + e * 16u * 512u + l * 8u) = u32x2{0u, 0u};
    }
    const auto src = [&] {
        if constexpr (TBL)
            return BsgTbl{(CU64)job.table, k, r};
        else
            return BsgKarg{kernarg_job<MatJob>()};
    }();
    // The walk's "stripes" are (row group, stripe) pairs, group-major (one group
    // without the table): a launch with few units of work per row group still
    // fills the chip, each workgroup building the combinations of its unit's
    // inputs for its group's rows.
    const uint32_t ns = job.nstripes;
    uint32_t nvs = ns;
    if constexpr (TBL) nvs = ns * job.ngroups;
    const uint32_t rpg = 4u * static_cast<uint32_t>(RT);  // rows per group
    const uint64_t sz = job.sz;
    // byte offset of unit c in a block: the last unit of a block ends at sz
    // (overlapping its neighbour)
    auto unit_off = [&](uint32_t cu) {
        uint64_t o = static_cast<uint64_t>(cu) * kBsgChunk;
        return o > sz - kBsgChunk ? sz - kBsgChunk : o;
    };
    auto stripe_of = [&](uint32_t vs) { return TBL ? vs % ns : vs; };
    const bool builder = wave < static_cast<uint32_t>(P);
    // the input this wave transposes next, loaded one phase ahead (the next
    // unit's first phase while the current unit's last phase computes), so a
    // phase never starts waiting on HBM
    u32x4 xin[4];
    auto load_input = [&](uint32_t vs, uint32_t cu, uint32_t j) {
        const uint8_t* ip = src.in(j) + (stripe_of(vs) * job.in_sstride + unit_off(cu) + lane * 16u);
        xin[0] = load16(ip);
        xin[1] = load16(ip + 1024);
        xin[2] = load16(ip + 2048);
        xin[3] = load16(ip + 3072);
    };
    uint32_t s = blockIdx.x / job.cps, c = blockIdx.x - s * job.cps;  // s: (group, stripe) index
    if (builder && s < nvs && wave < k) load_input(s, c, wave);
    while (s < nvs) {
        uint32_t s2 = s + job.gs_s, c2 = c + job.gs_c;  // this workgroup's next unit
        if (c2 >= job.cps) {
            c2 -= job.cps;
            ++s2;
        }
        const uint32_t g = TBL ? s / ns : 0u;  // row group
        const uint32_t row0 = g * rpg, rows = r - row0 < rpg ? r - row0 : rpg;
        const KWords cw = src.coef() + (g * 4u + wave) * nph * ND;  // this wave's phases
        const uint64_t ob = stripe_of(s) * job.out_sstride + unit_off(c) + lane * 16u;
        uint32_t acc[RT][2][8];
#pragma unroll
        for (int rr = 0; rr < RT; ++rr)
#pragma unroll
            for (int gg = 0; gg < 2; ++gg)
#pragma unroll
                for (int b = 0; b < 8; ++b) acc[rr][gg][b] = 0u;
        for (uint32_t f = 0; f < nph; ++f) {
            const uint32_t j0 = f * P;
            // build: input j0 + wave into slot wave
            const uint32_t jb = j0 + wave;
            if (builder && jb < k) {
                char* slot = bsg_lds + wave * kBsgSlotBytes;
                uint32_t g0[8] = {xin[0].x, xin[0].y, xin[0].z, xin[0].w, xin[1].x, xin[1].y, xin[1].z, xin[1].w};
                uint32_t g1[8] = {xin[2].x, xin[2].y, xin[2].z, xin[2].w, xin[3].x, xin[3].y, xin[3].z, xin[3].w};
                transpose8(g0);
                transpose8(g1);
                const uint32_t l0[4] = {g0[0], g0[1], g0[2], g0[3]}, l1[4] = {g1[0], g1[1], g1[2], g1[3]};
                const uint32_t h0[4] = {g0[4], g0[5], g0[6], g0[7]}, h1[4] = {g1[4], g1[5], g1[6], g1[7]};
                write_combos(slot, lane8, l0, l1, 0u);
                write_combos(slot, lane8, h0, h1, 16u);
            }
            if (builder) {  // prefetch: this unit's next phase, else the next unit's first
                if (f + 1 < nph) {
                    if (jb + P < k) load_input(s, c, jb + P);
                } else if (s2 < nvs && wave < k) {
                    load_input(s2, c2, wave);
                }
            }
            // this phase's coefficients (scalar loads, waited for before the barrier)
            uint32_t cwd[ND];
#pragma unroll
            for (int d = 0; d < ND; ++d) cwd[d] = cw[f * ND + d];
            auto coef_at = [&](int t) { return (cwd[t >> 2] >> ((t & 3) * 8)) & 0xFFu; };
            __syncthreads();
            const uint32_t jn = k - j0 < static_cast<uint32_t>(P) ? k - j0 : static_cast<uint32_t>(P);
            uint32_t o[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) o[b] = g_bsg.off[coef_at(0) * 16u + b];
#pragma unroll
            for (int t = 0; t < P * RT; ++t) {
                const int js = t / RT, rr = t % RT;
                if (static_cast<uint32_t>(js) >= jn) break;  // wave-uniform
                uint32_t on[16];
                if (t + 1 < P * RT) {  // the next step's offsets, in flight during this step
#pragma unroll
                    for (int b = 0; b < 16; ++b) on[b] = g_bsg.off[coef_at(t + 1) * 16u + b];
                }
                const char* base = bsg_lds + js * kBsgSlotBytes + lane8;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const u32x2 vl = *reinterpret_cast<const u32x2*>(base + o[b]);
                    const u32x2 vh = *reinterpret_cast<const u32x2*>(base + o[8 + b]);
                    acc[rr][0][b] = xor3(acc[rr][0][b], vl.x, vh.x);
                    acc[rr][1][b] = xor3(acc[rr][1][b], vl.y, vh.y);
                }
                if (t + 1 < P * RT) {
#pragma unroll
                    for (int b = 0; b < 16; ++b) o[b] = on[b];
                }
            }
            __syncthreads();  // every wave has read the slots before the next phase overwrites them
        }
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            const uint32_t i = wave + 4u * rr;
            if (i >= rows) break;  // wave-uniform
            transpose8(acc[rr][0]);
            transpose8(acc[rr][1]);
            uint8_t* op = src.out(row0 + i) + ob;
            store16_out<true>(op, u32x4{acc[rr][0][0], acc[rr][0][1], acc[rr][0][2], acc[rr][0][3]});
            store16_out<true>(op + 1024, u32x4{acc[rr][0][4], acc[rr][0][5], acc[rr][0][6], acc[rr][0][7]});
            store16_out<true>(op + 2048, u32x4{acc[rr][1][0], acc[rr][1][1], acc[rr][1][2], acc[rr][1][3]});
            store16_out<true>(op + 3072, u32x4{acc[rr][1][4], acc[rr][1][5], acc[rr][1][6], acc[rr][1][7]});
        }
        s = s2;
        c = c2;
    }
}

// ---------------------------------------------------------------------------
// matapply_bsr<RT>: bit-sliced with the coefficients as run-time data, at the
// instruction count of a specialised (JIT) kernel.  Multiplying the 32 bytes
// of a lane by c and adding them to an accumulator row is, on bit-planes, eight
// XOR3s whose operands depend on c only; gf_routines.inc holds those eight
// instructions for every c as a routine (zfec_gf_routines + 72 c) working on
// fixed registers: the input's combinations of planes (built once per input
// per wave) and accumulator row 0, offset to row rr by VGPR index mode.  A
// coefficient costs a call (a few scalar instructions and two jumps, no LDS
// read) instead of matapply_bsg's sixteen LDS reads or a compile per matrix.
//
// Unit = 2 KiB of every block of a stripe (32 bytes per lane, like the JIT
// kernels); rows in tiles of <= RT <= 10 (the accumulators of a tile live in
// v38..v37+8RT, gf_routines.inc).  Two forms:
//   matapply_bsr_solo<RT> (one tile, r <= 10): one wave per unit, no LDS; the
//       wave loads and transposes its inputs two ahead;
//   matapply_bsr<RT> ("lds", r > 10): one workgroup per unit, a wave per
//       tile; the unit's inputs go through LDS in phases, loaded straight into
//       LDS (LDS-DMA) and transposed in place into bit-planes, two phases
//       resident so the next phase loads while the waves walk the current one
//       (bsr_db_phase).  All k inputs in LDS at once (k * 2 KiB) capped the
//       workgroups per CU and measured 0.51 ms against 0.37-0.38 with phases
//       of 8 on cfg4's first-seen decodes (profiles/r04_bsr_ab.json).
// Coefficients: absolute routine addresses (BsrJob / BsrTblJob below).
// ---------------------------------------------------------------------------
// ZFEC_GF_ROUTINES_INC: another generated form of the routines (the A/B,
// tools/ab_bsr.sh: `tools/gen_gf_routines.py --form legacy --out ...`)
#ifdef ZFEC_GF_ROUTINES_INC
#include ZFEC_GF_ROUTINES_INC
#else
#include "gf_routines.inc"
#endif

constexpr uint32_t kBsrChunk = 2048;  // bytes of each block per unit
template <bool B>
struct BoolC {  // a compile-time flag passed to generic lambdas
    static constexpr bool value = B;
};
// ZFEC_BSR_EARLY_ADDR (default): the LDS-phase form loads the next input's
// routine addresses before the current input's calls, not after them
// (matapply_bsr; tools/ab_bsr.sh, profiles/r06_bsr_ab.json).
#ifndef ZFEC_BSR_EARLY_ADDR
#define ZFEC_BSR_EARLY_ADDR 1
#endif
// ZFEC_BSR_TBL_WRITER (A/B knob, tools/ab_build.sh; 0): 1 writes a new
// matrix's device-side address table with a kernel from the launch's
// arguments instead of copying it from pinned host memory.  Even: K=20/M=60
// first launches of new matrices 0.829-0.848 against 0.818-0.850 ms between
// events (profiles/r06_bsr_tblwrite_ab.json); the host's enqueue, not the copy,
// separates them from the compiled kernel's.
#ifndef ZFEC_BSR_TBL_WRITER
#define ZFEC_BSR_TBL_WRITER 0
#endif
// ZFEC_BSR_CMB_DB (A/B knob, tools/ab_build.sh; off): the combination-sharing
// form double-buffers its phases (one barrier per phase, half the waves build
// the next phase during the current one's calls).  It lost: 128/256 0.109 ->
// 0.112 ms, 160/256 0.112 -> 0.119, 64/112 0.051 -> 0.054
// (profiles/r06_bsr_cmb_db_ab.json).
#ifndef ZFEC_BSR_CMB_DB
#define ZFEC_BSR_CMB_DB 0
#endif
typedef __attribute__((address_space(1))) void GlobalVoid;
typedef __attribute__((address_space(3))) void LdsVoid;
// Inputs per phase of the combination-sharing form (7.5 KiB of combinations +
// 2 KiB of raw staging each): one per wave, so the 16 / nw workgroups a CU
// holds at 4 waves per SIMD take 152 KiB.
__host__ __device__ constexpr uint32_t bsr_cmb_phase(uint32_t nw) { return nw; }
// Inputs per phase of the plane-sharing form, whose LDS holds two phases: the
// 16 / nw workgroups a CU holds at 4 waves per SIMD keep within its 160 KiB.
__host__ __device__ constexpr uint32_t bsr_db_phase(uint32_t nw) { return nw <= 2 ? 2u : nw <= 4 ? 4u : 8u; }
constexpr int kBsrMaxOut = 4 * kBsrMaxRows;  // rows of the kernel-argument form (4 tiles)
constexpr int kBsrArgAddrs = 432;     // routine addresses the kernel-argument form holds

// Routine addresses: every coefficient reaches the kernel as the absolute
// address of its routine (zfec_gf_routines + 72 c on the launch's device,
// bsr_routine_base), in the kernel's walk order [group][wave][input][row],
// RT per (wave, input) -- rows past a wave's tile hold routine 0's address,
// which only returns.  Kernel-argument form (k <= 32, r <= 40, at most
// kBsrArgAddrs addresses): block pointers and addresses in the arguments.
struct alignas(16) BsrJob {
    uint64_t sz, in_sstride, out_sstride;
    uint32_t nstripes, k, r, cps, gs_c, gs_s;
    uint32_t nt;  // one-wave form: row tiles per unit
    uint32_t pad_;
    const uint8_t* in[kMaxIn];
    uint8_t* out[kBsrMaxOut];
    uint64_t addr[kBsrArgAddrs];
};
static_assert(sizeof(BsrJob) <= 4096, "kernel arguments are limited to 4 KiB");

// Table form (k > 32, or more addresses than the arguments hold): the block
// pointers in the arguments, the addresses in a device-side table the host
// uploads once per matrix and layout and keeps (bsr_addr_table), read with
// scalar loads.
constexpr int kBsrTblPtrs = 320;  // k + r block pointers of a table-form launch
struct alignas(16) BsrTblJob {
    uint64_t sz, in_sstride, out_sstride;
    uint32_t nstripes, k, r, cps, gs_c, gs_s;
    uint32_t ngroups;  // row groups: workgroup units are (group, stripe, unit) triples
    uint32_t pad_;
    const uint64_t* addr;             // device: [group][wave][input][RT] routine addresses
    const uint8_t* ptr[kBsrTblPtrs];  // k input block pointers, then r output block pointers
};
static_assert(sizeof(BsrTblJob) <= 4096, "kernel arguments are limited to 4 KiB");

// 32-bit argument form (LDS-phase kernel, one row group): block pointers and
// the routine addresses' low halves in the kernel arguments, the high half
// (the same for the whole routine table) once.  It holds twice the addresses
// of BsrJob -- K=20/M=60's 40-row encode needs 800 -- so a first launch of a
// new matrix copies no table to the device: the table form's upload (a
// hipMemcpyAsync the kernel waits for) cost a first launch ~65 us between its
// events (profiles/r06_bench_vs_trace.txt).
constexpr int kBsr32Ptrs = 72;  // k + r block pointers
struct alignas(16) BsrJob32 {
    uint64_t sz, in_sstride, out_sstride;
    uint32_t nstripes, k, r, cps, gs_c, gs_s;
    uint32_t ngroups;  // 1
    uint32_t addr_hi;  // high 32 bits of every routine address
    const uint8_t* ptr[kBsr32Ptrs];
    uint32_t addr[(4096 - 56 - 8 * kBsr32Ptrs) / 4];  // [wave][input][RT] low halves (56: the header)
};
[[maybe_unused]] constexpr int kBsr32Addrs = (4096 - 56 - 8 * kBsr32Ptrs) / 4;
static_assert(sizeof(BsrJob32) <= 4096, "kernel arguments are limited to 4 KiB");
typedef const __attribute__((address_space(4))) uint32_t* CU32;

// Where a wave's routine addresses come from: 64-bit values (kernel arguments
// or the device-side table) or the 32-bit argument form's low halves.
struct Addr64 {
    CU64 p;
    template <int RT>
    __device__ __forceinline__ void load(uint64_t (&ad)[RT], uint32_t j) const {
        const CU64 q = p + static_cast<uint64_t>(j) * RT;
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) ad[rr] = q[rr];
    }
};
struct Addr32 {
    CU32 p;
    uint32_t hi;
    template <int RT>
    __device__ __forceinline__ void load(uint64_t (&ad)[RT], uint32_t j) const {
        const CU32 q = p + static_cast<uint64_t>(j) * RT;
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) ad[rr] = (static_cast<uint64_t>(hi) << 32) | q[rr];
    }
};

// Writes a device-side routine-address table from its 32-bit low halves in the
// kernel arguments (one workgroup; the high half is one value for the whole
// table): a launch's upload of a new matrix's table without a host-to-device
// copy (bsr_addr_table).
constexpr int kBsrWriteMax = (4096 - 16) / 4;  // addresses per writer launch
struct alignas(16) BsrWriteJob {
    uint64_t* dst;
    uint32_t n, hi;
    uint32_t lo[kBsrWriteMax];
};
static_assert(sizeof(BsrWriteJob) <= 4096, "kernel arguments are limited to 4 KiB");
__global__ __launch_bounds__(256) void bsr_table_write(const BsrWriteJob job) {
    const KPtr<BsrWriteJob> kj = kernarg_job<BsrWriteJob>();
    for (uint32_t i = threadIdx.x; i < job.n; i += 256)
        job.dst[i] = (static_cast<uint64_t>(job.hi) << 32) | kj->lo[i];
}

// Reads input j's RT routine addresses (scalar loads).
// (The row offset is added to a 64-bit pointer, so the loads share one
// address and merge into s_load_dwordx16 / x4 with immediate offsets.)
template <int RT>
__device__ __forceinline__ void bsr_addrs(uint64_t (&ad)[RT], CU64 ca, uint32_t j) {
    const CU64 q = ca + static_cast<uint64_t>(j) * RT;
#pragma unroll
    for (int rr = 0; rr < RT; ++rr) ad[rr] = q[rr];
}

// The address of zfec_gf_routines on this device, computed the way a call
// site would (s_getpc + the rel32 relocation) and stored by lane 0 with a
// vector store; the host reads it once per device (bsr_routine_base).
__global__ void bsr_table_probe(uint64_t* out) {
    uint32_t lo, hi;
    asm volatile(
        "s_getpc_b64 s[26:27]\n\t"
        "s_add_u32 s26, s26, zfec_gf_routines@rel32@lo+4\n\t"
        "s_addc_u32 s27, s27, zfec_gf_routines@rel32@hi+12\n\t"
        "s_mov_b32 %0, s26\n\t"
        "s_mov_b32 %1, s27"
        : "=s"(lo), "=s"(hi)
        :
        : "s26", "s27", "scc");
    if (threadIdx.x == 0) out[0] = (static_cast<uint64_t>(hi) << 32) | lo;
}

// The 30 combinations of an input's bit-planes in bsr_input_c's register
// order (gf_routines.inc): planes p0..p7, then L[m] (planes 0-3) and H[m]
// (planes 4-7) for the eleven multi-plane m in increasing order.
__device__ __forceinline__ void bsr_combos(const uint32_t (&p)[8], uint32_t (&q)[30]) {
    constexpr int kMulti[11] = {3, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15};
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = p[i];
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        uint32_t c[16] = {};
#pragma unroll
        for (int i = 0; i < 4; ++i) c[1 << i] = p[4 * side + i];
#pragma unroll
        for (int x = 0; x < 11; ++x) {
            const int m = kMulti[x];
            const int top = m >= 8 ? 8 : m >= 4 ? 4 : 2;
            c[m] = c[m ^ top] ^ c[top];
            q[8 + 11 * side + x] = c[m];
        }
    }
}

// Bytes of LDS per input of a phase: the 8 planes, or (CMB) all 30 combinations.
template <bool CMB>
__host__ __device__ constexpr uint32_t bsr_in_bytes() {
    return CMB ? 30u * 256u : 8u * 256u;
}

template <int RT, bool TBL, bool CMB, class J>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void matapply_bsr(const J job) {
    // [input][half][lane] planes, or (CMB) [input][7 x (4 dwords)][lane] + [2 dwords][lane] combinations
    extern __shared__ u32x4 bsr_planes[];
    constexpr uint32_t kIn = bsr_in_bytes<CMB>() / 16;  // u32x4 per input
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = blockDim.x >> 6;
    const uint32_t k = job.k, r = job.r;
    // block pointers and routine addresses: kernel arguments (BsrJob) or the
    // device-side table (BsrTblJob); the walk's "stripes" are (row group,
    // stripe) pairs, group-major
    const uint32_t ns = job.nstripes;
    uint32_t ng = 1;
    KPtr<J> kj = kernarg_job<J>();
    constexpr bool A32 = std::is_same<J, BsrJob32>::value;  // 32-bit argument form
    constexpr bool PTR = TBL || A32;                         // block pointers in ptr[]
    if constexpr (TBL) ng = job.ngroups;
    auto in_ptr = [&](uint32_t j) -> const uint8_t* {
        if constexpr (PTR)
            return kj->ptr[j];
        else
            return kj->in[j];
    };
    auto out_ptr = [&](uint32_t i) -> uint8_t* {
        if constexpr (PTR)
            return const_cast<uint8_t*>(kj->ptr[k + i]);
        else
            return kj->out[i];
    };
    const uint64_t sz = job.sz;
    uint32_t s = blockIdx.x / job.cps, c = blockIdx.x - s * job.cps;
    while (s < ns * ng) {
        const uint32_t g = TBL && ng > 1 ? s / ns : 0u, stripe = s - g * ns;
        const uint32_t gr0 = g * r / ng, grn = (g + 1) * r / ng - gr0;
        const uint32_t r0 = gr0 + wave * grn / nw, rows = gr0 + (wave + 1) * grn / nw - r0;
        auto ca = [&] {
            if constexpr (A32)
                return Addr32{(CU32)kj->addr + wave * k * RT, job.addr_hi};
            else if constexpr (TBL)
                return Addr64{(CU64)job.addr + (g * nw + wave) * k * RT};
            else
                return Addr64{(CU64)kj->addr + wave * k * RT};
        }();
        uint64_t off = static_cast<uint64_t>(c) * kBsrChunk;
        if (off > sz - kBsrChunk) off = sz - kBsrChunk;  // the last unit ends at sz (overlapping its neighbour)
        const uint64_t ib = stripe * job.in_sstride + off + lane * 16u;
        const uint64_t ob = stripe * job.out_sstride + off + lane * 16u;
        uint32_t acc[RT][8];  // no zeroing: the wave's first input calls "set" routines (kBsrSetBase)
        // One input's calls: its planes (or, CMB, its 30 combinations) read from
        // LDS at b, its routine addresses in `cur`; the wave's first input
        // (global index 0) calls the set twins (bsr_input_first: every row
        // written).  `wait` runs between the LDS reads and the calls.
        constexpr int kVals = CMB ? 30 : 8;
        auto load = [&](const u32x4* b, uint32_t (&q)[kVals]) {
            if constexpr (CMB) {
#pragma unroll
                for (int g = 0; g < 7; ++g) {
                    const u32x4 t = b[g * 64 + lane];
                    q[4 * g] = t.x;
                    q[4 * g + 1] = t.y;
                    q[4 * g + 2] = t.z;
                    q[4 * g + 3] = t.w;
                }
                const u32x2 t2 = reinterpret_cast<const u32x2*>(b + 448)[lane];
                q[28] = t2.x;
                q[29] = t2.y;
            } else {
                const u32x4 pa = b[lane], pb = b[64u + lane];
                q[0] = pa.x, q[1] = pa.y, q[2] = pa.z, q[3] = pa.w;
                q[4] = pb.x, q[5] = pb.y, q[6] = pb.z, q[7] = pb.w;
            }
        };
        auto input = [&](auto first, const uint32_t (&q)[kVals], const uint64_t (&cur)[RT]) {
            if constexpr (CMB) {
                if constexpr (decltype(first)::value)
                    bsr_input_c_first<RT>(acc, q, cur);
                else
                    bsr_input_c<RT>(acc, q, cur);
            } else {
                if constexpr (decltype(first)::value)
                    bsr_input_first<RT>(acc, q, cur);
                else
                    bsr_input<RT>(acc, q, cur);
            }
        };
        // calls(first, ph, kn, o): the calls of one phase's kn inputs (ph, ph +
        // 1, ...), planes or combinations at LDS offset o (u32x4).  The first
        // phase is its own instance (first = BoolC<true>): its input 0 runs the
        // set twins, peeled at compile time -- a run-time choice between the two
        // statements made the compiler copy and spill the pinned accumulators.
#if ZFEC_BSR_EARLY_ADDR
        // Routine addresses, two sets by the parity of the input's global
        // index (phases hold an even number of inputs: bsr_db_phase,
        // bsr_cmb_phase).  Input g + 1's set is loaded (scalar loads) right
        // after input g's LDS data has been waited for and before g's calls,
        // so it arrives during them: the wait for g + 1's LDS data, which
        // drains scalar loads too (lgkmcnt), finds it landed.  Round 5 loaded
        // input g + 2's set after g's calls, and that wait stalled on it.
        uint64_t ad0[RT], ad1[RT];
        ca.template load<RT>(ad0, 0);
        auto step = [&](auto first, uint32_t gi, const u32x4* b, const uint64_t (&cur)[RT], uint64_t (&nxt)[RT]) {
            uint32_t q[kVals];
            load(b, q);
            // a use of every value read: the LDS wait goes here, before the scalar loads
            if constexpr (CMB)
                asm volatile("" ::"v"(q[3]), "v"(q[7]), "v"(q[11]), "v"(q[15]), "v"(q[19]), "v"(q[23]), "v"(q[27]),
                             "v"(q[29]));
            else
                asm volatile("" ::"v"(q[3]), "v"(q[7]));
            __builtin_amdgcn_sched_barrier(0);
            ca.template load<RT>(nxt, gi + 1 < k ? gi + 1 : k - 1);  // unconditional (clamped)
            __builtin_amdgcn_sched_barrier(0);
            input(first, q, cur);
        };
        auto calls = [&](auto first, uint32_t ph, uint32_t kn, uint32_t o) {
            uint32_t j = 0;
            if constexpr (decltype(first)::value) {  // ph == 0
                step(BoolC<true>{}, 0, bsr_planes + o, ad0, ad1);
                for (j = 1; j + 1 < kn; j += 2) {
                    step(BoolC<false>{}, j, bsr_planes + o + j * kIn, ad1, ad0);
                    step(BoolC<false>{}, j + 1, bsr_planes + o + (j + 1) * kIn, ad0, ad1);
                }
                if (j < kn) step(BoolC<false>{}, j, bsr_planes + o + j * kIn, ad1, ad0);  // k < the phase
                return;
            }
            for (; j + 1 < kn; j += 2) {
                step(first, ph + j, bsr_planes + o + j * kIn, ad0, ad1);
                step(first, ph + j + 1, bsr_planes + o + (j + 1) * kIn, ad1, ad0);
            }
            if (j < kn) step(first, ph + j, bsr_planes + o + j * kIn, ad0, ad1);  // the last phase
        };
#else
        // In pairs with fixed address registers (A: even, B: odd): after input
        // j's calls its set is reloaded (scalar loads, unconditional: clamped to
        // the phase's last input) with input j + 2's addresses (round 5's schedule)
        auto calls = [&](auto first, uint32_t ph, uint32_t kn, uint32_t o) {
            uint64_t ada[RT], adb[RT];
            ca.template load<RT>(ada, ph);
            ca.template load<RT>(adb, ph + (kn > 1 ? 1 : 0));
            auto step = [&](auto fst, uint32_t j, uint64_t (&ad)[RT]) {
                uint32_t q[kVals];
                load(bsr_planes + o + j * kIn, q);
                input(fst, q, ad);
                ca.template load<RT>(ad, ph + (j + 2 < kn ? j + 2 : kn - 1));
            };
            uint32_t j = 0;
            if constexpr (decltype(first)::value) {
                step(BoolC<true>{}, 0, ada);
                if (kn > 1) step(BoolC<false>{}, 1, adb);
                j = 2;
            }
            for (; j + 1 < kn; j += 2) {
                step(BoolC<false>{}, j, ada);
                step(BoolC<false>{}, j + 1, adb);
            }
            if (j < kn) step(BoolC<false>{}, j, ada);
        };
#endif
        if constexpr (!CMB) {
            // Planes: double-buffered phases of kq inputs.  A phase's inputs go
            // straight into LDS (LDS-DMA, global_load_lds: no registers in
            // flight) while the waves run the previous phase's calls, and are
            // then transposed in place -- lane l's 16 + 16 bytes land in the
            // slots its planes go to (b[l], b[64 + l]).  One barrier per phase.
            const uint32_t kq = bsr_db_phase(nw);
            auto dma = [&](uint32_t ph, uint32_t kn, uint32_t o) {
                for (uint32_t j = wave; j < kn; j += nw) {
                    const uint8_t* ip = in_ptr(ph + j) + ib;
                    u32x4* b = bsr_planes + o + j * kIn;
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip), (LdsVoid*)(b), 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip + 1024), (LdsVoid*)(b + 64), 16, 0, 0);
                }
            };
            auto xpose = [&](uint32_t kn, uint32_t o) {
                // hipcc does not order these LDS reads after the LDS-DMA writes
                // (no vmcnt wait of its own here): wait for them explicitly
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                for (uint32_t j = wave; j < kn; j += nw) {
                    u32x4* b = bsr_planes + o + j * kIn;
                    const u32x4 x0 = b[lane], x1 = b[64u + lane];
                    uint32_t v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                    transpose8(v);
                    b[lane] = u32x4{v[0], v[1], v[2], v[3]};
                    b[64u + lane] = u32x4{v[4], v[5], v[6], v[7]};
                }
            };
            uint32_t kn = k < kq ? k : kq, o = 0;
            dma(0, kn, 0);
            xpose(kn, 0);
            __syncthreads();
            auto phase = [&](auto first, uint32_t ph) {
                const uint32_t nx = ph + kq, knx = nx < k ? (k - nx < kq ? k - nx : kq) : 0u;
                const uint32_t ox = o ^ (kq * kIn);  // the other half
                if (knx) dma(nx, knx, ox);
                calls(first, ph, kn, o);
                if (knx) xpose(knx, ox);
                __syncthreads();  // phase ph's planes read, phase nx's written
                kn = knx;
                o = ox;
            };
            phase(BoolC<true>{}, 0);
            for (uint32_t ph = kq; ph < k; ph += kq) phase(BoolC<false>{}, ph);
        } else {
#if ZFEC_BSR_CMB_DB
            // Combinations, double-buffered: phases of kp = nw / 2 inputs, two
            // phases' combinations resident.  The waves are two halves of kp
            // (one wave of each per SIMD); wave i of half h owns input i of the
            // phases of parity h.  In phase p, half (p + 1) & 1 builds phase p +
            // 1 (its inputs arrived by LDS-DMA during phase p - 1: transpose, 30
            // combinations, into the other buffer) and half p & 1 starts the
            // LDS-DMA of phase p + 2 into the raw slots phase p has vacated;
            // then every wave runs phase p's calls; one barrier ends the phase.
            // (Single-buffered: phases of nw inputs, a barrier, every wave
            // building one input, a second barrier: the build stalled the calls.)
            const uint32_t kp = nw / 2, half = wave >= kp ? 1u : 0u, wi = wave - half * kp;
            const uint32_t ocmb = 0, oraw = 2 * kp * kIn;  // [2][kp] combinations, then [2][kp] raw inputs
            auto nin = [&](uint32_t ph) { return ph < k ? (k - ph < kp ? k - ph : kp) : 0u; };
            auto dma = [&](uint32_t p) {  // my input of phase p into raw slot p & 1
                if (wi < nin(p * kp)) {
                    const uint8_t* ip = in_ptr(p * kp + wi) + ib;
                    u32x4* b = bsr_planes + oraw + ((p & 1) * kp + wi) * 128u;
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip), (LdsVoid*)(b), 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip + 1024), (LdsVoid*)(b + 64), 16, 0, 0);
                }
            };
            auto build = [&](uint32_t p) {  // my input of phase p: raw slot -> combinations buffer p & 1
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (as in the planes form)
                if (wi < nin(p * kp)) {
                    const u32x4* r = bsr_planes + oraw + ((p & 1) * kp + wi) * 128u;
                    const u32x4 x0 = r[lane], x1 = r[64u + lane];
                    uint32_t v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                    transpose8(v);
                    uint32_t q30[30];
                    bsr_combos(v, q30);
                    u32x4* b = bsr_planes + ocmb + ((p & 1) * kp + wi) * kIn;
#pragma unroll
                    for (int g = 0; g < 7; ++g)
                        b[g * 64 + lane] = u32x4{q30[4 * g], q30[4 * g + 1], q30[4 * g + 2], q30[4 * g + 3]};
                    reinterpret_cast<u32x2*>(b + 448)[lane] = u32x2{q30[28], q30[29]};
                }
            };
            const uint32_t np = (k + kp - 1) / kp;  // phases
            dma(half);                              // phase 0 (half 0), phase 1 (half 1)
            if (half == 0) build(0);
            __syncthreads();
            auto phase = [&](auto first, uint32_t p) {
                if (half == ((p + 1) & 1)) {
                    if (p + 1 < np) build(p + 1);
                } else if (p + 2 < np) {
                    dma(p + 2);
                }
                calls(first, p * kp, nin(p * kp), ocmb + (p & 1) * kp * kIn);
                __syncthreads();  // phase p read, phase p + 1 written
            };
            phase(BoolC<true>{}, 0);
            for (uint32_t p = 1; p < np; ++p) phase(BoolC<false>{}, p);
#else
            // Combinations: phases of kp = nw inputs, one per wave.  A phase's
            // inputs go into a raw staging area (LDS-DMA) while the waves walk
            // the previous phase; after the barrier that ends it, each wave
            // transposes its own input, builds its 30 combinations and writes
            // them for every wave.
            const uint32_t kp = bsr_cmb_phase(nw), oraw = (k < kp ? k : kp) * kIn;  // staging after the combinations
            auto dma = [&](uint32_t ph, uint32_t kn) {
                for (uint32_t j = wave; j < kn; j += nw) {
                    const uint8_t* ip = in_ptr(ph + j) + ib;
                    u32x4* b = bsr_planes + oraw + j * 128u;
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip), (LdsVoid*)(b), 16, 0, 0);
                    __builtin_amdgcn_global_load_lds((const GlobalVoid*)(ip + 1024), (LdsVoid*)(b + 64), 16, 0, 0);
                }
            };
            auto build = [&](uint32_t kn) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (as in the planes form)
                for (uint32_t j = wave; j < kn; j += nw) {
                    const u32x4* r = bsr_planes + oraw + j * 128u;
                    const u32x4 x0 = r[lane], x1 = r[64u + lane];
                    uint32_t v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                    transpose8(v);
                    uint32_t q30[30];
                    bsr_combos(v, q30);
                    u32x4* b = bsr_planes + j * kIn;
#pragma unroll
                    for (int g = 0; g < 7; ++g)
                        b[g * 64 + lane] = u32x4{q30[4 * g], q30[4 * g + 1], q30[4 * g + 2], q30[4 * g + 3]};
                    reinterpret_cast<u32x2*>(b + 448)[lane] = u32x2{q30[28], q30[29]};
                }
            };
            uint32_t kn = k < kp ? k : kp;
            dma(0, kn);
            build(kn);
            __syncthreads();
            auto phase = [&](auto first, uint32_t ph) {
                const uint32_t nx = ph + kp, knx = nx < k ? (k - nx < kp ? k - nx : kp) : 0u;
                if (knx) dma(nx, knx);  // each wave's staging slot: read by its own build() before the barrier
                calls(first, ph, kn, 0);
                __syncthreads();  // every wave has read the combinations before they are overwritten
                if (knx) {
                    build(knx);
                    __syncthreads();
                }
                kn = knx;
            };
            phase(BoolC<true>{}, 0);
            for (uint32_t ph = kp; ph < k; ph += kp) phase(BoolC<false>{}, ph);
        #endif
        }
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            if (static_cast<uint32_t>(rr) < rows) {  // wave-uniform
                transpose8(acc[rr]);
                uint8_t* op = out_ptr(r0 + rr) + ob;
                store16_out<true>(op, u32x4{acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]});
                store16_out<true>(op + 1024, u32x4{acc[rr][4], acc[rr][5], acc[rr][6], acc[rr][7]});
            }
        }
        c += job.gs_c;
        s += job.gs_s;
        if (c >= job.cps) {
            c -= job.cps;
            ++s;
        }
    }
}

// One wave's walk over n inputs of a unit (the one-wave and ks forms): input
// j's two 16-byte pieces at ptr(j) + ib, its routine addresses at ca[j * RT].
// Unrolled by two with fixed register roles (A: even inputs, B: odd), so a
// load lands in the registers its input's transpose has just consumed (no
// copies) and is waited for two inputs later; the A and B routine-address
// sets are scalar-loaded the same way, and block pointers one step ahead of
// their use (a scalar wait drains every outstanding scalar load, so none is
// issued right before it is needed).
template <int RT, class P>
__device__ __forceinline__ void bsr_walk(uint32_t (&acc)[RT][8], uint32_t n, uint64_t ib, CU64 ca, P ptr) {
    u32x4 a0, a1, b0, b1;
    const uint8_t* pa = ptr(0);
    const uint8_t* pb = ptr(n > 1 ? 1 : 0);
    a0 = load16(pa + ib);
    a1 = load16(pa + ib + 1024);
    b0 = load16(pb + ib);
    b1 = load16(pb + ib + 1024);
    pa = ptr(n > 2 ? 2 : n - 1);
    pb = ptr(n > 3 ? 3 : n - 1);
    uint64_t ada[RT], adb[RT];
    bsr_addrs<RT>(ada, ca, 0);
    bsr_addrs<RT>(adb, ca, n > 1 ? 1 : 0);
    // the loads and scalar loads are unconditional (past the last input they
    // re-read input n - 1, from L2): a conditional load would make the compiler
    // merge its registers with a copy that waits for every load in flight
    auto step = [&](auto first, u32x4& x0, u32x4& x1, const uint8_t*& pn, uint64_t (&ad)[RT], uint32_t j) {
        uint32_t p[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        transpose8(p);
        if constexpr (decltype(first)::value)  // the walk's first input: the set twins (fill_bsr_addrs)
            bsr_input_first<RT>(acc, p, ad);
        else
            bsr_input<RT>(acc, p, ad);
        // input j + 2 into x0 / x1 / ad, which this input has consumed (after
        // the calls, so the compiler cannot keep the planes in them and copy)
        bsr_addrs<RT>(ad, ca, j + 2 < n ? j + 2 : n - 1);
        x0 = load16(pn + ib);
        x1 = load16(pn + ib + 1024);
        pn = ptr(j + 4 < n ? j + 4 : n - 1);
    };
    // whole pairs, then an odd last input: with no conditional step inside the
    // loop, input j's wait leaves input j + 1's loads in flight.  Input 0 is
    // peeled (the set twins, a statement of its own: a run-time choice between
    // the two made the compiler copy the pinned accumulators).
    step(BoolC<true>{}, a0, a1, pa, ada, 0);
    uint32_t j = 1;
    for (; j + 1 < n; j += 2) {
        step(BoolC<false>{}, b0, b1, pb, adb, j);
        step(BoolC<false>{}, a0, a1, pa, ada, j + 1);
    }
    if (j < n) step(BoolC<false>{}, b0, b1, pb, adb, j);
}

// One wave per (unit, row tile), no LDS: the wave loads and transposes every
// input of its unit itself (tiles of one unit are adjacent workgroups, so the
// second tile's loads hit L2), two inputs in flight ahead.
template <int RT>
__global__ __launch_bounds__(64) void matapply_bsr_solo(const BsrJob job) {
    const uint32_t lane = threadIdx.x;
    const uint32_t k = job.k, r = job.r, nt = job.nt;
    const KPtr<BsrJob> kj = kernarg_job<BsrJob>();
    const uint64_t sz = job.sz;
    const uint64_t total = uint64_t(job.nstripes) * job.cps * nt;
    for (uint64_t v = blockIdx.x; v < total; v += gridDim.x) {
        const uint32_t t = static_cast<uint32_t>(v % nt);
        const uint64_t u = v / nt;
        const uint32_t s = static_cast<uint32_t>(u / job.cps), c = static_cast<uint32_t>(u % job.cps);
        const uint32_t r0 = t * r / nt, rows = (t + 1) * r / nt - r0;
        const CU64 ca = (CU64)kj->addr + t * k * RT;
        uint64_t off = static_cast<uint64_t>(c) * kBsrChunk;
        if (off > sz - kBsrChunk) off = sz - kBsrChunk;
        const uint64_t ib = s * job.in_sstride + off + lane * 16u;
        const uint64_t ob = s * job.out_sstride + off + lane * 16u;
        uint32_t acc[RT][8];  // no zeroing: the wave's first input calls "set" routines (kBsrSetBase)
        bsr_walk<RT>(acc, k, ib, ca, [&](uint32_t j) { return kj->in[j]; });
#pragma unroll
        for (int rr = 0; rr < RT; ++rr) {
            if (static_cast<uint32_t>(rr) < rows) {
                transpose8(acc[rr]);
                uint8_t* op = kj->out[r0 + rr] + ob;
                store16_out<true>(op, u32x4{acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]});
                store16_out<true>(op + 1024, u32x4{acc[rr][4], acc[rr][5], acc[rr][6], acc[rr][7]});
            }
        }
    }
}

// Wide codes (k > 32) with one row tile (r <= 10), e.g. the reference
// benchmark's 94/100: a 64 MiB stripe is only a few hundred 2 KiB units, so
// the W waves of a workgroup split a unit's inputs (wave w: inputs
// [w k / W, (w + 1) k / W), loaded two ahead and transposed by the wave), XOR
// their partial accumulator planes into one LDS copy of the unit's rows
// (ds_xor_b32, [row][plane][lane]), and after a barrier wave w transposes and
// stores rows w, w + W, ...  Block pointers in the arguments, routine
// addresses ([group][input][RT]) in the device-side table (BsrTblJob).
template <int RT>
__global__ __launch_bounds__(512) void matapply_bsr_ks(const BsrTblJob job) {
    __shared__ uint32_t red[RT * 8 * 64];  // [row][plane][lane]
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nw = blockDim.x >> 6;
    const uint32_t k = job.k, r = job.r;
    const KPtr<BsrTblJob> kj = kernarg_job<BsrTblJob>();
    const uint32_t j0 = wave * k / nw, j1 = (wave + 1) * k / nw;
    const uint32_t ns = job.nstripes, ng = job.ngroups;  // row groups of <= RT rows: (group, stripe) walk
    const uint64_t sz = job.sz;
    for (uint32_t i = threadIdx.x; i < RT * 8 * 64; i += blockDim.x) red[i] = 0u;
    __syncthreads();
    uint32_t s = blockIdx.x / job.cps, c = blockIdx.x - s * job.cps;
    while (s < ns * ng) {
        const uint32_t g = s / ns, stripe = s - g * ns;
        const uint32_t gr0 = g * r / ng, rows = (g + 1) * r / ng - gr0;
        const CU64 ca = (CU64)job.addr + g * k * RT;
        uint64_t off = static_cast<uint64_t>(c) * kBsrChunk;
        if (off > sz - kBsrChunk) off = sz - kBsrChunk;
        const uint64_t ib = stripe * job.in_sstride + off + lane * 16u;
        const uint64_t ob = stripe * job.out_sstride + off + lane * 16u;
        if (j0 < j1) {  // wave-uniform
            uint32_t acc[RT][8];  // no zeroing: input j0 calls "set" routines (kBsrSetBase)
            bsr_walk<RT>(acc, j1 - j0, ib, ca + j0 * RT,
                         [&](uint32_t j) { return kj->ptr[j0 + j]; });
#pragma unroll
            for (int rr = 0; rr < RT; ++rr)
                if (static_cast<uint32_t>(rr) < rows)
#pragma unroll
                    for (int b = 0; b < 8; ++b)
                        __hip_atomic_fetch_xor(&red[(rr * 8 + b) * 64 + lane], acc[rr][b], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        for (uint32_t i = wave; i < rows; i += nw) {  // wave-uniform
            uint32_t v[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                v[b] = red[(i * 8 + b) * 64 + lane];
                red[(i * 8 + b) * 64 + lane] = 0u;  // ready for the next unit
            }
            transpose8(v);
            uint8_t* op = const_cast<uint8_t*>(kj->ptr[k + gr0 + i]) + ob;
            store16_out<true>(op, u32x4{v[0], v[1], v[2], v[3]});
            store16_out<true>(op + 1024, u32x4{v[4], v[5], v[6], v[7]});
        }
        __syncthreads();  // rows read and cleared before the next unit's partials
        c += job.gs_c;
        s += job.gs_s;
        if (c >= job.cps) {
            c -= job.cps;
            ++s;
        }
    }
}

// ---------------------------------------------------------------------------
// matapply_small: launches too small to fill the chip with the unit kernels,
// for codes beyond the register kernels (k > 4 or r > 8).  The unit kernels
// give each lane every output row of its slice: a K=20/M=60 stripe of 4 KiB
// (205-byte blocks) is 26 lanes doing 800 coefficient MACs each, ~30-40 us
// in one wave (tools/small_call_probe.py under rocprofv3,
// profiles/r02_small_calls.log).  Here a wave owns one output row (so its
// coefficients are wave-uniform: their tables are scalar loads from the
// bank) and 64 four-byte units of it, and each lane does k MACs with all k
// input loads in flight at once.  Inputs are re-read once per row, from L2
// (host calls stage wide codes through device memory, fec_abi.cpp).  Python
// bytes calls, K=20/M=60: 4 KiB stripe 57-59 -> 25-26 us per encode, 64 KiB
// 77-81 -> 43-52, 256 KiB 111-121 -> 68-79 (profiles/r02_small_calls.log).
// Launch: gs_c = waves per row, gs_s = bytes per unit (4, or 1 when sz < 4),
// cps = units per stripe.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void matapply_small(const MatJob job) {
    const uint32_t wave = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint32_t wpr = job.gs_c;
    const uint32_t row = __builtin_amdgcn_readfirstlane(wave / wpr);
    if (row >= job.r) return;
    const uint64_t unit = uint64_t(wave - row * wpr) * 64u + (threadIdx.x & 63u);
    const uint64_t cps = job.cps;
    if (unit >= cps * job.nstripes) return;
    const uint32_t ub = job.gs_s;
    const uint64_t s = unit / cps;
    uint64_t off = (unit - s * cps) * ub;
    // The last unit of a block: shifted back to end at sz (its neighbour
    // stores the same bytes), except when accumulating, where two lanes of
    // different waves would both read-modify-write the overlap: there it
    // takes only its own bytes (nb < 4), one at a time.
    uint32_t nb = ub;
    if (off + ub > job.sz) {
        if (job.accumulate)
            nb = static_cast<uint32_t>(job.sz - off);
        else
            off = job.sz - ub;
    }
    const uint64_t io = s * job.in_sstride + off, oo = s * job.out_sstride + off;
    uint32_t acc = 0;
    if (nb == 4u) {
        // every input load is issued before the first is used: one memory
        // latency per launch instead of one per input
        uint32_t xs[kMaxIn];
#pragma unroll
        for (uint32_t j = 0; j < static_cast<uint32_t>(kMaxIn); ++j)
            if (j < job.k) __builtin_memcpy(&xs[j], job.in[j] + io, 4);
#pragma unroll
        for (uint32_t j = 0; j < static_cast<uint32_t>(kMaxIn); ++j) {
            if (j < job.k) {
                const uint32_t* t = &g_bank.w[uint32_t(job.coef[row * job.k + j]) * 8u];
                const Sel sl = selectors(xs[j]);
                acc = xor3(acc, perm(t[1], t[0], sl.s0), perm(t[3], t[2], sl.s1)) ^ perm(t[4], t[4], sl.s2);
            }
        }
    } else {  // the bytes of a block shorter than 4, or an accumulating launch's tail
        for (uint32_t j = 0; j < job.k; ++j) {
            uint32_t x = 0;
            for (uint32_t q = 0; q < nb; ++q) x |= uint32_t(job.in[j][io + q]) << (8 * q);
            const uint32_t* t = &g_bank.w[uint32_t(job.coef[row * job.k + j]) * 8u];
            const Sel sl = selectors(x);
            acc = xor3(acc, perm(t[1], t[0], sl.s0), perm(t[3], t[2], sl.s1)) ^ perm(t[4], t[4], sl.s2);
        }
    }
    uint8_t* op = job.out[row] + oo;
    if (nb == 4u) {
        if (job.accumulate) {
            uint32_t o;
            __builtin_memcpy(&o, op, 4);
            acc ^= o;
        }
        __builtin_memcpy(op, &acc, 4);
    } else {
        for (uint32_t b = 0; b < nb; ++b) {
            const uint8_t v = static_cast<uint8_t>(acc >> (8 * b));
            op[b] = job.accumulate ? static_cast<uint8_t>(op[b] ^ v) : v;
        }
    }
}

// Launch through hipLaunchKernel itself: hipLaunchKernelGGL (<<<>>>) adds
// __hipPushCallConfiguration / __hipPopCallConfiguration around it, and the
// hipGetLastError after it is one more runtime call; together 0.2-0.35 us of
// host time per launch (tools/host_cost.hip: "launch, 560 B kernarg" against
// "hipLaunchKernel 560 B").  The returned status is the launch's.
template <class J>
hipError_t launch_job(const void* fn, uint32_t grid, uint32_t block, size_t lds, hipStream_t stream, const J& job) {
    void* args[] = {const_cast<J*>(&job)};
    return hipLaunchKernel(fn, dim3(grid), dim3(block), args, lds, stream);
}

// Launches whose unit kernels would run fewer lanes than Config::small_lanes
// (2048 by default) take matapply_small.
hipError_t launch_small(MatJob& job, hipStream_t stream) {
    const uint32_t ub = job.sz >= 4 ? 4u : 1u;
    const uint64_t cps = (job.sz + ub - 1) / ub;
    const uint64_t units = cps * job.nstripes;
    const uint64_t wpr = (units + 63) / 64;
    const uint64_t waves = wpr * job.r;
    if (waves > (1ull << 31)) return hipErrorNotSupported;
    job.cps = static_cast<uint32_t>(cps);
    job.gs_c = static_cast<uint32_t>(wpr);
    job.gs_s = ub;
    const uint32_t grid = static_cast<uint32_t>((waves + kBlock / 64 - 1) / (kBlock / 64));
    return launch_job(reinterpret_cast<const void*>(matapply_small), grid, kBlock, 0, stream, job);
}

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
typedef void (*KernelFn)(const MatJob);

std::once_flag g_dispatch_once;
int g_num_cu = 256;
// Grid cap of the unit kernels: CUs x 8 x 1024 workgroups, i.e. about one unit
// per lane for any launch this library makes (measured +9 % on 10^6 4 KiB
// stripes against a grid of 16 resident waves per SIMD); a launch past it
// walks grid-stride.
constexpr uint64_t kGridPerCu = 8 * 1024;

void init_dispatch() {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
            g_num_cu = prop.multiProcessorCount;
    }
}

thread_local const char* t_last_kernel = "";

thread_local uint32_t* t_signal_flag = nullptr;
thread_local uint32_t t_signal_seq = 0;
thread_local bool t_signal_used = false;

// ---- register kernels (k <= 4, r <= 8) ----------------------------------------
constexpr int kRegK = 4, kRegR = 8;
const char* const kRegNames[kRegK + 1][kRegR + 1] = {
    {},
    {"", "matapply_reg<1,1>", "matapply_reg<1,2>", "matapply_reg<1,3>", "matapply_reg<1,4>", "matapply_reg<1,5>",
     "matapply_reg<1,6>", "matapply_reg<1,7>", "matapply_reg<1,8>"},
    {"", "matapply_reg<2,1>", "matapply_reg<2,2>", "matapply_reg<2,3>", "matapply_reg<2,4>", "matapply_reg<2,5>",
     "matapply_reg<2,6>", "matapply_reg<2,7>", "matapply_reg<2,8>"},
    {"", "matapply_reg<3,1>", "matapply_reg<3,2>", "matapply_reg<3,3>", "matapply_reg<3,4>", "matapply_reg<3,5>",
     "matapply_reg<3,6>", "matapply_reg<3,7>", "matapply_reg<3,8>"},
    {"", "matapply_reg<4,1>", "matapply_reg<4,2>", "matapply_reg<4,3>", "matapply_reg<4,4>", "matapply_reg<4,5>",
     "matapply_reg<4,6>", "matapply_reg<4,7>", "matapply_reg<4,8>"}};

const char* const kRowsNames[kRegK + 1][kRegR + 1] = {
    {},
    {"", "matapply_rows<1,1>", "matapply_rows<1,2>", "matapply_rows<1,3>", "matapply_rows<1,4>",
     "matapply_rows<1,5>", "matapply_rows<1,6>", "matapply_rows<1,7>", "matapply_rows<1,8>"},
    {"", "matapply_rows<2,1>", "matapply_rows<2,2>", "matapply_rows<2,3>", "matapply_rows<2,4>",
     "matapply_rows<2,5>", "matapply_rows<2,6>", "matapply_rows<2,7>", "matapply_rows<2,8>"},
    {"", "matapply_rows<3,1>", "matapply_rows<3,2>", "matapply_rows<3,3>", "matapply_rows<3,4>",
     "matapply_rows<3,5>", "matapply_rows<3,6>", "matapply_rows<3,7>", "matapply_rows<3,8>"},
    {"", "matapply_rows<4,1>", "matapply_rows<4,2>", "matapply_rows<4,3>", "matapply_rows<4,4>",
     "matapply_rows<4,5>", "matapply_rows<4,6>", "matapply_rows<4,7>", "matapply_rows<4,8>"}};

// Output store policy of the register kernels: nt sc1 (written through the L2
// at device scope) for single-stripe launches -- a few long rows, where it measured faster: the
// cfg2 64 MiB K=3/M=10 stripe, encode 68.5 -> 69.1-69.9 % of HBM from cold
// caches, secondary decode 65.6 -> 68.0 %, bench value +1.2-1.5 % -- and nt for
// batches of many stripes, where nt sc1 measured slower (256 x 1 MiB
// object-major 69.5 -> 67.7 %, 10^6 x 4 KiB -1 %; tools/ab_store.sh,
// profiles/r02_store_ab.log; copy-walk probe: tools/mb_cold.exe tail).
// Fill a register kernel's argument block for `a`; returns its grid (0: more
// units than one launch walks -- the caller splits).  rows: matapply_rows'
// one-wave-per-stripe walk.
template <int K, int R>
uint32_t fill_regjob(const ApplySpec& a, RegJob<K, R>& job, bool rows) {
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.done_flag = nullptr;
    job.done_seq = 0;
    job.pad_ = 0;
    for (int j = 0; j < K; ++j) job.in[j] = a.in[j];
    for (int i = 0; i < R; ++i) job.out[i] = a.out[i];
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < K; ++j) {
            const uint32_t* w = &kHostBank.w[uint32_t(a.coef[size_t(i) * a.coef_stride + j]) * 8];
            uint32_t* t = &job.tab[(i * K + j) * 5];
            t[0] = w[0];
            t[1] = w[1];
            t[2] = w[2];
            t[3] = w[3];
            t[4] = w[4];
        }
    const uint64_t cps = (a.sz + kChunk - 1) / kChunk;
    if (cps * a.nstripes >= (1ull << 32) - (1ull << 24)) return 0;
    job.cps = static_cast<uint32_t>(cps);
    // one unit per lane up to the grid cap; beyond it a grid-stride loop
    const uint64_t lanes = rows ? a.nstripes * 64u : cps * a.nstripes;  // rows: one wave per stripe
    const uint64_t need = (lanes + kBlock - 1) / kBlock;
    const uint64_t cap = uint64_t(g_num_cu) * kGridPerCu;
    const uint32_t grid = static_cast<uint32_t>(need < cap ? need : cap);
    const uint64_t gstride = uint64_t(grid) * kBlock;
    job.gs_s = static_cast<uint32_t>(gstride / cps);
    job.gs_c = static_cast<uint32_t>(gstride % cps);
    return grid;
}

bool rows_shape(const ApplySpec& a) { return a.sz > kRowsMin && a.sz <= kRowsMax && a.nstripes >= 64; }

template <int K, int R>
hipError_t launch_reg(const ApplySpec& a, hipStream_t stream, uint32_t* sig) {
    // many outputs: the prefetching walk (K=3/M=10 encode 6.17 -> 6.41 TB/s,
    // tools/mb_encode.exe; no gain for the 3-row decode)
    constexpr bool kPrefetch = reg_prefetch(R);
    // more table dwords than the SGPRs hold next to the pointers: read them
    // where they are used (K=3/M=10 encode 35.9 -> 33.6 us, tools/mb_encode.exe
    // variant "PF AL"; the 3-row decode is unchanged either way)
    constexpr bool kArgLoad = reg_argload(K, R);
    RegJob<K, R> job;
    const bool rows = rows_shape(a);
    const uint32_t grid = fill_regjob<K, R>(a, job, rows);
    if (!grid) return hipErrorInvalidValue;  // the caller splits
    void (*fn)(const RegJob<K, R>);
    if (rows) {
        fn = matapply_rows<K, R, kArgLoad>;
        t_last_kernel = kRowsNames[K][R];
    } else {
        // Single stripes store nt sc1 -- unless an output row starts off a
        // 16-byte line: its 16-byte stores straddle two lines, and written
        // through (sc1) each straddling store costs a partial-line write; nt
        // alone lets the L2 merge the halves.  K=3/M=10 64 MiB, outputs at 6
        // (mod 16): nt sc1 47.2 us, nt 41.6-42.0 us, aligned 39.6
        // (tools/misaligned_bench.py, profiles/r04_misaligned_ab.json; staging
        // the rows through LDS to store aligned lines measured 56-62 us, and
        // assembling them across lanes with DPP 90 us).
        bool ma = false;
        for (int i = 0; i < R; ++i) ma = ma || (reinterpret_cast<uintptr_t>(a.out[i]) & 15u) != 0;
        fn = a.nstripes == 1 && !ma ? matapply_reg<K, R, 3, kPrefetch, kArgLoad>
                                    : matapply_reg<K, R, 0, kPrefetch, kArgLoad>;
        t_last_kernel = kRegNames[K][R];
        if (sig && grid == 1) {  // one workgroup: it signals its own completion
            job.done_flag = sig;
            job.done_seq = t_signal_seq;
            t_signal_used = true;
        }
    }
    return launch_job(reinterpret_cast<const void*>(fn), grid, kBlock, 0, stream, job);
}

typedef hipError_t (*RegLaunch)(const ApplySpec&, hipStream_t, uint32_t*);

template <int K, int... R>
constexpr std::array<RegLaunch, kRegR + 1> reg_row(std::integer_sequence<int, R...>) {
    return {{nullptr, launch_reg<K, R + 1>...}};
}

const std::array<RegLaunch, kRegR + 1> g_reg_launch[kRegK + 1] = {
    {}, reg_row<1>(std::make_integer_sequence<int, kRegR>()), reg_row<2>(std::make_integer_sequence<int, kRegR>()),
    reg_row<3>(std::make_integer_sequence<int, kRegR>()), reg_row<4>(std::make_integer_sequence<int, kRegR>())};

// ---- paired register launches (matapply_pair) ------------------------------------
char g_pair_names[kRegK + 1][kRegR + 1][kRegR + 1][32];

template <int K, int RA, int RB>
hipError_t launch_pair(const ApplySpec& a, const ApplySpec& b, hipStream_t stream) {
    PairJob<K, RA, RB> job;
    const uint32_t ga = fill_regjob<K, RA>(a, job.a, false), gb = fill_regjob<K, RB>(b, job.b, false);
    if (!ga || !gb || uint64_t(ga) + gb >= (1ull << 31)) return hipErrorNotSupported;
    job.blocks_a = ga;
    job.pad_[0] = job.pad_[1] = job.pad_[2] = 0;
    // the register kernels' store policy, single-stripe (nt sc1) only when both are
    const bool sc1 = a.nstripes == 1 && b.nstripes == 1;
    void (*fn)(const PairJob<K, RA, RB>) = sc1 ? matapply_pair<K, RA, RB, 3> : matapply_pair<K, RA, RB, 0>;
    t_last_kernel = g_pair_names[K][RA][RB];
    return launch_job(reinterpret_cast<const void*>(fn), ga + gb, kBlock, 0, stream, job);
}

typedef hipError_t (*PairLaunch)(const ApplySpec&, const ApplySpec&, hipStream_t);
typedef std::array<PairLaunch, kRegR + 1> PairRow;

template <int K, int RA, int RB>
constexpr PairLaunch pair_entry() {
    if constexpr (RB <= K && RB <= RA)
        return launch_pair<K, RA, RB>;
    else
        return nullptr;
}

template <int K, int RA, int... RB>
constexpr PairRow pair_row(std::integer_sequence<int, RB...>) {
    return {{nullptr, pair_entry<K, RA, RB + 1>()...}};
}

template <int K, int... RA>
constexpr std::array<PairRow, kRegR + 1> pair_plane(std::integer_sequence<int, RA...>) {
    return {{PairRow{}, pair_row<K, RA + 1>(std::make_integer_sequence<int, kRegR>())...}};
}

const std::array<PairRow, kRegR + 1> g_pair_launch[kRegK + 1] = {
    {}, pair_plane<1>(std::make_integer_sequence<int, kRegR>()), pair_plane<2>(std::make_integer_sequence<int, kRegR>()),
    pair_plane<3>(std::make_integer_sequence<int, kRegR>()), pair_plane<4>(std::make_integer_sequence<int, kRegR>())};

// ---- table kernels (matapply_lds, k <= 32, r <= 48) ----------------------------
struct LdsVariant {
    KernelFn fn;
    const char* name;
    int chunk;     // bytes per unit (a lane's slice of one block)
    int pad_tile;  // kTilesPadded: rows per tile (the LDS table is padded to whole tiles); 0: ragged
};

// Padded-tile variants by tile height: 1-8 rows in one tile (r <= 8), 9-20
// rows for wider codes split into ceil(r/20) near-equal tiles.
constexpr int kMaxTile = 20;
char g_pad_names[kMaxTile + 1][40];
LdsVariant g_lds_pad[kMaxTile + 1];
// measured (tools/mb_encode.exe MB_AB, interleaved medians): k <= 4
// (memory-bound) takes 16 bytes per lane in ragged 8-row tiles; wider codes
// take 8 bytes per lane in padded tiles (no per-row branches), as few tiles as
// 20-row register tiles allow (inputs are re-read per tile)
const LdsVariant g_lds_fewin{matapply_lds<false, true, 8, 4, 4>, "matapply_lds<8,4,4>", 16, 0};
const LdsVariant g_lds_acc{matapply_lds<true, false, 16, 2, 2>, "matapply_lds<16,2,2,acc>", 8, 0};

template <int RT>
void fill_pad() {
    constexpr int G = (RT <= 4 || RT == 8) ? 4 : 2;  // input group size: measured per tile height
    snprintf(g_pad_names[RT], sizeof g_pad_names[RT], "matapply_lds<%d,2,%d,pad>", RT, G);
    g_lds_pad[RT] = LdsVariant{matapply_lds<false, true, RT, 2, G, kTilesPadded>, g_pad_names[RT], 8, RT};
    if constexpr (RT < kMaxTile) fill_pad<RT + 1>();
}

std::once_flag g_pad_once;

const LdsVariant& pick_lds(uint32_t k, uint32_t r, bool acc) {
    std::call_once(g_pad_once, [] { fill_pad<1>(); });
    if (acc) return g_lds_acc;
    if (k <= 4) return g_lds_fewin;
    const uint32_t tiles = (r + kMaxTile - 1) / kMaxTile;
    return g_lds_pad[(r + tiles - 1) / tiles];
}

void fill_matjob(const ApplySpec& a, MatJob& job) {
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = a.k;
    job.r = a.r;
    job.cps = job.gs_c = job.gs_s = 0;
    job.accumulate = a.accumulate;
    job.pad_ = 0;
    for (uint32_t j = 0; j < a.k; ++j) job.in[j] = a.in[j];
    for (uint32_t i = 0; i < a.r; ++i) job.out[i] = a.out[i];
}

void fill_coef(const ApplySpec& a, MatJob& job) {
    for (uint32_t i = 0; i < a.r; ++i) std::memcpy(&job.coef[i * a.k], a.coef + size_t(i) * a.coef_stride, a.k);
}

hipError_t launch_lds(const ApplySpec& a, hipStream_t stream) {
    const LdsVariant& v = pick_lds(a.k, a.r, a.accumulate);
    const uint64_t cps = (a.sz + v.chunk - 1) / v.chunk;
    const uint64_t total = cps * a.nstripes;
    if (total >= (1ull << 32) - (1ull << 24)) return hipErrorInvalidValue;  // the caller splits larger jobs
    MatJob job;
    fill_matjob(a, job);
    fill_coef(a, job);
    job.cps = static_cast<uint32_t>(cps);
    const size_t rows = v.pad_tile ? (a.r + v.pad_tile - 1) / v.pad_tile * v.pad_tile : a.r;
    const size_t lds = size_t(a.k) * rows * 32;
    const uint64_t need = (total + kBlock - 1) / kBlock;
    const uint64_t cap = uint64_t(g_num_cu) * kGridPerCu;
    const uint32_t grid = static_cast<uint32_t>(need < cap ? need : cap);
    const uint64_t gstride = uint64_t(grid) * kBlock;
    job.gs_s = static_cast<uint32_t>(gstride / cps);
    job.gs_c = static_cast<uint32_t>(gstride % cps);
    t_last_kernel = v.name;
    return launch_job(reinterpret_cast<const void*>(v.fn), grid, kBlock, lds, stream, job);
}

// ---- matapply_bsg dispatch ------------------------------------------------------
// Rows per wave: the smallest instantiated RT >= ceil(r / 4).
constexpr int kBsgRT[] = {1, 2, 3, 4, 5, 6, 8, 10, 12};
constexpr int kBsgNumRT = sizeof(kBsgRT) / sizeof(kBsgRT[0]);
constexpr uint32_t kBsgMaxRows = 4u * 12u;

struct BsgVariant {
    const void* fn_karg = nullptr;  // matapply_bsg<RT, false, MatJob>
    const void* fn_tbl = nullptr;   // matapply_bsg<RT, true, BsgTblJob>
    char name[32] = "";
    char name_tbl[32] = "";
    int blocks_per_cu = 1;          // resident workgroups per CU (occupancy API), set once
};
BsgVariant g_bsg_var[kBsgNumRT];
std::once_flag g_bsg_once;
std::atomic<int> g_generic{-1};

template <int I>
void fill_bsg() {
    constexpr int RT = kBsgRT[I];
    BsgVariant& v = g_bsg_var[I];
    v.fn_karg = reinterpret_cast<const void*>(matapply_bsg<RT, false, MatJob>);
    v.fn_tbl = reinterpret_cast<const void*>(matapply_bsg<RT, true, BsgTblJob>);
    snprintf(v.name, sizeof v.name, "matapply_bsg<%d,2>", RT);
    snprintf(v.name_tbl, sizeof v.name_tbl, "matapply_bsg<%d,2,tbl>", RT);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, v.fn_karg, 256, kBsgPhase * kBsgSlotBytes) == hipSuccess &&
        nb > 0)
        v.blocks_per_cu = nb;
    else
        (void)hipGetLastError();
    if constexpr (I + 1 < kBsgNumRT) fill_bsg<I + 1>();
}

bool bsg_shape_ok(uint32_t k, uint32_t r, uint64_t sz) {
    // k * r >= 24, not a register-kernel shape; past 32 inputs (the table form)
    // up to 256 rows in one launch, otherwise one group of <= 48
    const uint32_t rmax = k > static_cast<uint32_t>(kMaxIn) ? 256u : kBsgMaxRows;
    return generic_mode() != 0 && sz >= kBsgChunk && k >= 1 && k <= static_cast<uint32_t>(kMaxWideIn) && r >= 1 &&
           r <= rmax && k * r >= 24 && !(k <= 4 && r <= 8);
}

// Device-side argument tables of wide matapply_bsg launches, per thread and
// device: a ring of slots in device memory filled by stream-ordered copies
// from a pinned mirror; a slot is reused once the event recorded after its
// last launch has completed.
// Events that only tell the host when a table slot's readers have finished
// (hipEventSynchronize before the slot is rewritten, hipStreamWaitEvent for
// another stream of the same device): no system-scope release, which would
// write the L2's dirty lines back at every launch that records one.
constexpr unsigned kSlotEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;

struct TableRing {
    static constexpr int kSlots = 8;
    static constexpr size_t kSlotBytes = size_t(160) << 10;  // k, r <= 256 with 64 row groups of 4
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    hipEvent_t ev[kSlots] = {};
    bool busy[kSlots] = {};
    unsigned next = 0;
};

struct Rings {
    std::unordered_map<int, TableRing> dev;
    ~Rings() {
        for (auto& kv : dev) {
            int cur = 0;
            if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(kv.first) != hipSuccess) continue;
            TableRing& t = kv.second;
            for (int i = 0; i < TableRing::kSlots; ++i)
                if (t.ev[i]) (void)hipEventSynchronize(t.ev[i]), (void)hipEventDestroy(t.ev[i]);
            if (t.dev) (void)hipFree(t.dev);
            if (t.host) (void)hipHostFree(t.host);
            (void)hipSetDevice(cur);
        }
    }
};
thread_local Rings t_rings;

hipError_t ring_slot(TableRing** ring, unsigned* slot) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    TableRing& t = t_rings.dev[dev];
    if (!t.dev) {
        if ((e = hipMalloc(&t.dev, TableRing::kSlots * TableRing::kSlotBytes)) != hipSuccess) return e;
        if ((e = hipHostMalloc(&t.host, TableRing::kSlots * TableRing::kSlotBytes, hipHostMallocDefault)) !=
            hipSuccess) {
            (void)hipFree(t.dev);
            t.dev = nullptr;
            return e;
        }
        for (int i = 0; i < TableRing::kSlots; ++i)
            if ((e = hipEventCreateWithFlags(&t.ev[i], kSlotEventFlags)) != hipSuccess) return e;
    }
    const unsigned s = t.next++ % TableRing::kSlots;
    if (t.busy[s] && (e = hipEventSynchronize(t.ev[s])) != hipSuccess) return e;  // its last launch has read it
    t.busy[s] = false;
    *ring = &t;
    *slot = s;
    return hipSuccess;
}

// matapply_bsg launch (the table form declines under graph capture: stream_capturing).
hipError_t launch_bsg(const ApplySpec& a, hipStream_t stream) {
    std::call_once(g_bsg_once, [] { fill_bsg<0>(); });
    const uint32_t k = a.k, r = a.r;
    const uint64_t cps = (a.sz + kBsgChunk - 1) / kBsgChunk;
    const uint64_t units = cps * a.nstripes;
    // Rows per wave: the smallest instantiated RT >= ceil(r / 4), at most 12
    // (48 rows per group of the walk).  A launch with fewer than ~4 workgroups
    // per CU of (unit, row group) work takes smaller row groups: each group's
    // workgroups rebuild the inputs' combinations, which costs less than idle
    // CUs (a 64 MiB stripe of a 128/256 code is 128 units of 4 KiB).  The
    // shrinking stops at RT 2: one row per wave re-reads every input per 4
    // rows, and measured slower than half-idle CUs (profiles/r03_bsg_wgs.json:
    // 200/256 at RT 2 0.207 ms, RT 1 0.278 ms; 128/256 at RT 4 0.249 ms, RT 10
    // 0.351 ms, RT 2 0.312 ms).
    constexpr uint32_t kBsgWgsPerCu = 4;
    const uint32_t need_rt = (r + 3) / 4;
    int ri = 0;
    while (ri + 1 < kBsgNumRT && kBsgRT[ri] < static_cast<int>(need_rt)) ++ri;
    const uint64_t target = uint64_t(kBsgWgsPerCu) * static_cast<uint64_t>(g_num_cu);
    auto groups_of = [&](int i) { return (r + 4u * kBsgRT[i] - 1) / (4u * kBsgRT[i]); };
    while (ri > 1 && units * groups_of(ri) < target) --ri;
    const uint32_t ngroups = groups_of(ri);
    const BsgVariant& v = g_bsg_var[ri];
    // coefficients in the kernel's walk order: group g, wave w, phase f at
    // ((g * 4 + w) * nph + f) * PB, (js, rr) in order: row g * 4 * RT + w + 4 * rr
    // of input 2 * f + js
    const uint32_t RT = static_cast<uint32_t>(kBsgRT[ri]), P = kBsgPhase;
    const uint32_t PB = (P * RT + 3) / 4 * 4, nph = (k + P - 1) / P;
    const uint32_t walk = ngroups * 4u * nph * PB;
    auto fill_walk = [&](uint8_t* cf) {
        std::memset(cf, 0, walk);
        for (uint32_t g = 0; g < ngroups; ++g)
            for (uint32_t w = 0; w < 4; ++w)
                for (uint32_t f = 0; f < nph; ++f)
                    for (uint32_t js = 0; js < P; ++js)
                        for (uint32_t rr = 0; rr < RT; ++rr) {
                            const uint32_t i = g * 4 * RT + w + 4 * rr, j = P * f + js;
                            if (i < r && j < k && w + 4 * rr < 4 * RT)
                                cf[((g * 4 + w) * nph + f) * PB + js * RT + rr] =
                                    a.coef[size_t(i) * a.coef_stride + j];
                        }
    };
    const size_t lds = size_t(P) * kBsgSlotBytes;
    const uint64_t vunits = units * ngroups;
    if (vunits >= (1ull << 32) - (1ull << 24)) return hipErrorInvalidValue;
    const uint64_t cap = uint64_t(g_num_cu) * v.blocks_per_cu * 8;
    const uint32_t grid = static_cast<uint32_t>(vunits < cap ? vunits : cap);
    const uint32_t gs_s = static_cast<uint32_t>(grid / cps), gs_c = static_cast<uint32_t>(grid % cps);
    if (ngroups == 1 && k <= static_cast<uint32_t>(kMaxIn) && r <= static_cast<uint32_t>(kMaxOut) &&
        walk <= static_cast<uint32_t>(kMaxCoef)) {
        MatJob job;
        fill_matjob(a, job);
        fill_walk(job.coef);
        job.cps = static_cast<uint32_t>(cps);
        job.gs_s = gs_s;
        job.gs_c = gs_c;
        t_last_kernel = v.name;
        return launch_job(v.fn_karg, grid, 256, lds, stream, job);
    }
    // pointers and coefficients in a device-side table
    if (stream_capturing(stream)) return hipErrorNotSupported;
    const size_t bytes = 8 * size_t(k + r) + walk;
    if (bytes > TableRing::kSlotBytes) return hipErrorNotSupported;
    TableRing* ring = nullptr;
    unsigned slot = 0;
    hipError_t e = ring_slot(&ring, &slot);
    if (e != hipSuccess) return e;
    uint8_t* h = ring->host + slot * TableRing::kSlotBytes;
    uint8_t* d = ring->dev + slot * TableRing::kSlotBytes;
    std::memcpy(h, a.in, 8 * size_t(k));
    std::memcpy(h + 8 * size_t(k), a.out, 8 * size_t(r));
    fill_walk(h + 8 * size_t(k + r));
    if ((e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream)) != hipSuccess) return e;
    BsgTblJob job;
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = k;
    job.r = r;
    job.cps = static_cast<uint32_t>(cps);
    job.gs_s = gs_s;
    job.gs_c = gs_c;
    job.ngroups = ngroups;
    job.pad_ = 0;
    job.table = d;
    if ((e = launch_job(v.fn_tbl, grid, 256, lds, stream, job)) != hipSuccess) return e;
    if ((e = hipEventRecord(ring->ev[slot], stream)) != hipSuccess) return e;
    ring->busy[slot] = true;
    t_last_kernel = v.name_tbl;
    return hipSuccess;
}

// ---- matapply_bsr dispatch ------------------------------------------------------
// Whether an nw-wave LDS-phase launch shares the inputs' 30 combinations through
// LDS (built once per workgroup, phases of one input per wave) instead of the 8
// planes (the 22 multi-plane combinations rebuilt by every wave): with 8 waves,
// where rebuilding is 8x the work (128/256 0.130 -> 0.122 ms per 64 MiB stripe);
// with 2 or 4 the short phases cost more than the XORs saved (cfg4's first-seen
// 20-row decode 0.439 -> 0.474 ms, 30/70 0.070 -> 0.074; profiles/r05_bsr_cmb_ab.json;
// on DMA-staged phases 0.419 -> 0.428 and 0.065 -> 0.067, r05_lds_dma_ab.json).
// ZFEC_BSR_CMB_MIN_NW: the least waves per workgroup that share combinations
// (default 8; the A/B knob of tools/ab_build.sh)
#ifndef ZFEC_BSR_CMB_MIN_NW
#define ZFEC_BSR_CMB_MIN_NW 8
#endif
// (the double-buffered form needs an even phase, nw / 2 >= 2: the kernel's
// routine-address sets alternate by input parity across phases)
bool bsr_cmb(uint32_t nw) { return nw >= ZFEC_BSR_CMB_MIN_NW && (!ZFEC_BSR_CMB_DB || nw >= 4); }

// LDS of an nw-wave LDS-phase launch over k inputs: one phase of combinations
// and its raw staging, or two phases of planes (one when a single phase holds
// all k).
size_t bsr_lds_bytes(uint32_t k, uint32_t nw, bool cmb) {
#if ZFEC_BSR_CMB_DB
    // two phases of nw / 2 inputs: combinations and raw staging each
    if (cmb) return size_t(2) * (nw / 2) * (bsr_in_bytes<true>() + bsr_in_bytes<false>());
#endif
    const uint32_t ph = cmb ? bsr_cmb_phase(nw) : bsr_db_phase(nw);
    if (cmb) return size_t(k < ph ? k : ph) * (bsr_in_bytes<true>() + bsr_in_bytes<false>());  // + raw staging
    return size_t(k <= ph ? k : 2 * ph) * bsr_in_bytes<false>();
}

// nw = ceil(r / 10) waves, one per row tile of <= RT = ceil(r / nw) rows.
struct BsrVariant {
    const void* fn = nullptr;
    const void* fn_cmb = nullptr;  // combination-sharing form (bsr_cmb)
    const void* fn_solo = nullptr;
    const void* fn_a32 = nullptr;  // 32-bit argument form (BsrJob32)
    const void* fn_a32_cmb = nullptr;
    char name[24] = "";
    char name_cmb[28] = "";
    char name_solo[32] = "";
    char name_a32[28] = "";
    char name_a32_cmb[32] = "";
};
BsrVariant g_bsr_var[kBsrMaxRows + 1];
std::once_flag g_bsr_once;

template <int RT>
void fill_bsr() {
    g_bsr_var[RT].fn = reinterpret_cast<const void*>(matapply_bsr<RT, false, false, BsrJob>);
    g_bsr_var[RT].fn_cmb = reinterpret_cast<const void*>(matapply_bsr<RT, false, true, BsrJob>);
    snprintf(g_bsr_var[RT].name, sizeof g_bsr_var[RT].name, "matapply_bsr<%d,lds>", RT);
    snprintf(g_bsr_var[RT].name_cmb, sizeof g_bsr_var[RT].name_cmb, "matapply_bsr<%d,lds,cmb>", RT);
    g_bsr_var[RT].fn_solo = reinterpret_cast<const void*>(matapply_bsr_solo<RT>);
    snprintf(g_bsr_var[RT].name_solo, sizeof g_bsr_var[RT].name_solo, "matapply_bsr<%d>", RT);
#if !ZFEC_BSR_NO_A32  // (instantiated only for the A/B)
    g_bsr_var[RT].fn_a32 = reinterpret_cast<const void*>(matapply_bsr<RT, false, false, BsrJob32>);
    g_bsr_var[RT].fn_a32_cmb = reinterpret_cast<const void*>(matapply_bsr<RT, false, true, BsrJob32>);
#endif
    snprintf(g_bsr_var[RT].name_a32, sizeof g_bsr_var[RT].name_a32, "matapply_bsr<%d,lds,a32>", RT);
    snprintf(g_bsr_var[RT].name_a32_cmb, sizeof g_bsr_var[RT].name_a32_cmb, "matapply_bsr<%d,lds,a32,cmb>", RT);
    if constexpr (RT < kBsrMaxRows) fill_bsr<RT + 1>();
}

// The address of the routine table on each device, read by bsr_table_probe
// (the host writes every coefficient's routine address into the launches'
// arguments).  Only a successful probe is latched: a failed one (stream,
// pinned buffer, launch or sync error) is reported on stderr under
// ZFEC_HIP_JIT_VERBOSE and retried by a later launch, up to kBsrProbeTries per
// device; until one succeeds the device gets no matapply_bsr launches
// (launch_apply hands them to matapply_bsg).
constexpr int kBsrMaxDevices = 64;
constexpr int kBsrProbeTries = 3;
struct BsrBase {
    std::mutex mu;
    std::atomic<uint64_t> addr{0};  // nonzero: the probe succeeded
    int tries = 0;
};
BsrBase g_bsr_base[kBsrMaxDevices];

hipError_t bsr_probe(uint64_t* addr) {
    hipStream_t st = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
    uint64_t* h = nullptr;
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(uint64_t), hipHostMallocDefault)) == hipSuccess) {
        *h = 0;
        hipLaunchKernelGGL(bsr_table_probe, dim3(1), dim3(64), 0, st, h);
        if ((e = hipGetLastError()) == hipSuccess && (e = hipStreamSynchronize(st)) == hipSuccess)
            *addr = *h;
        (void)hipHostFree(h);
    }
    (void)hipStreamDestroy(st);
    return e;
}

hipError_t bsr_routine_base(uint64_t* base, hipStream_t stream) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kBsrMaxDevices) return hipErrorNotSupported;
    BsrBase& b = g_bsr_base[dev];
    uint64_t a = b.addr.load(std::memory_order_acquire);
    if (!a) {
        // the probe synchronises a stream of its own: not while the launch
        // stream is being captured into a graph (the launch declines; a later one probes)
        if (stream_capturing(stream)) return hipErrorNotSupported;
        std::lock_guard<std::mutex> g(b.mu);
        a = b.addr.load(std::memory_order_acquire);
        if (!a && b.tries < kBsrProbeTries) {
            ++b.tries;
            uint64_t got = 0;
            const hipError_t e = bsr_probe(&got);
            if (e == hipSuccess && got) {
                b.addr.store(got, std::memory_order_release);
                a = got;
            } else {
                (void)hipGetLastError();
                if (getenv("ZFEC_HIP_JIT_VERBOSE"))
                    fprintf(stderr, "zfec_hip: routine-table probe on device %d failed (try %d of %d): %s\n", dev,
                            b.tries, kBsrProbeTries, e == hipSuccess ? "address 0" : hipGetErrorString(e));
            }
        }
        if (!a) return hipErrorNotSupported;
    }
    *base = a;
    return hipSuccess;
}

// Routine addresses in a bsr kernel's walk order, [group][wave][input][rt]:
// group g holds rows g*r/ng .. (g+1)*r/ng - 1, split over its nw waves as the
// kernels split them; routine 0 (which only returns) past a wave's rows.  The
// first input a wave walks -- input 0, or with the inputs split over `split`
// waves (the ks form) inputs s*k/split -- calls the "set" routines, which
// write the rows instead of adding to them (the kernels do not zero their
// accumulators).  False if a wave would hold more than rt rows (the kernel
// would drop them).
bool fill_bsr_addrs(uint64_t* dst, const ApplySpec& a, uint64_t base, uint32_t ng, uint32_t nw, uint32_t rt,
                    uint32_t split) {
    const uint32_t k = a.k, r = a.r;
    std::vector<uint8_t> first(k, 0);
    for (uint32_t w = 0; w < split; ++w)
        if (w * k / split < (w + 1) * k / split) first[w * k / split] = 1;
    for (uint32_t g = 0; g < ng; ++g) {
        const uint32_t gr0 = g * r / ng, grn = (g + 1) * r / ng - gr0;
        for (uint32_t w = 0; w < nw; ++w) {
            const uint32_t r0 = gr0 + w * grn / nw, rows = gr0 + (w + 1) * grn / nw - r0;
            if (rows > rt) return false;
            uint64_t* d = dst + size_t(g * nw + w) * k * rt;
            for (uint32_t j = 0; j < k; ++j) {
                const uint64_t tb = base + (first[j] ? kBsrSetBase : 0u);
                for (uint32_t rr = 0; rr < rt; ++rr)  // (row slot rr's table in the slots form)
                    d[size_t(j) * rt + rr] = tb + uint64_t(kBsrSlotStride) * rr +
                                             uint64_t(kBsrStride) * (rr < rows ? a.coef[size_t(r0 + rr) * a.coef_stride + j] : 0u);
            }
        }
    }
    return true;
}

// Device-side routine-address tables of the table forms, kept per (thread,
// device) by matrix and layout: a launch whose table is held reads it as is
// (its block pointers travel in the kernel arguments), so a matrix's table is
// copied to the device by its first launch only.  Copying the table per launch
// cost 19 us ahead of each 0.10 ms 200/256 launch (90 KB of addresses).  Slots
// are reused round-robin once the launches that read them have finished (an
// event per slot); a launch on another stream than the slot's last one is
// ordered after it (hipStreamWaitEvent), so one event covers every reader.
struct BsrTblCache {
    static constexpr int kSlots = 8;
    static constexpr size_t kSlotBytes = size_t(160) << 10;
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    hipEvent_t used[kSlots] = {};  // recorded after the last launch that read the slot (and its upload)
    bool busy[kSlots] = {};
    hipStream_t last[kSlots] = {};
    uint32_t dims[kSlots][6] = {};  // k, r, ng, nw, rt, split of the table held (k == 0: empty)
    std::vector<uint8_t> coef[kSlots];
    unsigned next = 0;
};

struct BsrTblCaches {
    std::unordered_map<int, BsrTblCache> dev;
    ~BsrTblCaches() {
        for (auto& kv : dev) {
            int cur = 0;
            if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(kv.first) != hipSuccess) continue;
            BsrTblCache& c = kv.second;
            for (int i = 0; i < BsrTblCache::kSlots; ++i)
                if (c.used[i]) (void)hipEventSynchronize(c.used[i]), (void)hipEventDestroy(c.used[i]);
            if (c.dev) (void)hipFree(c.dev);
            if (c.host) (void)hipHostFree(c.host);
            (void)hipSetDevice(cur);
        }
    }
};
thread_local BsrTblCaches t_bsr_tbl;

struct BsrTblRef {
    BsrTblCache* c = nullptr;
    unsigned slot = 0;
    const uint64_t* dev = nullptr;
};

hipError_t bsr_table_done(const BsrTblRef& t, hipStream_t stream) {
    const hipError_t e = hipEventRecord(t.c->used[t.slot], stream);
    if (e == hipSuccess) {
        t.c->busy[t.slot] = true;
        t.c->last[t.slot] = stream;
    }
    return e;
}

// The device-side address table of a (matrix, layout) for a launch on `stream`
// (ng row groups of nw waves of rt rows, inputs split over `split` waves),
// uploaded on a miss; the caller
// launches, then calls bsr_table_done.
hipError_t bsr_addr_table(const ApplySpec& a, hipStream_t stream, uint64_t base, uint32_t ng, uint32_t nw, uint32_t rt,
                          uint32_t split, BsrTblRef* ref) {
    const uint32_t k = a.k, r = a.r;
    const size_t n = size_t(ng) * nw * k * rt;
    if (n * 8 > BsrTblCache::kSlotBytes || stream_capturing(stream)) return hipErrorNotSupported;
    int devid = 0;
    hipError_t e = hipGetDevice(&devid);
    if (e != hipSuccess) return e;
    BsrTblCache& c = t_bsr_tbl.dev[devid];
    if (!c.dev) {
        if ((e = hipMalloc(&c.dev, BsrTblCache::kSlots * BsrTblCache::kSlotBytes)) != hipSuccess) return e;
        if ((e = hipHostMalloc(&c.host, BsrTblCache::kSlots * BsrTblCache::kSlotBytes, hipHostMallocDefault)) !=
            hipSuccess) {
            (void)hipFree(c.dev);
            c.dev = nullptr;
            return e;
        }
        for (int i = 0; i < BsrTblCache::kSlots; ++i)
            if ((e = hipEventCreateWithFlags(&c.used[i], kSlotEventFlags)) != hipSuccess) return e;
    }
    thread_local std::vector<uint8_t> m;  // the matrix, row-major: the key with the layout
    m.resize(size_t(r) * k);
    for (uint32_t i = 0; i < r; ++i) std::memcpy(&m[size_t(i) * k], a.coef + size_t(i) * a.coef_stride, k);
    const uint32_t dims[6] = {k, r, ng, nw, rt, split};
    for (unsigned i = 0; i < BsrTblCache::kSlots; ++i) {
        if (std::memcmp(c.dims[i], dims, sizeof dims) != 0 || c.coef[i] != m) continue;
        if (c.busy[i] && c.last[i] != stream && (e = hipStreamWaitEvent(stream, c.used[i], 0)) != hipSuccess)
            return e;
        *ref = BsrTblRef{&c, i, reinterpret_cast<const uint64_t*>(c.dev + i * BsrTblCache::kSlotBytes)};
        return hipSuccess;
    }
    const unsigned i = c.next++ % BsrTblCache::kSlots;
    if (c.busy[i] && (e = hipEventSynchronize(c.used[i])) != hipSuccess) return e;  // its readers have finished
    c.busy[i] = false;
    c.dims[i][0] = 0;  // empty until the upload is enqueued
    uint64_t* h = reinterpret_cast<uint64_t*>(c.host + i * BsrTblCache::kSlotBytes);
    uint8_t* d = c.dev + i * BsrTblCache::kSlotBytes;
    if (!fill_bsr_addrs(h, a, base, ng, nw, rt, split)) return hipErrorInvalidValue;
    const uint32_t hi = static_cast<uint32_t>(h[0] >> 32);
    bool one_hi = ZFEC_BSR_TBL_WRITER && n <= size_t(4) * kBsrWriteMax;
    for (size_t x = 0; one_hi && x < n; ++x) one_hi = static_cast<uint32_t>(h[x] >> 32) == hi;
    if (one_hi) {
        // up to 4 writer launches (~4 KB of arguments each) instead of the copy
        for (size_t x0 = 0; x0 < n; x0 += kBsrWriteMax) {
            BsrWriteJob w;
            w.dst = reinterpret_cast<uint64_t*>(d) + x0;
            w.n = static_cast<uint32_t>(n - x0 < size_t(kBsrWriteMax) ? n - x0 : kBsrWriteMax);
            w.hi = hi;
            for (uint32_t x = 0; x < w.n; ++x) w.lo[x] = static_cast<uint32_t>(h[x0 + x]);
            if ((e = launch_job(reinterpret_cast<const void*>(bsr_table_write), 1, 256, 0, stream, w)) != hipSuccess)
                return e;
        }
    } else if ((e = hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, stream)) != hipSuccess) {
        return e;
    }
    // (no event for the upload itself: the launch that follows on this stream records
    // the slot's event whether or not it is accepted, bsr_table_done, and that event
    // completes after the upload -- one hipEventRecord less in a first launch)
    std::memcpy(c.dims[i], dims, sizeof dims);
    c.coef[i] = m;
    *ref = BsrTblRef{&c, i, reinterpret_cast<const uint64_t*>(d)};
    return hipSuccess;
}

// Block pointers of a table-form launch into its arguments: false if k + r
// exceeds them.
bool bsr_tbl_ptrs(const ApplySpec& a, BsrTblJob& job) {
    if (size_t(a.k) + a.r > static_cast<size_t>(kBsrTblPtrs)) return false;
    for (uint32_t j = 0; j < a.k; ++j) job.ptr[j] = a.in[j];
    for (uint32_t i = 0; i < a.r; ++i) job.ptr[a.k + i] = a.out[i];
    return true;
}

// Waves (row tiles) per workgroup: one for r <= 10 (the one-wave form); 4 for
// r > 20 (tiles of <= 10 rows): 3 or 5 waves leave a SIMD of the CU with more
// of them than the others (one 64 MiB stripe: 20/50 0.062 ms with 3 tiles of
// 10 vs 0.056 with 4 of 8, 30/70 0.074 with 4 of 10 vs 0.091 with 5 of 8).
// 11-16 rows: 2 tiles of <= 8 (20/33: 0.031 ms, 4 tiles 0.035); 17-20 rows: 2
// tiles of 9-10 when the launch has units for >= 16 waves per CU (cfg4's
// 1024-stripe r = 20 decode: 0.469 ms, 3 tiles 0.475-0.48), else 4 tiles of 5
// (one 64 MiB 20/40 stripe: 0.044 ms, 2 tiles 0.053, 3 tiles 0.048).
// ZFEC_BSR_NW_WIDE: waves for r > 20 (default 4; the A/B knob of tools/ab_build.sh)
#ifndef ZFEC_BSR_NW_WIDE
#define ZFEC_BSR_NW_WIDE 4
#endif
void bsr_tiles(uint32_t r, uint64_t units, uint32_t* nw, uint32_t* rt) {
    if (r <= static_cast<uint32_t>(kBsrMaxRows))
        *nw = 1;
    else if (r <= 16 || (r <= 2u * kBsrMaxRows && units * 2 >= uint64_t(g_num_cu) * 16))
        *nw = 2;
    else
        *nw = ZFEC_BSR_NW_WIDE;
    *rt = (r + *nw - 1) / *nw;
}

bool bsr_shape_ok(uint32_t k, uint32_t r, uint64_t sz) {
    // kernel-argument form, or the table form past kBsrArgAddrs addresses
    return generic_mode() == 2 && k >= 1 && k <= static_cast<uint32_t>(kMaxIn) && r >= 1 &&
           r <= static_cast<uint32_t>(kBsrMaxOut) && sz >= kBsrChunk && k * r >= 24 && !(k <= 4 && r <= 8);
}

// Wide codes, one row tile: matapply_bsr_ks (table form).  Waves per unit:
// enough for ~8 waves per CU over the launch, 4-8, at least 4 inputs each.
constexpr uint32_t kBsrKsRows = 8;  // rows per group of the ks form past one tile
constexpr uint32_t kBsrTblTile = 8;

// The table form of the LDS-phase kernel (below) runs tiles of <= 8 rows in row
// groups of <= 8 tiles.  Round 4 used tiles of 4 for k > 64 in launches too
// small for 16 waves per CU; with the 8-wave groups sharing their inputs'
// combinations (bsr_cmb) a 4-row tile reads 30 LDS dwords per 4 rows and loses:
// 160/256 0.183 ms with tiles of 4 against 0.122 with 8 (profiles/r05_bsr_wide_ab.json).
//
// The ks form (inputs split over the waves of a workgroup) serves k > 32 with
// one row tile, and -- in row groups of 8, each re-reading the inputs -- launches
// of k >= 64 whose LDS-phase form would run fewer than 8 waves per CU (units x
// row groups x waves per group): 200/256 (164 units of 2 KiB per 64 MiB stripe,
// 1,312 waves) 0.082 ms on ks against 0.153, 96/128 (1,368 waves) 0.053 against
// 0.086; from there up the LDS-phase form wins: 160/256 (3,280 waves) 0.122,
// 64/112 (4,096) 0.070 -> 0.055, 128/256 0.121 (ks: 0.195 in round 4).
bool bsr_wide_ok(uint32_t k, uint32_t r, uint64_t sz, uint64_t nstripes) {
    if (generic_mode() != 2 || k <= static_cast<uint32_t>(kMaxIn) || k > static_cast<uint32_t>(kMaxWideIn) || r < 1 ||
        r > 256 || sz < kBsgChunk || k * r < 24)
        return false;
    if (r <= static_cast<uint32_t>(kBsrMaxRows)) return true;
    const uint64_t units = (sz + kBsrChunk - 1) / kBsrChunk * nstripes;
    const uint32_t ng = (r + 8 * kBsrTblTile - 1) / (8 * kBsrTblTile), rpg = (r + ng - 1) / ng;
    uint32_t nw = 1;  // as launch_bsr_tbl
    while (nw * kBsrTblTile < rpg) nw *= 2;
    return k >= 64 && units * ng * nw < uint64_t(g_num_cu) * 8;
}

struct BsrKsVariant {
    const void* fn = nullptr;
    char name[28] = "";
};
BsrKsVariant g_bsr_ks[kBsrMaxRows + 1];
std::once_flag g_bsr_ks_once;

template <int RT>
void fill_bsr_ks() {
    g_bsr_ks[RT].fn = reinterpret_cast<const void*>(matapply_bsr_ks<RT>);
    snprintf(g_bsr_ks[RT].name, sizeof g_bsr_ks[RT].name, "matapply_bsr<%d,ks,tbl>", RT);
    if constexpr (RT < kBsrMaxRows) fill_bsr_ks<RT + 1>();
}

hipError_t launch_bsr_wide(const ApplySpec& a, hipStream_t stream) {
    std::call_once(g_bsr_ks_once, [] { fill_bsr_ks<1>(); });
    uint64_t base = 0;
    if (bsr_routine_base(&base, stream) != hipSuccess) return hipErrorNotSupported;
    const uint32_t k = a.k, r = a.r;
    const uint32_t ng = r <= static_cast<uint32_t>(kBsrMaxRows) ? 1u : (r + kBsrKsRows - 1) / kBsrKsRows;
    const uint32_t rt = (r + ng - 1) / ng;
    const uint64_t cps = (a.sz + kBsrChunk - 1) / kBsrChunk;
    const uint64_t units = cps * a.nstripes * ng;
    if (units >= (1ull << 32) - (1ull << 24)) return hipErrorInvalidValue;
    // waves per unit: 8 when the launch has fewer than 2 units per CU, else 4
    // (>= 4 inputs per wave); 16 waves measured slower on 94/100 (0.027 ->
    // 0.031 ms per 64 MiB stripe) and the same on 255/256
    uint32_t nw = units * 2 < uint64_t(g_num_cu) * 4 ? 8u : 4u;
    while (nw > 1 && k / nw < 4) nw /= 2;
    BsrTblJob job;
    if (!bsr_tbl_ptrs(a, job)) return hipErrorNotSupported;
    BsrTblRef t;
    hipError_t e = bsr_addr_table(a, stream, base, ng, 1, rt, nw, &t);
    if (e != hipSuccess) return e;
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = k;
    job.r = r;
    job.ngroups = ng;
    job.pad_ = 0;
    const uint64_t cap = uint64_t(g_num_cu) * 1024;
    const uint32_t grid = static_cast<uint32_t>(units < cap ? units : cap);
    job.cps = static_cast<uint32_t>(cps);
    job.gs_s = static_cast<uint32_t>(grid / cps);
    job.gs_c = static_cast<uint32_t>(grid % cps);
    job.addr = t.dev;
    e = launch_job(g_bsr_ks[rt].fn, grid, 64 * nw, 0, stream, job);
    const hipError_t te = bsr_table_done(t, stream);  // also when the launch failed: the upload is a reader
    if (e != hipSuccess) return e;
    t_last_kernel = g_bsr_ks[rt].name;
    return te;
}

// Table form of the LDS-phase kernel: k > 32 with more than one row tile, or
// more rows than 4 tiles of 10.  Tiles of <= 8 rows (<= 127 VGPRs: 4 waves per
// SIMD), <= 8 waves per workgroup, so row groups of <= 64 rows; each group's
// workgroups read the unit's inputs again (L2 when they run together).
bool bsr_tbl_ok(uint32_t k, uint32_t r, uint64_t sz) {
    return generic_mode() == 2 && k >= 1 && k <= static_cast<uint32_t>(kMaxWideIn) && r >= 1 && r <= 256 &&
           sz >= kBsgChunk && k * r >= 24 && !(k <= 4 && r <= 8) &&
           (k > static_cast<uint32_t>(kMaxIn) ? r > static_cast<uint32_t>(kBsrMaxRows) : r > 4u * kBsrMaxRows);
}

struct BsrTblVariant {
    const void* fn = nullptr;
    const void* fn_cmb = nullptr;
    char name[28] = "";
    char name_cmb[32] = "";
};
BsrTblVariant g_bsr_tbl[kBsrMaxRows + 1];
std::once_flag g_bsr_tbl_once;

template <int RT>
void fill_bsr_tbl() {
    g_bsr_tbl[RT].fn = reinterpret_cast<const void*>(matapply_bsr<RT, true, false, BsrTblJob>);
    g_bsr_tbl[RT].fn_cmb = reinterpret_cast<const void*>(matapply_bsr<RT, true, true, BsrTblJob>);
    snprintf(g_bsr_tbl[RT].name, sizeof g_bsr_tbl[RT].name, "matapply_bsr<%d,lds,tbl>", RT);
    snprintf(g_bsr_tbl[RT].name_cmb, sizeof g_bsr_tbl[RT].name_cmb, "matapply_bsr<%d,lds,tbl,cmb>", RT);
    if constexpr (RT < kBsrMaxRows) fill_bsr_tbl<RT + 1>();
}

// One table-form launch of the LDS-phase kernel: ng row groups of nw waves of
// <= rt rows each.
hipError_t launch_bsr_lds_tbl(const ApplySpec& a, hipStream_t stream, uint64_t base, uint32_t ng, uint32_t nw,
                              uint32_t rt) {
    std::call_once(g_bsr_tbl_once, [] { fill_bsr_tbl<1>(); });
    const uint32_t k = a.k, r = a.r;
    const uint64_t cps = (a.sz + kBsrChunk - 1) / kBsrChunk;
    const uint64_t vunits = cps * a.nstripes * ng;
    if (vunits >= (1ull << 32) - (1ull << 24) || rt < 1 || rt > static_cast<uint32_t>(kBsrMaxRows))
        return hipErrorInvalidValue;
    BsrTblJob job;
    if (!bsr_tbl_ptrs(a, job)) return hipErrorNotSupported;
    BsrTblRef t;
    hipError_t e = bsr_addr_table(a, stream, base, ng, nw, rt, 1, &t);
    if (e != hipSuccess) return e;
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = k;
    job.r = r;
    job.ngroups = ng;
    job.pad_ = 0;
    const uint64_t cap = uint64_t(g_num_cu) * 1024;
    const uint32_t grid = static_cast<uint32_t>(vunits < cap ? vunits : cap);
    job.cps = static_cast<uint32_t>(cps);
    job.gs_s = static_cast<uint32_t>(grid / cps);
    job.gs_c = static_cast<uint32_t>(grid % cps);
    job.addr = t.dev;
    const bool cmb = bsr_cmb(nw);
    e = launch_job(cmb ? g_bsr_tbl[rt].fn_cmb : g_bsr_tbl[rt].fn, grid, 64 * nw, bsr_lds_bytes(k, nw, cmb), stream, job);
    const hipError_t te = bsr_table_done(t, stream);  // also when the launch failed: the upload is a reader
    if (e != hipSuccess) return e;
    t_last_kernel = cmb ? g_bsr_tbl[rt].name_cmb : g_bsr_tbl[rt].name;
    return te;
}

hipError_t launch_bsr_tbl(const ApplySpec& a, hipStream_t stream) {
    uint64_t base = 0;
    if (bsr_routine_base(&base, stream) != hipSuccess) return hipErrorNotSupported;
    const uint32_t r = a.r, tile = kBsrTblTile;
    const uint32_t ng = (r + 8 * tile - 1) / (8 * tile);  // row groups of <= 8 waves
    const uint32_t rpg = (r + ng - 1) / ng;            // rows of the largest group
    uint32_t nw = 1;                                   // 1, 2, 4 or 8 waves: see bsr_tiles
    while (nw * tile < rpg) nw *= 2;
    return launch_bsr_lds_tbl(a, stream, base, ng, nw, (rpg + nw - 1) / nw);
}

// ZFEC_BSR_NO_A32 (A/B knob, tools/ab_build.sh; 1 = off): 0 puts launches of
// 433-866 addresses on the 32-bit argument form.  It lost: K=20/M=60's 40-row
// encode 0.69 -> 0.74 ms back to back (each address needs its 64-bit SGPR pair
// assembled: ~20 more scalar instructions per input and wave), and its first
// launches of new matrices too (profiles/r06_bsr_a32_ab.json); the table form
// stays, its upload written by a kernel (bsr_table_write).
#ifndef ZFEC_BSR_NO_A32
#define ZFEC_BSR_NO_A32 1
#endif

// The LDS-phase kernel in its 32-bit argument form (BsrJob32): one row group of
// nw waves of rt rows.
hipError_t launch_bsr_a32(const ApplySpec& a, hipStream_t stream, uint64_t base, uint32_t nw, uint32_t rt,
                          uint64_t units, uint64_t cps) {
    const uint32_t k = a.k, r = a.r;
    BsrJob32 job;
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = k;
    job.r = r;
    job.ngroups = 1;
    job.addr_hi = static_cast<uint32_t>(base >> 32);
    for (uint32_t j = 0; j < k; ++j) job.ptr[j] = a.in[j];
    for (uint32_t i = 0; i < r; ++i) job.ptr[k + i] = a.out[i];
    thread_local std::vector<uint64_t> full;
    full.resize(size_t(nw) * k * rt);
    if (!fill_bsr_addrs(full.data(), a, base, 1, nw, rt, 1)) return hipErrorInvalidValue;
    for (size_t i = 0; i < full.size(); ++i) job.addr[i] = static_cast<uint32_t>(full[i]);
    const uint64_t cap = uint64_t(g_num_cu) * 1024;
    const uint32_t grid = static_cast<uint32_t>(units < cap ? units : cap);
    job.cps = static_cast<uint32_t>(cps);
    job.gs_s = static_cast<uint32_t>(grid / cps);
    job.gs_c = static_cast<uint32_t>(grid % cps);
    const bool cmb = bsr_cmb(nw);
    t_last_kernel = cmb ? g_bsr_var[rt].name_a32_cmb : g_bsr_var[rt].name_a32;
    return launch_job(cmb ? g_bsr_var[rt].fn_a32_cmb : g_bsr_var[rt].fn_a32, grid, 64 * nw,
                      bsr_lds_bytes(k, nw, cmb), stream, job);
}

hipError_t launch_bsr(const ApplySpec& a, hipStream_t stream) {
    std::call_once(g_bsr_once, [] { fill_bsr<1>(); });
    uint64_t base = 0;
    if (bsr_routine_base(&base, stream) != hipSuccess) return hipErrorNotSupported;
    const uint32_t k = a.k, r = a.r;
    const uint64_t cps = (a.sz + kBsrChunk - 1) / kBsrChunk;
    const uint64_t units = cps * a.nstripes;
    uint32_t nw, rt;
    bsr_tiles(r, units, &nw, &rt);
    if (units >= (1ull << 32) - (1ull << 24)) return hipErrorInvalidValue;
    // more addresses than the arguments hold as 64-bit values (e.g. K=20/M=60's
    // 40-row encode, 800): their low halves in the arguments (BsrJob32) when
    // they fit and the routine table's high half is one value; else the same
    // kernel reading them from a device-side table
    if (size_t(nw) * k * rt > static_cast<size_t>(kBsrArgAddrs)) {
        const uint64_t top = base + uint64_t(kBsrSlotStride ? kBsrSlotStride * kBsrMaxRows : kBsrSetBase * 2);
#if !ZFEC_BSR_NO_A32
        if (nw > 1 && size_t(nw) * k * rt <= static_cast<size_t>(kBsr32Addrs) && k + r <= uint32_t(kBsr32Ptrs) &&
            (base >> 32) == (top >> 32))
            return launch_bsr_a32(a, stream, base, nw, rt, units, cps);
#else
        (void)top;
#endif
        return launch_bsr_lds_tbl(a, stream, base, 1, nw, rt);
    }
    BsrJob job;
    job.sz = a.sz;
    job.in_sstride = a.in_sstride;
    job.out_sstride = a.out_sstride;
    job.nstripes = static_cast<uint32_t>(a.nstripes);
    job.k = k;
    job.r = r;
    job.nt = nw;
    job.pad_ = 0;
    for (uint32_t j = 0; j < k; ++j) job.in[j] = a.in[j];
    for (uint32_t i = 0; i < r; ++i) job.out[i] = a.out[i];
    if (!fill_bsr_addrs(job.addr, a, base, 1, nw, rt, 1)) return hipErrorInvalidValue;
    const uint64_t cap = uint64_t(g_num_cu) * 1024;
    const uint32_t grid = static_cast<uint32_t>(units < cap ? units : cap);
    job.cps = static_cast<uint32_t>(cps);
    job.gs_s = static_cast<uint32_t>(grid / cps);
    job.gs_c = static_cast<uint32_t>(grid % cps);
    if (nw == 1) {  // one row tile: one wave per unit, no LDS
        t_last_kernel = g_bsr_var[rt].name_solo;
        return launch_job(g_bsr_var[rt].fn_solo, grid, 64, 0, stream, job);
    }
    const bool cmb = bsr_cmb(nw);
    t_last_kernel = cmb ? g_bsr_var[rt].name_cmb : g_bsr_var[rt].name;
    return launch_job(cmb ? g_bsr_var[rt].fn_cmb : g_bsr_var[rt].fn, grid, 64 * nw, bsr_lds_bytes(k, nw, cmb), stream,
                      job);
}

}  // namespace

int generic_mode() {
    int g = g_generic.load();
    if (g < 0) {
        const char* e = getenv("ZFEC_HIP_GENERIC");
        g = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 2;
        int expect = -1;
        if (!g_generic.compare_exchange_strong(expect, g)) g = expect;  // set_generic_mode won the race
    }
    return g;
}

void set_generic_mode(int mode) { g_generic.store(mode < 0 ? 0 : mode > 2 ? 2 : mode); }

const char* matapply_variant_name(uint32_t k, uint32_t r, bool accumulate) {
    if (!accumulate && k >= 1 && k <= static_cast<uint32_t>(kRegK) && r >= 1 && r <= static_cast<uint32_t>(kRegR))
        return kRegNames[k][r];
    return pick_lds(k, r, accumulate).name;
}

const char* matapply_last_kernel() { return t_last_kernel; }

void matapply_request_signal(uint32_t* flag_dev, uint32_t seq) {
    t_signal_flag = flag_dev;
    t_signal_seq = seq;
}

bool matapply_signal_used() { return t_signal_used; }

// Whether `stream` is being captured into a HIP graph.  The table forms read a
// device-side table the host fills (and reuses) at enqueue time: a captured
// graph would replay its copy from a host slot rewritten since, and the bsr
// address cache would hold a slot whose upload never ran (the copy is only
// recorded).  Under capture those forms decline (hipErrorNotSupported) and a
// kernel whose whole description travels in its arguments takes the launch.
bool stream_capturing(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

bool wide_launch_ok(uint32_t k, uint32_t r, uint64_t sz, uint64_t nstripes) {
    // (forced) a specialised kernel of the whole matrix
    if (jit_mode() == kJitForce && sz >= static_cast<uint64_t>(kBsChunk) && k * r <= kJitMaxCoef) return true;
    // launches too small to fill the chip: matapply_small's passes of 32 inputs
    // (a wave per output row, every input load in flight at once) beat one
    // matapply_bsg launch walking all inputs in phases of 2
    if ((sz + 7) / 8 * nstripes < config().small_lanes) return false;
    return bsg_shape_ok(k, r, sz);  // matapply_bsg's table form
}

hipError_t launch_apply(const ApplySpec& a, hipStream_t stream) {
    uint32_t* const sig = t_signal_flag;  // a request covers this launch only
    t_signal_flag = nullptr;
    t_signal_used = false;
    std::call_once(g_dispatch_once, init_dispatch);
    const uint32_t k = a.k, r = a.r;
    const bool wide = k > static_cast<uint32_t>(kMaxIn);
    if (k == 0 || r == 0 || a.nstripes == 0 || a.sz == 0 || a.nstripes >= (1ull << 32) || a.coef_stride < k ||
        k > static_cast<uint32_t>(kMaxWideIn) || r > (wide ? 256u : static_cast<uint32_t>(kMaxOut)))
        return hipErrorInvalidValue;
    if (!wide && k * r > static_cast<uint32_t>(kMaxCoef)) return hipErrorInvalidValue;
    if (!a.accumulate) {  // a run-time specialised bit-sliced kernel, where one applies and is compiled
        const char* jit_name = nullptr;
        const hipError_t je = launch_matapply_jit(a, stream, &jit_name);
        if (je == hipSuccess) {
            t_last_kernel = jit_name;
            return hipSuccess;
        }
        if (je != hipErrorNotSupported && je != hipErrorNotReady) return je;
    }
    const bool reg = k <= static_cast<uint32_t>(kRegK) && r <= static_cast<uint32_t>(kRegR);
    if (wide) {
        if (a.accumulate || !bsg_shape_ok(k, r, a.sz)) return hipErrorNotSupported;
        // matapply_bsr, or matapply_bsg where it declines (hipErrorNotSupported:
        // a table past its ring slot, or no routine table on this device)
        hipError_t e = hipErrorNotSupported;
        if (bsr_wide_ok(k, r, a.sz, a.nstripes))
            e = launch_bsr_wide(a, stream);
        else if (bsr_tbl_ok(k, r, a.sz))
            e = launch_bsr_tbl(a, stream);
        if (e != hipErrorNotSupported) return e;
        return launch_bsg(a, stream);
    }
    const Config& cfg = config();
    if (!reg && (a.sz + 7) / 8 * a.nstripes < cfg.small_lanes) {
        MatJob job;
        fill_matjob(a, job);
        fill_coef(a, job);
        const hipError_t se = launch_small(job, stream);
        if (se != hipErrorNotSupported) {
            t_last_kernel = "matapply_small";
            return se;
        }
    }
    if (!a.accumulate) {
        hipError_t e = hipErrorNotSupported;
        if (bsr_shape_ok(k, r, a.sz))
            e = launch_bsr(a, stream);
        else if (bsr_tbl_ok(k, r, a.sz))
            e = launch_bsr_tbl(a, stream);
        if (e != hipErrorNotSupported) return e;
    }
    if (!a.accumulate && bsg_shape_ok(k, r, a.sz)) {
        const hipError_t e = launch_bsg(a, stream);
        if (e != hipErrorNotSupported) return e;  // (its table form declines under graph capture)
    }
    if (reg && !a.accumulate) return g_reg_launch[k][r](a, stream, sig);
    return launch_lds(a, stream);
}

hipError_t launch_one(const ApplySpec& a, hipStream_t stream, uint32_t* flag_dev, uint32_t seq,
                      const uint8_t* const* host_in, uint64_t host_sz) {
    static const char* const kOneNames[2][5] = {
        {"", "matapply_one<1>", "matapply_one<2>", "matapply_one<3>", "matapply_one<4>"},
        {"", "matapply_one<1,inline>", "matapply_one<2,inline>", "matapply_one<3,inline>", "matapply_one<4,inline>"}};
    if (a.k < 1 || a.k > 4 || a.r < 1 || a.r > 8 || a.nstripes != 1 || a.sz == 0 || a.sz % 16 || a.sz > 4096 ||
        a.accumulate || a.coef_stride < a.k)
        return hipErrorInvalidValue;
    t_signal_flag = nullptr;  // an unconsumed launch_apply request must not outlive this launch
    t_signal_used = false;
    const uint32_t units = static_cast<uint32_t>(a.sz / 16);
    // host_in: the caller has NOT copied the inputs anywhere the kernel can
    // read; they must fit the argument block, or the launch is refused (no
    // fallback to the bounce-buffer form, which would read stale memory)
    const bool inl = host_in != nullptr;
    if (inl && !one_inline_fits(a.k, a.sz, host_sz)) return hipErrorInvalidValue;
    thread_local OneJobInline big;  // ~5 KiB: not on the stack of every call
    OneJob& job = big.job;
    std::memset(&job, 0, sizeof job);
    for (uint32_t j = 0; j < a.k; ++j) job.in[j] = a.in[j];
    for (uint32_t i = 0; i < a.r; ++i) job.out[i] = a.out[i];
    job.done_flag = flag_dev;
    job.done_seq = seq;
    job.units = units;
    job.r = a.r;
    for (uint32_t i = 0; i < a.r; ++i)
        for (uint32_t j = 0; j < a.k; ++j) {
            const uint32_t* w = &kHostBank.w[uint32_t(a.coef[size_t(i) * a.coef_stride + j]) * 8];
            std::memcpy(&job.tab[(i * a.k + j) * 5], w, 5 * sizeof(uint32_t));
        }
    typedef void (*OneFn)(const OneJob);
    typedef void (*OneInlFn)(const OneJobInline);
    static const OneFn kOne[5] = {nullptr, matapply_one<1, false, OneJob>, matapply_one<2, false, OneJob>,
                                  matapply_one<3, false, OneJob>, matapply_one<4, false, OneJob>};
    static const OneInlFn kOneInl[5] = {nullptr, matapply_one<1, true, OneJobInline>,
                                        matapply_one<2, true, OneJobInline>, matapply_one<3, true, OneJobInline>,
                                        matapply_one<4, true, OneJobInline>};
    t_last_kernel = kOneNames[inl ? 1 : 0][a.k];
    if (!inl) return launch_job(reinterpret_cast<const void*>(kOne[a.k]), 1, kBlock, 0, stream, job);
    // the caller's host blocks, each padded with zeros to its whole units
    uint8_t* d = reinterpret_cast<uint8_t*>(big.data);
    for (uint32_t j = 0; j < a.k; ++j) {
        std::memcpy(d + size_t(j) * units * 16, host_in[j], host_sz);
        std::memset(d + size_t(j) * units * 16 + host_sz, 0, size_t(units) * 16 - host_sz);
    }
    return launch_job(reinterpret_cast<const void*>(kOneInl[a.k]), 1, kBlock, 0, stream, big);
}

hipError_t launch_apply_pair(const ApplySpec& x, const ApplySpec& y, hipStream_t stream) {
    std::call_once(g_dispatch_once, init_dispatch);
    static std::once_flag names_once;
    std::call_once(names_once, [] {
        for (int k = 1; k <= kRegK; ++k)
            for (int ra = 1; ra <= kRegR; ++ra)
                for (int rb = 1; rb <= kRegR; ++rb)
                    snprintf(g_pair_names[k][ra][rb], sizeof g_pair_names[k][ra][rb], "matapply_pair<%d,%d,%d>", k,
                             ra, rb);
    });
    // the shapes launch_apply runs on matapply_reg (not matapply_rows, not a
    // forced JIT kernel), each within one launch
    auto reg_shape = [](const ApplySpec& a) {
        return !a.accumulate && a.k >= 1 && a.k <= static_cast<uint32_t>(kRegK) && a.r >= 1 &&
               a.r <= static_cast<uint32_t>(kRegR) && a.sz > 0 && a.nstripes > 0 && a.nstripes < (1ull << 32) &&
               a.coef_stride >= a.k && !rows_shape(a);
    };
    if (x.k != y.k || !reg_shape(x) || !reg_shape(y) || jit_mode() == kJitForce) return hipErrorNotSupported;
    const ApplySpec& a = x.r >= y.r ? x : y;
    const ApplySpec& b = x.r >= y.r ? y : x;
    const PairLaunch f = g_pair_launch[a.k][a.r][b.r];
    if (!f) return hipErrorNotSupported;
    t_signal_flag = nullptr;
    t_signal_used = false;
    return f(a, b, stream);
}

}  // namespace zfec_hip
