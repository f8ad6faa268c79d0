// kernels.hip -- GF(2^8) matrix-apply kernels for gfx950 (MI355X, CDNA4).
//
// The hot loop of zfec is _addmul1 (zfec/fec.c:170-204): dst[i] ^= c*src[i]
// by a 256-byte table row per coefficient, driven by fec_encode
// (fec.c:487-505) and fec_decode (fec.c:527-557).  Here one kernel reads each
// input chunk from HBM once and produces every requested output from it:
//
//   * each lane owns a 16-byte column slice (one global_load_dwordx4 per input
//     block, 1 KiB coalesced per wave);
//   * the GF multiply is table-free in memory: multiplication by a constant c
//     is GF(2)-linear, so c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6] with
//     three 8/8/4-entry byte tables, and v_perm_b32 looks up four bytes at
//     once from an 8-byte table held in two VGPRs;
//   * the three partial products and the accumulator are merged by
//     v_bitop3_b32 (gfx950's 3-input logic op, truth table 0x96 = XOR3);
//   * the per-coefficient tables (5 dwords) are built once per workgroup in
//     LDS from the raw coefficients, then either hoisted into VGPRs for the
//     whole launch (small k*r, `matapply_reg`) or read per use with
//     wave-uniform (broadcast, conflict-free) LDS reads (`matapply_lds`).
//
// Per input byte this costs ~(5 + 4.5*r)/4 VALU ops and m/k bytes of HBM
// traffic; at K=3/M=10 that is ~9 ops per input byte, far under the VALU
// budget at the HBM roofline, so the kernels are bandwidth-bound there.
#include "kernels.hpp"

#include <hip/hip_runtime.h>

#include <mutex>

namespace zfec_hip {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// v_perm_b32: byte i of the result = byte sel_i of the 8-byte value {hi:lo}
// (selector 0-3 -> lo, 4-7 -> hi).
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

__device__ __forceinline__ uint32_t xtime(uint32_t v) {
    v <<= 1;
    return (v & 0x100u) ? (v ^ 0x11Du) : v;
}

// Tables for multiplication by c (one byte):
//   t0 = c*{0..7}          (bits 0-2 of x)   -> t[0] (entries 0-3), t[1] (4-7)
//   t1 = c*{0,8,..,56}     (bits 3-5 of x)   -> t[2], t[3]
//   t2 = c*{0,64,128,192}  (bits 6-7 of x)   -> t[4]
__device__ inline void make_tables(uint32_t c, uint32_t t[5]) {
    uint32_t p[8];
    p[0] = c;
#pragma unroll
    for (int i = 1; i < 8; ++i) p[i] = xtime(p[i - 1]);
    auto e3 = [&](int n, int b) -> uint32_t {
        return ((n & 1) ? p[b] : 0u) ^ ((n & 2) ? p[b + 1] : 0u) ^ ((n & 4) ? p[b + 2] : 0u);
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        t[2 * h + 0] = e3(0, 3 * h) | (e3(1, 3 * h) << 8) | (e3(2, 3 * h) << 16) | (e3(3, 3 * h) << 24);
        t[2 * h + 1] = e3(4, 3 * h) | (e3(5, 3 * h) << 8) | (e3(6, 3 * h) << 16) | (e3(7, 3 * h) << 24);
    }
    t[4] = (p[6] << 8) | (p[7] << 16) | ((p[6] ^ p[7]) << 24);
}

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
    return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// acc ^ c*x for four bytes: 3 v_perm_b32 + 2 v_bitop3_b32.
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, const uint32_t t[5], Sel s) {
    const uint32_t a = perm(t[1], t[0], s.s0);
    const uint32_t b = perm(t[3], t[2], s.s1);
    const uint32_t d = perm(t[4], t[4], s.s2);
    return xor3(xor3(acc, a, b), d, 0u);
}

// Partial-chunk helpers for the last (sz % 16) bytes of a block.
__device__ inline u32x4 load_tail(const uint8_t* p, uint32_t nb) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t b = 0; b < nb; ++b) w[b >> 2] |= static_cast<uint32_t>(p[b]) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ inline void store_tail(uint8_t* p, u32x4 v, uint32_t nb) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t b = 0; b < nb; ++b) p[b] = static_cast<uint8_t>(w[b >> 2] >> (8 * (b & 3)));
}

__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);  // global_load_dwordx4; unaligned addresses are legal on gfx950
    return v;
}

__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) { __builtin_memcpy(p, &v, 16); }

// Walks this lane's (stripe, chunk) units in grid-stride order without a
// division per step.
struct UnitIter {
    uint32_t s, c;
    __device__ UnitIter(const MatJob& job) {
        const uint32_t gid = blockIdx.x * kBlock + threadIdx.x;
        s = gid / job.cps;
        c = gid - s * job.cps;
    }
    __device__ __forceinline__ void next(const MatJob& job) {
        c += job.gs_c;
        s += job.gs_s;
        if (c >= job.cps) {
            c -= job.cps;
            ++s;
        }
    }
};

// ---------------------------------------------------------------------------
// Variant 1: compile-time k = K and r = R, tables hoisted into VGPRs.
// ---------------------------------------------------------------------------
template <int K, int R>
__global__ __launch_bounds__(kBlock) void matapply_reg(const MatJob job) {
    __shared__ uint32_t lds_tab[K * R * 5];
    for (int i = threadIdx.x; i < K * R; i += kBlock) {
        uint32_t t[5];
        make_tables(job.coef[i], t);
#pragma unroll
        for (int q = 0; q < 5; ++q) lds_tab[i * 5 + q] = t[q];
    }
    __syncthreads();
    uint32_t T[R][K][5];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int q = 0; q < 5; ++q) T[r][j][q] = lds_tab[(r * K + j) * 5 + q];

    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    for (UnitIter u(job); u.s < job.nstripes; u.next(job)) {
        const uint64_t off = static_cast<uint64_t>(u.c) * kChunk;
        const uint64_t ib = u.s * job.in_sstride + off;
        const uint64_t ob = u.s * job.out_sstride + off;
        const bool full = u.c < nfull;
        const uint32_t nb = full ? kChunk : static_cast<uint32_t>(sz - off);
        u32x4 x[K];
        if (full) {
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + ib);
        } else {
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = load_tail(job.in[j] + ib, nb);
        }
        Sel sel[K][4];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            sel[j][0] = selectors(x[j].x);
            sel[j][1] = selectors(x[j].y);
            sel[j][2] = selectors(x[j].z);
            sel[j][3] = selectors(x[j].w);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t a[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < K; ++j)
#pragma unroll
                for (int v = 0; v < 4; ++v) a[v] = gf_mac(a[v], T[r][j], sel[j][v]);
            const u32x4 y{a[0], a[1], a[2], a[3]};
            if (full)
                store16(job.out[r] + ob, y);
            else
                store_tail(job.out[r] + ob, y, nb);
        }
    }
}

// ---------------------------------------------------------------------------
// Variant 2: runtime r (<= kMaxOut, in passes of RT rows); k compile-time
// (KT > 0, inputs stay in VGPRs across passes) or runtime (KT == 0, inputs are
// re-read per pass from L1/L2).  Tables stay in LDS and are read with
// wave-uniform addresses.  ACC: XOR into the existing output (k > kMaxIn).
// ---------------------------------------------------------------------------
constexpr int RT = 8;

template <int KT, bool ACC>
__global__ __launch_bounds__(kBlock) void matapply_lds(const MatJob job) {
    __shared__ u32x4 lds_a[kMaxCoef];   // t0lo t0hi t1lo t1hi
    __shared__ uint32_t lds_b[kMaxCoef];  // t2
    const uint32_t k = KT > 0 ? static_cast<uint32_t>(KT) : job.k;
    const uint32_t r = job.r;
    const uint32_t rpad = (r + RT - 1) / RT * RT;
    for (uint32_t i = threadIdx.x; i < rpad * k; i += kBlock) {
        uint32_t t[5];
        make_tables(i < r * k ? job.coef[i] : 0u, t);
        lds_a[i] = u32x4{t[0], t[1], t[2], t[3]};
        lds_b[i] = t[4];
    }
    __syncthreads();

    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    for (UnitIter u(job); u.s < job.nstripes; u.next(job)) {
        const uint64_t off = static_cast<uint64_t>(u.c) * kChunk;
        const uint64_t ib = u.s * job.in_sstride + off;
        const uint64_t ob = u.s * job.out_sstride + off;
        const bool full = u.c < nfull;
        const uint32_t nb = full ? kChunk : static_cast<uint32_t>(sz - off);

        u32x4 xk[KT > 0 ? KT : 1];
        if constexpr (KT > 0) {
#pragma unroll
            for (int j = 0; j < KT; ++j) xk[j] = full ? load16(job.in[j] + ib) : load_tail(job.in[j] + ib, nb);
        }
        for (uint32_t rb = 0; rb < rpad; rb += RT) {
            uint32_t a[RT][4];
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) a[rr][0] = a[rr][1] = a[rr][2] = a[rr][3] = 0u;
#pragma unroll 2
            for (uint32_t j = 0; j < k; ++j) {
                u32x4 x;
                if constexpr (KT > 0)
                    x = xk[j];
                else
                    x = full ? load16(job.in[j] + ib) : load_tail(job.in[j] + ib, nb);
                const Sel s[4] = {selectors(x.x), selectors(x.y), selectors(x.z), selectors(x.w)};
#pragma unroll
                for (int rr = 0; rr < RT; ++rr) {
                    const uint32_t idx = (rb + rr) * k + j;
                    const u32x4 ta = lds_a[idx];
                    const uint32_t t[5] = {ta.x, ta.y, ta.z, ta.w, lds_b[idx]};
#pragma unroll
                    for (int v = 0; v < 4; ++v) a[rr][v] = gf_mac(a[rr][v], t, s[v]);
                }
            }
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) {
                if (rb + rr >= r) break;
                uint8_t* op = job.out[rb + rr] + ob;
                u32x4 y{a[rr][0], a[rr][1], a[rr][2], a[rr][3]};
                if constexpr (ACC) y ^= full ? load16(op) : load_tail(op, nb);
                if (full)
                    store16(op, y);
                else
                    store_tail(op, y, nb);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Dispatch
// ---------------------------------------------------------------------------
typedef void (*KernelFn)(const MatJob);

struct Variant {
    KernelFn fn;
    const char* name;
    int max_blocks_per_cu;  // from the occupancy API, cached
};

template <int K, int R>
Variant make_reg() {
    return Variant{matapply_reg<K, R>, "matapply_reg", 0};
}

// Register-table variants: k <= 4, r <= 8 and k*r <= 24 (<= 120 table VGPRs).
constexpr int kRegK = 4, kRegR = 8;
Variant g_reg[kRegK + 1][kRegR + 1];
Variant g_lds_k0, g_lds_k0_acc;
std::once_flag g_dispatch_once;
int g_num_cu = 0;

template <int K>
void fill_reg_row() {
    g_reg[K][1] = make_reg<K, 1>();
    g_reg[K][2] = make_reg<K, 2>();
    g_reg[K][3] = make_reg<K, 3>();
    g_reg[K][4] = make_reg<K, 4>();
    g_reg[K][5] = make_reg<K, 5>();
    g_reg[K][6] = make_reg<K, 6>();
    if constexpr (K * 7 <= 24) g_reg[K][7] = make_reg<K, 7>();
    if constexpr (K * 8 <= 24) g_reg[K][8] = make_reg<K, 8>();
}

void init_dispatch() {
    fill_reg_row<1>();
    fill_reg_row<2>();
    fill_reg_row<3>();
    fill_reg_row<4>();
    g_lds_k0 = Variant{matapply_lds<0, false>, "matapply_lds<k>", 0};
    g_lds_k0_acc = Variant{matapply_lds<0, true>, "matapply_lds<k,acc>", 0};
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) g_num_cu = prop.multiProcessorCount;
    }
    if (g_num_cu <= 0) g_num_cu = 256;
}

Variant* pick(uint32_t k, uint32_t r, bool acc) {
    std::call_once(g_dispatch_once, init_dispatch);
    if (acc) return &g_lds_k0_acc;
    if (k >= 1 && k <= static_cast<uint32_t>(kRegK) && r >= 1 && r <= static_cast<uint32_t>(kRegR) && g_reg[k][r].fn)
        return &g_reg[k][r];
    return &g_lds_k0;
}

}  // namespace

const char* matapply_variant_name(uint32_t k, uint32_t r, bool accumulate) {
    return pick(k, r, accumulate)->name;
}

hipError_t launch_matapply(MatJob& job, hipStream_t stream) {
    if (job.k == 0 || job.k > static_cast<uint32_t>(kMaxIn) || job.r == 0 || job.r > static_cast<uint32_t>(kMaxOut) ||
        job.r * job.k > static_cast<uint32_t>(kMaxCoef) || job.nstripes == 0 || job.sz == 0)
        return hipErrorInvalidValue;
    const uint64_t cps = (job.sz + kChunk - 1) / kChunk;
    const uint64_t total = cps * job.nstripes;
    if (total >= (1ull << 32) - 2ull * kBlock * 4096ull) return hipErrorInvalidValue;  // caller splits
    job.cps = static_cast<uint32_t>(cps);

    Variant* v = pick(job.k, job.r, job.accumulate != 0);
    if (v->max_blocks_per_cu == 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(v->fn), kBlock, 0) !=
                hipSuccess ||
            nb <= 0)
            nb = 1;
        v->max_blocks_per_cu = nb;
    }
    const uint64_t need = (total + kBlock - 1) / kBlock;
    const uint64_t cap = static_cast<uint64_t>(g_num_cu) * v->max_blocks_per_cu;
    const uint32_t grid = static_cast<uint32_t>(need < cap ? need : cap);
    const uint64_t gstride = static_cast<uint64_t>(grid) * kBlock;
    job.gs_s = static_cast<uint32_t>(gstride / cps);
    job.gs_c = static_cast<uint32_t>(gstride % cps);
    hipLaunchKernelGGL(v->fn, dim3(grid), dim3(kBlock), 0, stream, job);
    return hipGetLastError();
}

}  // namespace zfec_hip
