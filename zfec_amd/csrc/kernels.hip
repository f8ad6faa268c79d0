// kernels.hip -- GF(2^8) matrix-apply kernels for gfx950 (MI355X, CDNA4).
//
// The hot loop of zfec is _addmul1 (zfec/fec.c:170-204): dst[i] ^= c*src[i]
// through a 256-byte table row per coefficient, driven by fec_encode
// (fec.c:487-505) and fec_decode (fec.c:527-557).  Here one kernel reads each
// input chunk from HBM once and produces every requested output from it:
//
//   * each lane owns a 16-byte column slice of every block (one
//     global_load_dwordx4 per input block, 1 KiB coalesced per wave);
//   * multiplication by a constant c is GF(2)-linear, so
//       c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
//     with three 8/8/4-entry byte tables; v_perm_b32 looks up four bytes at
//     once in an 8-byte table held in a register pair;
//   * partial products are merged by v_bitop3_b32 (gfx950's 3-input logic
//     op; truth table 0x96 = XOR3);
//   * the tables of all 256 byte values are a compile-time bank in constant
//     memory (8 KiB); a wave-uniform coefficient becomes two scalar loads, so
//     tables live in SGPRs and never cost LDS bandwidth or VGPRs.
//
// Two shapes of kernel:
//   matapply_reg<K, R>  compile-time k <= 4 and r <= 8 (encode K=3/M=10 is
//                       <3,7>, its decode <3,3>): every table is loaded once
//                       per lane, the per-chunk body is straight-line code.
//   matapply_gen        any k <= 32, r <= 48: rows in register tiles of RT,
//                       inputs streamed in groups of G with loads one group
//                       ahead, tables fetched per use by scalar loads.
//
// Cost per input byte: 3 v_perm + ~1.5 v_bitop3 per output row / 4 bytes,
// i.e. ~9 VALU ops at K=3/M=10; the HBM roofline needs ~15 T ops/s of the
// chip's ~78 T, so the K=3/M=10 kernels are memory-bound (measured: they move
// bytes as fast as a copy kernel with the same load/store pattern).
#include "kernels.hpp"

#include <hip/hip_runtime.h>

#include <cstdlib>
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

// Host copy of the bank: launch_matapply places small launches' tables
// directly in the kernel arguments.
constexpr TableBank kHostBank = make_bank();

struct Tab {
    uint32_t w0, w1, w2, w3, w4;
};

__device__ __forceinline__ Tab table_of(uint32_t c) {
    const uint32_t* t = &g_bank.w[c * 8];
    return Tab{t[0], t[1], t[2], t[3], t[4]};
}

// Table of coefficient i (row-major r x k) from the kernel arguments.
__device__ __forceinline__ Tab karg_table(const MatJob& job, uint32_t i) {
    const uint32_t* t = &job.tab[i * 5];
    return Tab{t[0], t[1], t[2], t[3], t[4]};
}

// Byte i of the kernarg coefficient array, fetched as a scalar dword.
__device__ __forceinline__ uint32_t coef_at(const MatJob& job, uint32_t i) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(job.coef)[i >> 2];
    return (w >> (8 * (i & 3))) & 0xFFu;
}

// ---- arithmetic ---------------------------------------------------------------

struct Sel {
    uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel selectors(uint32_t x) {
    return Sel{x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u};
}

// acc ^ c*x for four bytes: 3 v_perm_b32 + 2 v_bitop3_b32.
__device__ __forceinline__ uint32_t gf_mac(uint32_t acc, const Tab& t, Sel s) {
    const uint32_t a = perm(t.w1, t.w0, s.s0);
    const uint32_t b = perm(t.w3, t.w2, s.s1);
    const uint32_t d = perm(t.w4, t.w4, s.s2);
    return xor3(xor3(acc, a, b), d, 0u);
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
// division per step.
struct UnitIter {
    uint32_t s, c;
    __device__ explicit UnitIter(const MatJob& job) {
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
// matapply_reg<K, R>: compile-time k and r.  All K*R tables come with the
// kernel arguments (prefetched scalar loads); the compiler keeps the high
// words in SGPRs and copies the low words to VGPRs once, outside the loop.
// ---------------------------------------------------------------------------
// One (stripe, chunk) unit: load K x 16 bytes, store R x 16 bytes.
template <int K, int R, bool NT>
__device__ __forceinline__ void reg_compute_store(const MatJob& job, const Tab (&T)[R][K], const u32x4 (&x)[K],
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
        const u32x4 y{gf_dot<K>(T[r], sel[0]), gf_dot<K>(T[r], sel[1]), gf_dot<K>(T[r], sel[2]),
                      gf_dot<K>(T[r], sel[3])};
        if (full)
            store16_out<NT>(job.out[r] + ob, y);
        else
            store_tail(job.out[r] + ob, y, nb);
    }
}

template <int K>
__device__ __forceinline__ void reg_load(const MatJob& job, u32x4 (&x)[K], uint64_t ib, bool full, uint32_t nb) {
    if (full) {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + ib);
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load_tail(job.in[j] + ib, nb);
    }
}

// U: units per lane per loop trip (U = 2 puts 2K loads in flight per lane).
template <int K, int R, bool NT, int U = 1>
__global__ __launch_bounds__(kBlock) void matapply_reg(const MatJob job) {
    Tab T[R][K];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j) T[r][j] = karg_table(job, r * K + j);

    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    UnitIter u(job);
    while (u.s < job.nstripes) {
        uint64_t ib[U], ob[U];
        uint32_t nb[U];
        bool full[U], live[U];
        u32x4 x[U][K];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            live[i] = u.s < job.nstripes;
            const uint64_t off = static_cast<uint64_t>(u.c) * kChunk;
            ib[i] = u.s * job.in_sstride + off;
            ob[i] = u.s * job.out_sstride + off;
            full[i] = u.c < nfull;
            nb[i] = full[i] ? kChunk : static_cast<uint32_t>(sz - off);
            if (live[i]) reg_load<K>(job, x[i], ib[i], full[i], nb[i]);
            u.next(job);
        }
#pragma unroll
        for (int i = 0; i < U; ++i)
            if (live[i]) reg_compute_store<K, R, NT>(job, T, x[i], ob[i], full[i], nb[i]);
    }
}

// ---------------------------------------------------------------------------
// matapply_gen: runtime k (<= kMaxIn) and r (<= kMaxOut).  Rows are produced
// in register tiles of RT; inside a tile the inputs stream through in groups
// of G blocks whose loads are issued one group ahead.  Each (row, input)
// table arrives by scalar loads: from the kernel arguments when k*r <=
// kMaxKernargTables (KTAB), else coefficient byte -> bank.  ACC: XOR into the
// existing output (continuation launches for k > kMaxIn).
// ---------------------------------------------------------------------------
constexpr int RT = 8;
constexpr int G = 4;

__device__ __forceinline__ void load_group(u32x4 (&x)[G], const MatJob& job, uint32_t g, uint32_t k, uint64_t ib,
                                           bool full, uint32_t nb) {
#pragma unroll
    for (int jj = 0; jj < G; ++jj) {
        const uint32_t j = g + jj;
        if (j < k)
            x[jj] = full ? load16(job.in[j] + ib) : load_tail(job.in[j] + ib, nb);
        else
            x[jj] = u32x4{0u, 0u, 0u, 0u};
    }
}

template <bool ACC, bool NT, bool KTAB>
__global__ __launch_bounds__(kBlock) void matapply_gen(const MatJob job) {
    const uint32_t k = job.k;
    const uint32_t r = job.r;
    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    for (UnitIter u(job); u.s < job.nstripes; u.next(job)) {
        const uint64_t off = static_cast<uint64_t>(u.c) * kChunk;
        const uint64_t ib = u.s * job.in_sstride + off;
        const uint64_t ob = u.s * job.out_sstride + off;
        const bool full = u.c < nfull;
        const uint32_t nb = full ? kChunk : static_cast<uint32_t>(sz - off);
        for (uint32_t rb = 0; rb < r; rb += RT) {
            uint32_t a[RT][4];
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) a[rr][0] = a[rr][1] = a[rr][2] = a[rr][3] = 0u;
            u32x4 xa[G];
            load_group(xa, job, 0, k, ib, full, nb);
            for (uint32_t g = 0; g < k; g += G) {
                u32x4 xb[G];
                load_group(xb, job, g + G, k, ib, full, nb);
#pragma unroll
                for (int jj = 0; jj < G; ++jj) {
                    const uint32_t j = g + jj;
                    if (j >= k) break;
                    const Sel s[4] = {selectors(xa[jj].x), selectors(xa[jj].y), selectors(xa[jj].z),
                                      selectors(xa[jj].w)};
#pragma unroll
                    for (int rr = 0; rr < RT; ++rr) {
                        const uint32_t row = rb + rr;
                        Tab t;
                        if constexpr (KTAB)
                            t = row < r ? karg_table(job, row * k + j) : table_of(0u);
                        else
                            t = table_of(row < r ? coef_at(job, row * k + j) : 0u);
#pragma unroll
                        for (int v = 0; v < 4; ++v) a[rr][v] = gf_mac(a[rr][v], t, s[v]);
                    }
                }
#pragma unroll
                for (int jj = 0; jj < G; ++jj) xa[jj] = xb[jj];
            }
#pragma unroll
            for (int rr = 0; rr < RT; ++rr) {
                if (rb + rr >= r) break;
                uint8_t* op = job.out[rb + rr] + ob;
                u32x4 y{a[rr][0], a[rr][1], a[rr][2], a[rr][3]};
                if constexpr (ACC) y ^= full ? load16(op) : load_tail(op, nb);
                if (full)
                    store16_out<NT>(op, y);
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
    bool kernarg_tables;    // the kernel reads job.tab[] instead of job.coef[]
    int units_per_lane = 1; // units a lane handles per loop trip (grid sizing)
};

// Register-table variants: k <= 4, r <= 8.
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
Variant g_reg[kRegK + 1][kRegR + 1];
Variant g_gen, g_gen_acc, g_gen_tab;
std::once_flag g_dispatch_once;
int g_num_cu = 0;
int g_grid_mult = 16;  // grid cap = CUs x resident blocks per CU x g_grid_mult

template <int K, int R>
void set_reg() {
    g_reg[K][R] = Variant{matapply_reg<K, R, true>, kRegNames[K][R], 0, true};
}

template <int K>
void fill_reg_row() {
    set_reg<K, 1>();
    set_reg<K, 2>();
    set_reg<K, 3>();
    set_reg<K, 4>();
    set_reg<K, 5>();
    set_reg<K, 6>();
    set_reg<K, 7>();
    set_reg<K, 8>();
}

void init_dispatch() {
    fill_reg_row<1>();
    fill_reg_row<2>();
    fill_reg_row<3>();
    fill_reg_row<4>();
    g_gen = Variant{matapply_gen<false, true, false>, "matapply_gen", 0, false};
    g_gen_tab = Variant{matapply_gen<false, true, true>, "matapply_gen<ktab>", 0, true};
    g_gen_acc = Variant{matapply_gen<true, false, false>, "matapply_gen<acc>", 0, false};
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) g_num_cu = prop.multiProcessorCount;
    }
    if (g_num_cu <= 0) g_num_cu = 256;
    if (const char* e = getenv("ZFEC_HIP_GRID_MULT")) g_grid_mult = atoi(e) > 0 ? atoi(e) : g_grid_mult;
}

Variant* pick(uint32_t k, uint32_t r, bool acc) {
    std::call_once(g_dispatch_once, init_dispatch);
    if (acc) return &g_gen_acc;
    if (k >= 1 && k <= static_cast<uint32_t>(kRegK) && r >= 1 && r <= static_cast<uint32_t>(kRegR)) return &g_reg[k][r];
    if (k * r <= static_cast<uint32_t>(kMaxKernargTables)) return &g_gen_tab;
    return &g_gen;
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
    if (total >= (1ull << 32) - (1ull << 24)) return hipErrorInvalidValue;  // the caller splits larger jobs
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
    // One 16-byte unit per lane up to 16x the resident capacity; beyond that a
    // grid-stride loop (the 64 MiB config fits in a single pass).
    const uint64_t lanes = (total + v->units_per_lane - 1) / v->units_per_lane;
    const uint64_t need = (lanes + kBlock - 1) / kBlock;
    const uint64_t cap = static_cast<uint64_t>(g_num_cu) * v->max_blocks_per_cu * g_grid_mult;
    const uint32_t grid = static_cast<uint32_t>(need < cap ? need : cap);
    const uint64_t gstride = static_cast<uint64_t>(grid) * kBlock;
    job.gs_s = static_cast<uint32_t>(gstride / cps);
    job.gs_c = static_cast<uint32_t>(gstride % cps);
    if (v->kernarg_tables && !job.tables) {  // idempotent: a job may be relaunched
        uint8_t c[kMaxKernargTables];
        const uint32_t n = job.k * job.r;
        for (uint32_t i = 0; i < n; ++i) c[i] = job.coef[i];
        for (uint32_t i = 0; i < n; ++i)
            for (int q = 0; q < 5; ++q) job.tab[i * 5 + q] = kHostBank.w[c[i] * 8 + q];
        job.tables = 1;
    }
    hipLaunchKernelGGL(v->fn, dim3(grid), dim3(kBlock), 0, stream, job);
    return hipGetLastError();
}

}  // namespace zfec_hip
