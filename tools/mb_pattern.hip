// mb_pattern.hip -- the K=20/M=60 encode's memory pattern (BASELINE cfg4:
// 1024 stripes of 20 input rows and 40 output rows of 52,429 bytes, rows
// 52,480 bytes apart, inputs [stripe][20][row] and outputs [stripe][40][row]
// in separate arrays), from cold caches, with no GF arithmetic: each unit
// loads its 20 input pieces, XORs them, stores 40 output pieces.  The
// bit-sliced JIT kernel gives each wave a 2 KiB piece of every row of a
// stripe per unit; its no-arithmetic probe (same loads and stores) took
// 623 us, 5.2 TB/s (profiles/r03_jit_probe.json).  Which piece length and
// walk order does HBM serve fastest?
//
//   wave<P>   one wave per unit of P bytes of every row (lanes 16 B apart,
//             P / 1024 instructions per row), units in (stripe, piece) order
//   split<P>  as wave<P>, the 40 output rows stored by the 4 waves of a
//             workgroup, 10 rows each, after all 4 waves loaded the unit's
//             inputs (the unit's input pieces read 4 times, mostly from L2)
//   rows      one 16-byte unit per lane (a 1 KiB piece per wave per row)
//   *_occ3    the same with 48 KiB of dynamic LDS per workgroup: at most 3
//             workgroups (12 waves) per CU, the JIT kernel's residency (156
//             VGPRs: 3 waves per SIMD) -- round 4: is the piece length or the
//             residency what separates wave1k from the JIT kernel?
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_pattern.hip -o tools/mb_pattern.exe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int K = 20, R = 40;
constexpr uint32_t kSz = 52429, kLd = 52480, kNs = 1024;

struct Set {
    const uint8_t* in;
    uint8_t* out;
};

__device__ __forceinline__ void st(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

// a wave per unit of P bytes; piece c of stripe s; lanes 16 B apart
template <int P>
__global__ __launch_bounds__(256) void wave_unit(Set s) {
    constexpr int I = P / 1024;  // 1 KiB instructions per row
    constexpr uint32_t cps = (kSz + P - 1) / P;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (wave >= cps * kNs) return;
    const uint32_t st_ = wave / cps, c = wave % cps;
    const uint8_t* ib = s.in + uint64_t(st_) * K * kLd;
    uint8_t* ob = s.out + uint64_t(st_) * R * kLd;
    u32x4 acc[I];
#pragma unroll
    for (int i = 0; i < I; ++i) acc[i] = u32x4{0u, 0u, 0u, 0u};
    // clamped (in-bounds) addresses: every load issued before the first wait
    uint32_t offc[I];
#pragma unroll
    for (int i = 0; i < I; ++i) offc[i] = min(c * P + i * 1024 + lane * 16, kLd - 16);
    u32x4 x[K][I];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < I; ++i) x[j][i] = *reinterpret_cast<const u32x4*>(ib + uint64_t(j) * kLd + offc[i]);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < I; ++i) acc[i] ^= x[j][i];
#pragma unroll 4
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t off = c * P + i * 1024 + lane * 16;
            if (off < kLd) st(ob + uint64_t(r) * kLd + off, acc[i] ^ uint32_t(r));
        }
}

// the 4 waves of a workgroup share one unit of P bytes: each wave loads the
// whole unit's inputs and stores 10 of the 40 output rows
template <int P>
__global__ __launch_bounds__(256) void split_unit(Set s) {
    constexpr int I = P / 1024;
    constexpr uint32_t cps = (kSz + P - 1) / P;
    const uint32_t unit = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (unit >= cps * kNs) return;
    const uint32_t st_ = unit / cps, c = unit % cps;
    const uint8_t* ib = s.in + uint64_t(st_) * K * kLd;
    uint8_t* ob = s.out + uint64_t(st_) * R * kLd;
    u32x4 acc[I];
#pragma unroll
    for (int i = 0; i < I; ++i) acc[i] = u32x4{0u, 0u, 0u, 0u};
    // clamped (in-bounds) addresses: every load issued before the first wait
    uint32_t offc[I];
#pragma unroll
    for (int i = 0; i < I; ++i) offc[i] = min(c * P + i * 1024 + lane * 16, kLd - 16);
    u32x4 x[K][I];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < I; ++i) x[j][i] = *reinterpret_cast<const u32x4*>(ib + uint64_t(j) * kLd + offc[i]);
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < I; ++i) acc[i] ^= x[j][i];
#pragma unroll
    for (int q = 0; q < R / 4; ++q) {
        const int r = w * (R / 4) + q;
#pragma unroll
        for (int i = 0; i < I; ++i) {
            const uint32_t off = c * P + i * 1024 + lane * 16;
            if (off < kLd) st(ob + uint64_t(r) * kLd + off, acc[i] ^ uint32_t(r));
        }
    }
}

// one 16-byte unit per lane of the (stripe, 16-byte column) sequence
__global__ __launch_bounds__(256) void rows16(Set s) {
    constexpr uint32_t cps = kLd / 16;
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    if (u >= cps * kNs) return;
    const uint32_t st_ = u / cps, c = u % cps;
    const uint8_t* ib = s.in + uint64_t(st_) * K * kLd + c * 16;
    uint8_t* ob = s.out + uint64_t(st_) * R * kLd + c * 16;
    u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < K; ++j) acc ^= *reinterpret_cast<const u32x4*>(ib + uint64_t(j) * kLd);
#pragma unroll 8
    for (int r = 0; r < R; ++r) st(ob + uint64_t(r) * kLd, acc ^ uint32_t(r));
}

typedef void (*Fn)(Set);

float run(Fn fn, uint32_t grid, const std::vector<Set>& sets, int reps, uint32_t lds = 0) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 4; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, 0, sets[i % sets.size()]);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), lds, 0, sets[(i + 4) % sets.size()]);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    CK(hipGetLastError());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<Set> sets(2);
    for (auto& s : sets) {
        uint8_t *i, *o;
        CK(hipMalloc(&i, uint64_t(kNs) * K * kLd));
        CK(hipMalloc(&o, uint64_t(kNs) * R * kLd));
        CK(hipMemset(i, 0x3c, uint64_t(kNs) * K * kLd));
        s.in = i;
        s.out = o;
    }
    CK(hipDeviceSynchronize());
    const double bytes = double(kNs) * (K + R) * kSz;  // algorithmic bytes, as the bench counts them
    auto g_wave = [](uint32_t P) { return ((kSz + P - 1) / P * kNs + 3) / 4; };
    auto g_split = [](uint32_t P) { return (kSz + P - 1) / P * kNs; };
    struct V {
        const char* name;
        Fn fn;
        uint32_t grid;
        uint32_t lds;
    };
    const V vs[] = {
        {"wave1k", wave_unit<1024>, g_wave(1024), 0},   {"wave2k", wave_unit<2048>, g_wave(2048), 0},
        {"wave4k", wave_unit<4096>, g_wave(4096), 0},   {"split1k", split_unit<1024>, g_split(1024), 0},
        {"split2k", split_unit<2048>, g_split(2048), 0}, {"rows16", rows16, (kLd / 16 * kNs + 255) / 256, 0},
        {"wave1k_occ3", wave_unit<1024>, g_wave(1024), 48u << 10},
        {"wave2k_occ3", wave_unit<2048>, g_wave(2048), 48u << 10},
        {"split1k_occ3", split_unit<1024>, g_split(1024), 48u << 10},
        {"split2k_occ3", split_unit<2048>, g_split(2048), 48u << 10},
    };
    printf("K=20/M=60 pattern, %u stripes of %u-byte rows (row stride %u), 2 sets of %.2f GB, %d reps\n", kNs, kSz,
           kLd, (double(kNs) * (K + R) * kLd) / 1e9, reps);
    for (int round = 0; round < 3; ++round) {
        printf("-- round %d\n", round);
        for (const V& v : vs) {
            const float ms = run(v.fn, v.grid, sets, reps, v.lds);
            printf("%-8s %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)  grid %u\n", v.name, ms * 1e3,
                   bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12, v.grid);
            fflush(stdout);
        }
    }
    for (auto& s : sets) {
        CK(hipFree(const_cast<uint8_t*>(s.in)));
        CK(hipFree(s.out));
    }
    return 0;
}
