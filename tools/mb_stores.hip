// mb_stores.hip -- shapes of a cold HBM store stream at the cfg2 encode's size
// (7 output rows of 22,369,792 bytes = 156.6 MB per launch), launches rotated
// over buffer sets spanning > 768 MiB so no launch finds its lines in the
// 256 MiB Infinity Cache.  Writes are 70 % of the K=3/M=10 encode's traffic and
// the stores alone run at 5.66-5.80 TB/s (profiles/r02_mb_cold.log, 16-byte
// nt stores, one unit per lane, 7 rows interleaved), below the 6.0-6.2 TB/s
// MI355X_MICROARCH.md measured for plain stores of another shape.  Which
// store shape writes fastest?
//
//   rows7_*    one 16-byte unit per lane, the 7 rows interleaved as the
//              encode writes them (nt / plain / nt sc1 policy)
//   seq_nt     the same stores, one long stream (the 7 rows back to back)
//   wave4k     each wave writes 4 KiB contiguous of every row (4 x 1 KiB
//              instructions per row)
//   lane32     two adjacent 16-byte stores per lane (2 KiB per wave per row)
//   dword      4-byte stores, 4 per row per lane (256 B per wave-instruction)
//   persist    rows7_nt as a persistent grid (CUs x 8 workgroups, grid-stride)
//   copy_rows3 3 rows read, the same 3 rows' bytes written elsewhere (1:1)
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_stores.hip -o tools/mb_stores.exe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
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

constexpr int R = 7;
constexpr uint64_t kRow = 22369792;  // cfg2 block row (22,369,622 rounded up to 256)
constexpr uint32_t kUnits = kRow / 16;  // 16-byte units per row

struct Set {
    uint8_t* out;  // R rows of kRow
    uint8_t* in;   // 3 rows of kRow (copy variant)
};

template <int POL>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
    if constexpr (POL == 0)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else if constexpr (POL == 1)
        *reinterpret_cast<u32x4*>(p) = v;
    else
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
}

template <int POL>
__global__ __launch_bounds__(256) void rows7(Set s) {
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    if (u >= kUnits) return;
    const u32x4 v = {u, u ^ 1u, u ^ 2u, u ^ 3u};
#pragma unroll
    for (int r = 0; r < R; ++r) st16<POL>(s.out + r * kRow + uint64_t(u) * 16, v ^ uint32_t(r));
}

__global__ __launch_bounds__(256) void seq_nt(Set s) {
    // the same 7 x kUnits stores as one stream: lane u stores units u, u + kUnits, ... in one long row
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    const uint64_t total = uint64_t(kUnits) * R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint64_t g = uint64_t(blockIdx.x) * 256 * R + uint64_t(r) * 256 + threadIdx.x;  // 4 KiB runs per WG
        if (g < total) {
            const u32x4 v = {u, u ^ 1u, u ^ 2u, uint32_t(r)};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(s.out + g * 16));
        }
    }
}

__global__ __launch_bounds__(256) void wave4k(Set s) {
    // wave w owns units [256 w, 256 w + 256) of every row: 4 x 1 KiB per row
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t u = wave * 256 + p * 64 + lane;
            if (u < kUnits) {
                const u32x4 v = {u, u ^ 1u, u ^ 2u, uint32_t(r)};
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(s.out + r * kRow + uint64_t(u) * 16));
            }
        }
}

__global__ __launch_bounds__(256) void lane32(Set s) {
    const uint32_t u = (blockIdx.x * 256 + threadIdx.x) * 2;
    if (u >= kUnits) return;
    const u32x4 v = {u, u ^ 1u, u ^ 2u, u ^ 3u};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* p = s.out + r * kRow + uint64_t(u) * 16;
        __builtin_nontemporal_store(v ^ uint32_t(r), reinterpret_cast<u32x4*>(p));
        __builtin_nontemporal_store(v ^ uint32_t(r + 8), reinterpret_cast<u32x4*>(p + 16));
    }
}

__global__ __launch_bounds__(256) void dword4(Set s) {
    // each lane 4 dwords per row, 256 B apart: a wave covers 1 KiB per row in 4 instructions
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t base = uint64_t(wave) * 1024;
    if (base >= kRow) return;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint64_t o = base + p * 256 + lane * 4;
            if (o < kRow)  // kRow is not a multiple of 1 KiB
                __builtin_nontemporal_store(uint32_t(o + r), reinterpret_cast<uint32_t*>(s.out + r * kRow + o));
        }
}

__global__ __launch_bounds__(256) void persist(Set s) {
    for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < kUnits; u += gridDim.x * 256) {
        const u32x4 v = {u, u ^ 1u, u ^ 2u, u ^ 3u};
#pragma unroll
        for (int r = 0; r < R; ++r) st16<0>(s.out + r * kRow + uint64_t(u) * 16, v ^ uint32_t(r));
    }
}

__global__ __launch_bounds__(256) void copy_rows3(Set s) {
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    if (u >= kUnits) return;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(s.in + r * kRow + uint64_t(u) * 16);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(s.out + r * kRow + uint64_t(u) * 16));
    }
}

typedef void (*Fn)(Set);

float run(Fn fn, uint32_t grid, const std::vector<Set>& sets, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, sets[i % sets.size()]);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, sets[(i + 20) % sets.size()]);
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
    const int nsets = argc > 1 ? atoi(argv[1]) : 6;
    const int reps = argc > 2 ? atoi(argv[2]) : 60;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Set> sets(nsets);
    for (auto& s : sets) {
        CK(hipMalloc(&s.out, R * kRow));
        CK(hipMalloc(&s.in, 3 * kRow));
        CK(hipMemset(s.in, 0x5a, 3 * kRow));
        CK(hipMemset(s.out, 0, R * kRow));
    }
    CK(hipDeviceSynchronize());
    const uint32_t g1 = (kUnits + 255) / 256;
    struct V {
        const char* name;
        Fn fn;
        uint32_t grid;
        double bytes;
    };
    const double wb = double(R) * kRow;
    const V vs[] = {
        {"rows7_nt", rows7<0>, g1, wb},
        {"rows7_plain", rows7<1>, g1, wb},
        {"rows7_ntsc1", rows7<2>, g1, wb},
        {"seq_nt", seq_nt, uint32_t((uint64_t(kUnits) * R + 256 * R - 1) / (256 * R)), wb},
        {"wave4k", wave4k, (kUnits / 256 + 3) / 4 + 1, wb},
        {"lane32", lane32, (kUnits / 2 + 255) / 256, wb},
        {"dword4", dword4, uint32_t((kRow / 1024 + 3) / 4), wb},
        {"persist", persist, uint32_t(ncu * 8), wb},
        {"copy_rows3", copy_rows3, g1, 6.0 * kRow},
    };
    printf("cold store shapes: %d sets of %.1f MB written per launch (%.0f MiB rotation), %d reps, %d CUs\n", nsets,
           wb / 1e6, nsets * (R + 3) * kRow / 1048576.0, reps, ncu);
    for (int round = 0; round < 3; ++round) {
        printf("-- round %d\n", round);
        for (const V& v : vs) {
            const float ms = run(v.fn, v.grid, sets, reps);
            printf("%-12s %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)  grid %u\n", v.name, ms * 1e3, v.bytes / (ms * 1e-3) / 1e9,
                   v.bytes / (ms * 1e-3) / 8e12, v.grid);
            fflush(stdout);
        }
    }
    for (auto& s : sets) {
        CK(hipFree(s.out));
        CK(hipFree(s.in));
    }
    return 0;
}
