// mb_cold.hip -- HBM ceilings of the K=3/M=10 encode's memory pattern from
// cold caches: 256 stripes x 1 MiB (bench.py's batched_1MiB layout,
// [stripe][block][row], rows of 349,696 bytes), launches rotated over buffer
// sets spanning > 768 MiB so no launch finds its bytes in the 256 MiB
// Infinity Cache.  Every variant moves the same bytes: 3 x 16-byte loads and
// 7 x 16-byte stores per lane per unit; the arithmetic is an XOR (a copy
// ceiling), except "prod", which is the production dispatcher's kernel.
//
// Walk variants:
//   lane     one 16-byte unit per lane, grid = units / 256 (production walk)
//   persist  persistent grid (CUs x 8 workgroups), grid-stride over units
//   xcd      as `lane`, but workgroups dealt so that the 8 XCDs (blockIdx % 8)
//            each sweep one contiguous eighth of the units
//   wave4    each wave owns 4 consecutive 1 KiB pieces of every block
//            (4 KiB contiguous per block per wave), lanes 1 KiB apart
//   plain    `lane` with default-policy stores instead of nt
//   ntload   `lane` with nt loads too
//   prod / prod_xcd: the production kernel without / with XCD-contiguous
//            workgroup order (ZFEC_HIP_XCD)
//   prod_gmN the production kernel with its grid capped at N x the resident
//            workgroups (a grid-stride walk of ~units / (N x resident lanes)
//            units per lane; the default cap is 1024, i.e. one unit per lane)
//   prod_bm  the production kernel on the same stripes stored block-major
//            (one long row per block, as fec_encode_batch collapses them)
// usage: tools/mb_cold.exe [buffer sets] [stripes] | tools/mb_cold.exe sweep
// Ceilings: read3 (only the 3 loads), write7 (only the 7 stores), copy1
// (1 load, 1 store per unit).
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_cold.hip zfec_amd/csrc/bitslice.cpp \
//          zfec_amd/csrc/gf256.cpp -ldl -o tools/mb_cold.exe
#include "../zfec_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <vector>

using namespace zfec_hip;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

namespace {

constexpr int K = 3, R = 7;

struct Lay {
    uint8_t* in;
    uint8_t* out;
    uint64_t ld;       // row bytes
    uint32_t cps;      // 16-byte chunks per row
    uint32_t units;    // cps * nstripes
};

__device__ __forceinline__ void unit_io(const Lay& L, uint32_t u, bool ntload, bool ntstore, int mode) {
    const uint32_t s = u / L.cps, c = u - s * L.cps;
    const uint64_t ib = uint64_t(s) * K * L.ld + uint64_t(c) * 16;
    const uint64_t ob = uint64_t(s) * R * L.ld + uint64_t(c) * 16;
    u32x4 acc = {0u, 0u, 0u, 0u};
    if (mode != 2) {  // loads
        const int nl = mode == 3 ? 1 : K;
        for (int j = 0; j < nl; ++j) {
            const u32x4* p = reinterpret_cast<const u32x4*>(L.in + ib + j * L.ld);
            acc ^= ntload ? __builtin_nontemporal_load(p) : *p;
        }
    } else {
        acc = u32x4{u, u + 1, u + 2, u + 3};
    }
    if (mode == 1) {  // read only: keep the loads alive
        if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) *reinterpret_cast<u32x4*>(L.out + ob) = acc;
        return;
    }
    const int ns = mode == 3 ? 1 : R;
    for (int r = 0; r < ns; ++r) {
        u32x4* q = reinterpret_cast<u32x4*>(L.out + ob + r * L.ld);
        if (ntstore)
            __builtin_nontemporal_store(acc ^ uint32_t(r), q);
        else
            *q = acc ^ uint32_t(r);
    }
}

// walk: 0 lane, 1 persist, 2 xcd, 3 wave4.  mode: 0 encode-shaped, 1 read3, 2 write7, 3 copy1
template <int WALK, bool NTL, bool NTS, int MODE>
__global__ __launch_bounds__(256) void mb(const Lay L) {
    if constexpr (WALK == 0) {
        const uint32_t u = blockIdx.x * 256 + threadIdx.x;
        if (u < L.units) unit_io(L, u, NTL, NTS, MODE);
    } else if constexpr (WALK == 1) {
        for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < L.units; u += gridDim.x * 256)
            unit_io(L, u, NTL, NTS, MODE);
    } else if constexpr (WALK == 2) {
        const uint32_t nwg = gridDim.x, q = nwg / 8, rr = nwg % 8, x = blockIdx.x % 8;
        const uint32_t wg = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + blockIdx.x / 8;
        const uint32_t u = wg * 256 + threadIdx.x;
        if (u < L.units) unit_io(L, u, NTL, NTS, MODE);
    } else {
        // wave w of the grid owns 64-lane pieces 4w..4w+3 of the unit sequence
        const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
        for (int p = 0; p < 4; ++p) {
            const uint32_t u = (wave * 4 + p) * 64 + lane;
            if (u < L.units) unit_io(L, u, NTL, NTS, MODE);
        }
    }
}

// Encode-shaped copy walk (`lane`) whose last workgroups store with a
// write-through policy (SP: 1 sc1, 2 sc0 sc1, 3 nt sc1) and the rest with nt:
// does the end-of-kernel write-back of dirty L2 lines set part of the fixed
// per-launch cost?  Workgroups >= tail_wg take the write-through stores.
template <int SP>
__global__ __launch_bounds__(256) void mb_tail(const Lay L, uint32_t tail_wg) {
    const uint32_t u = blockIdx.x * 256 + threadIdx.x;
    if (u >= L.units) return;
    const uint32_t s = u / L.cps, c = u - s * L.cps;
    const uint64_t ib = uint64_t(s) * K * L.ld + uint64_t(c) * 16;
    const uint64_t ob = uint64_t(s) * R * L.ld + uint64_t(c) * 16;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int j = 0; j < K; ++j) acc ^= *reinterpret_cast<const u32x4*>(L.in + ib + j * L.ld);
    const bool wt = blockIdx.x >= tail_wg;
    for (int r = 0; r < R; ++r) {
        uint8_t* q = L.out + ob + r * L.ld;
        if (wt)
            store16_pol<true, SP>(q, acc ^ uint32_t(r));
        else
            __builtin_nontemporal_store(acc ^ uint32_t(r), reinterpret_cast<u32x4*>(q));
    }
}

template <int SP>
float run_tail(const std::vector<Lay>& sets, int reps, uint32_t grid, uint32_t tail_wg) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(mb_tail<SP>, dim3(grid), dim3(256), 0, 0, sets[i % sets.size()], tail_wg);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(mb_tail<SP>, dim3(grid), dim3(256), 0, 0, sets[(i + 3) % sets.size()], tail_wg);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int WALK, bool NTL, bool NTS, int MODE>
float run(const std::vector<Lay>& sets, int reps, uint32_t grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((mb<WALK, NTL, NTS, MODE>), dim3(grid), dim3(256), 0, 0, sets[i % sets.size()]);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((mb<WALK, NTL, NTS, MODE>), dim3(grid), dim3(256), 0, 0, sets[(i + 3) % sets.size()]);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

float run_prod(const std::vector<Lay>& sets, int reps, uint64_t sz, uint32_t ns) {
    std::vector<MatJob> jobs(sets.size());
    static const uint8_t coef[R * K] = {15, 8, 6, 45, 48, 28, 153, 224, 120, 11, 231, 237, 137, 59, 179, 70, 241, 182, 186, 217, 98};
    for (size_t i = 0; i < sets.size(); ++i) {
        MatJob& j = jobs[i];
        std::memset(&j, 0, sizeof j);
        j.sz = sz;
        j.in_sstride = K * sets[i].ld;
        j.out_sstride = R * sets[i].ld;
        j.nstripes = ns;
        j.k = K;
        j.r = R;
        for (int q = 0; q < K; ++q) j.in[q] = sets[i].in + q * sets[i].ld;
        for (int q = 0; q < R; ++q) j.out[q] = sets[i].out + q * sets[i].ld;
        std::memcpy(j.coef, coef, sizeof coef);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) CK(launch_matapply(jobs[i % jobs.size()], 0));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) CK(launch_matapply(jobs[(i + 3) % jobs.size()], 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// The same stripes stored block-major (block j of every stripe back to back:
// one row of ns * sz bytes per block), as fec_encode_batch collapses them:
// one launch over 10 long streams.
float run_prod_bm(const std::vector<Lay>& sets, int reps, uint64_t sz, uint32_t ns) {
    std::vector<MatJob> jobs(sets.size());
    static const uint8_t coef[R * K] = {15, 8, 6, 45, 48, 28, 153, 224, 120, 11, 231, 237, 137, 59, 179, 70, 241, 182, 186, 217, 98};
    for (size_t i = 0; i < sets.size(); ++i) {
        MatJob& j = jobs[i];
        std::memset(&j, 0, sizeof j);
        j.sz = sz * ns;
        j.nstripes = 1;
        j.k = K;
        j.r = R;
        for (int q = 0; q < K; ++q) j.in[q] = sets[i].in + q * sz * ns;
        for (int q = 0; q < R; ++q) j.out[q] = sets[i].out + q * sz * ns;
        std::memcpy(j.coef, coef, sizeof coef);
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) CK(launch_matapply(jobs[i % jobs.size()], 0));
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) CK(launch_matapply(jobs[(i + 3) % jobs.size()], 0));
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

}  // namespace

// Walk variants of matapply_reg<3,7> on one stripe per block (block-major),
// cold: U units per lane per loop trip, prefetch of the next unit, and the grid
// (one unit per lane, or capped at `cap` x the resident workgroups with a
// grid-stride loop), launched directly (tables in the kernel arguments as
// launch_matapply puts them).
template <int U, bool PF>
float run_walk(const std::vector<Lay>& sets, int reps, uint64_t sz, uint32_t ns, int cap) {
    typedef void (*Fn)(const MatJob);
    Fn fn = matapply_reg<K, R, true, U, 0, PF, 0, true>;
    static const uint8_t coef[R * K] = {15, 8, 6, 45, 48, 28, 153, 224, 120, 11, 231, 237, 137, 59, 179, 70, 241, 182, 186, 217, 98};
    int nb = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(fn), kBlock, 0));
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::vector<MatJob> jobs(sets.size());
    for (size_t i = 0; i < sets.size(); ++i) {
        MatJob& j = jobs[i];
        std::memset(&j, 0, sizeof j);
        j.sz = sz * ns;
        j.nstripes = 1;
        j.k = K;
        j.r = R;
        for (int q = 0; q < K; ++q) j.in[q] = sets[i].in + q * sz * ns;
        for (int q = 0; q < R; ++q) j.out[q] = sets[i].out + q * sz * ns;
        for (int c = 0; c < K * R; ++c)
            for (int q = 0; q < 5; ++q) j.tab[c * 5 + q] = kHostBank.w[coef[c] * 8 + q];
        j.tables = 1;
        const uint64_t cps = (j.sz + kChunk - 1) / kChunk;
        j.cps = static_cast<uint32_t>(cps);
        const uint64_t lanes = (cps + U - 1) / U;
        const uint64_t need = (lanes + kBlock - 1) / kBlock;
        const uint64_t capb = cap ? uint64_t(ncu) * nb * cap : need;
        const uint32_t grid = static_cast<uint32_t>(need < capb ? need : capb);
        const uint64_t gstride = uint64_t(grid) * kBlock;
        j.gs_s = static_cast<uint32_t>(gstride / cps);
        j.gs_c = static_cast<uint32_t>(gstride % cps);
        j.pad_ = grid;  // (unused by the kernel) the grid to launch
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(fn, dim3(jobs[i % jobs.size()].pad_), dim3(kBlock), 0, 0, jobs[i % jobs.size()]);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) {
        const MatJob& j = jobs[(i + 3) % jobs.size()];
        hipLaunchKernelGGL(fn, dim3(j.pad_), dim3(kBlock), 0, 0, j);
    }
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int walks() {
    const uint64_t sz1 = (1u << 20) / 3 + 1;
    for (uint32_t ns : {64u, 256u}) {
        const uint64_t fp = uint64_t(K + R) * sz1 * ns;
        const int nsets = std::max<int>(2, int((1536ull << 20) / fp) + 1);
        std::vector<Lay> sets(nsets);
        for (auto& L : sets) {
            CK(hipMalloc(&L.in, ns * K * sz1));
            CK(hipMalloc(&L.out, ns * R * sz1));
            CK(hipMemset(L.in, 0x5A, ns * K * sz1));
            L.ld = sz1;
        }
        CK(hipDeviceSynchronize());
        const double bytes = double(K + R) * sz1 * ns;
        for (int rnd = 0; rnd < 2; ++rnd) {
            struct V {
                const char* name;
                float ms;
            } vs[] = {
                {"prod (dispatcher)", run_prod_bm(sets, 20, sz1, ns)},
                {"U1 PF grid=units", run_walk<1, true>(sets, 20, sz1, ns, 0)},
                {"U1 noPF grid=units", run_walk<1, false>(sets, 20, sz1, ns, 0)},
                {"U2 grid=units/2", run_walk<2, false>(sets, 20, sz1, ns, 0)},
                {"U4 grid=units/4", run_walk<4, false>(sets, 20, sz1, ns, 0)},
                {"U2 cap=2", run_walk<2, false>(sets, 20, sz1, ns, 2)},
                {"U4 cap=1", run_walk<4, false>(sets, 20, sz1, ns, 1)},
                {"U1 PF cap=4", run_walk<1, true>(sets, 20, sz1, ns, 4)},
            };
            for (const V& v : vs)
                printf("walk ns=%4u %-20s %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)\n", ns, v.name, v.ms * 1e3,
                       bytes / (v.ms * 1e-3) / 1e9, bytes / (v.ms * 1e-3) / 8e12);
        }
        for (auto& L : sets) {
            CK(hipFree(L.in));
            CK(hipFree(L.out));
        }
    }
    return 0;
}

// Size sweep of the production kernel on one long stripe per block (block-major),
// cold: how the HBM fraction of a K=3/M=10 encode grows with the launch's size.
int sweep() {
    const uint64_t sz1 = (1u << 20) / 3 + 1;
    for (uint32_t ns : {16u, 32u, 64u, 128u, 256u, 512u, 1024u}) {
        const uint64_t fp = uint64_t(K + R) * sz1 * ns;
        const int nsets = std::max<int>(2, int((1536ull << 20) / fp) + 1);
        std::vector<Lay> sets(nsets);
        for (auto& L : sets) {
            CK(hipMalloc(&L.in, ns * K * sz1));
            CK(hipMalloc(&L.out, ns * R * sz1));
            CK(hipMemset(L.in, 0x5A, ns * K * sz1));
            L.ld = sz1;
        }
        CK(hipDeviceSynchronize());
        float best = 1e9f, sum = 0.f;
        for (int rnd = 0; rnd < 3; ++rnd) {
            const float ms = run_prod_bm(sets, 20, sz1, ns);
            best = std::min(best, ms);
            sum += ms;
        }
        const double bytes = double(K + R) * sz1 * ns;
        printf("sweep ns=%4u  %8.1f MB/launch  %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s) mean-of-3 %.1f us  sets=%d\n", ns,
               bytes / 1e6, best * 1e3, bytes / (best * 1e-3) / 1e9, bytes / (best * 1e-3) / 8e12, sum / 3 * 1e3, nsets);
        for (auto& L : sets) {
            CK(hipFree(L.in));
            CK(hipFree(L.out));
        }
    }
    return 0;
}

// Row-stride sweep of the production kernel on 256 object-major 1 MiB stripes
// (rows of sz = 349,526 bytes at stride ld): does the HBM fraction depend on
// where the 10 rows of a stripe fall relative to each other?
int ldsweep() {
    const uint32_t ns = 256;
    const uint64_t sz = (1u << 20) / 3 + 1;
    const uint64_t lds[] = {349696, 349696 + 128, 349696 + 512, 349696 + 2048, 352256, 352256 + 4096,
                            356352 + 8192, 393216, 1u << 19, (1u << 19) + 4096};
    for (int rnd = 0; rnd < 2; ++rnd)
        for (uint64_t ld : lds) {
            const uint64_t fp = uint64_t(K + R) * ld * ns;
            const int nsets = std::max<int>(2, int((1536ull << 20) / fp) + 1);
            std::vector<Lay> sets(nsets);
            for (auto& L : sets) {
                CK(hipMalloc(&L.in, ns * K * ld));
                CK(hipMalloc(&L.out, ns * R * ld));
                CK(hipMemset(L.in, 0x5A, ns * K * ld));
                L.ld = ld;
            }
            CK(hipDeviceSynchronize());
            const float ms = run_prod(sets, 20, sz, ns);
            const double bytes = double(K + R) * sz * ns;
            printf("ldsweep ld=%8llu (ld %% 4096 = %4llu)  %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)  sets=%d\n",
                   (unsigned long long)ld, (unsigned long long)(ld % 4096), ms * 1e3, bytes / (ms * 1e-3) / 1e9,
                   bytes / (ms * 1e-3) / 8e12, nsets);
            for (auto& L : sets) {
                CK(hipFree(L.in));
                CK(hipFree(L.out));
            }
        }
    return 0;
}

// cfg2's shape (one 64 MiB K=3/M=10 stripe: 3 + 7 rows of 22,369,792 bytes),
// cold rotation: the nt copy walk with its last fraction f of workgroups
// storing write-through, against the production kernel.
int tail() {
    const uint64_t sz = (64ull << 20) / 3 + 1, ld = (sz + 255) / 256 * 256;
    const int nsets = int((1536ull << 20) / (10 * ld)) + 1;
    std::vector<Lay> sets(nsets);
    for (auto& L : sets) {
        CK(hipMalloc(&L.in, K * ld));
        CK(hipMalloc(&L.out, R * ld));
        CK(hipMemset(L.in, 0x5A, K * ld));
        CK(hipMemset(L.out, 0, R * ld));
        L.ld = ld;
        L.cps = static_cast<uint32_t>(ld / 16);
        L.units = L.cps;
    }
    CK(hipDeviceSynchronize());
    const uint32_t grid = (sets[0].units + 255) / 256;
    const double bytes = double(K + R) * ld;
    auto rep = [&](const char* name, float ms) {
        printf("tail %-24s %7.2f us  %7.1f GB/s  (%.3f of 8 TB/s)  sets=%d\n", name, ms * 1e3,
               bytes / (ms * 1e-3) / 1e9, bytes / (ms * 1e-3) / 8e12, nsets);
    };
    for (int rnd = 0; rnd < 3; ++rnd) {
        printf("-- round %d\n", rnd);
        rep("prod", run_prod(sets, 40, sz, 1));
        for (double f : {0.0, 0.02, 0.05, 0.1, 0.2, 1.0}) {
            const uint32_t tw = grid - static_cast<uint32_t>(f * grid);
            char nm[64];
            snprintf(nm, sizeof nm, "f=%.2f sc0sc1", f);
            rep(nm, run_tail<2>(sets, 40, grid, tw));
            snprintf(nm, sizeof nm, "f=%.2f ntsc1", f);
            rep(nm, run_tail<3>(sets, 40, grid, tw));
            snprintf(nm, sizeof nm, "f=%.2f sc1", f);
            rep(nm, run_tail<1>(sets, 40, grid, tw));
        }
    }
    return 0;
}

// The `lane` copy walk with BS-thread workgroups (256 in production): fewer,
// larger workgroups cost less to dispatch (launch_cost) -- does the walk gain?
template <int BS>
__global__ __launch_bounds__(BS) void mb_bs(const Lay L) {
    const uint32_t u = blockIdx.x * BS + threadIdx.x;
    if (u < L.units) unit_io(L, u, false, true, 0);
}

template <int BS>
float run_bs(const std::vector<Lay>& sets, int reps) {
    const uint32_t grid = (sets[0].units + BS - 1) / BS;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(mb_bs<BS>, dim3(grid), dim3(BS), 0, 0, sets[i % sets.size()]);
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(mb_bs<BS>, dim3(grid), dim3(BS), 0, 0, sets[(i + 3) % sets.size()]);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

// 256 object-major 1 MiB stripes (as main) and the cfg2 stripe, cold: the
// copy walk at 256 / 512 / 1024 threads per workgroup.
int blocks() {
    for (int shape = 0; shape < 2; ++shape) {
        const uint32_t ns = shape == 0 ? 256 : 1;
        const uint64_t sz = shape == 0 ? (1u << 20) / 3 + 1 : (64ull << 20) / 3 + 1;
        const uint64_t ld = (sz + 255) / 256 * 256;
        const int nsets = std::max<int>(2, int((1536ull << 20) / (10 * ld * ns)) + 1);
        std::vector<Lay> sets(nsets);
        for (auto& L : sets) {
            CK(hipMalloc(&L.in, ns * K * ld));
            CK(hipMalloc(&L.out, ns * R * ld));
            CK(hipMemset(L.in, 0x5A, ns * K * ld));
            L.ld = ld;
            L.cps = static_cast<uint32_t>(ld / 16);
            L.units = L.cps * ns;
        }
        CK(hipDeviceSynchronize());
        const double bytes = double(K + R) * ld * ns;
        for (int rnd = 0; rnd < 3; ++rnd) {
            const float t256 = run_bs<256>(sets, 20), t512 = run_bs<512>(sets, 20), t1024 = run_bs<1024>(sets, 20);
            printf("blocks %s  256: %7.2f us (%.3f)  512: %7.2f us (%.3f)  1024: %7.2f us (%.3f)\n",
                   shape == 0 ? "256 x 1 MiB object-major" : "cfg2 64 MiB stripe      ", t256 * 1e3,
                   bytes / (t256 * 1e-3) / 8e12, t512 * 1e3, bytes / (t512 * 1e-3) / 8e12, t1024 * 1e3,
                   bytes / (t1024 * 1e-3) / 8e12);
        }
        for (auto& L : sets) {
            CK(hipFree(L.in));
            CK(hipFree(L.out));
        }
    }
    return 0;
}

// Fixed cost of a launch: back-to-back launches of a kernel that does no
// memory work, with one workgroup and with the cfg2 encode's grid (one
// 16-byte unit per lane of a 22,369,792-byte row: 5,462 workgroups of 256).
__global__ __launch_bounds__(256) void mb_empty(uint32_t* out, uint32_t v) {
    if (v == 0x12345678u && threadIdx.x == 0) out[blockIdx.x] = v;
}

int launch_cost() {
    uint32_t* out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint32_t grid : {1u, 256u, 5462u, 21845u, 87381u}) {
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(mb_empty, dim3(grid), dim3(256), 0, 0, out, 1u);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(mb_empty, dim3(grid), dim3(256), 0, 0, out, 1u);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("launch grid=%6u x 256  %6.2f us per launch (back to back, empty kernel)\n", grid, ms * 1e3 / 200);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "sweep") return sweep();
    if (argc > 1 && std::string(argv[1]) == "launch") return launch_cost();
    if (argc > 1 && std::string(argv[1]) == "blocks") return blocks();
    if (argc > 1 && std::string(argv[1]) == "tail") return tail();
    if (argc > 1 && std::string(argv[1]) == "ldsweep") return ldsweep();
    if (argc > 1 && std::string(argv[1]) == "walks") return walks();
    const uint32_t ns = argc > 2 ? atoi(argv[2]) : 256;
    const uint64_t sz = (1u << 20) / 3 + 1;  // 349,526
    const uint64_t ld = (sz + 255) / 256 * 256;
    const int nsets = argc > 1 ? atoi(argv[1]) : 2;
    const int reps = 20;
    std::vector<Lay> sets(nsets);
    for (auto& L : sets) {
        CK(hipMalloc(&L.in, ns * K * ld));
        CK(hipMalloc(&L.out, ns * R * ld));
        CK(hipMemset(L.in, 0x5A, ns * K * ld));
        CK(hipMemset(L.out, 0, ns * R * ld));
        L.ld = ld;
        L.cps = static_cast<uint32_t>(ld / 16);
        L.units = L.cps * ns;
    }
    CK(hipDeviceSynchronize());
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t units = sets[0].units;
    const uint32_t g_lane = (units + 255) / 256, g_persist = ncu * 8, g_wave4 = (units + 1023) / 1024;
    const double enc_bytes = double(K + R) * ld * ns;
    auto rep = [&](const char* name, float ms, double bytes) {
        printf("%-10s %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)  sets=%d\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9,
               bytes / (ms * 1e-3) / 8e12, nsets);
    };
    for (int round = 0; round < 3; ++round) {
        printf("-- round %d\n", round);
        setenv("ZFEC_HIP_XCD", "1", 1);
        rep("prod_xcd", run_prod(sets, reps, sz, ns), double(K + R) * sz * ns);
        setenv("ZFEC_HIP_XCD", "0", 1);
        rep("prod", run_prod(sets, reps, sz, ns), double(K + R) * sz * ns);
        rep("prod_bm", run_prod_bm(sets, reps, sz, ns), double(K + R) * sz * ns);
        for (int gm : {1, 2, 4, 16}) {  // grid cap = CUs x resident workgroups x gm (grid-stride beyond)
            char nm[32];
            snprintf(nm, sizeof nm, "prod_gm%d", gm);
            const int keep = g_grid_mult;
            g_grid_mult = gm;
            rep(nm, run_prod(sets, reps, sz, ns), double(K + R) * sz * ns);
            g_grid_mult = keep;
        }
        rep("lane", run<0, false, true, 0>(sets, reps, g_lane), enc_bytes);
        rep("persist", run<1, false, true, 0>(sets, reps, g_persist), enc_bytes);
        rep("xcd", run<2, false, true, 0>(sets, reps, g_lane), enc_bytes);
        rep("wave4", run<3, false, true, 0>(sets, reps, g_wave4), enc_bytes);
        rep("plain", run<0, false, false, 0>(sets, reps, g_lane), enc_bytes);
        rep("ntload", run<0, true, true, 0>(sets, reps, g_lane), enc_bytes);
        rep("read3", run<0, false, true, 1>(sets, reps, g_lane), double(K) * ld * ns);
        rep("write7", run<0, false, true, 2>(sets, reps, g_lane), double(R) * ld * ns);
        rep("copy1", run<0, false, true, 3>(sets, reps, g_lane), 2.0 * ld * ns);
        rep("copy1_pl", run<0, false, false, 3>(sets, reps, g_lane), 2.0 * ld * ns);
    }
    return 0;
}
