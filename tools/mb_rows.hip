// mb_rows.hip -- short rows (cfg5: 10^6 stripes of K=3 x 1366-byte blocks):
// the production unit walk (16-byte units numbered stripe-major, so one wave
// instruction spans the end of one stripe's row and the start of the next)
// against a row walk (one wave per stripe: lane l owns bytes 16l and
// 1024 + 16l of every row, the last chunk shifted back to end at sz), each as
// a pure copy and with the GF arithmetic.  Random input bytes; back-to-back
// launches, medians of interleaved rounds.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_rows.hip zfec_amd/csrc/bitslice.cpp \
//          zfec_amd/csrc/gf256.cpp -ldl -lpthread -o tools/mb_rows.exe
#include "../zfec_amd/csrc/kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
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

__global__ void fill_random(uint32_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        uint32_t x = uint32_t(i) * 2654435761u ^ seed;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        p[i] = x;
    }
}

// the production walk as a copy (tools/mb_encode.hip copy_walk)
template <int K, int R>
__global__ __launch_bounds__(256) void unit_copy(const MatJob job) {
    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    for (UnitIter u(job); u.s < job.nstripes; u.next(job)) {
        const Span sp = chunk_span<kChunk, true>(u.c, sz, nfull);
        const uint64_t ib = u.s * job.in_sstride + sp.off, ob = u.s * job.out_sstride + sp.off;
        u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= load16(job.in[j] + ib);
#pragma unroll
        for (int r = 0; r < R; ++r) store16_out<true>(job.out[r] + ob, acc ^ uint32_t(r));
    }
}

// one wave per stripe; 1024 < sz <= 2048
template <int K, int R, bool GF>
__global__ __launch_bounds__(256) void row_walk(const MatJob job) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * 4u;
    const uint64_t sz = job.sz;
    Tab T[R][K];
    for (uint32_t s = blockIdx.x * 4u + (threadIdx.x >> 6); s < job.nstripes; s += nw) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint64_t off = uint64_t(h) * 1024u + lane * 16u;
            if (h == 1) {
                if (off >= sz) continue;  // lanes past the row end
                if (off + 16u > sz) off = sz - 16u;
            }
            const uint64_t ib = s * job.in_sstride + off, ob = s * job.out_sstride + off;
            u32x4 x[K];
#pragma unroll
            for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + ib);
            if constexpr (GF) {
                reg_compute_store<K, R, true, 0, true>(job, T, x, ob, true, 16u);
            } else {
                u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < K; ++j) acc ^= x[j];
#pragma unroll
                for (int r = 0; r < R; ++r) store16_out<true>(job.out[r] + ob, acc ^ uint32_t(r));
            }
        }
    }
}

// row walk over a contiguous range of stripes per wave (grid below one wave per stripe)
template <int K, int R>
__global__ __launch_bounds__(256) void row_walk_chunked(const MatJob job) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nw = gridDim.x * 4u, w = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t sz = job.sz;
    const uint32_t per = (job.nstripes + nw - 1) / nw;
    const uint32_t s0 = w * per, s1 = min(job.nstripes, s0 + per);
    Tab T[R][K];
    for (uint32_t s = s0; s < s1; ++s)
        for (uint64_t off = lane * 16u; off < sz; off += 1024u) {
            const uint64_t o = off + 16u <= sz ? off : sz - 16u;
            u32x4 x[K];
            reg_load<K>(job, x, s * job.in_sstride + o, true, 16u);
            reg_compute_store<K, R, true, 0, true>(job, T, x, s * job.out_sstride + o, true, 16u);
        }
}

// variants of the row walk: MODE 1 = 32 bytes per lane (bytes 32l and 32l + 16),
// MODE 2 = two stripes per wave (half-wave per stripe, 16 bytes at 16l' + 512h)
template <int K, int R, bool GF, int MODE>
__global__ __launch_bounds__(256) void row_walk2(const MatJob job) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t sz = job.sz;
    Tab T[R][K];
    auto unit = [&](uint64_t s, uint64_t off) {
        const uint64_t o = off + 16u <= sz ? off : sz - 16u;
        const uint64_t ib = s * job.in_sstride + o, ob = s * job.out_sstride + o;
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = load16(job.in[j] + ib);
        if constexpr (GF) {
            reg_compute_store<K, R, true, 0, true>(job, T, x, ob, true, 16u);
        } else {
            u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int j = 0; j < K; ++j) acc ^= x[j];
#pragma unroll
            for (int r = 0; r < R; ++r) store16_out<true>(job.out[r] + ob, acc ^ uint32_t(r));
        }
    };
    if constexpr (MODE == 1) {
        const uint32_t nw = gridDim.x * 4u;
        for (uint32_t s = blockIdx.x * 4u + (threadIdx.x >> 6); s < job.nstripes; s += nw)
            for (uint64_t off = lane * 32u; off < sz; off += 2048u) {
                unit(s, off);
                if (off + 16u < sz) unit(s, off + 16u);
            }
    } else {
        const uint32_t nw = gridDim.x * 8u;
        const uint32_t l = lane & 31u;
        for (uint32_t s = blockIdx.x * 8u + (threadIdx.x >> 5); s < job.nstripes; s += nw)
            for (uint64_t off = l * 16u; off < sz; off += 512u) unit(s, off);
    }
}

}  // namespace

int main() {
    std::call_once(g_dispatch_once, init_dispatch);
    set_jit_mode(kJitOff);
    const int k = 3, r = 7;
    const size_t sz = 1366, ns = 1000000;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (size_t ld : {size_t(1536), size_t(1408), size_t(1366), size_t(1664)}) {
        uint8_t *in, *out;
        CK(hipMalloc(&in, ns * k * ld));
        CK(hipMalloc(&out, ns * r * ld));
        hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(in),
                           ns * k * ld / 4, 12345u);
        CK(hipDeviceSynchronize());
        MatJob j;
        memset(&j, 0, sizeof j);
        j.sz = sz;
        j.nstripes = ns;
        j.k = k;
        j.r = r;
        j.in_sstride = k * ld;
        j.out_sstride = r * ld;
        for (int q = 0; q < k; ++q) j.in[q] = in + q * ld;
        for (int q = 0; q < r; ++q) j.out[q] = out + q * ld;
        for (int q = 0; q < k * r; ++q) j.coef[q] = uint8_t(q * 37 + 11);
        // tables as launch_matapply places them in the kernel arguments
        MatJob jt = j;
        {
            uint8_t c[kMaxKernargTables];
            for (int q = 0; q < k * r; ++q) c[q] = jt.coef[q];
            for (int q = 0; q < k * r; ++q)
                for (int w = 0; w < 5; ++w) jt.tab[q * 5 + w] = kHostBank.w[c[q] * 8 + w];
            jt.tables = 1;
        }
        int nb = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(row_walk<3, 7, true>), 256, 0));
        const uint32_t g_full = uint32_t((ns + 3) / 4), g_cap = uint32_t(256 * std::max(nb, 1) * 16);
        struct V {
            const char* name;
            int kind;  // 0 production, 1 unit copy, 2 row copy, 3 row GF, 4-7 row_walk2 copy / GF
            uint32_t grid;
        } vs[] = {{"production reg<3,7>", 0, 0},
                  {"unit-walk copy", 1, 0},
                  {"row-walk copy, 1 stripe/wave", 2, g_full},
                  {"row-walk copy, 16x resident", 2, std::min(g_full, g_cap)},
                  {"row-walk GF, 1 stripe/wave", 3, g_full},
                  {"row-walk GF, 16x resident", 3, std::min(g_full, g_cap)},
                  {"row-walk GF, 4x resident", 3, std::min(g_full, g_cap / 4)},
                  {"row-walk GF, 64x resident", 3, std::min(g_full, g_cap * 4)},
                  {"row-walk GF chunked, 16x res", 8, std::min(g_full, g_cap)},
                  {"row-walk GF chunked, 4x res", 8, std::min(g_full, g_cap / 4)}};
        const int nv = sizeof(vs) / sizeof(vs[0]);
        std::vector<std::vector<float>> t(nv);
        std::vector<uint8_t> ref, got(size_t(2000) * r * ld);
        for (int round = 0; round < 5; ++round)
            for (int v = 0; v < nv; ++v) {
                auto launch = [&] {
                    if (vs[v].kind == 0) {
                        MatJob jj = j;
                        CK(launch_matapply(jj, 0));
                    } else if (vs[v].kind == 1) {
                        MatJob jj = j;
                        jj.cps = uint32_t((sz + 15) / 16);
                        const uint64_t total = uint64_t(jj.cps) * ns;
                        const uint32_t grid = uint32_t((total + 255) / 256);
                        jj.gs_s = uint32_t(uint64_t(grid) * 256 / jj.cps);
                        jj.gs_c = uint32_t(uint64_t(grid) * 256 % jj.cps);
                        hipLaunchKernelGGL((unit_copy<3, 7>), dim3(grid), dim3(256), 0, 0, jj);
                    } else if (vs[v].kind == 2) {
                        hipLaunchKernelGGL((row_walk<3, 7, false>), dim3(vs[v].grid), dim3(256), 0, 0, j);
                    } else if (vs[v].kind == 3) {
                        hipLaunchKernelGGL((row_walk<3, 7, true>), dim3(vs[v].grid), dim3(256), 0, 0, jt);
                    } else if (vs[v].kind == 8) {
                        hipLaunchKernelGGL((row_walk_chunked<3, 7>), dim3(vs[v].grid), dim3(256), 0, 0, jt);
                    } else if (vs[v].kind == 4) {
                        hipLaunchKernelGGL((row_walk2<3, 7, false, 1>), dim3(vs[v].grid), dim3(256), 0, 0, j);
                    } else if (vs[v].kind == 5) {
                        hipLaunchKernelGGL((row_walk2<3, 7, true, 1>), dim3(vs[v].grid), dim3(256), 0, 0, jt);
                    } else if (vs[v].kind == 6) {
                        hipLaunchKernelGGL((row_walk2<3, 7, false, 2>), dim3(vs[v].grid), dim3(256), 0, 0, j);
                    } else {
                        hipLaunchKernelGGL((row_walk2<3, 7, true, 2>), dim3(vs[v].grid), dim3(256), 0, 0, jt);
                    }
                };
                launch();
                launch();
                CK(hipDeviceSynchronize());
                if (round == 0 && (vs[v].kind == 0 || vs[v].kind == 3 || vs[v].kind == 5 || vs[v].kind == 7 ||
                                   vs[v].kind == 8)) {
                    CK(hipMemcpy(got.data(), out, got.size(), hipMemcpyDeviceToHost));
                    if (vs[v].kind == 0)
                        ref = got;
                    else if (memcmp(ref.data(), got.data(), got.size()))
                        printf("MISMATCH %s ld=%zu\n", vs[v].name, ld);
                }
                CK(hipEventRecord(a, 0));
                for (int i = 0; i < 5; ++i) launch();
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                t[v].push_back(ms / 5);
            }
        for (int v = 0; v < nv; ++v) {
            std::sort(t[v].begin(), t[v].end());
            printf("ld=%zu %-30s %8.4f ms  %7.1f GB/s\n", ld, vs[v].name, t[v][2],
                   double(k + r) * sz * ns / (t[v][2] * 1e-3) / 1e9);
        }
        CK(hipFree(in));
        CK(hipFree(out));
    }
    return 0;
}
