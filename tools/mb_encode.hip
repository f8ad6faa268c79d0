// mb_encode.hip -- microbenchmark of the matrix-apply kernels on one GPU.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_encode.hip zfec_amd/csrc/bitslice.cpp \
//          zfec_amd/csrc/gf256.cpp -ldl -o tools/mb_encode.exe
// Run:   ./tools/mb_encode.exe [stripe_bytes]
//
// 1. A copy-shaped ceiling kernel that moves the K=3/M=10 encode's bytes
//    (3 16-byte loads, 7 16-byte stores per lane) with trivial arithmetic.
// 2. The production dispatcher (kernels.hip, included in this TU) over
//    (k, r) shapes, 16-byte-aligned vs misaligned block bases, and grid caps.
// Bandwidth = algorithmic bytes (k + r) * block size / kernel time.
#include "../zfec_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#include <array>

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

template <int K, int R, bool NT>
__global__ __launch_bounds__(256) void copy_like(const MatJob job) {
    const uint32_t n = static_cast<uint32_t>(job.sz / 16);
    for (uint32_t c = blockIdx.x * 256 + threadIdx.x; c < n; c += gridDim.x * 256) {
        const uint64_t off = uint64_t(c) * 16;
        u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < K; ++j) acc ^= load16(job.in[j] + off);
#pragma unroll
        for (int r = 0; r < R; ++r) store16_out<NT>(job.out[r] + off, acc ^ uint32_t(r));
    }
}

// The encode kernel's exact unit walk and memory pattern (K=3 loads, R=7
// stores per unit, overlapping tail chunk) with the GF arithmetic replaced by
// an XOR: the layout's copy ceiling.
template <int K, int R>
__global__ __launch_bounds__(256) void copy_walk(const MatJob job) {
    const uint64_t sz = job.sz;
    const uint32_t nfull = static_cast<uint32_t>(sz / kChunk);
    for (UnitIter u(job); u.s < job.nstripes; u.next(job)) {
        const Span sp = chunk_span<kChunk, true>(u.c, sz, nfull);
        const uint64_t ib = u.s * job.in_sstride + sp.off, ob = u.s * job.out_sstride + sp.off;
        u32x4 acc = {0u, 0u, 0u, 0u};
        if (sp.full) {
#pragma unroll
            for (int j = 0; j < K; ++j) acc ^= load16(job.in[j] + ib);
#pragma unroll
            for (int r = 0; r < R; ++r) store16_out<true>(job.out[r] + ob, acc ^ uint32_t(r));
        }
    }
}

template <class F>
float time_ms(F&& launch, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / iters;
}

MatJob make_job(uint8_t* in, uint8_t* out, int k, int r, size_t sz, size_t stride, size_t ostride = 0) {
    if (!ostride) ostride = stride;
    MatJob j;
    memset(&j, 0, sizeof j);
    j.sz = sz;
    j.nstripes = 1;
    j.k = k;
    j.r = r;
    for (int i = 0; i < k; ++i) j.in[i] = in + i * stride;
    for (int i = 0; i < r; ++i) j.out[i] = out + i * ostride;
    for (int i = 0; i < k * r; ++i) j.coef[i] = uint8_t(i * 37 + 11);
    return j;
}

}  // namespace

int main(int argc, char** argv) {
    const size_t S = argc > 1 ? strtoull(argv[1], nullptr, 0) : (size_t(64) << 20);
    std::call_once(g_dispatch_once, init_dispatch);
    {  // copy-shaped ceiling for K=3/M=10
        const size_t sz = (S / 3 + 255) / 256 * 256;
        uint8_t *in, *out;
        CK(hipMalloc(&in, 3 * sz));
        CK(hipMalloc(&out, 7 * sz));
        CK(hipMemset(in, 0x5a, 3 * sz));
        MatJob j = make_job(in, out, 3, 7, sz, sz);
        for (int nt = 0; nt < 2; ++nt) {
            const size_t grid = (sz / 16 + 255) / 256;
            auto fn = nt ? copy_like<3, 7, true> : copy_like<3, 7, false>;
            float ms = time_ms([&] { hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, j); }, 20);
            printf("copy_like k=3 r=7 nt=%d                         %8.4f ms  hbm %7.1f GB/s\n", nt, ms,
                   10.0 * sz / (ms * 1e-3) / 1e9);
        }
        {  // the encode kernel's unit walk with the GF arithmetic replaced by an XOR
            const Variant saved = g_reg[3][7];
            g_reg[3][7] = Variant{copy_walk<3, 7>, "copy_walk", 0, true, 1};
            for (int gm : {2, 16}) {
                g_grid_mult = gm;
                MatJob jj = make_job(in, out, 3, 7, sz, sz);
                float ms = time_ms([&] { MatJob j2 = jj; CK(launch_matapply(j2, 0)); }, 20);
                printf("copy_walk k=3 r=7 gm=%2d                         %8.4f ms  hbm %7.1f GB/s\n", gm, ms,
                       10.0 * sz / (ms * 1e-3) / 1e9);
            }
            g_reg[3][7] = saved;
        }
        {  // the same for the decode shape (3 inputs, 3 outputs)
            const Variant saved = g_reg[3][3];
            g_reg[3][3] = Variant{copy_walk<3, 3>, "copy_walk", 0, true, 1};
            for (int gm : {2, 16}) {
                g_grid_mult = gm;
                MatJob jj = make_job(in, out, 3, 3, sz, sz);
                float ms = time_ms([&] { MatJob j2 = jj; CK(launch_matapply(j2, 0)); }, 20);
                printf("copy_walk k=3 r=3 gm=%2d                         %8.4f ms  hbm %7.1f GB/s\n", gm, ms,
                       6.0 * sz / (ms * 1e-3) / 1e9);
            }
            g_reg[3][3] = saved;
        }
        CK(hipFree(in));
        CK(hipFree(out));
    }
    {  // misalignment split: inputs only / outputs only (K=3/M=10 encode)
        const int k = 3, r = 7;
        const size_t bsz = (S / k + 255) / 256 * 256;
        for (int mi : {0, 6}) for (int mo : {0, 6}) {
            uint8_t *xin, *xout;
            CK(hipMalloc(&xin, k * (bsz + mi) + 256));
            CK(hipMalloc(&xout, r * (bsz + mo) + 256));
            CK(hipMemset(xin, 0x5a, k * (bsz + mi) + 256));
            g_grid_mult = 16;
            MatJob j = make_job(xin, xout, k, r, bsz, bsz + mi, bsz + mo);
            float ms = time_ms([&] { CK(launch_matapply(j, 0)); }, 20);
            printf("k=3 r=7 mis_in=%d mis_out=%d %8.4f ms  hbm %7.1f GB/s\n", mi, mo, ms, 10.0 * bsz / (ms * 1e-3) / 1e9);
            CK(hipFree(xin));
            CK(hipFree(xout));
        }
    }
    if (getenv("MB_BATCH")) {  // cfg5 shape: 1e6 stripes of K=3 x 1366 B, rows 1536 apart; U and grid cap
        const int k = 3, r = 7;
        const size_t sz = 1366, ns = 1000000;
        const size_t ld = getenv("MB_LD") ? strtoull(getenv("MB_LD"), nullptr, 0) : 1536;
        printf("BATCH layout: rows of %zu B at stride %zu\n", sz, ld);
        uint8_t *xin, *xout;
        CK(hipMalloc(&xin, ns * k * ld));
        CK(hipMalloc(&xout, ns * r * ld));
        CK(hipMemset(xin, 0x5a, ns * k * ld));
        struct V {
            const char* name;
            KernelFn fn;
            int upl;
        } vs[] = {{"reg<3,7>PF-AL", matapply_reg<3, 7, true, 1, 0, true, 0, true>, 1}, {"copy_walk", copy_walk<3, 7>, 1},
                  {"reg<3,7>U2", matapply_reg<3, 7, true, 2>, 2}};
        std::vector<std::vector<float>> t(3 * 4);
        const int gms[4] = {16, 64, 256, 1024};
        for (int round = 0; round < 5; ++round)
            for (int i = 0; i < 3; ++i)
                for (int g = 0; g < 4; ++g) {
                    const Variant saved = g_reg[3][7];
                    g_reg[3][7] = Variant{vs[i].fn, vs[i].name, 0, true, vs[i].upl};
                    g_grid_mult = gms[g];
                    MatJob j = make_job(xin, xout, k, r, sz, ld);
                    j.nstripes = ns;
                    j.in_sstride = k * ld;
                    j.out_sstride = r * ld;
                    for (int b = 0; b < k; ++b) j.in[b] = xin + b * ld;
                    for (int b = 0; b < r; ++b) j.out[b] = xout + b * ld;
                    t[i * 4 + g].push_back(time_ms([&] { MatJob jj = j; CK(launch_matapply(jj, 0)); }, 5));
                    g_reg[3][7] = saved;
                }
        for (int i = 0; i < 3; ++i)
            for (int g = 0; g < 4; ++g) {
                auto& v = t[i * 4 + g];
                std::sort(v.begin(), v.end());
                printf("BATCH %-12s gm=%4d median %8.4f ms  hbm %7.1f GB/s\n", vs[i].name, gms[g], v[2],
                       double(k + r) * sz * ns / (v[2] * 1e-3) / 1e9);
            }
        return 0;
    }
    if (getenv("MB_AB")) {  // interleaved A/B of general-kernel variants: 7 rounds, median (guide §5.4 rule 24)
        struct V {
            const char* name;
            KernelFn fn;
            bool ktab, lds;
            int chunk;
        } vs[] = {
            {"auto", nullptr, false, true, 8},
            {"pad6", matapply_lds<false, true, 6, 2, 2, kTilesPadded>, false, true, 8},
            {"pad6-nomem", matapply_lds<false, true, 6, 2, 2, kTilesPadded, 1>, false, true, 8},
            {"pad6-noalu", matapply_lds<false, true, 6, 2, 2, kTilesPadded, 2>, false, true, 8},
            {"pad20", matapply_lds<false, true, 20, 2, 2, kTilesPadded>, false, true, 8},
            {"pad20-nomem", matapply_lds<false, true, 20, 2, 2, kTilesPadded, 1>, false, true, 8},
            {"pad20-noalu", matapply_lds<false, true, 20, 2, 2, kTilesPadded, 2>, false, true, 8},
        };
        const int shapes_all[][2] = {{10, 6}, {16, 6}, {20, 40}, {20, 20}};
        std::vector<std::array<int, 2>> shapes;
        if (const char* e = getenv("MB_SHAPE")) {  // "k,r": one shape only (for counter runs)
            int a = 0, b = 0;
            sscanf(e, "%d,%d", &a, &b);
            shapes.push_back({a, b});
        } else {
            for (auto& sh : shapes_all) shapes.push_back({sh[0], sh[1]});
        }
        const char* only = getenv("MB_VARIANT");  // one variant name only
        const int nv = sizeof(vs) / sizeof(vs[0]);
        for (auto& sh : shapes) {
            const int k = sh[0], r = sh[1];
            const size_t bsz = (S / k + 255) / 256 * 256;
            uint8_t *xin, *xout;
            CK(hipMalloc(&xin, k * bsz));
            CK(hipMalloc(&xout, r * bsz));
            CK(hipMemset(xin, 0x5a, k * bsz));
            std::vector<std::vector<float>> t(nv);
            std::vector<uint8_t> want(r * bsz), got(r * bsz);
            {
                MatJob j = make_job(xin, xout, k, r, bsz, bsz);
                CK(launch_matapply(j, 0));
                CK(hipMemcpy(want.data(), xout, r * bsz, hipMemcpyDeviceToHost));
            }
            for (int round = 0; round < 7; ++round)
                for (int i = 0; i < nv; ++i) {
                    if (vs[i].ktab && k * r > kMaxKernargTables) continue;
                    if (only && strcmp(only, vs[i].name)) continue;
                    if (!strncmp(vs[i].name, "pad", 3) && atoi(vs[i].name + 3) != (int)pick(k, r, false)->pad_tile) continue;
                    Variant* slot = pick(k, r, false);
                    const Variant saved = *slot;
                    if (vs[i].fn) *slot = Variant{vs[i].fn, vs[i].name, 0, vs[i].ktab, 1, vs[i].lds, vs[i].chunk};
                    g_grid_mult = getenv("MB_GM") ? atoi(getenv("MB_GM")) : 16;
                    MatJob j = make_job(xin, xout, k, r, bsz, bsz);
                    if (round == 0) CK(hipMemset(xout, 0, r * bsz));
                    t[i].push_back(time_ms([&] { MatJob jj = j; CK(launch_matapply(jj, 0)); }, 10));
                    *slot = saved;
                    if (round == 0) {
                        CK(hipMemcpy(got.data(), xout, r * bsz, hipMemcpyDeviceToHost));
                        if (!strstr(vs[i].name, "-no") && memcmp(got.data(), want.data(), r * bsz)) printf("MISMATCH k=%d r=%d %s\n", k, r, vs[i].name);
                    }
                }
            for (int i = 0; i < nv; ++i) {
                if (t[i].empty()) continue;
                std::sort(t[i].begin(), t[i].end());
                const double by = double(k + r) * bsz;
                printf("AB k=%2d r=%2d %-10s median %8.4f ms  hbm %7.1f GB/s  input %7.1f GB/s\n", k, r, vs[i].fn ? vs[i].name : pick(k, r, false)->name,
                       t[i][3], by / (t[i][3] * 1e-3) / 1e9, double(k) * bsz / (t[i][3] * 1e-3) / 1e9);
            }
            CK(hipFree(xin));
            CK(hipFree(xout));
        }
        return 0;
    }
    {  // kernel variants of the K=3 register path, aligned layout
        struct V {
            const char* name;
            KernelFn fn;
            int upl;
            int k, r;
        } vs[] = {
            {"reg<3,7> nt U1", matapply_reg<3, 7, true, 1>, 1, 3, 7},
            {"reg<3,7> nt U2", matapply_reg<3, 7, true, 2>, 2, 3, 7},
            {"reg<3,7> plain U1", matapply_reg<3, 7, false, 1>, 1, 3, 7},
            {"reg<3,7> plain U2", matapply_reg<3, 7, false, 2>, 2, 3, 7},
            {"reg<3,3> nt U1", matapply_reg<3, 3, true, 1>, 1, 3, 3},
            {"reg<3,3> nt U2", matapply_reg<3, 3, true, 2>, 2, 3, 3},
            {"reg<3,3> plain U1", matapply_reg<3, 3, false, 1>, 1, 3, 3},
            {"reg<3,7> nt PF", matapply_reg<3, 7, true, 1, 0, true>, 1, 3, 7},
            {"reg<3,7> nt W7", matapply_reg<3, 7, true, 1, 0, false, 7>, 1, 3, 7},
            {"reg<3,7> nt W8", matapply_reg<3, 7, true, 1, 0, false, 8>, 1, 3, 7},
            {"reg<3,7> nt PF W7", matapply_reg<3, 7, true, 1, 0, true, 7>, 1, 3, 7},
            {"reg<3,3> nt W8", matapply_reg<3, 3, true, 1, 0, false, 8>, 1, 3, 3},
            {"reg<3,3> nt PF", matapply_reg<3, 3, true, 1, 0, true>, 1, 3, 3},
            {"reg<3,7> nt PF AL", matapply_reg<3, 7, true, 1, 0, true, 0, true>, 1, 3, 7},
            {"reg<3,7> nt U1 AL", matapply_reg<3, 7, true, 1, 0, false, 0, true>, 1, 3, 7},
            {"reg<3,3> nt U1 AL", matapply_reg<3, 3, true, 1, 0, false, 0, true>, 1, 3, 3},
            {"reg<3,3> nt PF AL", matapply_reg<3, 3, true, 1, 0, true, 0, true>, 1, 3, 3},
            {"reg<3,3> nt U2 AL", matapply_reg<3, 3, true, 2, 0, false, 0, true>, 2, 3, 3},
        };
        for (auto& v : vs) {
            const Variant saved = g_reg[v.k][v.r];
            g_reg[v.k][v.r] = Variant{v.fn, v.name, 0, true, v.upl};
            const size_t bsz = (S / v.k + 255) / 256 * 256;
            uint8_t *xin, *xout;
            CK(hipMalloc(&xin, v.k * bsz));
            CK(hipMalloc(&xout, v.r * bsz));
            CK(hipMemset(xin, 0x5a, v.k * bsz));
            hipFuncAttributes attr;
            CK(hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(v.fn)));
            for (int gm : {1, 2, 16}) {
                g_grid_mult = gm;
                MatJob j = make_job(xin, xout, v.k, v.r, bsz, bsz);
                float ms = time_ms([&] { CK(launch_matapply(j, 0)); }, 20);
                printf("variant %-18s vgpr=%3d sgpr=%3d gm=%2d %8.4f ms  hbm %7.1f GB/s\n", v.name, attr.numRegs,
                       0, gm, ms, double(v.k + v.r) * bsz / (ms * 1e-3) / 1e9);
            }
            CK(hipFree(xin));
            CK(hipFree(xout));
            g_reg[v.k][v.r] = saved;
        }
    }
    if (getenv("MB_MIS_ONLY")) return 0;
    const int shapes[][2] = {{3, 7}, {3, 3}, {10, 6}, {10, 4}, {20, 40}, {20, 20}, {16, 16}, {32, 32}, {5, 8}};
    for (auto& sh : shapes) {
        const int k = sh[0], r = sh[1];
        const size_t bsz = (S / k + 255) / 256 * 256;
        for (int mis : {0, 6}) {
            const size_t stride = bsz + mis;
            uint8_t *xin, *xout;
            CK(hipMalloc(&xin, k * stride + 256));
            CK(hipMalloc(&xout, r * stride + 256));
            CK(hipMemset(xin, 0x5a, k * stride + 256));
            for (int gm : {1, 4, 16}) {
                g_grid_mult = gm;
                MatJob j = make_job(xin, xout, k, r, bsz, stride);
                float ms = time_ms([&] { CK(launch_matapply(j, 0)); }, 20);
                const double by = double(k + r) * bsz;
                printf("k=%2d r=%2d mis=%d gm=%2d %-14s %8.4f ms  hbm %7.1f GB/s  input %7.1f GB/s\n", k, r, mis, gm,
                       matapply_variant_name(k, r, false), ms, by / (ms * 1e-3) / 1e9,
                       double(k) * bsz / (ms * 1e-3) / 1e9);
            }
            CK(hipFree(xin));
            CK(hipFree(xout));
        }
    }
    return 0;
}
