// mb_store.hip -- cache policy of the output stores of the K=3/M=10 register
// kernels (matapply_reg<3,7> encode, <3,3> decode): nt (production), sc1, sc0 sc1,
// over K=3 single stripes of 8-512 MiB, batches of 1 MiB stripes and cfg5.
//
// A kernel that streams ~150 MB of stores ends with the XCD L2s full of dirty
// lines; the end-of-kernel release writes them back before the next kernel of
// the stream starts (MI355X_MICROARCH.md, row "boundary": + B / 6 TB/s).  sc1
// stores leave nothing dirty behind.  Timed: back-to-back launches between
// two events (per-launch wall time, boundaries included) and single launches
// between their own events; interleaved rounds, medians; outputs compared.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_store.hip zfec_amd/csrc/bitslice.cpp \
//          zfec_amd/csrc/gf256.cpp -ldl -o tools/mb_store.exe
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

int main() {
    std::call_once(g_dispatch_once, init_dispatch);
    set_jit_mode(kJitOff);
    struct V {
        const char* name;
        int r;
        KernelFn fn;
    } vs[] = {{"nt", 7, matapply_reg<3, 7, true, 1, 0, true>},
              {"sc1", 7, matapply_reg<3, 7, true, 1, 1, true>},
              {"sc0sc1", 7, matapply_reg<3, 7, true, 1, 2, true>},
              {"dec-nt", 3, matapply_reg<3, 3, true, 1, 0>},
              {"dec-sc0sc1", 3, matapply_reg<3, 3, true, 1, 2>}};
    const int nv = sizeof(vs) / sizeof(vs[0]);
    // K=3 single stripes of 8 MiB .. 512 MiB, batches of 1 MiB stripes, and cfg5
    struct Shape {
        char name[32];
        size_t sz, ld, ns;
    };
    std::vector<Shape> shapes;
    for (size_t mib : {8, 16, 32, 64, 96, 128, 192, 256, 512}) {
        Shape sh;
        snprintf(sh.name, sizeof sh.name, "%zu MiB x1", mib);
        sh.sz = ((mib << 20) + 2) / 3;
        sh.ld = (sh.sz + 255) / 256 * 256;
        sh.ns = 1;
        shapes.push_back(sh);
    }
    for (size_t ns : {32, 64, 128, 256}) {
        Shape sh;
        snprintf(sh.name, sizeof sh.name, "1 MiB x%zu", ns);
        sh.sz = 349526;
        sh.ld = 349696;
        sh.ns = ns;
        shapes.push_back(sh);
    }
    if (!getenv("MB_NO_CFG5")) shapes.push_back(Shape{"cfg5 4KiB x1e6", 1366, 1536, 1000000});
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (const Shape& sh : shapes) {
        const int k = 3, r = 7;  // buffers sized for the widest variant
        uint8_t *in, *out;
        CK(hipMalloc(&in, sh.ns * k * sh.ld));
        CK(hipMalloc(&out, sh.ns * r * sh.ld));
        CK(hipMemset(in, 0x5a, sh.ns * k * sh.ld));
        CK(hipMemset(out, 0, sh.ns * r * sh.ld));
        // each variant's previous output is compared with the same-r variant's
        std::vector<uint8_t> want[8], got(sh.ns * r * sh.ld);
        std::vector<std::vector<float>> t_b2b(nv), t_one(nv);
        const int reps = sh.ns > 1000 ? 5 : 20;
        for (int round = 0; round < 5; ++round)
            for (int v = 0; v < nv; ++v) {
                const int r = vs[v].r;
                Variant* slot = &g_reg[3][r];
                const Variant saved = *slot;
                *slot = Variant{vs[v].fn, vs[v].name, 0, true, 1};
                MatJob j;
                memset(&j, 0, sizeof j);
                j.sz = sh.sz;
                j.nstripes = sh.ns;
                j.k = k;
                j.r = r;
                j.in_sstride = k * sh.ld;
                j.out_sstride = r * sh.ld;
                for (int q = 0; q < k; ++q) j.in[q] = in + q * sh.ld;
                for (int q = 0; q < r; ++q) j.out[q] = out + q * sh.ld;
                for (int q = 0; q < k * r; ++q) j.coef[q] = uint8_t(q * 37 + 11);
                auto launch = [&] {
                    MatJob jj = j;
                    CK(launch_matapply(jj, 0));
                };
                launch();
                CK(hipDeviceSynchronize());
                if (round == 0) {
                    CK(hipMemcpy(got.data(), out, got.size(), hipMemcpyDeviceToHost));
                    if (want[r].empty())
                        want[r] = got;
                    else if (memcmp(want[r].data(), got.data(), got.size()))
                        printf("MISMATCH %s %s\n", sh.name, vs[v].name);
                }
                CK(hipEventRecord(a, 0));
                for (int i = 0; i < reps; ++i) launch();
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t_b2b[v].push_back(ms / reps);
                std::vector<float> one;
                for (int i = 0; i < 5; ++i) {
                    CK(hipEventRecord(a, 0));
                    launch();
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    one.push_back(ms);
                }
                std::sort(one.begin(), one.end());
                t_one[v].push_back(one[2]);
                *slot = saved;
            }
        for (int v = 0; v < nv; ++v) {
            std::sort(t_b2b[v].begin(), t_b2b[v].end());
            std::sort(t_one[v].begin(), t_one[v].end());
            const double bytes = double(k + vs[v].r) * sh.sz * sh.ns;
            printf("%-16s %-10s back-to-back %8.4f ms (%6.1f GB/s)   single %8.4f ms (%6.1f GB/s)\n", sh.name, vs[v].name,
                   t_b2b[v][2], bytes / (t_b2b[v][2] * 1e-3) / 1e9, t_one[v][2], bytes / (t_one[v][2] * 1e-3) / 1e9);
        }
        CK(hipFree(in));
        CK(hipFree(out));
    }
    return 0;
}
