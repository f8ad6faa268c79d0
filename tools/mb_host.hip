// mb_host.hip -- host-memory paths for one K=3/M=10 64 MiB stripe:
//   copies: H2D alone, D2H alone, both at once on two streams (does PCIe run
//   both directions together through hipMemcpyAsync?);
//   zero-copy: the encode kernel reading / writing pinned host memory directly.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_host.hip -o tools/mb_host.exe
#include "../zfec_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <algorithm>

using namespace zfec_hip;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

template <class F>
float time_ms(F&& f, int iters, hipStream_t s = 0) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b, s));
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / iters;
}

int main() {
    const int k = 3, r = 7;
    const size_t sz = (size_t(64) << 20) / k / 256 * 256;
    uint8_t *hin, *hout, *din, *dout;
    CK(hipHostMalloc(&hin, k * sz, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, r * sz, hipHostMallocDefault));
    CK(hipMalloc(&din, k * sz));
    CK(hipMalloc(&dout, r * sz));
    memset(hin, 0x5a, k * sz);
    memset(hout, 0, r * sz);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    float h2d = time_ms([&] { CK(hipMemcpyAsync(din, hin, k * sz, hipMemcpyHostToDevice, s1)); }, 5, s1);
    float d2h = time_ms([&] { CK(hipMemcpyAsync(hout, dout, r * sz, hipMemcpyDeviceToHost, s2)); }, 5, s2);
    printf("H2D %zu B: %.3f ms %.1f GB/s\n", k * sz, h2d, k * sz / (h2d * 1e-3) / 1e9);
    printf("D2H %zu B: %.3f ms %.1f GB/s\n", r * sz, d2h, r * sz / (d2h * 1e-3) / 1e9);
    auto both = [&] {
        CK(hipMemcpyAsync(din, hin, k * sz, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(hout, dout, r * sz, hipMemcpyDeviceToHost, s2));
    };
    both();
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 5; ++i) both();
    CK(hipDeviceSynchronize());
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / 5;
    printf("H2D+D2H concurrently: %.3f ms (serial sum %.3f)\n", ms, h2d + d2h);
    // chunked: 2 MiB pieces per block, the pipeline's copy pattern
    const size_t C = 2 << 20;
    auto chunked = [&] {
        for (size_t off = 0; off < sz; off += C) {
            const size_t len = std::min(C, sz - off);
            for (int j = 0; j < k; ++j)
                CK(hipMemcpyAsync(din + j * sz + off, hin + j * sz + off, len, hipMemcpyHostToDevice, s1));
            for (int i = 0; i < r; ++i)
                CK(hipMemcpyAsync(hout + i * sz + off, dout + i * sz + off, len, hipMemcpyDeviceToHost, s2));
        }
    };
    chunked();
    CK(hipDeviceSynchronize());
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 5; ++i) chunked();
    CK(hipDeviceSynchronize());
    ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / 5;
    printf("chunked 2 MiB both directions: %.3f ms\n", ms);
    // zero-copy kernels
    auto job = [&](uint8_t* in, uint8_t* out) {
        MatJob j;
        memset(&j, 0, sizeof j);
        j.sz = sz;
        j.nstripes = 1;
        j.k = k;
        j.r = r;
        for (int i = 0; i < k; ++i) j.in[i] = in + i * sz;
        for (int i = 0; i < r; ++i) j.out[i] = out + i * sz;
        for (int i = 0; i < k * r; ++i) j.coef[i] = uint8_t(i * 37 + 11);
        return j;
    };
    struct {
        const char* name;
        uint8_t *in, *out;
    } cases[] = {{"dev->dev", din, dout}, {"host->dev", hin, dout}, {"dev->host", din, hout}, {"host->host", hin, hout}};
    for (auto& c : cases) {
        MatJob j = job(c.in, c.out);
        float t = time_ms([&] { MatJob jj = j; CK(launch_matapply(jj, s1)); }, 5, s1);
        printf("zero-copy encode %-10s %.3f ms  %.1f GB/s of input\n", c.name, t, k * sz / (t * 1e-3) / 1e9);
    }
    return 0;
}
