// argsize_ab.hip -- host cost of hipLaunchKernel by argument-block size,
// interleaved: blocks of 2000 launches of each size in turn, 15 rounds, so the
// drift of the launch rate within a process (tools/host_cost.hip) hits every
// size alike.  Medians of the per-block means.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/argsize_ab.hip -o tools/argsize_ab.exe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int N>
struct Arg {
    unsigned char b[N];
};

template <int N>
__global__ void empty_kernel(const Arg<N> a) {
    if (a.b[0] == 0xEE && threadIdx.x == 9999) asm volatile("s_nop 0");
}

template <int N>
double block_us(hipStream_t st, int n) {
    Arg<N> a{};
    void* args[] = {&a};
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i)
        (void)hipLaunchKernel(reinterpret_cast<const void*>(empty_kernel<N>), dim3(1), dim3(256), args, 0, st);
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipStreamSynchronize(st);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    for (int i = 0; i < 50000; ++i) (void)block_us<16>(st, 1);
    const int sizes[] = {16, 64, 112, 128, 256, 560, 1024};
    std::vector<double> t[7];
    for (int round = 0; round < 15; ++round) {
        t[0].push_back(block_us<16>(st, 2000));
        t[1].push_back(block_us<64>(st, 2000));
        t[2].push_back(block_us<112>(st, 2000));
        t[3].push_back(block_us<128>(st, 2000));
        t[4].push_back(block_us<256>(st, 2000));
        t[5].push_back(block_us<560>(st, 2000));
        t[6].push_back(block_us<1024>(st, 2000));
    }
    printf("hipLaunchKernel host cost by argument size, interleaved blocks of 2000, 15 rounds (median / min / max us)\n");
    for (int i = 0; i < 7; ++i) {
        std::vector<double> v = t[i];
        std::sort(v.begin(), v.end());
        printf("  %5d B  %.2f  %.2f  %.2f\n", sizes[i], v[v.size() / 2], v.front(), v.back());
    }
    return 0;
}
