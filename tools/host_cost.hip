// host_cost.hip -- what one batched C-ABI call costs the host, piece by piece
// (VERDICT r02 "cut the per-launch host cost").  Device buffers, a 4 KiB
// K=3/M=10 stripe (so the GPU never limits the enqueue rate), N calls timed on
// the host clock, against the HIP calls the library makes per call.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/host_cost.hip -Iinclude \
//          -Lzfec_amd -lzfec_hip -Wl,-rpath,$PWD/zfec_amd -o tools/host_cost.exe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "zfec_hip.h"

template <int N>
struct Arg {
    unsigned char b[N];
};

template <int N>
__global__ void empty_kernel(const Arg<N> a) {
    if (a.b[0] == 0xEE && threadIdx.x == 9999) asm volatile("s_nop 0");
}

template <class F>
double per_call_us(F f, int n = 20000) {
    for (int i = 0; i < 200; ++i) f();
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) f();
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipDeviceSynchronize();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    fec_init();
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const size_t sz = 4096, ld = 4096;
    unsigned char *src, *dst;
    (void)hipMalloc(&src, 3 * ld);
    (void)hipMalloc(&dst, 7 * ld);
    fec_t* code = fec_new(3, 10);
    const unsigned nums[7] = {3, 4, 5, 6, 7, 8, 9};
    const unsigned slots[3] = {7, 8, 9};
    hipPointerAttribute_t attr;
    int dev = 0, cnt = 0;
    Arg<16> a16{};
    Arg<64> a64{};
    Arg<72> a72{};
    Arg<80> a80{};
    Arg<96> a96{};
    Arg<112> a112{};
    Arg<128> a128{};
    Arg<192> a192{};
    Arg<256> a256{};
    Arg<384> a384{};
    Arg<560> a560{};
    Arg<1024> a1024{};
    Arg<2240> a2240{};
    // the launch rate climbs over the first ~10^5 launches of a process (CPU
    // clock, runtime pools): without this warm-up the first rows read up to
    // 1 us slower than the same launches later in the run
    for (int i = 0; i < 100000; ++i) hipLaunchKernelGGL(empty_kernel<16>, dim3(1), dim3(256), 0, st, a16);
    (void)hipDeviceSynchronize();
    printf("host cost per call (us), %s (after 10^5 warm-up launches)\n", fec_version());
    printf("  hipGetDeviceCount          %6.2f\n", per_call_us([&] { (void)hipGetDeviceCount(&cnt); }));
    printf("  hipGetDevice               %6.2f\n", per_call_us([&] { (void)hipGetDevice(&dev); }));
    printf("  hipPointerGetAttributes    %6.2f\n", per_call_us([&] { (void)hipPointerGetAttributes(&attr, src); }));
    printf("  hipGetLastError            %6.2f\n", per_call_us([&] { (void)hipGetLastError(); }));
    printf("  launch, 16 B kernarg       %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<16>, dim3(1), dim3(256), 0, st, a16); }));
    printf("  launch, 64 B kernarg       %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<64>, dim3(1), dim3(256), 0, st, a64); }));
    printf("  launch, 72 B kernarg       %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<72>, dim3(1), dim3(256), 0, st, a72); }));
    printf("  launch, 80 B kernarg       %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<80>, dim3(1), dim3(256), 0, st, a80); }));
    printf("  launch, 96 B kernarg       %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<96>, dim3(1), dim3(256), 0, st, a96); }));
    printf("  launch, 112 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<112>, dim3(1), dim3(256), 0, st, a112); }));
    printf("  launch, 128 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<128>, dim3(1), dim3(256), 0, st, a128); }));
    printf("  launch, 192 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<192>, dim3(1), dim3(256), 0, st, a192); }));
    printf("  launch, 256 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<256>, dim3(1), dim3(256), 0, st, a256); }));
    printf("  launch, 384 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<384>, dim3(1), dim3(256), 0, st, a384); }));
    printf("  launch, 1024 B kernarg     %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<1024>, dim3(1), dim3(256), 0, st, a1024); }));
    printf("  launch, 560 B kernarg      %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<560>, dim3(1), dim3(256), 0, st, a560); }));
    printf("  launch, 2240 B kernarg     %6.2f\n",
           per_call_us([&] { hipLaunchKernelGGL(empty_kernel<2240>, dim3(1), dim3(256), 0, st, a2240); }));
    {
        // the same 560-byte launch through the module API with one argument buffer
        hipFunction_t f = nullptr;
        if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(empty_kernel<560>)) == hipSuccess && f) {
            size_t size = sizeof a560;
            void* conf[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a560, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                            HIP_LAUNCH_PARAM_END};
            printf("  module launch, 560 B buffer %5.2f\n", per_call_us([&] {
                       (void)hipModuleLaunchKernel(f, 1, 1, 1, 256, 1, 1, 0, st, nullptr, conf);
                   }));
            void* args[] = {&a560};
            printf("  module launch, 560 B params %5.2f\n", per_call_us([&] {
                       (void)hipModuleLaunchKernel(f, 1, 1, 1, 256, 1, 1, 0, st, args, nullptr);
                   }));
        } else {
            printf("  hipGetFuncBySymbol failed\n");
        }
        void* args[] = {&a560};
        printf("  hipLaunchKernel 560 B      %6.2f\n", per_call_us([&] {
                   (void)hipLaunchKernel(reinterpret_cast<const void*>(empty_kernel<560>), dim3(1), dim3(256), args, 0,
                                         st);
               }));
        printf("  hipExtLaunchKernel 560 B   %6.2f\n", per_call_us([&] {
                   (void)hipExtLaunchKernel(reinterpret_cast<const void*>(empty_kernel<560>), dim3(1), dim3(256),
                                            args, 0, st, nullptr, nullptr, 0);
               }));
    }
    printf("  fec_encode_batch 3->7      %6.2f\n", per_call_us([&] {
               fec_encode_batch(code, src, ld, 3 * ld, dst, ld, 7 * ld, nums, 7, sz, 1, st,
                                FEC_FLAG_ASYNC | FEC_FLAG_ROW_PADDING);
           }));
    printf("  fec_decode_batch 3->3      %6.2f\n", per_call_us([&] {
               fec_decode_batch(code, dst + 4 * ld, ld, 3 * ld, src, ld, 3 * ld, slots, sz, 1, st,
                                FEC_FLAG_ASYNC | FEC_FLAG_ROW_PADDING);
           }));
    const gf* in[3] = {src, src + ld, src + 2 * ld};
    gf* out[7];
    for (int i = 0; i < 7; ++i) out[i] = dst + i * ld;
    printf("  fec_encode_ex 3->7         %6.2f\n",
           per_call_us([&] { fec_encode_ex(code, in, out, nums, 7, sz, st, FEC_FLAG_ASYNC); }));
    printf("  last status %d (%s), kernel %s\n", fec_last_status(), fec_last_error_message(), fec_last_kernel_name());
    {
        // synchronous small calls from pageable host memory, launch to return:
        // the Python bytes API's 4 KiB K=3/M=10 stripe (sz = 1366) without Python
        const size_t hs = 1366;
        std::vector<unsigned char> h(10 * hs, 7);
        const gf* hin[3] = {&h[0], &h[hs], &h[2 * hs]};
        gf* hout[7];
        for (int i = 0; i < 7; ++i) hout[i] = &h[(3 + i) * hs];
        printf("  sync 4 KiB encode, host, FEC_FLAG_HOST_MEMORY %6.2f\n",
               per_call_us([&] { fec_encode_ex(code, hin, hout, nums, 7, hs, nullptr, FEC_FLAG_HOST_MEMORY); }, 5000));
        printf("  sync 4 KiB encode, host, classified           %6.2f\n",
               per_call_us([&] { fec_encode(code, hin, hout, nums, 7, hs); }, 5000));
        const gf* dinb[3] = {hout[4], hout[5], hout[6]};
        gf* doutb[3] = {&h[0], &h[hs], &h[2 * hs]};
        printf("  sync 4 KiB decode 3->3, host, FEC_FLAG_HOST_MEMORY %6.2f\n",
               per_call_us([&] { fec_decode_ex(code, dinb, doutb, slots, hs, nullptr, FEC_FLAG_HOST_MEMORY); }, 5000));
        printf("  last status %d (%s), kernel %s, signal wait %d\n", fec_last_status(), fec_last_error_message(),
               fec_last_kernel_name(), fec_last_wait());
    }
    fec_free(code);
    return 0;
}
