// mb_sync.hip -- round trip of one small launch as a synchronous host call
// sees it (the floor of a small fec_encode from host memory): enqueue a tiny
// kernel and wait for it, four ways, on an otherwise idle GPU.
//   stream_sync  hipStreamSynchronize on the launch stream (what fec_abi.cpp does)
//   event_sync   hipEventRecord + hipEventSynchronize
//   event_query  hipEventRecord + spin on hipEventQuery
//   host_flag    the kernel's last store is a flag in pinned host memory (vector
//                store, system scope, after a system-scope release fence); the
//                host spins on it, then calls hipStreamSynchronize only every
//                64th call so the stream's bookkeeping keeps up
//   write_value  the kernel as usual, then hipStreamWriteValue32 of the flag
//                on the same stream; the host spins on the flag
//   flag_kernel  the kernel as usual, then a one-lane kernel that writes the flag
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mb_sync.hip -o tools/mb_sync.exe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
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

// one workgroup: copies 4 KiB and, when flag != nullptr, publishes `seq`
__global__ __launch_bounds__(256) void tiny(const uint4* in, uint4* out, volatile uint32_t* flag, uint32_t seq) {
    out[threadIdx.x] = in[threadIdx.x];
    if (flag) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(const_cast<uint32_t*>(flag), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

int main() {
    uint4 *in, *out;
    CK(hipMalloc(&in, 4096));
    CK(hipMalloc(&out, 4096));
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocDefault));
    *flag = 0;
    uint32_t* flag_dev = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_dev), flag, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int n = 2000;
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (int round = 0; round < 3; ++round) {
        for (int mode = 0; mode < 6; ++mode) {
            std::vector<double> us;
            us.reserve(n);
            uint32_t seq = 0;
            for (int i = 0; i < n + 50; ++i) {
                const auto t0 = now();
                if (mode >= 3) {
                    ++seq;
                    if (mode == 3) {
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, st, in, out, flag_dev, seq);
                    } else {
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, st, in, out, nullptr, 0u);
                        if (mode == 4)
                            CK(hipStreamWriteValue32(st, flag_dev, seq, 0));
                        else
                            hipLaunchKernelGGL(tiny, dim3(1), dim3(1), 0, st, in, out, flag_dev, seq);
                    }
                    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
                    }
                    if ((i & 63) == 63) CK(hipStreamSynchronize(st));
                } else {
                    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, st, in, out, nullptr, 0u);
                    if (mode == 0) {
                        CK(hipStreamSynchronize(st));
                    } else {
                        CK(hipEventRecord(ev, st));
                        if (mode == 1)
                            CK(hipEventSynchronize(ev));
                        else
                            while (hipEventQuery(ev) == hipErrorNotReady) {
                            }
                    }
                }
                const auto t1 = now();
                if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            CK(hipStreamSynchronize(st));
            std::sort(us.begin(), us.end());
            static const char* names[] = {"stream_sync", "event_sync", "event_query", "host_flag", "write_value",
                                          "flag_kernel"};
            printf("round %d %-12s median %6.2f us  p10 %6.2f  p90 %6.2f\n", round, names[mode], us[n / 2], us[n / 10],
                   us[n * 9 / 10]);
        }
    }
    return 0;
}
