// inline_probe.hip -- a synchronous 4 KiB K=3/M=10 encode from host memory
// (the Python bytes API's smallest call), launch to completion seen by the
// host, with the k input blocks reaching the kernel two ways:
//
//   pinned   the inputs copied into a pinned host buffer, the kernel loads
//            them over PCIe (the library's small-call path, fec_abi.cpp
//            run_single): a PCIe read round trip inside the kernel
//   inline   the inputs copied into the kernel's argument block; HIP copies
//            the arguments to device memory with the launch (posted writes),
//            and the kernel reads them from there
//
// Both write the 7 output blocks to pinned host memory and then a completion
// word (system-scope release); the host spins on it and copies the outputs
// out.  Also: how large an argument block hipLaunchKernel accepts.
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/inline_probe.hip -o tools/inline_probe.exe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

constexpr int K = 3, R = 7;
constexpr uint32_t kSz = 1366;
constexpr uint32_t kSlot = 1376;  // 16-byte multiple

struct PinnedArgs {
    const uint8_t* in;  // K slots of kSlot bytes (pinned host)
    uint8_t* out;       // R slots (pinned host)
    uint32_t* flag;
    uint32_t seq;
};

template <int BYTES>
struct InlineArgs {
    uint8_t* out;
    uint32_t* flag;
    uint32_t seq;
    uint32_t pad;
    u32x4 data[BYTES / 16];
};

template <int SP>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
    if constexpr (SP == 0)
        *reinterpret_cast<u32x4*>(p) = v;
    else if constexpr (SP == 1)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void finish(uint32_t* flag, uint32_t seq) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int SP>
__global__ __launch_bounds__(256) void enc_pinned(const PinnedArgs a) {
    const uint32_t u = threadIdx.x;
    if (u < kSlot / 16) {
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = *reinterpret_cast<const u32x4*>(a.in + j * kSlot + u * 16);
#pragma unroll
        for (int r = 0; r < R; ++r)
            st16<SP>(a.out + r * kSlot + u * 16, x[0] ^ x[1] ^ x[2] ^ uint32_t(r));
    }
    finish(a.flag, a.seq);
}

template <int BYTES, int SP>
__global__ __launch_bounds__(256) void enc_inline(const InlineArgs<BYTES> a) {
    const uint32_t u = threadIdx.x;
    if (u < kSlot / 16) {
        u32x4 x[K];
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = a.data[j * (kSlot / 16) + u];
#pragma unroll
        for (int r = 0; r < R; ++r)
            st16<SP>(a.out + r * kSlot + u * 16, x[0] ^ x[1] ^ x[2] ^ uint32_t(r));
    }
    finish(a.flag, a.seq);
}

template <int BYTES>
__global__ void big_arg(const InlineArgs<BYTES> a) {
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int i = 0; i < BYTES / 16; ++i) s += a.data[i].x + a.data[i].w;
        __hip_atomic_store(a.flag, s + a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

template <int BYTES>
static void try_size(uint32_t* flag, uint32_t* flag_dev) {
    auto* a = new InlineArgs<BYTES>();
    a->flag = flag_dev;
    a->seq = 5;
    uint32_t want = 5;
    for (int i = 0; i < BYTES / 16; ++i) {
        a->data[i] = u32x4{uint32_t(i), 0u, 0u, 1u};
        want += uint32_t(i) + 1u;
    }
    *flag = 0;
    hipLaunchKernelGGL(big_arg<BYTES>, dim3(1), dim3(64), 0, 0, *a);
    const hipError_t e = hipGetLastError();
    const hipError_t s = hipDeviceSynchronize();
    printf("argument block %6d B: launch %s, sync %s, result %s\n", int(sizeof(InlineArgs<BYTES>)),
           hipGetErrorString(e), hipGetErrorString(s), *flag == want ? "correct" : "WRONG");
    (void)hipGetLastError();
    delete a;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 3000;
    CK(hipSetDevice(0));
    uint32_t *flag, *flag_dev;
    uint8_t *hin, *hin_dev, *hout, *hout_dev;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_dev), flag, 0));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hin), K * kSlot, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hin_dev), hin, 0));
    CK(hipHostMalloc(reinterpret_cast<void**>(&hout), R * kSlot, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hout_dev), hout, 0));
    try_size<2048>(flag, flag_dev);
    try_size<4000>(flag, flag_dev);
    try_size<4096>(flag, flag_dev);
    try_size<8192>(flag, flag_dev);

    // the caller's blocks (pageable) and outputs
    std::vector<uint8_t> src(K * kSz), dst(R * kSz), ref(R * kSz);
    for (size_t i = 0; i < src.size(); ++i) src[i] = uint8_t(i * 131 + 7);
    for (int r = 0; r < R; ++r)
        for (uint32_t b = 0; b < kSz; ++b) {
            const uint8_t x = src[b] ^ src[kSz + b] ^ src[2 * kSz + b];
            ref[r * kSz + b] = x ^ ((b & 3) == 0 ? uint8_t(r) : 0);
        }
    uint32_t seq = 0;
    auto spin = [&](uint32_t s) {
        const double t0 = now_us();
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s)
            if (now_us() - t0 > 1e6) {
                fprintf(stderr, "flag timeout\n");
                exit(1);
            }
    };
    auto* ia = new InlineArgs<K * kSlot>();
    auto call_pinned = [&](auto fn) {
        for (int j = 0; j < K; ++j) memcpy(hin + j * kSlot, &src[j * kSz], kSz);
        PinnedArgs a{hin_dev, hout_dev, flag_dev, ++seq};
        hipLaunchKernelGGL(fn, dim3(1), dim3(256), 0, 0, a);
        spin(a.seq);
        for (int r = 0; r < R; ++r) memcpy(&dst[r * kSz], hout + r * kSlot, kSz);
    };
    auto call_inline = [&](auto fn) {
        for (int j = 0; j < K; ++j) memcpy(reinterpret_cast<uint8_t*>(ia->data) + j * kSlot, &src[j * kSz], kSz);
        ia->out = hout_dev;
        ia->flag = flag_dev;
        ia->seq = ++seq;
        hipLaunchKernelGGL(fn, dim3(1), dim3(256), 0, 0, *ia);
        spin(ia->seq);
        for (int r = 0; r < R; ++r) memcpy(&dst[r * kSz], hout + r * kSlot, kSz);
    };
    call_pinned(enc_pinned<2>);
    printf("pinned result %s\n", memcmp(dst.data(), ref.data(), dst.size()) ? "WRONG" : "correct");
    memset(dst.data(), 0, dst.size());
    call_inline(enc_inline<K * kSlot, 2>);
    printf("inline result %s (argument block %zu B)\n", memcmp(dst.data(), ref.data(), dst.size()) ? "WRONG" : "correct",
           sizeof(*ia));
    const char* names[6] = {"pinned plain", "pinned nt", "pinned nt sc1", "inline plain", "inline nt", "inline nt sc1"};
    for (int round = 0; round < 3; ++round) {
        std::vector<double> t[6];
        for (int i = 0; i < n; ++i) {
            for (int v = 0; v < 6; ++v) {
                const double t0 = now_us();
                switch (v) {
                    case 0: call_pinned(enc_pinned<0>); break;
                    case 1: call_pinned(enc_pinned<1>); break;
                    case 2: call_pinned(enc_pinned<2>); break;
                    case 3: call_inline(enc_inline<K * kSlot, 0>); break;
                    case 4: call_inline(enc_inline<K * kSlot, 1>); break;
                    default: call_inline(enc_inline<K * kSlot, 2>); break;
                }
                t[v].push_back(now_us() - t0);
            }
        }
        printf("round %d (medians of %d, interleaved):", round, n);
        for (int v = 0; v < 6; ++v) printf("  %s %.2f", names[v], median(t[v]));
        printf(" us\n");
    }
    CK(hipDeviceSynchronize());
    delete ia;
    return 0;
}
