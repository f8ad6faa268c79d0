// mb_valu.hip -- issue rate of the VALU ops the GF(2^8) kernels are made of
// (v_perm_b32, v_bitop3_b32, v_and_b32, v_lshrrev_b32), one SGPR operand vs
// none, at several waves per SIMD.  Prints lane-ops/s chip-wide.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mb_valu.hip -o tools/mb_valu.exe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int ITERS = 4096;

// 8 independent chains, each op depends on the previous op of its chain.
template <int OP>
__global__ __launch_bounds__(256) void valu_loop(uint32_t* out, uint32_t s0, uint32_t s1) {
    uint32_t v[8];
    for (int i = 0; i < 8; ++i) v[i] = threadIdx.x * 0x01010101u + i;
    uint32_t t = threadIdx.x ^ 0x5a5a5a5au;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0)  // v_perm, hi from SGPR, lo VGPR
                asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "s"(s0), "v"(t));
            else if constexpr (OP == 1)  // v_perm, same SGPR twice
                asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(v[i]) : "s"(s0));
            else if constexpr (OP == 2)  // v_perm, all VGPR
                asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(t), "v"(t));
            else if constexpr (OP == 3)  // xor3
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(t), "v"(t));
            else if constexpr (OP == 4)  // v_and
                asm volatile("v_and_b32 %0, %1, %0" : "+v"(v[i]) : "v"(t));
            else if constexpr (OP == 5)  // v_xor (VOP2)
                asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(t));
            else if constexpr (OP == 6)  // v_lshlrev_b32 (VOP2 shift)
                asm volatile("v_lshlrev_b32 %0, 4, %0" : "+v"(v[i]));
            else if constexpr (OP == 7)  // v_lshl_or_b32 (VOP3)
                asm volatile("v_lshl_or_b32 %0, %0, 4, %1" : "+v"(v[i]) : "v"(t));
        }
    }
    uint32_t acc = 0;
    for (int i = 0; i < 8; ++i) acc ^= v[i];
    if (acc == 0x12345678u) out[0] = acc;
}

// 64-bit shifts of register pairs (8 independent chains of 64 bits): one
// v_lshlrev_b64 moves two 32-bit words; counted here as 2 lane-ops (the two
// dwords it shifts), so equal to v_lshlrev_b32's figure means full rate.
__global__ __launch_bounds__(256) void valu_loop64(uint32_t* out) {
    uint64_t v[8];
    for (int i = 0; i < 8; ++i) v[i] = (uint64_t(threadIdx.x) << 32) * 0x01010101ull + i;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_lshlrev_b64 %0, 4, %0" : "+v"(v[i]));
    }
    uint64_t acc = 0;
    for (int i = 0; i < 8; ++i) acc ^= v[i];
    if (acc == 0x12345678ull) out[0] = uint32_t(acc);
}

int main() {
    uint32_t* out;
    CK(hipMalloc(&out, 4));
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const char* names[] = {"v_perm s,v,v", "v_perm s,s,v", "v_perm v,v,v", "v_bitop3 xor3", "v_and_b32",
                           "v_xor_b32",   "v_lshlrev_b32", "v_lshl_or_b32", "v_lshlrev_b64 (x2)"};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int op = 0; op < 9; ++op) {
        for (int wps : {1, 2, 4, 8}) {  // waves per SIMD
            const int grid = p.multiProcessorCount * wps;  // 256-thread blocks = 4 waves = 1 per SIMD
            auto launch = [&] {
                switch (op) {
                    case 0: hipLaunchKernelGGL(valu_loop<0>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 1: hipLaunchKernelGGL(valu_loop<1>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 2: hipLaunchKernelGGL(valu_loop<2>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 3: hipLaunchKernelGGL(valu_loop<3>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 4: hipLaunchKernelGGL(valu_loop<4>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 5: hipLaunchKernelGGL(valu_loop<5>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 6: hipLaunchKernelGGL(valu_loop<6>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 7: hipLaunchKernelGGL(valu_loop<7>, grid, 256, 0, 0, out, 1u, 2u); break;
                    case 8: hipLaunchKernelGGL(valu_loop64, grid, 256, 0, 0, out); break;
                }
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int i = 0; i < 5; ++i) launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double ops = 5.0 * grid * 256.0 * ITERS * 8 * (op == 8 ? 2 : 1);
            printf("%-14s waves/SIMD=%d  %7.2f T lane-ops/s\n", names[op], wps, ops / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
