// isa_probe.hip -- checks of three gfx950 behaviours the kernels may rely on,
// each against a host-computed expectation:
//   1. VGPR index mode (s_set_gpr_idx_on ... gpr_idx(SRC0)) applied to the
//      src0 of v_xor_b32 (VOP2) and of v_bitop3_b32 (VOP3);
//   2. ds_write_b128 / ds_read_b128 at LDS addresses that are not 16-byte
//      (or 4-byte) multiples;
//   3. DPP wave_shl:1 (lane l reads lane l+1).
// build: hipcc --offload-arch=gfx950 -O3 tools/isa_probe.hip -o tools/isa_probe.exe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void gpr_idx_probe(unsigned* out, unsigned idx) {
    // v40..v47 hold lane*16 + i; with idx, v_xor dst, v40(+idx), src1 reads v[40+idx]
    unsigned r0, r1;
    unsigned a0 = threadIdx.x * 16 + 0, a1 = threadIdx.x * 16 + 1, a2 = threadIdx.x * 16 + 2, a3 = threadIdx.x * 16 + 3;
    unsigned a4 = threadIdx.x * 16 + 4, a5 = threadIdx.x * 16 + 5, a6 = threadIdx.x * 16 + 6, a7 = threadIdx.x * 16 + 7;
    unsigned k = 0x5A5A0000u;
    asm volatile(
        "s_set_gpr_idx_on %[i], gpr_idx(SRC0)\n"
        "v_xor_b32 %[r0], v40, %[k]\n"
        "v_bitop3_b32 %[r1], v40, %[k], %[k] bitop3:0x96\n"
        "s_set_gpr_idx_off\n"
        : [r0] "=&v"(r0), [r1] "=&v"(r1), "+{v40}"(a0), "+{v41}"(a1), "+{v42}"(a2), "+{v43}"(a3), "+{v44}"(a4),
          "+{v45}"(a5), "+{v46}"(a6), "+{v47}"(a7)
        : [i] "s"(idx), [k] "v"(k));
    out[threadIdx.x * 2] = r0;
    out[threadIdx.x * 2 + 1] = r1;
}

__global__ void lds_unaligned_probe(unsigned* out, unsigned off) {
    __shared__ unsigned char buf[64 * 16 + 64];
    for (unsigned i = threadIdx.x; i < sizeof buf; i += 64) buf[i] = 0xEE;
    __syncthreads();
    const u32x4 v = {threadIdx.x * 0x01010101u, 0x11223344u, 0x55667788u, threadIdx.x ^ 0xA5A5A5A5u};
    const unsigned addr = static_cast<unsigned>(reinterpret_cast<uintptr_t>(buf)) + off + threadIdx.x * 16;
    asm volatile("ds_write_b128 %0, %1\n s_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(v) : "memory");
    __syncthreads();
    u32x4 w;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(addr) : "memory");
    out[threadIdx.x * 4 + 0] = w.x;
    out[threadIdx.x * 4 + 1] = w.y;
    out[threadIdx.x * 4 + 2] = w.z;
    out[threadIdx.x * 4 + 3] = w.w;
}

__global__ void dpp_probe(unsigned* out) {
    const unsigned v = threadIdx.x * 3 + 1;
    out[threadIdx.x] = __builtin_amdgcn_update_dpp(0xFFFFFFFFu, v, 0x130, 0xF, 0xF, false);
}

int main() {
    unsigned* d;
    hipMalloc(&d, 64 * 4 * 4);
    unsigned h[256];
    int bad = 0;
    for (unsigned idx = 0; idx < 8; ++idx) {
        hipLaunchKernelGGL(gpr_idx_probe, dim3(1), dim3(64), 0, 0, d, idx);
        hipMemcpy(h, d, 64 * 2 * 4, hipMemcpyDeviceToHost);
        for (unsigned l = 0; l < 64; ++l) {
            const unsigned want = (l * 16 + idx) ^ 0x5A5A0000u;
            if (h[2 * l] != want || h[2 * l + 1] != ((l * 16 + idx) ^ 0x5A5A0000u ^ 0x5A5A0000u)) {
                if (bad++ < 4) printf("gpr_idx idx %u lane %u: xor %08x bitop3 %08x want %08x\n", idx, l, h[2 * l],
                                      h[2 * l + 1], want);
            }
        }
    }
    printf("gpr_idx on VOP2/VOP3 src0: %s\n", bad ? "MISMATCH" : "ok");
    int bad2 = 0;
    for (unsigned off : {0u, 1u, 2u, 4u, 6u, 8u, 13u}) {
        hipLaunchKernelGGL(lds_unaligned_probe, dim3(1), dim3(64), 0, 0, d, off);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("lds unaligned off %u: launch failed\n", off);
            bad2++;
            break;
        }
        hipMemcpy(h, d, 64 * 4 * 4, hipMemcpyDeviceToHost);
        for (unsigned l = 0; l < 64; ++l)
            if (h[4 * l] != l * 0x01010101u || h[4 * l + 1] != 0x11223344u || h[4 * l + 2] != 0x55667788u ||
                h[4 * l + 3] != (l ^ 0xA5A5A5A5u)) {
                if (bad2++ < 4) printf("lds off %u lane %u: %08x %08x %08x %08x\n", off, l, h[4 * l], h[4 * l + 1],
                                       h[4 * l + 2], h[4 * l + 3]);
            }
    }
    printf("ds b128 at unaligned LDS addresses: %s\n", bad2 ? "MISMATCH" : "ok");
    hipLaunchKernelGGL(dpp_probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
    int bad3 = 0;
    for (unsigned l = 0; l < 63; ++l)
        if (h[l] != (l + 1) * 3 + 1) bad3++;
    printf("dpp wave_shl:1 lane l reads lane l+1: %s (lane 63 got %08x)\n", bad3 ? "MISMATCH" : "ok", h[63]);
    return bad || bad2 || bad3;
}
