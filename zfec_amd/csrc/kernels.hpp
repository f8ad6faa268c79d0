// kernels.hpp -- launch interface of the GF(2^8) matrix-apply kernels.
//
// One kernel family serves both directions of the code:
//   encode: out_i = sum_j E[block_nums[i]][j] * in_j   (zfec/fec.c:487-505)
//   decode: out_r = sum_c D[r][c] * in_c                (zfec/fec.c:527-557)
// i.e. an r x k coefficient matrix applied byte-wise to k input blocks, for
// `nstripes` independent stripes that share the matrix.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace zfec_hip {

constexpr int kMaxIn = 32;     // input blocks per launch (larger k: XOR-accumulating passes)
constexpr int kMaxOut = 48;    // output blocks per launch
constexpr int kMaxCoef = 1536; // r*k coefficients per launch
constexpr int kChunk = 16;     // bytes per lane per block per step (one dwordx4)
constexpr int kMinChunk = 4;   // smallest unit any kernel variant uses (launch splitting)
constexpr int kBlock = 256;    // threads per workgroup

// Kernel argument block (passed by value; ~2.2 KiB, well inside the kernarg limit).
struct alignas(16) MatJob {
    uint64_t sz;           // bytes per block
    uint64_t in_sstride;   // stripe stride added to every input pointer
    uint64_t out_sstride;  // stripe stride added to every output pointer
    uint32_t nstripes;
    uint32_t k;            // inputs in this launch
    uint32_t r;            // outputs in this launch
    uint32_t cps;          // 16-byte chunks per stripe = ceil(sz / 16)
    uint32_t gs_c, gs_s;   // grid stride expressed as (chunks, stripes): stride = gs_s*cps + gs_c
    uint32_t accumulate;   // 1: out ^= result (continuation pass for k > kMaxIn)
    uint32_t tables;       // set by launch_matapply: 1 = tab[] holds the per-coefficient tables,
                           // 2 = coef[] is in matapply_bsg's walk order
    uint32_t xcd_swizzle;  // set by launch_matapply: 1 = workgroups dealt XCD-contiguously (UnitIter)
    uint32_t pad_;
    uint32_t* done_flag;   // set by launch_matapply: pinned host word the kernel's one workgroup
    uint32_t done_seq;     //   stores done_seq into when it has finished (matapply_request_signal)
    uint32_t pad2_;
    const uint8_t* in[kMaxIn];
    uint8_t* out[kMaxOut];
    union {
        uint8_t coef[kMaxCoef];          // r x k coefficients, row-major (filled by the caller)
        uint32_t tab[kMaxCoef / 4];      // or their v_perm tables, 5 dwords each (filled by launch_matapply)
    };
};

constexpr int kMaxKernargTables = kMaxCoef / 4 / 5;  // 76 coefficients

// Enqueue one launch on `stream`.  Validates shapes against the kernel's
// compile-time limits before launching (returns hipErrorInvalidValue
// otherwise); chooses the specialised variant for (k, r) when one exists.
hipError_t launch_matapply(MatJob& job, hipStream_t stream);

// Ask the calling thread's next launch_matapply to have its kernel publish
// `seq` at flag_dev (pinned host memory) when it has finished -- honoured
// only by the register kernels in a one-workgroup launch (a stripe of at
// most 4 KiB per block); matapply_signal_used() says whether it was.
void matapply_request_signal(uint32_t* flag_dev, uint32_t seq);
bool matapply_signal_used();

// Name of the table-kernel variant launch_matapply uses for (k, r) when no
// run-time specialised kernel applies (for tests / profiling).
const char* matapply_variant_name(uint32_t k, uint32_t r, bool accumulate);

// Name of the kernel the calling thread launched last (table variant,
// run-time-data bit-sliced kernel matapply_bsg, or bit-sliced JIT kernel,
// bitslice.hpp).
const char* matapply_last_kernel();

// matapply_bsg (bit-sliced, coefficients as run-time data) for wide-code
// launches that no specialised JIT kernel serves: 1 = on (default; env
// ZFEC_HIP_GENERIC=0 starts it off), 0 = off (the table kernels serve).
int generic_mode();
void set_generic_mode(int on);

}  // namespace zfec_hip
