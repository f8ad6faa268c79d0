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

constexpr int kMaxIn = 32;       // inputs per launch of the table / small kernels (wider: XOR-accumulating passes)
constexpr int kMaxOut = 48;      // outputs per launch
constexpr int kMaxCoef = 1536;   // r*k coefficients per launch of the table kernels
constexpr int kMaxWideIn = 256;  // inputs per launch of the bit-sliced kernels (a device-side table past kMaxIn)
constexpr int kChunk = 16;       // bytes per lane per block per step (one dwordx4)
constexpr int kMinChunk = 4;     // smallest unit any kernel variant uses (launch splitting)
constexpr int kBlock = 256;      // threads per workgroup

// One matrix application, as the host describes it (not a kernel argument:
// every kernel family builds its own, sized to what it reads).
struct ApplySpec {
    const uint8_t* coef;          // r x k coefficients, row i at coef + i * coef_stride
    uint32_t coef_stride;         // >= k
    uint32_t k, r;
    const uint8_t* const* in;     // k input block bases (stripe 0), kernel-visible addresses
    uint8_t* const* out;          // r output block bases (stripe 0)
    uint64_t sz;                  // bytes per block
    uint64_t nstripes;
    uint64_t in_sstride, out_sstride;  // stripe strides added to every input / output pointer
    bool accumulate;              // out ^= result (continuation pass of a code split by input groups)
};

// Kernel argument block of the table (matapply_lds), small and run-time-data
// bit-sliced (matapply_bsg) kernels: ~2.2 KiB, k <= kMaxIn, r <= kMaxOut.
// The register kernels (k <= 4, r <= 8) take a block sized to k + r pointers
// and their tables instead (kernels.hip, RegJob).
struct alignas(16) MatJob {
    uint64_t sz;           // bytes per block
    uint64_t in_sstride;   // stripe stride added to every input pointer
    uint64_t out_sstride;  // stripe stride added to every output pointer
    uint32_t nstripes;
    uint32_t k;            // inputs in this launch
    uint32_t r;            // outputs in this launch
    uint32_t cps;          // units per stripe
    uint32_t gs_c, gs_s;   // grid stride expressed as (units, stripes): stride = gs_s*cps + gs_c
    uint32_t accumulate;   // 1: out ^= result
    uint32_t pad_;
    const uint8_t* in[kMaxIn];
    uint8_t* out[kMaxOut];
    uint8_t coef[kMaxCoef];  // r x k row-major (matapply_bsg: its walk order)
};

// Enqueue one launch on `stream` (the current device's).  Returns
// hipErrorInvalidValue for shapes no kernel accepts (the caller splits),
// hipErrorNotSupported when a wide launch (k > kMaxIn) has no kernel for its
// shape (the caller splits it into XOR-accumulating passes).
hipError_t launch_apply(const ApplySpec& a, hipStream_t stream);

// Two independent applications over the same k in ONE launch (matapply_pair):
// both register-kernel shapes (k <= 4, r <= 8, not matapply_rows' short
// blocks), the narrower one's r <= k.  hipErrorNotSupported otherwise (the
// caller launches them one at a time).  Neither may read what the other writes.
hipError_t launch_apply_pair(const ApplySpec& x, const ApplySpec& y, hipStream_t stream);

// Whether `stream` is being captured into a HIP graph.  The table forms (a
// device-side table the host fills and reuses at enqueue time) decline then:
// a captured graph would replay copies from host slots rewritten since, or
// read a cached device table whose upload was only recorded.  launch_apply
// falls back to kernels whose whole description travels in their arguments;
// wide launches (k > kMaxIn) are split into passes by the caller.
bool stream_capturing(hipStream_t stream);

// Whether launch_apply takes all k > kMaxIn inputs of a launch of r <= kMaxOut
// rows, sz-byte blocks and nstripes stripes in one pass (bit-sliced kernels).
bool wide_launch_ok(uint32_t k, uint32_t r, uint64_t sz, uint64_t nstripes);

// Ask the calling thread's next launch_apply to have its kernel publish `seq`
// at flag_dev (pinned host memory) when it has finished -- honoured only by
// the register kernels in a one-workgroup launch (a stripe of at most 4 KiB
// per block); matapply_signal_used() says whether it was.
void matapply_request_signal(uint32_t* flag_dev, uint32_t seq);
bool matapply_signal_used();

// The synchronous small call's launch (fec_abi.cpp run_single, every block in
// the thread's pinned bounce buffer): k <= 4, r <= 8, one stripe of sz bytes,
// sz a multiple of 16 and at most 4096 (whole 16-byte units, one workgroup).
// matapply_one publishes `seq` at flag_dev (pinned host memory, may be null)
// when it has finished.  host_in (may be null): the k input blocks of host_sz
// bytes each in host memory; where they fit (k x sz rounded to 16 bytes at
// most 4,352 bytes) they are copied into the kernel's argument block and
// a.in is not read.  hipErrorInvalidValue for other shapes.
constexpr uint32_t kOneInlineBytes = 4352;  // inline input capacity of matapply_one's argument block
// Whether k host inputs of host_sz bytes, padded to ksz (a whole number of
// 16-byte units), go inside matapply_one's argument block: the one test both
// run_single (which then skips the copy into the bounce buffer) and
// launch_one use.
constexpr bool one_inline_fits(uint32_t k, uint64_t ksz, uint64_t host_sz) {
    return host_sz <= ksz && ksz % 16 == 0 && uint64_t(k) * ksz <= kOneInlineBytes;
}
hipError_t launch_one(const ApplySpec& a, hipStream_t stream, uint32_t* flag_dev, uint32_t seq,
                      const uint8_t* const* host_in = nullptr, uint64_t host_sz = 0);

// Name of the table-kernel variant launch_apply uses for (k, r) when no
// run-time specialised kernel applies (for tests / profiling).
const char* matapply_variant_name(uint32_t k, uint32_t r, bool accumulate);

// Name of the kernel the calling thread launched last (table variant,
// run-time-data bit-sliced kernel matapply_bsg, or bit-sliced JIT kernel,
// bitslice.hpp).
const char* matapply_last_kernel();

// The bit-sliced kernels with the coefficients as run-time data, for wide-code
// launches that no specialised JIT kernel serves: 2 = matapply_bsr (default;
// matapply_bsg for the few shapes it does not take); 1 = matapply_bsg only;
// 0 = off (the table kernels serve).  Env ZFEC_HIP_GENERIC=0/1/2 starts
// in that mode.
int generic_mode();
void set_generic_mode(int mode);

}  // namespace zfec_hip
