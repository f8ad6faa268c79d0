/*
 * zfec_hip.h -- C-ABI of libzfec_hip.so, the MI355X (gfx950) erasure-coding engine.
 *
 * Part 1 is a drop-in for zfec's own C interface (/root/reference/zfec/fec.h):
 * same names, same argument meaning, same ownership rules, bit-identical
 * results.  A program (or FFI binding: zfec/_fecmodule.c, haskell/Codec/FEC.hs)
 * written against fec.h links against this library unchanged.  Buffers may be
 * host memory or device memory (hipMalloc / torch CUDA tensors); the library
 * detects which per pointer.  The GF(2^8) multiply-accumulate always runs in
 * HIP kernels on the GPU -- there is no CPU compute path.
 *
 * Part 2 adds what a GPU caller needs: status codes instead of assert(),
 * stream-ordered asynchronous variants, and batched strided entry points
 * that encode/decode many independent stripes in one launch.
 *
 * Plain C types only (stream handles are passed as void*, i.e. hipStream_t).
 */
#ifndef ZFEC_HIP_H
#define ZFEC_HIP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zfec/fec.h:9 */
typedef unsigned char gf;

/* zfec/fec.h:11-15.  The first three fields keep the reference layout (C callers
 * may read k and n); `priv` is library-private and follows them. */
typedef struct {
    unsigned long magic;
    unsigned short k, n; /* parameters of the code */
    gf* enc_matrix;      /* n x k row-major systematic encoding matrix (host memory) */
    void* priv;
} fec_t;

/* ---------------------------------------------------------------------------
 * Part 1: zfec/fec.h drop-in
 * ------------------------------------------------------------------------- */

/* Replaces zfec/fec.h:33 / fec.c:406-413.  Builds the GF(2^8) tables.  Unlike
 * the reference it is idempotent and thread-safe (std::call_once). */
void fec_init(void);

/* Replaces zfec/fec.h:39 / fec.c:430-479.  Returns NULL (and sets the
 * thread-local status) on invalid parameters (k < 1, m > 256, k > m) instead
 * of assert(); returns NULL if fec_init() was never called, like the reference
 * (fec.c:442-444). */
fec_t* fec_new(unsigned short k, unsigned short m);

/* Replaces zfec/fec.h:40 / fec.c:423-428. */
void fec_free(fec_t* p);

/* Replaces zfec/fec.h:49 / fec.c:487-505.  fecs[i] receives block
 * block_nums[i] (sz bytes) for i < num_block_nums.  Synchronous: the outputs
 * are complete when it returns.  Errors (block number >= n, HIP failure) set
 * the thread-local status and leave outputs unspecified; they never abort.
 * Extension: a block number < k yields a copy of that primary block (the
 * reference asserts, fec.c:498). */
void fec_encode(const fec_t* code, const gf* const* src, gf* const* fecs,
                const unsigned* block_nums, size_t num_block_nums, size_t sz);

/* Replaces zfec/fec.h:57 / fec.c:527-557.  inpkts[i] holds block index[i];
 * a present primary block i must sit at slot i.  outpkts receives the missing
 * primaries in ascending order.  Synchronous. */
void fec_decode(const fec_t* code, const gf* const* inpkts, gf* const* outpkts,
                const unsigned* index, size_t sz);

/* Exported by the reference too (fec.c:512-525, fec.c:341-394). */
void build_decode_matrix_into_space(const fec_t* code, const unsigned* index, const unsigned k, gf* matrix);
void _invert_vdm(gf* src, unsigned k);

/* ---------------------------------------------------------------------------
 * Part 2: extensions
 * ------------------------------------------------------------------------- */

enum {
    FEC_OK = 0,
    FEC_EINVAL = 1,     /* bad argument (k/m range, block number, duplicate, NULL) */
    FEC_ENODEV = 2,     /* no usable GPU */
    FEC_EHIP = 3,       /* a HIP runtime call failed */
    FEC_ENOMEM = 4,     /* allocation failed */
    FEC_ESINGULAR = 5,  /* decode matrix singular (duplicate block numbers) */
    FEC_EUNINIT = 6     /* fec_init() not called */
};

#define FEC_FLAG_ASYNC 1u          /* do not synchronize; all buffers device or page-locked host memory */
#define FEC_FLAG_LIBRARY_STREAM 2u /* ignore `stream`; use the library's per-thread stream */
#define FEC_FLAG_ALL_PRIMARIES 4u  /* decode: output all k primaries in order (present ones copied),
                                      not only the missing ones: the output is the stripe itself */
#define FEC_FLAG_HOST_MEMORY 8u    /* every block is host memory (pageable or page-locked): skip the
                                      per-pointer device queries (small calls from Python bytes) */
#define FEC_FLAG_ROW_PADDING 16u   /* batched calls: every block row may be read (inputs) and written
                                      (outputs) up to the next multiple of 128 bytes past its end, so
                                      each row ends on a whole cache line; output bytes past sz are
                                      then unspecified.  Used only when the block and stripe strides
                                      leave that much room; otherwise ignored */
#define FEC_FLAG_NO_POPULATE 32u   /* accepted and ignored (round 2's page-locking host path, which
                                      pre-faulted outputs, was removed: the staged path never locks) */

/* Status of the last library call made by this thread, and its message. */
int fec_last_status(void);
const char* fec_last_error_message(void);

/* fec_encode / fec_decode returning a status, on a caller-chosen HIP stream.
 * `stream` follows HIP's convention: NULL is the null (legacy default) stream,
 * which is what torch's default stream hands out.  FEC_FLAG_LIBRARY_STREAM
 * selects the library's own per-thread non-blocking stream instead (what the
 * synchronous fec_encode / fec_decode use).  With FEC_FLAG_ASYNC and device or
 * page-locked host buffers the call only enqueues work on the stream.
 *
 * Host buffers: page-locked ones (fec_host_alloc, hipHostMalloc,
 * hipHostRegister) are read and written by the kernel in place over PCIe;
 * large pageable ones are copied through pinned staging slots by the
 * library's host threads, chunk by chunk, overlapped with the kernels; small
 * pageable ones go through a bounce buffer.  Calls with pageable host buffers
 * are synchronous whatever the flags. */
int fec_encode_ex(const fec_t* code, const gf* const* src, gf* const* fecs,
                  const unsigned* block_nums, size_t num_block_nums, size_t sz,
                  void* stream, unsigned flags);
int fec_decode_ex(const fec_t* code, const gf* const* inpkts, gf* const* outpkts,
                  const unsigned* index, size_t sz, void* stream, unsigned flags);

/* Batched encode of nstripes independent stripes in one launch (device memory
 * on one device, or page-locked host memory).  Pageable host memory on either
 * side is accepted too: it is staged through pinned slots in groups of stripes
 * by the library's host threads (only the rows are written; the call is then
 * synchronous and FEC_FLAG_ROW_PADDING does not apply).  Block j of stripe s is read from src + s*src_stripe_stride +
 * j*src_block_stride; output i of stripe s (block block_nums[i]) is written to
 * dst + s*dst_stripe_stride + i*dst_block_stride.  Packed [stripe][block][sz]
 * layouts use block_stride = sz, stripe_stride = k*sz (input) / num*sz (output).
 * Block-major layouts (block j of every stripe back to back: stripe_stride = sz
 * on both sides, block_stride >= nstripes*sz) run as one stripe of nstripes*sz
 * bytes, the fastest shape for many small objects. */
int fec_encode_batch(const fec_t* code,
                     const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                     gf* dst, size_t dst_block_stride, size_t dst_stripe_stride,
                     const unsigned* block_nums, size_t num_block_nums, size_t sz,
                     size_t nstripes, void* stream, unsigned flags);

/* Batched decode: every stripe received the same block numbers (index[slot],
 * primaries at their own slot as in fec_decode).  Slot j of stripe s at
 * src + s*src_stripe_stride + j*src_block_stride; the recovered primaries
 * (ascending) at dst + s*dst_stripe_stride + i*dst_block_stride. */
int fec_decode_batch(const fec_t* code,
                     const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                     gf* dst, size_t dst_block_stride, size_t dst_stripe_stride,
                     const unsigned* index, size_t sz, size_t nstripes,
                     void* stream, unsigned flags);

/* Batched calls over several GPUs of this process.  The nstripes stripes are
 * split into contiguous, balanced ranges, one per entry of devices[] (entry d
 * gets stripes [d*q + min(d, e), ...), q = nstripes / ndevices, e = the
 * remainder: zfec_amd.shard.shard_range), and every range runs on its device
 * from a persistent host thread of the library bound to that device, with its
 * own stream and pinned staging slots; the call returns when all are done.
 * src / dst must be host memory (pageable: staged per device; page-locked:
 * read and written in place), each GPU moving its share over its own PCIe
 * link.  A device may be listed more than once (several threads on one GPU).
 * Layout, block numbers and flags as fec_encode_batch / fec_decode_batch
 * (FEC_FLAG_ASYNC and FEC_FLAG_LIBRARY_STREAM do not apply: the call is
 * synchronous on the library's streams).  The first failing range's status
 * is returned, its message prefixed with the device. */
int fec_encode_batch_multi(const fec_t* code,
                           const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                           gf* dst, size_t dst_block_stride, size_t dst_stripe_stride,
                           const unsigned* block_nums, size_t num_block_nums, size_t sz, size_t nstripes,
                           const int* devices, size_t ndevices, unsigned flags);
int fec_decode_batch_multi(const fec_t* code,
                           const gf* src, size_t src_block_stride, size_t src_stripe_stride,
                           gf* dst, size_t dst_block_stride, size_t dst_stripe_stride,
                           const unsigned* index, size_t sz, size_t nstripes,
                           const int* devices, size_t ndevices, unsigned flags);

/* Several batched calls in one: job i is exactly the fec_encode_batch
 * (kind FEC_JOB_ENCODE: nums = block_nums, num_nums entries) or
 * fec_decode_batch (kind FEC_JOB_DECODE: nums = index, k entries; num_nums
 * ignored) call its fields describe, with its own flags (only
 * FEC_FLAG_ROW_PADDING and FEC_FLAG_ALL_PRIMARIES apply per job).  The jobs
 * are independent: they may run concurrently and in any order, so no job may
 * read or write a buffer another job writes.  Two consecutive jobs on one
 * device, over codes with the same k and of register-kernel shape (k <= 4,
 * at most 8 outputs each, the narrower job at most k outputs; blocks longer
 * than 4 KiB or fewer than 64 stripes) share ONE launch, which pays one launch
 * ramp-up and drain instead of two (a stripe's encode next to another
 * stripe's decode); other jobs launch one at a time on the same stream.
 * `stream` and `flags` (FEC_FLAG_ASYNC, FEC_FLAG_LIBRARY_STREAM) apply to the
 * whole call.  The first failing job's status is returned, its message
 * prefixed "job i".  (An extension: zfec/fec.h has no batched calls.)  On the
 * cfg2 step (a 64 MiB K=3/M=10 stripe's encode and another's decode) one
 * paired launch per step measured 2465-2514 GB/s against 2506-2529 for the
 * two launches on two streams and about 2350 on one stream
 * (profiles/r03_pair_ab.json). */
#define FEC_JOB_ENCODE 0u
#define FEC_JOB_DECODE 1u
typedef struct fec_batch_job {
    const fec_t* code;
    unsigned kind;
    unsigned flags;
    const gf* src;
    size_t src_block_stride, src_stripe_stride;
    gf* dst;
    size_t dst_block_stride, dst_stripe_stride;
    const unsigned* nums;
    size_t num_nums;
    size_t sz, nstripes;
} fec_batch_job;
int fec_run_batch_jobs(const fec_batch_job* jobs, size_t njobs, void* stream, unsigned flags);

/* Page-locked host memory (hipHostMalloc): host buffers passed to fec_encode /
 * fec_decode from here are read and written by the kernel in place (no
 * per-call pinning, no staging copies).  NULL on failure (status set). */
void* fec_host_alloc(size_t bytes);
void fec_host_free(void* p);

/* Number of visible GPUs (0 when none; never aborts). */
int fec_device_count(void);

/* Library version string. */
const char* fec_version(void);

/* Name of the table-kernel variant a launch with k inputs and r outputs uses
 * when no run-time specialised kernel applies (diagnostics and profiling;
 * k <= 32, r <= 48 per launch). */
const char* fec_kernel_name(unsigned k, unsigned r);

/* Name of the kernel the calling thread launched last. */
const char* fec_last_kernel_name(void);

/* Run-time specialised bit-sliced kernels (hipRTC; zfec_amd/csrc/bitslice.cpp):
 * the coefficient matrix of a launch compiled into the instruction stream.
 * mode 0 = off; 1 = auto (default; launches of >= 8 MiB of wide codes: a
 * matrix's second such launch queues its compile in a background thread while
 * the table kernels serve; kernels are cached in memory and in jit_cache/ next
 * to the library, at most 512); 2 = force (every launch with blocks of
 * >= 2048 bytes, compiled synchronously).  The environment variable
 * ZFEC_HIP_JIT=0|auto|force sets the initial mode.  Returns the previous
 * mode; any other value of `mode` only queries.  Results are bit-identical in
 * every mode. */
int fec_jit_mode(int mode);

/* Wide-code launches that no compiled specialised kernel serves (a decode of
 * an erasure pattern seen for the first time, small launches, JIT off) run on
 * the bit-sliced kernels that take the coefficient matrix as run-time data (no
 * compile step): mode 2 = matapply_bsr (default; the specialised kernels'
 * instruction stream, one call per coefficient, any k, r up to 256/256);
 * 1 = matapply_bsg only; 0 = off (the table-lookup
 * kernels serve them; environment ZFEC_HIP_GENERIC=0 / 1 / 2 starts in that
 * mode).  Returns the previous mode; any other value only queries.  Results are
 * bit-identical in every mode. */
int fec_generic_mode(int mode);

/* Wait for background compiles; returns the number of compiled kernels. */
int fec_jit_wait(void);

/* Diagnostics and A/B runs.  The ZFEC_HIP_* environment knobs are read once,
 * at the library's first call; fec_reload_config re-reads them (returns
 * FEC_OK).  fec_last_wait: how the calling thread's last synchronous
 * small-object call waited for its kernel -- 1 = on the completion word the
 * kernel itself wrote to pinned host memory, 0 = hipStreamSynchronize. */
int fec_reload_config(void);
int fec_last_wait(void);

/* Compile now (no GPU needed) the kernels an fec_encode of block_nums, or an
 * fec_decode from `index` (flags as fec_decode_ex), would use.  FEC_OK, or
 * FEC_EHIP with the compiler's message. */
int fec_jit_prepare_encode(const fec_t* code, const unsigned* block_nums, size_t num_block_nums);
int fec_jit_prepare_decode(const fec_t* code, const unsigned* index, unsigned flags);

#ifdef __cplusplus
}
#endif

#endif /* ZFEC_HIP_H */
