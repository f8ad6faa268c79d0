// bitslice.hpp -- run-time specialised ("JIT") bit-sliced GF(2^8) kernels.
//
// For codes with many coefficients (K=10/M=16, K=20/M=60) the table-lookup
// kernels of kernels.hip are bound by VALU issue: 4.5 VOP3 per coefficient per
// 4 bytes.  Multiplication by a constant c is a GF(2)-linear map on the 8 bits
// of a byte, so after an 8x8 bit transpose of 32 bytes into 8 bit-planes, c*x
// is, for every output plane, an XOR of a subset of the input planes -- a
// subset that is known once the coefficient matrix is known.  This module
// writes a HIP kernel for one r x k matrix with those subsets baked into the
// instruction stream (four-Russians: per input, the XOR combinations of planes
// 0-3 and of planes 4-7, then one XOR3 per output plane), compiles it with
// hipRTC and caches the code object in memory and on disk.  Cost per
// coefficient per 32 bytes: 8 XOR3 plus the amortised transposes and tables.
//
// Compilation takes about a second, so in the default mode a launch only uses
// a kernel that is already compiled, and otherwise queues a background compile
// and returns hipErrorNotReady: the caller runs the table kernel this time.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "kernels.hpp"

namespace zfec_hip {

constexpr int kBsChunk = 2048;    // bytes of a block per wave per unit (32 per lane, two 1 KiB halves)
constexpr int kBsMaxTile = 10;    // output rows per register tile (8 accumulator planes each)

// The generator's shape choices.  Fixed: the variants that lost their A/Bs
// (Gray-code combination order, launch-bound hints, tile heights, no prefetch,
// no scheduling barriers, pointers loaded up front, 32-bit-shift transposes,
// other store policies; DESIGN.md §4 and the committed profiles/r0*_jit_*
// logs) were removed in round 4, and so were the measurement-only probe
// variants, whose outputs were not the code's.  Only the LDS sharing of the
// planes depends on the matrix (options_for: k <= 32).
struct BsOptions {
    unsigned max_tile = kBsMaxTile;  // rows per tile (tiles are near-equal)
    unsigned prefetch = 2;           // input steps loaded ahead of the one being computed
    bool split = true;               // one wave per row tile of a unit (a workgroup shares the unit's inputs)
    bool share = true;               // split: inputs transposed once per unit, bit-planes shared through LDS
    unsigned phase = 8;              // share: inputs per LDS phase (0: all k at once, k x 2 KiB of LDS)
    bool dma = true;                 // share: inputs loaded with LDS-DMA, several phases double-buffered
    bool ksplit = true;              // one row tile and k > 32: a unit's inputs split over the 4 waves of a
                                     // workgroup, partial planes reduced through LDS (4x the waves per unit)
};

// Largest matrix (k * r coefficients per launch) the generator specialises:
// the kernel's code grows with it (~10 instructions per coefficient), and so
// does its compile time; larger launches run on matapply_bsg.
constexpr unsigned kJitMaxCoef = 1600;

// Row tiles of an r-row matrix, and whether they go to the waves of one
// workgroup (2-8 tiles) or each wave walks all of them.
unsigned bitslice_tiles(unsigned r, const BsOptions& opt);
bool bitslice_split(unsigned r, const BsOptions& opt);
// Whether the kernel for k inputs and r rows splits its inputs over the waves
// of a workgroup (BsOptions::ksplit).
bool bitslice_ksplit(unsigned k, unsigned r, const BsOptions& opt);

// Source of the kernel `name` for the r x k matrix `coef` (row-major).
std::string bitslice_source(const uint8_t* coef, unsigned k, unsigned r, const BsOptions& opt, const char* name);

enum JitMode {
    kJitOff = 0,    // never (ZFEC_HIP_JIT=0)
    kJitAuto = 1,   // large launches of wide codes; compile in the background (default)
    kJitForce = 2,  // every launch the kernel supports; compile synchronously (ZFEC_HIP_JIT=force)
};
JitMode jit_mode();
void set_jit_mode(JitMode m);

// Compile (synchronously; no GPU needed) the kernel for an r x k matrix.
// 0 on success, else -1 (jit_last_error() says why).
int jit_prepare(const uint8_t* coef, unsigned k, unsigned r);

// Auto mode, a code's construction (fec_new): if the disk cache already holds
// the compiled kernel of this r x k matrix (an earlier process compiled it),
// load it in the background -- no compile, nothing waits -- together with its
// module on the calling thread's current device, so the matrix's first large
// launch can run it instead of the run-time-data kernel.
void jit_prefetch(const uint8_t* coef, unsigned k, unsigned r);

// Launch the specialised kernel for the matrix application `a`.
// hipErrorNotSupported: not used for this launch (caller uses the other kernels);
// hipErrorNotReady: not compiled yet (a background compile is queued).
hipError_t launch_matapply_jit(const ApplySpec& a, hipStream_t stream, const char** name_out);

// Block until every queued compile has finished; returns the number of
// specialised kernels compiled so far (failures excluded).
int jit_wait();

// Last compile failure (empty if none): hipRTC missing, compile log, ...
std::string jit_last_error();

}  // namespace zfec_hip
