// config.hpp -- the library's ZFEC_HIP_* environment knobs, read once.
//
// Every knob is parsed at the first call into one immutable Config object;
// the launch path reads it through one atomic pointer load, so no getenv runs
// per call and no knob is ever read while another thread rewrites it.
// fec_reload_config() (include/zfec_hip.h) re-reads the environment into a
// new object (tests and A/B runs; objects are never freed, so a reader holding
// the old one stays valid).
#pragma once

#include <cstddef>
#include <cstdint>

#include "bitslice.hpp"

namespace zfec_hip {

enum StorePolicy { kStoreNt = 0, kStoreNtSc1 = 1, kStoreAuto = 2 };

struct Config {
    // launches
    size_t launch_units;   // ZFEC_HIP_LAUNCH_UNITS: units per launch (tests lower it to reach the split paths)
    bool batch_collapse;   // ZFEC_HIP_BATCH_COLLAPSE=0: block-major batches are not collapsed into one stripe
    StorePolicy store;     // ZFEC_HIP_STORE=auto|nt|ntsc1: output store policy of the register kernels
    uint64_t small_lanes;  // ZFEC_HIP_SMALL_LANES: launches below this many lanes take matapply_small (0: never)
    unsigned bsg_wgs_per_cu;  // ZFEC_HIP_BSG_WGS: matapply_bsg takes smaller row groups below this many workgroups per CU
    BsOptions jit;         // ZFEC_HIP_JIT_*: code-generation options of the bit-sliced JIT kernels
    unsigned jit_lds;      // ZFEC_HIP_JIT_LDS: extra dynamic LDS bytes per JIT workgroup (A/B: caps residency)
    // host paths
    bool wait_signal;      // ZFEC_HIP_WAIT=sync: small calls wait in hipStreamSynchronize
    size_t pack_limit;     // ZFEC_HIP_PACK_LIMIT: host bytes a call packs into the bounce buffer
    size_t stage_min;      // ZFEC_HIP_STAGE_MIN: host bytes from which blocks >= 64 KiB are staged
    size_t pool_copy_min;  // ZFEC_HIP_POOL_COPY_MIN: bounce-buffer copies on the host pool from this size
    size_t stage_chunk;    // ZFEC_HIP_STAGE_CHUNK: bytes of each block per staged chunk (0: automatic)
    bool zc_wide;          // ZFEC_HIP_ZC_WIDE=1: wide codes read the bounce buffer in place too
    size_t zc_wide_limit;  // ZFEC_HIP_ZC_WIDE_LIMIT: host bytes up to which wide codes' kernels use it in place (0: off)
    size_t zc_limit;       // ZFEC_HIP_ZC_LIMIT: host bytes up to which small calls' kernels use the bounce buffer in place (1.5 MiB)
    bool small_one;        // ZFEC_HIP_SMALL_ONE=0: small synchronous calls launch matapply_reg (A/B)
    bool small_inline;     // ZFEC_HIP_SMALL_INLINE=0: matapply_one reads its inputs from the bounce buffer (A/B)
    bool trace_host;       // ZFEC_HIP_TRACE_HOST: per-phase times of staged calls on stderr
    bool quiet;            // ZFEC_HIP_QUIET=1: no stderr report of a failed void fec_encode / fec_decode
};

const Config& config();
void reload_config();

}  // namespace zfec_hip
