// config.hpp -- the library's ZFEC_HIP_* environment knobs, read once.
//
// Every knob is parsed at the first call into one immutable Config object;
// the launch path reads it through one atomic pointer load, so no getenv runs
// per call and no knob is ever read while another thread rewrites it.
// fec_reload_config() (include/zfec_hip.h) re-reads the environment into a
// new object (tests; objects are never freed, so a reader holding the old one
// stays valid).
//
// No knob changes the bytes a call returns.  Round 4 removed the knobs whose
// variants lost their A/Bs (and the code they selected); what is left is the
// host-path policy a caller may tune and three test hooks that only change how
// work is cut into launches (INTEGRATION.md "Environment").  Read elsewhere,
// once: ZFEC_HIP_JIT / ZFEC_HIP_JIT_CACHE / ZFEC_HIP_JIT_VERBOSE /
// ZFEC_HIP_JIT_DUMP (bitslice.cpp), ZFEC_HIP_GENERIC (kernels.hip),
// ZFEC_HIP_HOST_THREADS (host_pool.cpp).
#pragma once

#include <cstddef>
#include <cstdint>

namespace zfec_hip {

struct Config {
    // host paths (policy)
    bool wait_signal;      // ZFEC_HIP_WAIT=sync: small calls wait in hipStreamSynchronize
    size_t pack_limit;     // ZFEC_HIP_PACK_LIMIT: host bytes a call packs into the bounce buffer (4 MiB)
    size_t stage_min;      // ZFEC_HIP_STAGE_MIN: host bytes from which blocks >= 64 KiB are staged (512 KiB)
    size_t zc_limit;       // ZFEC_HIP_ZC_LIMIT: host bytes up to which small calls' kernels use the bounce buffer in place (1.5 MiB)
    bool quiet;            // ZFEC_HIP_QUIET=1: no stderr report of a failed void fec_encode / fec_decode
    // test hooks: reach the split paths at sizes a test can afford
    size_t launch_units;   // ZFEC_HIP_LAUNCH_UNITS: units per launch (long rows cut into byte ranges, batches into groups)
    uint64_t small_lanes;  // ZFEC_HIP_SMALL_LANES: launches below this many lanes take matapply_small (0: never)
    size_t stage_chunk;    // ZFEC_HIP_STAGE_CHUNK: bytes of each block per staged chunk (0: automatic)
};

const Config& config();
void reload_config();

}  // namespace zfec_hip
