// config.cpp -- see config.hpp.
#include "config.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace zfec_hip {
namespace {

const char* env(const char* name) {
    const char* v = getenv(name);
    return v && *v ? v : nullptr;
}

size_t env_size(const char* name, size_t dflt) {
    const char* v = env(name);
    return v ? static_cast<size_t>(strtoull(v, nullptr, 10)) : dflt;
}

unsigned env_uint(const char* name, unsigned dflt) {
    const char* v = env(name);
    return v ? static_cast<unsigned>(strtoul(v, nullptr, 10)) : dflt;
}

bool env_flag(const char* name, bool dflt) {
    const char* v = env(name);
    return v ? v[0] != '0' : dflt;
}

Config* read_env() {
    Config* c = new Config;
    const unsigned long long u = env_size("ZFEC_HIP_LAUNCH_UNITS", 0);
    // the kernels' own bound is < 2^32 units per launch
    c->launch_units = u >= 1024 && u < (1ull << 31) ? static_cast<size_t>(u) : size_t(1) << 31;
    c->batch_collapse = env_flag("ZFEC_HIP_BATCH_COLLAPSE", true);
    const char* s = env("ZFEC_HIP_STORE");
    c->store = s && !strcmp(s, "nt") ? kStoreNt : s && !strcmp(s, "ntsc1") ? kStoreNtSc1 : kStoreAuto;
    c->small_lanes = env_size("ZFEC_HIP_SMALL_LANES", 2048);
    c->bsg_wgs_per_cu = env_uint("ZFEC_HIP_BSG_WGS", 4);

    BsOptions& o = c->jit;
    o.max_tile = env_uint("ZFEC_HIP_JIT_TILE", o.max_tile);
    if (o.max_tile == 0 || o.max_tile > 32) o.max_tile = kBsMaxTile;
    o.prefetch = env_uint("ZFEC_HIP_JIT_PREFETCH", o.prefetch);
    if (o.prefetch > 4) o.prefetch = 4;
    o.barriers = env_uint("ZFEC_HIP_JIT_BARRIER", 1) != 0;
    o.store_aux = env_uint("ZFEC_HIP_JIT_STORE", o.store_aux) & 0x1Fu;
    o.gray = env_uint("ZFEC_HIP_JIT_ORDER", o.gray ? 1 : 0) != 0;
    o.waves = env_uint("ZFEC_HIP_JIT_WAVES", o.waves);
    if (o.waves > 8) o.waves = 8;
    o.split = env_uint("ZFEC_HIP_JIT_SPLIT", o.split ? 1 : 0) != 0;
    o.share = env_uint("ZFEC_HIP_JIT_SHARE", o.share ? 1 : 0) != 0;
    o.argload = env_uint("ZFEC_HIP_JIT_ARGLOAD", o.argload ? 1 : 0) != 0;
    o.shift64 = env_uint("ZFEC_HIP_JIT_SHIFT64", o.shift64 ? 1 : 0) != 0;
    o.ksplit = env_uint("ZFEC_HIP_JIT_KSPLIT", o.ksplit ? 1 : 0) != 0;
    c->jit_lds = env_uint("ZFEC_HIP_JIT_LDS", 0);
    if (c->jit_lds > (96u << 10)) c->jit_lds = 96u << 10;
    o.probe = env_uint("ZFEC_HIP_JIT_PROBE", 0);
    if (o.probe > 2) o.probe = 0;

    const char* w = env("ZFEC_HIP_WAIT");
    c->wait_signal = !(w && !strcmp(w, "sync"));
    c->pack_limit = env_size("ZFEC_HIP_PACK_LIMIT", size_t(4) << 20);
    c->stage_min = env_size("ZFEC_HIP_STAGE_MIN", size_t(512) << 10);
    c->pool_copy_min = env_size("ZFEC_HIP_POOL_COPY_MIN", SIZE_MAX);
    const size_t sc = env_size("ZFEC_HIP_STAGE_CHUNK", 0);
    c->stage_chunk = sc >= (64u << 10) ? sc / 4096 * 4096 : 0;
    c->zc_wide = env_flag("ZFEC_HIP_ZC_WIDE", false);
    c->zc_limit = env_size("ZFEC_HIP_ZC_LIMIT", size_t(3) << 19);  // 1.5 MiB
    c->zc_wide_limit = env_size("ZFEC_HIP_ZC_WIDE_LIMIT", 0);
    c->small_one = env_flag("ZFEC_HIP_SMALL_ONE", true);
    c->small_inline = env_flag("ZFEC_HIP_SMALL_INLINE", true);
    c->trace_host = env("ZFEC_HIP_TRACE_HOST") != nullptr;
    const char* q = env("ZFEC_HIP_QUIET");
    c->quiet = q && q[0] == '1';
    return c;
}

std::atomic<const Config*> g_cfg{nullptr};
std::mutex g_mu;

}  // namespace

const Config& config() {
    const Config* c = g_cfg.load(std::memory_order_acquire);
    if (c) return *c;
    std::lock_guard<std::mutex> g(g_mu);
    c = g_cfg.load(std::memory_order_relaxed);
    if (!c) {
        c = read_env();
        g_cfg.store(c, std::memory_order_release);
    }
    return *c;
}

void reload_config() {
    std::lock_guard<std::mutex> g(g_mu);
    g_cfg.store(read_env(), std::memory_order_release);  // the old object is kept: readers may hold it
}

}  // namespace zfec_hip
