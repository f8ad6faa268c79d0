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

Config* read_env() {
    Config* c = new Config;
    const char* w = env("ZFEC_HIP_WAIT");
    c->wait_signal = !(w && !strcmp(w, "sync"));
    c->pack_limit = env_size("ZFEC_HIP_PACK_LIMIT", size_t(4) << 20);
    c->stage_min = env_size("ZFEC_HIP_STAGE_MIN", size_t(512) << 10);
    c->zc_limit = env_size("ZFEC_HIP_ZC_LIMIT", size_t(3) << 19);  // 1.5 MiB
    const char* q = env("ZFEC_HIP_QUIET");
    c->quiet = q && q[0] == '1';
    const unsigned long long u = env_size("ZFEC_HIP_LAUNCH_UNITS", 0);
    // the kernels' own bound is < 2^32 units per launch
    c->launch_units = u >= 1024 && u < (1ull << 31) ? static_cast<size_t>(u) : size_t(1) << 31;
    c->small_lanes = env_size("ZFEC_HIP_SMALL_LANES", 2048);
    const size_t sc = env_size("ZFEC_HIP_STAGE_CHUNK", 0);
    c->stage_chunk = sc >= (64u << 10) ? sc / 4096 * 4096 : 0;
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
