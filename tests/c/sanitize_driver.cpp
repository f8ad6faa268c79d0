// sanitize_driver.cpp -- host-side concurrency and validation checks of the
// library, built with AddressSanitizer or ThreadSanitizer (make asan / make
// tsan: every host object of libzfec_hip.so compiled with the sanitizer and
// linked into this program).  Runs without a GPU: what it exercises is the
// host code a GIL-releasing caller reaches from several threads at once --
// field / matrix construction (zfec/fec.c:406-479), argument validation and
// the void entry points' failure report (fec.h:33-57), decode-matrix
// inversion (fec.c:512-525), the hipRTC JIT registry, the configuration
// object, and the host copy pool of the staged path.  The reference's own
// race test is the parallel-init property of haskell/test/FECTest.hs:118-135.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zfec_hip.h"
#include "../../zfec_amd/csrc/config.hpp"
#include "../../zfec_amd/csrc/gf256.hpp"
#include "../../zfec_amd/csrc/host_pool.hpp"

namespace {

std::atomic<int> g_fail{0};

#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail.fetch_add(1);                                              \
        }                                                                     \
    } while (0)

template <class F>
void in_threads(int n, F f) {
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) th.emplace_back(f, i);
    for (auto& t : th) t.join();
}

// fec_init / fec_new / fec_free from many threads at once, the reference's
// parallel-init property (haskell/test/FECTest.hs:118-135): k = 1 parity
// rows equal the primary (fec.c's matrix for k = 1 is all ones).
void check_parallel_init() {
    in_threads(8, [](int t) {
        fec_init();
        for (int i = 0; i < 50; ++i) {
            const unsigned short k = static_cast<unsigned short>(1 + (t * 37 + i) % 40);
            fec_t* c = fec_new(k, static_cast<unsigned short>(k + 1 + i % 20));
            CHECK(c != nullptr);
            if (!c) continue;
            if (k == 1)
                for (unsigned r = 1; r < c->n; ++r) CHECK(c->enc_matrix[r] == 1);
            fec_free(c);
        }
    });
}

// Argument validation on every entry point, from several threads: statuses
// and messages are per thread.
void check_rejects() {
    in_threads(8, [](int t) {
        fec_t* c = fec_new(3, 10);
        CHECK(c != nullptr);
        uint8_t a[16] = {}, b[16] = {}, d[16] = {};
        const gf* src[3] = {a, b, d};
        uint8_t o1[16], o2[16];
        gf* out[2] = {o1, o2};
        for (int i = 0; i < 100; ++i) {
            const unsigned bad[2] = {3, 10 + static_cast<unsigned>(t)};
            CHECK(fec_encode_ex(c, src, out, bad, 2, 16, nullptr, 0) == FEC_EINVAL);
            CHECK(std::strstr(fec_last_error_message(), "out of range") != nullptr);
            const unsigned dup[3] = {4, 4, 5};
            CHECK(fec_decode_ex(c, src, out, dup, 16, nullptr, 0) == FEC_EINVAL);
            CHECK(std::strstr(fec_last_error_message(), "duplicate") != nullptr);
            const unsigned mis[3] = {1, 0, 5};
            CHECK(fec_decode_ex(c, src, out, mis, 16, nullptr, 0) == FEC_EINVAL);
            CHECK(fec_last_status() == FEC_EINVAL);
            // valid arguments, no GPU: a status, never an abort
            const unsigned ok[2] = {3, 9};
            const int st = fec_encode_ex(c, src, out, ok, 2, 16, nullptr, 0);
            CHECK(st == FEC_ENODEV || st == FEC_OK);
            fec_encode(c, src, out, ok, 2, 16);  // void entry point: the first failure is reported once
            const unsigned ix[3] = {7, 1, 9};
            gf mat[9];
            build_decode_matrix_into_space(c, ix, 3, mat);
            CHECK(fec_last_status() == FEC_OK);
            const int devs[2] = {0, 0};
            const int mst = fec_encode_batch_multi(c, a, 4, 12, o1, 4, 8, ok, 2, 4, 1, devs, 2, 0);
            CHECK(mst == FEC_ENODEV || mst == FEC_OK);
            fec_batch_job jobs[2] = {
                {c, FEC_JOB_ENCODE, 0, a, 4, 12, o1, 4, 8, ok, 2, 4, 1},
                {c, FEC_JOB_DECODE, 0, a, 4, 12, o2, 4, 12, dup, 0, 4, 1},
            };
            const int jst = fec_run_batch_jobs(jobs, 2, nullptr, 0);
            CHECK(jst == FEC_ENODEV || jst == FEC_EINVAL);  // no GPU here, or job 1's duplicate
            jobs[1].kind = 9;
            CHECK(fec_run_batch_jobs(jobs, 2, nullptr, 0) == FEC_EINVAL);
            CHECK(std::strstr(fec_last_error_message(), "job 1: kind 9") != nullptr);
        }
        fec_free(c);
    });
}

// Decode-matrix inversion from many threads (thread-local work buffers):
// D * E_rows == I for random erasure patterns of K=20/M=60.
void check_decode_matrices() {
    const zfec_hip::Field& f = zfec_hip::field();
    in_threads(8, [&](int t) {
        fec_t* c = fec_new(20, 60);
        unsigned seed = 12345u + 77u * static_cast<unsigned>(t);
        for (int it = 0; it < 50; ++it) {
            // a random 20 of the 60 blocks, primaries at their own slot (fec.c:549)
            unsigned perm[60];
            for (unsigned i = 0; i < 60; ++i) perm[i] = i;
            for (unsigned i = 59; i > 0; --i) {
                seed = seed * 1103515245u + 12345u;
                std::swap(perm[i], perm[(seed >> 8) % (i + 1)]);
            }
            unsigned idx[20];
            bool filled[20] = {};
            for (unsigned q = 0; q < 20; ++q)
                if (perm[q] < 20) {
                    idx[perm[q]] = perm[q];
                    filled[perm[q]] = true;
                }
            unsigned slot = 0;
            for (unsigned q = 0; q < 20; ++q)
                if (perm[q] >= 20) {
                    while (filled[slot]) ++slot;
                    idx[slot] = perm[q];
                    filled[slot] = true;
                }
            gf d[400];
            build_decode_matrix_into_space(c, idx, 20, d);
            CHECK(fec_last_status() == FEC_OK);
            for (unsigned i = 0; i < 20; ++i)
                for (unsigned j = 0; j < 20; ++j) {
                    unsigned v = 0;
                    for (unsigned q = 0; q < 20; ++q) v ^= f.mul[d[i * 20 + q]][c->enc_matrix[idx[q] * 20 + j]];
                    CHECK(v == (i == j ? 1u : 0u));
                }
        }
        fec_free(c);
    });
}

// The configuration object: readers on several threads while another
// re-reads the environment (objects are never freed, so a reader keeps a
// valid one).
void check_config_reload() {
    std::atomic<bool> stop{false};
    std::thread w([&] {
        for (int i = 0; i < 200; ++i) fec_reload_config();
        stop = true;
    });
    in_threads(4, [&](int) {
        while (!stop) {
            const zfec_hip::Config& c = zfec_hip::config();
            CHECK(c.launch_units >= 1024);
            CHECK(c.zc_limit > 0 && c.pack_limit > 0);
        }
    });
    w.join();
}

// The host copy pool: several callers queue copies and tasks with latches of
// their own and wait for them (the staged path's pattern).
void check_host_pool() {
    zfec_hip::HostPool& pool = zfec_hip::HostPool::get();
    in_threads(6, [&](int t) {
        std::vector<uint8_t> src(3 << 20), dst(3 << 20);
        for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<uint8_t>(i * 7 + t);
        for (int it = 0; it < 10; ++it) {
            zfec_hip::CopyLatch a, b;
            std::atomic<int> ran{0};
            pool.copy_async(dst.data(), src.data(), src.size(), &a, 256u << 10);
            for (int q = 0; q < 8; ++q) pool.run_async([&ran] { ran.fetch_add(1); }, &b);
            pool.wait(&a);
            pool.wait(&b);
            CHECK(ran.load() == 8);
            CHECK(std::memcmp(dst.data(), src.data(), src.size()) == 0);
            std::memset(dst.data(), 0, dst.size());
        }
    });
}

// The hipRTC JIT registry from several threads: the same and different
// matrices at once, one compile each (no GPU needed).
void check_jit_registry() {
    in_threads(6, [](int t) {
        const unsigned short k = (t % 2) ? 5 : 6, m = (t % 2) ? 9 : 11;
        fec_t* c = fec_new(k, m);
        unsigned nums[8];
        for (unsigned i = 0; i < static_cast<unsigned>(m - k); ++i) nums[i] = k + i;
        const int st = fec_jit_prepare_encode(c, nums, m - k);
        if (st != FEC_OK) fprintf(stderr, "jit prepare: %s\n", fec_last_error_message());
        CHECK(st == FEC_OK);
        fec_free(c);
    });
    CHECK(fec_jit_wait() >= 2);
}

}  // namespace

int main() {
    check_parallel_init();
    check_rejects();
    check_decode_matrices();
    check_config_reload();
    check_host_pool();
    check_jit_registry();
    const int f = g_fail.load();
    printf("sanitize_driver: %s (%d failed checks)\n", f ? "FAILED" : "ok", f);
    return f ? 1 : 0;
}
