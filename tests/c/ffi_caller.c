/* ffi_caller.c -- a plain C program that uses libzfec_hip.so exactly the way
 * the reference's FFI bindings use fec.h: host (malloc) buffers, fec_init /
 * fec_new / fec_encode / fec_decode / fec_free, several threads at once.
 *
 * Mirrors the properties of haskell/test/FECTest.hs (the Haskell binding
 * `foreign import ccall`s these same symbols, haskell/Codec/FEC.hs:79-114):
 *   - prop_primary_copies (:109-115): with k = 1 every secondary block is a
 *     copy of the primary; run from many threads at once, first thing after
 *     start-up, because it once caught a multi-threaded initialisation bug
 *     (:127-140);
 *   - testFEC / prop_decode (:58-89, :97-102): block j = byte j repeated,
 *     encode all secondaries, decode from a random k of the n blocks, get the
 *     primaries back.
 * Build and run: tests/test_ffi_caller.py (gpu).  Exit status 0 = pass. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zfec_hip.h"

static unsigned xs(unsigned* s) { /* xorshift32 */
    unsigned x = *s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return *s = x;
}

static int fail(const char* what, unsigned k, unsigned n, size_t len) {
    fprintf(stderr, "FAIL %s k=%u n=%u len=%zu: %s\n", what, k, n, len, fec_last_error_message());
    return 1;
}

/* prop_primary_copies */
static int primary_copies(unsigned seed) {
    const unsigned n = 2 + xs(&seed) % 254;
    const size_t len = 1 + xs(&seed) % 3000;
    fec_t* code = fec_new(1, (unsigned short)n);
    if (!code) return fail("fec_new", 1, n, len);
    gf* prim = malloc(len);
    for (size_t i = 0; i < len; ++i) prim[i] = (gf)xs(&seed);
    gf** outs = malloc((n - 1) * sizeof(gf*));
    unsigned* nums = malloc((n - 1) * sizeof(unsigned));
    for (unsigned i = 0; i < n - 1; ++i) {
        outs[i] = malloc(len);
        nums[i] = i + 1;
    }
    const gf* ins[1] = {prim};
    int bad = 0;
    fec_encode(code, ins, outs, nums, n - 1, len);
    if (fec_last_status() != FEC_OK) bad = fail("fec_encode", 1, n, len);
    for (unsigned i = 0; i < n - 1 && !bad; ++i)
        if (memcmp(outs[i], prim, len)) bad = fail("secondary is not a copy of the primary", 1, n, len);
    for (unsigned i = 0; i < n - 1; ++i) free(outs[i]);
    free(outs);
    free(nums);
    free(prim);
    fec_free(code);
    return bad;
}

/* testFEC */
static int roundtrip(unsigned seed) {
    const unsigned k = 1 + xs(&seed) % 255;
    const unsigned n = k + xs(&seed) % (256 - k);
    const size_t len = xs(&seed) % 2049;
    fec_t* code = fec_new((unsigned short)k, (unsigned short)n);
    if (!code) return fail("fec_new", k, n, len);
    gf** blocks = malloc(n * sizeof(gf*));
    for (unsigned j = 0; j < n; ++j) {
        blocks[j] = malloc(len ? len : 1);
        if (j < k) memset(blocks[j], (int)j, len);
    }
    int bad = 0;
    if (n > k) {
        unsigned* nums = malloc((n - k) * sizeof(unsigned));
        for (unsigned i = 0; i < n - k; ++i) nums[i] = k + i;
        fec_encode(code, (const gf* const*)blocks, blocks + k, nums, n - k, len);
        if (fec_last_status() != FEC_OK) bad = fail("fec_encode", k, n, len);
        free(nums);
    }
    /* a random k of the n blocks; primaries at their own slot, secondaries fill the rest */
    unsigned* perm = malloc(n * sizeof(unsigned));
    for (unsigned j = 0; j < n; ++j) perm[j] = j;
    for (unsigned j = n - 1; j > 0; --j) {
        const unsigned t = xs(&seed) % (j + 1), u = perm[j];
        perm[j] = perm[t];
        perm[t] = u;
    }
    unsigned* index = malloc(k * sizeof(unsigned));
    const gf** in = malloc(k * sizeof(gf*));
    char* used = calloc(k, 1);
    unsigned nsec = 0;
    for (unsigned i = 0; i < k; ++i)
        if (perm[i] < k) {
            index[perm[i]] = perm[i];
            in[perm[i]] = blocks[perm[i]];
            used[perm[i]] = 1;
        }
    unsigned slot = 0;
    for (unsigned i = 0; i < k; ++i)
        if (perm[i] >= k) {
            while (used[slot]) ++slot;
            index[slot] = perm[i];
            in[slot] = blocks[perm[i]];
            used[slot] = 1;
            ++nsec;
        }
    gf** out = malloc((nsec ? nsec : 1) * sizeof(gf*));
    for (unsigned i = 0; i < nsec; ++i) out[i] = malloc(len ? len : 1);
    if (!bad) {
        fec_decode(code, in, out, index, len);
        if (fec_last_status() != FEC_OK) bad = fail("fec_decode", k, n, len);
    }
    /* recovered primaries come out in ascending order of their numbers */
    unsigned o = 0;
    for (unsigned j = 0; j < k && !bad; ++j) {
        int have = 0;
        for (unsigned i = 0; i < k; ++i) have |= index[i] == j;
        if (have) continue;
        for (size_t b = 0; b < len; ++b)
            if (out[o][b] != (gf)j) {
                bad = fail("decoded block differs", k, n, len);
                break;
            }
        ++o;
    }
    for (unsigned i = 0; i < nsec; ++i) free(out[i]);
    for (unsigned j = 0; j < n; ++j) free(blocks[j]);
    free(out);
    free(blocks);
    free(perm);
    free(index);
    free(in);
    free(used);
    fec_free(code);
    return bad;
}

struct Job {
    unsigned seed;
    int iters, bad;
};

static void* copies_thread(void* p) {
    struct Job* j = p;
    fec_init();
    for (int i = 0; i < j->iters && !j->bad; ++i) j->bad |= primary_copies(j->seed + 7919u * i);
    return NULL;
}

static void* roundtrip_thread(void* p) {
    struct Job* j = p;
    for (int i = 0; i < j->iters && !j->bad; ++i) j->bad |= roundtrip(j->seed + 104729u * i);
    return NULL;
}

static int run(void* (*fn)(void*), int nthreads, int iters, unsigned seed) {
    pthread_t t[64];
    struct Job jobs[64];
    for (int i = 0; i < nthreads; ++i) {
        jobs[i] = (struct Job){seed + 1000u * i + 1u, iters, 0};
        pthread_create(&t[i], NULL, fn, &jobs[i]);
    }
    int bad = 0;
    for (int i = 0; i < nthreads; ++i) {
        pthread_join(t[i], NULL);
        bad |= jobs[i].bad;
    }
    return bad;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    /* no fec_init() here: the threads race to initialise, as in FECTest.hs */
    if (run(copies_thread, 20, 5, 1u)) return 1;
    if (run(roundtrip_thread, 8, iters, 99u)) return 1;
    printf("ok: %d primary-copy and %d round-trip cases\n", 20 * 5, 8 * iters);
    return 0;
}
