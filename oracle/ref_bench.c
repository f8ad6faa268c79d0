/* ref_bench.c -- TEST INFRASTRUCTURE (bench.py's cpu_baseline leg only).
 *
 * Times the reference's own CPU path, zfec/fec.c compiled in place from
 * /root/reference by oracle/Makefile (`make -C oracle ref`), from C threads:
 * each thread repeats one step on its own stripe -- fec_encode of the m-k
 * secondaries (zfec/fec.c:487-505) and fec_decode from the last k blocks
 * (zfec/fec.c:527-557) -- the same step bench.py times on the GPU.  Calling
 * fec.c from C threads keeps the Python binding's per-call cost and the GIL
 * out of the CPU figure (for 4 KiB objects they dominate it).
 *
 *   int ref_bench(k, m, sz, nthreads, seconds, steps_out, seconds_out)
 *
 * returns 0, or -1 when memory or threads cannot be had.  The decoded blocks
 * are compared with the data once per thread (a wrong baseline is no baseline).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "fec.h"

typedef struct {
    const fec_t* code;
    unsigned k, m;
    size_t sz;
    int* ready;  /* threads done with their setup */
    int* stop;
    uint64_t steps;
    int ok;
} Job;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    const unsigned k = j->k, m = j->m, r = m - k;
    const size_t sz = j->sz;
    gf* mem = (gf*)malloc(sz * (k + r + k));
    gf** data = (gf**)malloc(sizeof(gf*) * k);
    gf** par = (gf**)malloc(sizeof(gf*) * r);
    gf** out = (gf**)malloc(sizeof(gf*) * k);
    const gf** in = (const gf**)malloc(sizeof(gf*) * k);
    unsigned* nums = (unsigned*)malloc(sizeof(unsigned) * r);
    unsigned* index = (unsigned*)malloc(sizeof(unsigned) * k);
    j->ok = 0;
    if (!mem || !data || !par || !out || !in || !nums || !index) {
        __atomic_add_fetch(j->ready, 1, __ATOMIC_RELEASE);
        goto done;
    }
    unsigned seed = 12345u + (unsigned)(uintptr_t)j;
    for (unsigned i = 0; i < k; ++i) {
        data[i] = mem + i * sz;
        for (size_t b = 0; b < sz; ++b) data[i][b] = (gf)(rand_r(&seed) >> 7);
    }
    for (unsigned i = 0; i < r; ++i) par[i] = mem + (k + i) * sz, nums[i] = k + i;
    for (unsigned i = 0; i < k; ++i) out[i] = mem + (k + r + i) * sz;
    /* receive blocks m-k .. m-1: a present primary sits at its own slot, the
       present secondaries (from max(m-k, k) up) fill the other slots in order
       (fec.h:51-57) -- bench.py's place() */
    {
        unsigned nxt = m - k > k ? m - k : k;
        for (unsigned i = 0; i < k; ++i) index[i] = i >= m - k ? i : nxt++;
    }
    for (unsigned i = 0; i < k; ++i) in[i] = index[i] < k ? data[index[i]] : par[index[i] - k];
    __atomic_add_fetch(j->ready, 1, __ATOMIC_RELEASE);
    uint64_t n = 0;
    while (!__atomic_load_n(j->stop, __ATOMIC_ACQUIRE)) {
        fec_encode(j->code, (const gf* const*)data, par, nums, r, sz);
        fec_decode(j->code, in, out, index, sz);
        ++n;
    }
    /* the decoded primaries are the missing ones, in index order */
    {
        unsigned q = 0;
        int ok = 1;
        for (unsigned i = 0; i < k; ++i)
            if (index[i] >= k) ok = ok && memcmp(out[q++], data[i], sz) == 0;
        j->ok = ok ? 1 : 0;
    }
    j->steps = n;
done:
    free(mem);
    free(data);
    free(par);
    free(out);
    free(in);
    free(nums);
    free(index);
    return NULL;
}

int ref_bench(unsigned k, unsigned m, size_t sz, int nthreads, double seconds, uint64_t* steps_out,
              double* seconds_out) {
    if (k < 1 || m <= k || m > 256 || nthreads < 1 || sz < 1) return -1;
    fec_init();
    fec_t* code = fec_new((unsigned short)k, (unsigned short)m);
    if (!code) return -1;
    int stop = 0, ready = 0;
    Job* jobs = (Job*)calloc((size_t)nthreads, sizeof(Job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) return -1;
    int started = 0;
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (Job){code, k, m, sz, &ready, &stop, 0, 0};
        if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) break;
        ++started;
    }
    /* the clock starts once every thread has its stripe (setup is not timed) */
    while (__atomic_load_n(&ready, __ATOMIC_ACQUIRE) < started) {
        struct timespec w = {0, 100000};
        nanosleep(&w, NULL);
    }
    const double t0 = now();
    struct timespec ts = {(time_t)seconds, (long)((seconds - (double)(time_t)seconds) * 1e9)};
    nanosleep(&ts, NULL);
    __atomic_store_n(&stop, 1, __ATOMIC_RELEASE);
    uint64_t total = 0;
    int ok = started == nthreads;
    for (int t = 0; t < started; ++t) {
        pthread_join(th[t], NULL);
        total += jobs[t].steps;
        ok = ok && jobs[t].ok;
    }
    *seconds_out = now() - t0; /* every thread's step in flight at the stop is counted */
    *steps_out = total;
    free(jobs);
    free(th);
    fec_free(code);
    return ok ? 0 : -1;
}
