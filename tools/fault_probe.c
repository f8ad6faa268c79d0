// fault_probe.c -- how fast can fresh host pages be made writable on this
// host (the cost behind the bytes API's fresh output buffers)?  Maps 156 MB
// (7 x 22.4 MB, one K=3/M=10 64 MiB stripe's parity) and faults it in:
//   touch-N    N threads each writing one byte per 4 KiB page of its share
//   populate-N N threads each madvise(MADV_POPULATE_WRITE) on its share
//   memcpy-N   N threads copying a warm buffer into the fresh mapping
//   warm-N     N threads copying into already-faulted pages (the copy alone)
// build: gcc -O2 -pthread tools/fault_probe.c -o tools/fault_probe.exe
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/utsname.h>
#include <time.h>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static size_t N = 7ul * 22369622ul;
static char* src;

struct job { char* p; size_t n; int mode; int rc; };

static void* work(void* a) {
    struct job* j = a;
    if (j->mode == 0) {
        for (size_t i = 0; i < j->n; i += 4096) j->p[i] = 1;
    } else if (j->mode == 1) {
        j->rc = madvise(j->p, j->n, MADV_POPULATE_WRITE);
    } else {
        memcpy(j->p, src + (j->p - (char*)0) % 4096 * 0, j->n);
    }
    return NULL;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static double run(int mode, int nt, int fresh, int* rc) {
    char* p = mmap(NULL, N, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (!fresh) memset(p, 0, N);
    pthread_t th[64];
    struct job js[64];
    size_t per = (N / nt + 4095) / 4096 * 4096;
    double t0 = now();
    for (int i = 0; i < nt; ++i) {
        size_t off = per * i;
        js[i].p = p + off;
        js[i].n = off >= N ? 0 : (off + per > N ? N - off : per);
        js[i].mode = mode;
        js[i].rc = 0;
        pthread_create(&th[i], NULL, work, &js[i]);
    }
    for (int i = 0; i < nt; ++i) pthread_join(th[i], NULL);
    double t = now() - t0;
    *rc = 0;
    for (int i = 0; i < nt; ++i) *rc |= js[i].rc;
    munmap(p, N);
    return t;
}

int main(void) {
    struct utsname u;
    uname(&u);
    printf("kernel %s, %zu bytes\n", u.release, N);
    src = malloc(N);
    memset(src, 7, N);
    const char* names[] = {"touch", "populate", "memcpy"};
    for (int mode = 0; mode < 3; ++mode)
        for (int nt = 1; nt <= 16; nt *= 2) {
            int rc;
            double best = 1e9;
            for (int r = 0; r < 3; ++r) {
                double t = run(mode, nt, 1, &rc);
                if (t < best) best = t;
            }
            printf("%-9s %2d threads: %7.2f ms  (%.1f GB/s)%s\n", names[mode], nt, best * 1e3, N / best / 1e9,
                   rc ? "  [madvise failed]" : "");
        }
    for (int nt = 1; nt <= 16; nt *= 2) {
        int rc;
        double best = 1e9;
        for (int r = 0; r < 3; ++r) {
            double t = run(2, nt, 0, &rc);
            if (t < best) best = t;
        }
        printf("warm-copy %2d threads: %7.2f ms  (%.1f GB/s)\n", nt, best * 1e3, N / best / 1e9);
    }
    return 0;
}
