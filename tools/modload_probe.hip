// modload_probe.hip -- how long does it take to load a run-time specialised
// kernel's code object (hipModuleLoadData + hipModuleGetFunction) and launch
// it once?  Decides whether patching a pre-compiled template per erasure
// pattern (instead of a hipRTC compile) could serve first-seen patterns.
// usage: tools/modload_probe.exe <code object .co> <kernel name> [iterations]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    std::vector<char> code;
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) code.insert(code.end(), buf, buf + n);
    fclose(f);
    const int it = argc > 3 ? atoi(argv[3]) : 20;
    if (hipFree(nullptr) != hipSuccess) return 4;  // context up
    double tot = 0, mn = 1e9, mx = 0;
    for (int i = 0; i < it; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        hipModule_t m;
        hipFunction_t fn;
        if (hipModuleLoadData(&m, code.data()) != hipSuccess) return 5;
        if (hipModuleGetFunction(&fn, m, argv[2]) != hipSuccess) return 6;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        tot += us;
        mn = us < mn ? us : mn;
        mx = us > mx ? us : mx;
        if (hipModuleUnload(m) != hipSuccess) return 7;
    }
    printf("code object %zu bytes: load+getfunction mean %.1f us, min %.1f, max %.1f over %d\n", code.size(), tot / it,
           mn, mx, it);
    return 0;
}
