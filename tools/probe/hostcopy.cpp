// Host memcpy bandwidth into/out of HIP pinned memory (flags 0 vs non-coherent) vs
// pageable memory, 1 and N threads -- sizing the host-frame pipeline's gather/scatter.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double bw(void *dst, const void *src, size_t n, int threads, int reps) {
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) {
        std::vector<std::thread> ts;
        for (int t = 0; t < threads; t++)
            ts.emplace_back([=] {
                size_t a = n * t / threads, b = n * (t + 1) / threads;
                memcpy((char *)dst + a, (const char *)src + a, b - a);
            });
        for (auto &t : ts) t.join();
    }
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return (double)n * reps / s / (1 << 30);
}

int main() {
    const size_t n = 256u << 20;
    char *pg1 = (char *)aligned_alloc(4096, n), *pg2 = (char *)aligned_alloc(4096, n);
    memset(pg1, 1, n);
    memset(pg2, 2, n);
    struct { const char *name; unsigned flags; } kinds[] = {{"pinned(default)", 0},
                                                            {"pinned(noncoherent)", hipHostMallocNonCoherent},
                                                            {"pinned(coherent)", hipHostMallocCoherent}};
    printf("pageable->pageable: 1t %.1f  8t %.1f  16t %.1f GiB/s\n", bw(pg2, pg1, n, 1, 3), bw(pg2, pg1, n, 8, 5),
           bw(pg2, pg1, n, 16, 5));
    for (auto &k : kinds) {
        char *h = nullptr;
        if (hipHostMalloc((void **)&h, n, k.flags) != hipSuccess) { printf("%s: alloc failed\n", k.name); continue; }
        memset(h, 3, n);
        printf("%s: in(pageable->pinned) 1t %.1f 8t %.1f 16t %.1f | out(pinned->pageable) 1t %.1f 8t %.1f 16t %.1f GiB/s\n",
               k.name, bw(h, pg1, n, 1, 3), bw(h, pg1, n, 8, 5), bw(h, pg1, n, 16, 5), bw(pg2, h, n, 1, 3),
               bw(pg2, h, n, 8, 5), bw(pg2, h, n, 16, 5));
        hipHostFree(h);
    }
    return 0;
}
