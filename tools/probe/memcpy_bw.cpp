// Host copy bandwidth probe for the host-frame path: T threads each copy their share of
// N frames of L bytes (gather from a pageable array into a second array), with glibc
// memcpy and with 32-byte non-temporal stores.  Prints GB/s of payload copied.
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <thread>
#include <vector>

__attribute__((target("avx2"))) static void copy_nt(uint8_t *d, const uint8_t *s, size_t n) {
    size_t head = (32 - ((uintptr_t)d & 31)) & 31;
    if (head > n) head = n;
    memcpy(d, s, head);
    d += head; s += head; n -= head;
    for (; n >= 128; n -= 128, d += 128, s += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *)s), b = _mm256_loadu_si256((const __m256i *)(s + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *)(s + 64)), e = _mm256_loadu_si256((const __m256i *)(s + 96));
        _mm256_stream_si256((__m256i *)d, a); _mm256_stream_si256((__m256i *)(d + 32), b);
        _mm256_stream_si256((__m256i *)(d + 64), c); _mm256_stream_si256((__m256i *)(d + 96), e);
    }
    for (; n >= 32; n -= 32, d += 32, s += 32) _mm256_stream_si256((__m256i *)d, _mm256_loadu_si256((const __m256i *)s));
    memcpy(d, s, n);
}

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 16;
    const size_t L = 1024, N = 1 << 20;
    std::vector<uint8_t> a(N * L, 1), b(N * L, 0);
    for (int mode = 0; mode < 2; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < T; t++)
                th.emplace_back([&, t] {
                    for (size_t i = N * t / T; i < N * (t + 1) / T; i++) {
                        if (mode == 0) memcpy(&b[i * L], &a[i * L], L);
                        else copy_nt(&b[i * L], &a[i * L], L);
                    }
                    _mm_sfence();
                });
            for (auto &x : th) x.join();
            double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            printf("%s threads=%d rep=%d %.1f GB/s\n", mode ? "nt" : "memcpy", T, rep, N * L / dt / 1e9);
        }
    }
}
