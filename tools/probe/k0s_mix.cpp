// Small-call servers (K0s) beside batch kernels, both ways -- native threads (VERDICT r04
// item 4; tools/bench_k0s.py measured the same from Python, whose GIL hand-offs between a
// spinning per-call thread and the timing thread added ~0.9 ms to every timed call).
//
//   * batch call wall time (host clock around call + engine sync, median of reps) on the
//     main engine while N threads (N = 0, 1, 4, 16), each with its own engine and stream,
//     issue 1 KiB per-call decrypts back to back through fpnn_aes_cfb_host (the drop-in's
//     PackageEncryptor::decrypt shape, which keeps a K0s server alive per engine):
//     C2 (1M x 1 KiB AES-256 package) encrypt / decrypt and a C4-shaped ragged batch
//     (Zipf 64 B..64 KiB, 1 GiB) encrypt / decrypt;
//   * per-call decrypt latency alone and while the main engine runs C4-shaped encrypts
//     back to back.
// Prints JSON lines.
//   g++ -O2 -std=c++17 -I include tools/probe/k0s_mix.cpp -o tools/probe/k0s_mix -L fpnn_amd -lfpnn_aes \
//       -Wl,-rpath,$PWD/fpnn_amd -pthread
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "fpnn_aes.h"

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                                     \
    do {                                                                                          \
        int rc_ = (x);                                                                            \
        if (rc_) {                                                                                \
            fprintf(stderr, "%s failed: %d %s\n", #x, rc_, fpnn_aes_last_error());               \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

static double pct(std::vector<double> v, double p) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(p / 100.0 * (v.size() - 1) + 0.5))];
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 7;
    fpnn_aes_engine *e;
    CK(fpnn_aes_engine_create(0, FPNN_AES_OWN_STREAM, &e));
    uint8_t key[32], iv[16];
    for (int i = 0; i < 32; i++) key[i] = (uint8_t)(i * 7 + 1);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)(i * 3 + 2);
    fpnn_aes_keyset *ks;
    CK(fpnn_aes_keyset_create(e, 1, 32, key, iv, 1, &ks));
    // C2
    const uint32_t P = 1u << 20, L = 1024;
    void *a, *b;
    CK(fpnn_aes_device_alloc(e, (size_t)P * L, &a));
    CK(fpnn_aes_device_alloc(e, (size_t)P * L, &b));
    CK(fpnn_aes_fill_synthetic(e, (uint8_t *)a, (uint64_t)P * L, 2, 0));
    // C4-shaped: Zipf(1.1) over 1..1024 units of 64 B until 1 GiB
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    {
        std::vector<double> cdf(1024);
        double acc = 0;
        for (int r = 1; r <= 1024; r++) cdf[r - 1] = (acc += pow((double)r, -1.1));
        std::mt19937_64 rng(4);
        std::uniform_real_distribution<double> u(0, acc);
        uint64_t at = 0;
        while (at < (1ull << 30)) {
            const int r = (int)(std::lower_bound(cdf.begin(), cdf.end(), u(rng)) - cdf.begin()) + 1;
            offs.push_back(at);
            lens.push_back(64u * r);
            at += 64u * r;
        }
    }
    const uint32_t n4 = (uint32_t)lens.size();
    const uint64_t t4 = offs.back() + lens.back();
    void *a4, *b4, *d_off, *d_len;
    CK(fpnn_aes_device_alloc(e, t4, &a4));
    CK(fpnn_aes_device_alloc(e, t4, &b4));
    CK(fpnn_aes_device_alloc(e, 8ull * n4, &d_off));
    CK(fpnn_aes_device_alloc(e, 4ull * n4, &d_len));
    CK(fpnn_aes_fill_synthetic(e, (uint8_t *)a4, t4, 4, 0));
    CK(fpnn_aes_copy_async(e, d_off, offs.data(), 8ull * n4));
    CK(fpnn_aes_copy_async(e, d_len, lens.data(), 4ull * n4));
    CK(fpnn_aes_engine_sync(e));

    fpnn_aes_batch c2e{}, c2d{}, c4e{}, c4d{};
    c2e.in = (const uint8_t *)a; c2e.out = (uint8_t *)b; c2e.count = P; c2e.uniform_len = L; c2e.stride = L; c2e.keys = ks;
    c2d = c2e; c2d.in = (const uint8_t *)b; c2d.out = (uint8_t *)a;
    c4e.in = (const uint8_t *)a4; c4e.out = (uint8_t *)b4; c4e.count = n4; c4e.in_off = (const uint64_t *)d_off;
    c4e.len = (const uint32_t *)d_len; c4e.keys = ks;
    c4d = c4e; c4d.in = (const uint8_t *)b4; c4d.out = (uint8_t *)a4;
    struct Call {
        const char *name;
        std::function<void()> fn;
    };
    std::vector<Call> calls = {
        {"C2_encrypt", [&] { CK(fpnn_aes_package_encrypt(e, &c2e)); }},
        {"C2_decrypt", [&] { CK(fpnn_aes_package_decrypt(e, &c2d)); }},
        {"C4_encrypt", [&] { CK(fpnn_aes_package_encrypt(e, &c4e)); }},
        {"C4_decrypt", [&] { CK(fpnn_aes_package_decrypt(e, &c4d)); }},
    };
    auto wall = [&](const Call &c) {
        std::vector<double> t;
        for (int r = 0; r < reps; r++) {
            const double t0 = now();
            c.fn();
            CK(fpnn_aes_engine_sync(e));
            t.push_back(now() - t0);
        }
        return pct(t, 50);
    };
    for (double t_end = now() + 0.5; now() < t_end;)  // clocks up, scratch grown
        for (auto &c : calls) {
            c.fn();
            CK(fpnn_aes_engine_sync(e));
        }

    std::atomic<bool> stop{false};
    auto per_call = [&](std::vector<double> *lat, std::atomic<int> *ready) {
        fpnn_aes_engine *pe;
        CK(fpnn_aes_engine_create(0, FPNN_AES_OWN_STREAM, &pe));
        fpnn_aes_schedule ctx;
        CK(fpnn_aes_setup_encrypt(&ctx, key, 32));
        uint8_t in[1024], out[1024];
        for (int i = 0; i < 1024; i++) in[i] = (uint8_t)(i * 13);
        uint8_t v[16];
        size_t num = 0;
        memcpy(v, iv, 16);
        CK(fpnn_aes_cfb_host(pe, &ctx, 0, in, out, 1024, v, &num));
        ready->fetch_add(1);
        while (!stop.load(std::memory_order_relaxed)) {
            memcpy(v, iv, 16);
            num = 0;
            const double t0 = now();
            CK(fpnn_aes_cfb_host(pe, &ctx, 0, in, out, 1024, v, &num));
            lat->push_back(now() - t0);
        }
        CK(fpnn_aes_engine_destroy(pe));
    };
    auto with_threads = [&](int n, std::function<void()> body, std::vector<std::vector<double>> &lats) {
        stop = false;
        lats.assign(n, {});
        std::atomic<int> ready{0};
        std::vector<std::thread> th;
        for (int i = 0; i < n; i++) th.emplace_back(per_call, &lats[i], &ready);
        while (ready.load() < n) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
        body();
        stop = true;
        for (auto &t : th) t.join();
    };

    std::vector<double> base;
    for (int n : {0, 1, 4, 16}) {
        std::vector<double> ms(calls.size());
        std::vector<std::vector<double>> lats;
        with_threads(n, [&] { for (size_t i = 0; i < calls.size(); i++) ms[i] = 1e3 * wall(calls[i]); }, lats);
        if (n == 0) base = ms;
        std::string row = "{\"servers\": " + std::to_string(n);
        char buf[256];
        for (size_t i = 0; i < calls.size(); i++) {
            snprintf(buf, sizeof buf, ", \"%s_ms\": %.3f, \"%s_vs_none\": %.3f", calls[i].name, ms[i], calls[i].name,
                     ms[i] / base[i]);
            row += buf;
        }
        std::vector<double> all;
        for (auto &l : lats) all.insert(all.end(), l.begin(), l.end());
        snprintf(buf, sizeof buf, ", \"per_call_n\": %zu, \"per_call_p50_us\": %.1f, \"per_call_p99_us\": %.1f}", all.size(),
                 1e6 * pct(all, 50), 1e6 * pct(all, 99));
        row += buf;
        printf("%s\n", row.c_str());
        fflush(stdout);
    }
    // per-call latency alone / during back-to-back C4-shaped encrypts
    std::vector<std::vector<double>> alone, during;
    with_threads(1, [&] { std::this_thread::sleep_for(std::chrono::milliseconds(500)); }, alone);
    int flushes = 0;
    with_threads(1, [&] {
        for (double t_end = now() + 0.5; now() < t_end; flushes++) calls[2].fn();
        CK(fpnn_aes_engine_sync(e));
    }, during);
    auto q = [&](const std::vector<double> &v) {
        char buf[256];
        snprintf(buf, sizeof buf, "{\"n\": %zu, \"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}", v.size(),
                 1e6 * pct(v, 50), 1e6 * pct(v, 90), 1e6 * pct(v, 99), 1e6 * pct(v, 100));
        return std::string(buf);
    };
    printf("{\"per_call_decrypt_us\": {\"alone\": %s, \"during_c4_encrypts\": %s, \"c4_encrypts\": %d, \"c4_encrypt_ms\": %.3f}}\n",
           q(alone[0]).c_str(), q(during[0]).c_str(), flushes, base[2]);
    return 0;
}
