// Per-call cost of the drop-in Encryptor (VERDICT r01 item 6 / config C1's shape: 10 000
// frames of 1 KiB through PackageEncryptor, one call per frame as FPNN's SendBuffer and
// EncryptedPackageReceiver make them, core/IOBuffer.cpp:36-45, core/EncryptedPackageReceiver.cpp:110).
//
// The same source is built twice:
//   * against the reference's core/Encryptor.h + base/rijndael.c + core/Encryptor.cpp
//     (oracle/Makefile `percall` -> oracle/_ref/percall_ref; TEST INFRASTRUCTURE: the CPU
//     baseline), and
//   * against include/Encryptor.h + libfpnn_aes.so (tools/bench_percall.py), which adds
//     the batched form (fpnn::EncryptorBatch: the 10 000 calls queued, one flush).
// Both print one JSON line with a checksum of every output byte, so the two builds are
// checked against each other.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "Encryptor.h"
#ifdef FPNN_AMD_ENCRYPTOR_H
#include "EncryptorBatch.h"
#endif

static uint64_t fnv(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 10000, len = argc > 2 ? atoi(argv[2]) : 1024;
    uint8_t key[32], iv[16];
    for (int i = 0; i < 32; i++) key[i] = (uint8_t)(7 * i + 1);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)(13 * i + 5);
    std::vector<uint8_t> src((size_t)n * len), enc(src.size()), dec(src.size());
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &b : src) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = (uint8_t)x;
    }
    fpnn::PackageEncryptor pe(key, 32, iv);
    pe.encrypt(enc.data(), src.data(), len);  // warm-up (GPU build: engine creation)
    double t0 = now();
    for (int i = 0; i < n; i++) pe.encrypt(enc.data() + (size_t)i * len, src.data() + (size_t)i * len, len);
    const double te = now() - t0;
    t0 = now();
    for (int i = 0; i < n; i++) pe.decrypt(dec.data() + (size_t)i * len, enc.data() + (size_t)i * len, len);
    const double td = now() - t0;
    if (memcmp(dec.data(), src.data(), src.size()) != 0) {
        fprintf(stderr, "round trip failed\n");
        return 1;
    }
    std::vector<std::string> wire(n);
    t0 = now();
    for (int i = 0; i < n; i++) {  // SendBuffer::encryptData's call: encrypt(std::string*) adds the length prefix
        wire[i].assign(reinterpret_cast<const char *>(src.data()) + (size_t)i * len, len);
        pe.encrypt(&wire[i]);
    }
    const double ts = now() - t0;
    uint64_t h = 0xcbf29ce484222325ull;
    h = fnv(h, enc.data(), enc.size());
    for (const auto &w : wire) h = fnv(h, reinterpret_cast<const uint8_t *>(w.data()), w.size());
    printf("{\"frames\": %d, \"len\": %d, \"us_per_encrypt\": %.3f, \"us_per_decrypt\": %.3f, "
           "\"us_per_encrypt_string\": %.3f, \"checksum\": \"%016llx\"", n, len, 1e6 * te / n, 1e6 * td / n,
           1e6 * ts / n, (unsigned long long)h);
#ifdef FPNN_AMD_ENCRYPTOR_H
    // the same frames queued in one EncryptorBatch and flushed once
    std::vector<uint8_t> benc(src.size());
    fpnn::EncryptorBatch batch;
    for (int i = 0; i < n; i++) batch.encrypt(&pe, benc.data() + (size_t)i * len, src.data() + (size_t)i * len, len);
    batch.flush();  // warm-up of the batch path
    t0 = now();
    for (int i = 0; i < n; i++) batch.encrypt(&pe, benc.data() + (size_t)i * len, src.data() + (size_t)i * len, len);
    batch.flush();
    const double tb = now() - t0;
    printf(", \"us_per_frame_batched\": %.3f, \"batched_matches\": %s", 1e6 * tb / n,
           memcmp(benc.data(), enc.data(), enc.size()) == 0 ? "true" : "false");
#endif
    printf("}\n");
    return 0;
}
