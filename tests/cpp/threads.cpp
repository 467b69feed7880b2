// threads.cpp -- the engine pool behind the C++ classes (fpnn_amd/csrc/thread_engine.hpp)
// under FPNN's threading: Encryptors used from several IO / worker threads, an
// EncryptorBatch and a StreamReceiverBatch that outlive the thread that first flushed them
// (flushed on a worker thread, the thread joined, then flushed and destroyed
// on the main thread), and more threads than the pool has engines (FPNN_AES_MAX_ENGINES,
// set by the caller: threads then share engines and their calls serialise).
//
// Every frame is a deterministic function of (thread, frame); the program prints one line
// per (thread, kind) with an FNV-1a checksum of the ciphertexts, which the test recomputes
// with the oracle:
//   percall <t> <fnv>   PackageEncryptor::encrypt of frames 0..n-1 of thread t, one call each
//   batch <t> <fnv>     the same frames through one EncryptorBatch flush (must equal percall)
//   stream <t> <fnv>    StreamEncryptor::encrypt of the frames in order (one stream)
//   roundtrip <t> <ok>  decrypt(encrypt(x)) == x for the per-call and stream paths
//   migrate <fnv> <ok>  batch + receiver first flushed on a joined thread, then on main
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "Encryptor.h"
#include "EncryptorBatch.h"
#include "StreamReceiverBatch.h"

namespace {

uint64_t fnv(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}

std::vector<uint8_t> bytes_of(uint64_t seed, size_t n) {
    std::vector<uint8_t> v(n);
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    for (auto &b : v) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        b = (uint8_t)x;
    }
    return v;
}

size_t frame_len(int t, int i) { return (size_t)(1 + (t * 131 + i * 977) % 3000); }

std::mutex out_mu;

void worker(int t, int frames) {
    std::vector<uint8_t> key = bytes_of(1000 + t, 32), iv = bytes_of(2000 + t, 16);
    const size_t keylen = t % 3 == 0 ? 16 : t % 3 == 1 ? 24 : 32;
    fpnn::PackageEncryptor pe(key.data(), keylen, iv.data());
    fpnn::StreamEncryptor se(key.data(), keylen, iv.data()), sd(key.data(), keylen, iv.data());
    std::vector<std::vector<uint8_t>> plain(frames), enc(frames), benc(frames), senc(frames);
    uint64_t hp = 0xcbf29ce484222325ull, hb = hp, hs = hp;
    bool ok = true;
    fpnn::EncryptorBatch batch;
    for (int i = 0; i < frames; i++) {
        plain[i] = bytes_of(((uint64_t)t << 32) | (uint64_t)i, frame_len(t, i));
        const int n = (int)plain[i].size();
        enc[i].resize(n);
        benc[i].resize(n);
        senc[i].resize(n);
        pe.encrypt(enc[i].data(), plain[i].data(), n);
        std::vector<uint8_t> back(n);
        pe.decrypt(back.data(), enc[i].data(), n);
        ok = ok && back == plain[i];
        se.encrypt(senc[i].data(), plain[i].data(), n);
        std::vector<uint8_t> sback(n);
        sd.decrypt(sback.data(), senc[i].data(), n);
        ok = ok && sback == plain[i];
        batch.encrypt(&pe, benc[i].data(), plain[i].data(), n);
        hp = fnv(hp, enc[i].data(), n);
        hs = fnv(hs, senc[i].data(), n);
    }
    batch.flush();
    for (int i = 0; i < frames; i++) hb = fnv(hb, benc[i].data(), benc[i].size());
    std::lock_guard<std::mutex> lk(out_mu);
    printf("percall %d %016llx\nbatch %d %016llx\nstream %d %016llx\nroundtrip %d %d\n", t, (unsigned long long)hp, t,
           (unsigned long long)hb, t, (unsigned long long)hs, t, ok ? 1 : 0);
}

}  // namespace

int main(int argc, char **argv) {
    const int nthreads = argc > 1 ? atoi(argv[1]) : 6;
    const int frames = argc > 2 ? atoi(argv[2]) : 60;

    // ---- migration: first flush on a thread that then exits, the rest on main ----
    {
        std::vector<uint8_t> key = bytes_of(77, 32), iv = bytes_of(78, 16);
        std::unique_ptr<fpnn::PackageEncryptor> pe(new fpnn::PackageEncryptor(key.data(), 32, iv.data()));
        std::unique_ptr<fpnn::StreamEncryptor> rxenc(new fpnn::StreamEncryptor(key.data(), 32, iv.data()));
        std::unique_ptr<fpnn::EncryptorBatch> batch(new fpnn::EncryptorBatch());
        std::unique_ptr<fpnn::StreamReceiverBatch> rx(new fpnn::StreamReceiverBatch());
        const int conn = rx->open(rxenc.get());
        std::vector<std::vector<uint8_t>> plain(8), out(8);
        for (int i = 0; i < 8; i++) {
            plain[i] = bytes_of(500 + i, 100 + 37 * i);
            out[i].resize(plain[i].size());
        }
        const std::vector<uint8_t> junk = bytes_of(9, 40);  // not an FPNN message: the receiver closes
        {  // main leases its engine first, so the thread below works on another one
            std::vector<uint8_t> x(64), y(64);
            pe->encrypt(y.data(), x.data(), 64);
        }
        std::thread th([&] {
            for (int i = 0; i < 4; i++) batch->encrypt(pe.get(), out[i].data(), plain[i].data(), (int)plain[i].size());
            batch->flush();
            rx->received(conn, junk.data(), 5);  // a partial header: nothing to hand out yet
            rx->flush();
        });
        th.join();
        for (int i = 4; i < 8; i++) batch->encrypt(pe.get(), out[i].data(), plain[i].data(), (int)plain[i].size());
        batch->flush();  // on main's engine now
        rx->received(conn, junk.data() + 5, 35);
        rx->flush();
        uint64_t h = 0xcbf29ce484222325ull;
        bool ok = rx->status(conn) != 0;  // bad magic once the header is complete
        for (int i = 0; i < 8; i++) {
            h = fnv(h, out[i].data(), out[i].size());
            std::vector<uint8_t> back(out[i].size());
            pe->decrypt(back.data(), out[i].data(), (int)out[i].size());
            ok = ok && back == plain[i];
        }
        printf("migrate %016llx %d\n", (unsigned long long)h, ok ? 1 : 0);
        batch.reset();  // destroyed on main, after the first thread is gone
        rx.reset();
    }

    std::vector<std::thread> ths;
    for (int t = 0; t < nthreads; t++) ths.emplace_back(worker, t, frames);
    for (auto &th : ths) th.join();
    return 0;
}
