// TEST INFRASTRUCTURE ONLY -- drives the reference's own ECDH key exchange to produce the
// golden fixtures tests/golden/ecdh_cases.json; never part of the product.
//
// core/KeyExchange.cpp (ECCKeyExchange::init / calcKey, ECCKeysMaker::setCurve /
// publicKey / calcKey) and the vendored core/micro-ecc/uECC.c are compiled where they lie
// under /root/reference with their real dependencies (base/md5.c, base/sha256.c, FPLog,
// Setting, FileSystemUtil, ...; oracle/Makefile target `ecdh`).  The only hook is
// uECC_set_rng (micro-ecc's public API): the harness RNG hands out queued bytes first --
// so that uECC_make_key draws a chosen private key -- and a fixed xorshift stream after
// that (the random initial Z of uECC_shared_secret).
//
// stdin, one request per line (hex without spaces):
//   S <curve> <server_private> <peer_public> <keylen>   ECCKeyExchange::init + calcKey
//       -> "R <init_ok> <calc_ok> <key> <iv>"   (FPLog writes its records to stdout too)
//   T <curve> <server_private> <peer_public> <reps>     time `reps` calcKey calls (CPU baseline)
//       -> "R <seconds> <calc_ok>"
//   C <curve> <rng_bytes> <server_public> <keylen>      ECCKeysMaker: setCurve, publicKey
//       (private key drawn from rng_bytes), setPeerPublicKey, calcKey
//       -> "R <public> <private> <calc_ok> <key> <iv>"
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <iostream>
#include <string>
#include <vector>

#include "KeyExchange.h"
#include "Setting.h"

using namespace fpnn;

namespace {

std::vector<uint8_t> g_queue;
uint64_t g_state = 0x9E3779B97F4A7C15ull;

int harness_rng(uint8_t *dest, unsigned size) {
    for (unsigned i = 0; i < size; i++) {
        if (!g_queue.empty()) {
            dest[i] = g_queue.front();
            g_queue.erase(g_queue.begin());
        } else {
            g_state ^= g_state << 13;
            g_state ^= g_state >> 7;
            g_state ^= g_state << 17;
            dest[i] = (uint8_t)g_state;
        }
    }
    return 1;
}

std::string unhex(const std::string &h) {
    std::string o;
    if (h == "-") return o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return o;
}

std::string hex(const uint8_t *p, size_t n) {
    static const char *d = "0123456789abcdef";
    std::string o;
    for (size_t i = 0; i < n; i++) {
        o.push_back(d[p[i] >> 4]);
        o.push_back(d[p[i] & 15]);
    }
    return o.empty() ? "-" : o;
}

struct MakerProbe : ECCKeysMaker {
    const std::string &privateKey() const { return _privateKey; }
};

}  // namespace

int main() {
    Setting::set("FP.server.local.ip4", "127.0.0.1");  // see framing_ref.cpp
    uECC_set_rng(&harness_rng);
    std::string op, curve, a, b;
    int keylen;
    while (std::cin >> op >> curve >> a >> b >> keylen) {
        uint8_t key[32] = {0}, iv[16] = {0};
        if (op == "S") {
            ECCKeyExchange ex;
            const bool init_ok = ex.init(curve, unhex(a));
            const bool ok = init_ok && ex.calcKey(key, iv, keylen, unhex(b));
            printf("R %d %d %s %s\n", init_ok ? 1 : 0, ok ? 1 : 0, hex(key, ok ? keylen : 0).c_str(),
                   hex(iv, ok ? 16 : 0).c_str());
        } else if (op == "T") {
            ECCKeyExchange ex;
            ex.init(curve, unhex(a));
            const std::string peer = unhex(b);
            const auto t0 = std::chrono::steady_clock::now();
            bool ok = true;
            for (int r = 0; r < keylen; r++) ok = ex.calcKey(key, iv, 32, peer) && ok;
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            printf("R %.6f %d\n", dt, ok ? 1 : 0);
        } else if (op == "C") {
            const std::string q = unhex(a);
            g_queue.assign(q.begin(), q.end());
            MakerProbe m;
            if (!m.setCurve(curve)) {
                printf("R - - 0 - -\n");
                continue;
            }
            const std::string pub = m.publicKey();
            g_queue.clear();
            m.setPeerPublicKey(unhex(b));
            const bool ok = m.calcKey(key, iv, keylen);
            const std::string &priv = m.privateKey();
            printf("R %s %s %d %s %s\n", hex((const uint8_t *)pub.data(), pub.size()).c_str(),
                   hex((const uint8_t *)priv.data(), priv.size()).c_str(), ok ? 1 : 0,
                   hex(key, ok ? keylen : 0).c_str(), hex(iv, ok ? 16 : 0).c_str());
        } else {
            return 2;
        }
        fflush(stdout);
    }
    fflush(stdout);
    _exit(0);
}
