// TEST INFRASTRUCTURE ONLY -- SURVEY.md section 8f rows 2 and 4 through the reference's own
// UDP caller: core/UDP.v2/UDPCommon.v2.cpp, compiled unchanged, drives
// the cipher and the key exchange the way FPNN's reliable-UDP stack does:
//   server  UDPEncryptor::createPair(keyExchanger, clientPublicKey, reinforce)   :127-144
//           UDPEncryptor::createPair(kx, packagePublicKey, reinforcePackage,
//                                    dataPublicKey, reinforceData)               :146-172
//           (the ECDH of core/KeyExchange.cpp:87-127 on the accepted client's keys,
//            as core/UDP.v2/UDPParser.v2.cpp:953-993 calls it)
//   client  ECCKeyExchange::calcKey on the server's public key, then
//           UDPEncryptor::configPackageEncryptor / configDataEncryptor           :174-187
//           (core/UDP.v2/UDPIOBuffer.v2.cpp:153-156, 231-236), one UDPEncryptor to send
//           and one to parse, as the IO buffer and its ARQParser each hold one
//   traffic packageEncrypt -> packageDecrypt per datagram (UDPIOBuffer.v2.cpp:351,
//           UDPParser.v2.cpp:91), dataEncrypt -> dataDecrypt per data segment in order
//           (UDPAssembler.v2.cpp:578,622,701, UDPParser.v2.cpp:702,773,827), both ways.
//
// One source, two builds (oracle/Makefile `udp`):
//   _ref/udp_v2_ref     UDPCommon.v2.cpp + core/KeyExchange.cpp + core/Encryptor.cpp +
//                       base/rijndael.c, all where they lie (the CPU reference);
//   _ref/udp_v2_dropin  UDPCommon.v2.cpp compiled unchanged through a header overlay whose
//                       core/Encryptor.h, core/KeyExchange.h and base/rijndael.h are this
//                       repo's include/ headers, linked with fpnn_amd/libfpnn_aes.so (the
//                       cipher and the ECDH on the GPU).
// stdin, one case per line:
//   <curve> <server_priv> <server_pub> <c1_priv> <c1_pub> <c2_priv> <c2_pub>
//   <reinforce_pkg 0|1> <reinforce_data 0|1> <datagrams> <seed>
// (hex keys as tests/golden/ecdh_cases.json holds them).  Per case one JSON line: FNV-1a
// digests of every ciphertext byte per channel and direction, whether every decrypt gave
// back its plaintext, and whether createPair refused a malformed public key -- the two
// builds must print the same digests.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <iostream>
#include <string>
#include <vector>

#include "KeyExchange.h"
#include "UDP.v2/UDPCommon.v2.h"

using namespace fpnn;

namespace {

std::string unhex(const std::string &h) {
    std::string o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return o;
}

struct Rng {
    uint64_t s;
    uint64_t next() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    }
};

struct Digest {
    uint64_t h = 0xcbf29ce484222325ull, n = 0;
    void add(const uint8_t *p, size_t len) {
        for (size_t i = 0; i < len; i++) h = (h ^ p[i]) * 0x100000001b3ull;
        n += len;
    }
};

// one end's two UDPEncryptors (sending, parsing), configured the client's way
struct ClientEnd {
    UDPEncryptor send, parse;
    bool ok = true;
    void config(const std::string &curve, const std::string &priv, const std::string &serverPub, bool reinforcePkg,
                const std::string *dataPriv, bool reinforceData) {
        uint8_t key[32], iv[16];
        ECCKeyExchange kx;
        ok = ok && kx.init(curve, priv);
        const int kl = reinforcePkg ? 32 : 16;
        ok = ok && kx.calcKey(key, iv, kl, serverPub);
        send.configPackageEncryptor(key, kl, iv);
        parse.configPackageEncryptor(key, kl, iv);
        if (dataPriv) {
            ECCKeyExchange dk;
            ok = ok && dk.init(curve, *dataPriv);
            const int dl = reinforceData ? 32 : 16;
            ok = ok && dk.calcKey(key, iv, dl, serverPub);
            send.configDataEncryptor(key, dl, iv);
            parse.configDataEncryptor(key, dl, iv);
        }
    }
};

// datagrams both ways through one (server pair, client end); `data` adds a data-segment
// stream both ways (segments of one message split across datagrams)
void traffic(UDPEncryptor *sSend, UDPEncryptor *sRecv, ClientEnd &c, bool data, int datagrams, Rng &rng,
             Digest &pkgS2C, Digest &pkgC2S, Digest &dataS2C, Digest &dataC2S, bool &rt_ok) {
    std::vector<uint8_t> plain(1472), enc(1472), dec(1472);
    for (int i = 0; i < datagrams; i++) {
        // MTU-sized datagrams mostly (UDPIOBuffer.v2.h:14), short ones (acks, heartbeats)
        // in between
        const uint64_t r = rng.next();
        const int len = (r & 3) ? 1472 - (int)((r >> 8) % 64) : 1 + (int)((r >> 8) % 96);
        for (int k = 0; k < len; k++) plain[k] = (uint8_t)rng.next();
        for (int dir = 0; dir < 2; dir++) {
            UDPEncryptor *tx = dir ? &c.send : sSend, *rx = dir ? sRecv : &c.parse;
            Digest &dg = dir ? pkgC2S : pkgS2C;
            tx->packageEncrypt(enc.data(), plain.data(), len);
            dg.add(enc.data(), len);
            rx->packageDecrypt(dec.data(), enc.data(), len);
            rt_ok = rt_ok && memcmp(dec.data(), plain.data(), len) == 0;
            if (data) {
                // a data section inside the datagram: one segment of the stream
                const int seg = (int)(rng.next() % (uint64_t)len) + 1;
                Digest &dd = dir ? dataC2S : dataS2C;
                tx->dataEncrypt(enc.data(), plain.data(), seg);
                dd.add(enc.data(), seg);
                rx->dataDecrypt(dec.data(), enc.data(), seg);
                rt_ok = rt_ok && memcmp(dec.data(), plain.data(), seg) == 0;
            }
        }
    }
}

}  // namespace

int main() {
    std::string curve, sPriv, sPub, c1Priv, c1Pub, c2Priv, c2Pub;
    int rPkg, rData, datagrams;
    unsigned long long seed;
    while (std::cin >> curve >> sPriv >> sPub >> c1Priv >> c1Pub >> c2Priv >> c2Pub >> rPkg >> rData >> datagrams >>
           seed) {
        const auto t0 = std::chrono::steady_clock::now();
        ECCKeyExchange server;
        const bool init_ok = server.init(curve, unhex(sPriv));
        Rng rng{seed | 1};
        Digest pS2C, pC2S, dS2C, dC2S, qS2C, qC2S, eS2C, eC2S;
        bool rt_ok = true;

        // package-only session (createPair, 3 arguments)
        UDPEncryptor::EncryptorPair a = UDPEncryptor::createPair(&server, unhex(c1Pub), rPkg != 0);
        ClientEnd ca;
        ca.config(curve, unhex(c1Priv), unhex(sPub), rPkg != 0, nullptr, false);
        const bool pair_a = a.sender && a.receiver;
        if (pair_a) traffic(a.sender, a.receiver, ca, false, datagrams, rng, pS2C, pC2S, eS2C, eC2S, rt_ok);

        // package + reinforced data session (createPair, 5 arguments)
        UDPEncryptor::EncryptorPair b =
            UDPEncryptor::createPair(&server, unhex(c1Pub), rPkg != 0, unhex(c2Pub), rData != 0);
        ClientEnd cb;
        const std::string c2 = unhex(c2Priv);
        cb.config(curve, unhex(c1Priv), unhex(sPub), rPkg != 0, &c2, rData != 0);
        const bool pair_b = b.sender && b.receiver;
        if (pair_b) traffic(b.sender, b.receiver, cb, true, datagrams, rng, qS2C, qC2S, dS2C, dC2S, rt_ok);

        // a malformed public key: createPair returns an empty pair
        UDPEncryptor::EncryptorPair bad = UDPEncryptor::createPair(&server, std::string("\x04short", 6), false);
        const bool bad_refused = bad.sender == nullptr && bad.receiver == nullptr;
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"curve\": \"%s\", \"init_ok\": %d, \"pair_a\": %d, \"pair_b\": %d, \"client_ok\": %d, "
               "\"roundtrip_ok\": %d, \"bad_key_refused\": %d, "
               "\"a_pkg_s2c\": \"%016llx\", \"a_pkg_c2s\": \"%016llx\", \"b_pkg_s2c\": \"%016llx\", "
               "\"b_pkg_c2s\": \"%016llx\", \"b_data_s2c\": \"%016llx\", \"b_data_c2s\": \"%016llx\", "
               "\"bytes\": %llu, \"seconds\": %.6f}\n",
               curve.c_str(), init_ok, pair_a, pair_b, ca.ok && cb.ok, rt_ok, bad_refused,
               (unsigned long long)pS2C.h, (unsigned long long)pC2S.h, (unsigned long long)qS2C.h,
               (unsigned long long)qC2S.h, (unsigned long long)dS2C.h, (unsigned long long)dC2S.h,
               (unsigned long long)(pS2C.n + pC2S.n + qS2C.n + qC2S.n + dS2C.n + dC2S.n), secs);
        fflush(stdout);
        delete a.sender;
        delete a.receiver;
        delete b.sender;
        delete b.receiver;
    }
    return 0;
}
