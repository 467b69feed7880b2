// Drop-in check for include/KeyExchange.h: the reference's ECCKeyExchange / ECCKeysMaker
// call sequence (core/TCPEpollServer.h:375-383 server, core/TCPClient.cpp:225-236 client)
// against libfpnn_aes.so alone.  Driven by tests/test_gpu_ecdh.py::test_cpp_keyexchange_dropin.
//   S <curve> <private hex> <peer hex> <keylen>  -> "<init_ok> <ok> <key hex> <iv hex>"
//   R <curve> - - <keylen>                       -> "roundtrip <1|0>"
#include <stdio.h>
#include <string.h>

#include <iostream>
#include <string>

#include "KeyExchange.h"

static std::string unhex(const std::string &h) {
    std::string o;
    if (h == "-") return o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return o;
}

static std::string hex(const uint8_t *p, size_t n) {
    static const char *d = "0123456789abcdef";
    std::string o;
    for (size_t i = 0; i < n; i++) {
        o.push_back(d[p[i] >> 4]);
        o.push_back(d[p[i] & 15]);
    }
    return o.empty() ? "-" : o;
}

int main() {
    std::string op, curve, a, b;
    int keylen;
    while (std::cin >> op >> curve >> a >> b >> keylen) {
        if (op == "S") {
            fpnn::ECCKeyExchange ex;
            uint8_t key[32], iv[16];
            const bool init_ok = ex.init(curve, unhex(a));
            const bool ok = ex.calcKey(key, iv, keylen, unhex(b));
            printf("%d %d %s %s\n", init_ok ? 1 : 0, ok ? 1 : 0, hex(key, ok ? keylen : 0).c_str(),
                   hex(iv, ok ? 16 : 0).c_str());
        } else {
            fpnn::ECCKeysMaker client, server;
            if (!client.setCurve(curve) || !server.setCurve(curve)) return 3;
            const std::string cpub = client.publicKey(), spub = server.publicKey();
            client.setPeerPublicKey(spub);
            server.setPeerPublicKey(cpub);
            uint8_t k1[32], v1[16], k2[32], v2[16], k3[32], v3[16], ok3 = 0;
            const bool ok1 = client.calcKey(k1, v1, keylen);
            const bool ok2 = server.calcKey(k2, v2, keylen);
            const bool ok4 = server.calcKeys(1, reinterpret_cast<const uint8_t *>(cpub.data()), keylen, k3, v3, &ok3);
            const bool same = ok1 && ok2 && ok4 && ok3 && !cpub.empty() && cpub != spub &&
                              memcmp(k1, k2, keylen) == 0 && memcmp(v1, v2, 16) == 0 &&
                              memcmp(k1, k3, keylen) == 0 && memcmp(v1, v3, 16) == 0;
            printf("roundtrip %d\n", same ? 1 : 0);
        }
        fflush(stdout);
    }
    return 0;
}
