// stream_recv.cpp -- an EncryptedStreamReceiver-shaped IO loop (core/EncryptedStreamReceiver.cpp:72-163)
// over fpnn::StreamReceiverBatch: every connection's wire bytes arrive in pieces of a fixed
// size, one piece per connection per cycle; each cycle ends with one flush() for all
// connections.  Input (stdin), one connection per line:
//   <max_len> <key hex> <iv hex> <wire hex>
// argv[1] = piece size.  Output, one line per connection, in input order:
//   <status> <pending> <iv hex> <pos> <bytes fed> <message hex>...   (message = header + body plaintext)
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "Encryptor.h"
#include "StreamReceiverBatch.h"

namespace {

std::string unhex(const std::string &h) {
    std::string out(h.size() / 2, '\0');
    for (size_t i = 0; i < out.size(); i++) out[i] = (char)strtol(h.substr(2 * i, 2).c_str(), nullptr, 16);
    return out;
}

std::string hex(const std::string &b) {
    static const char *d = "0123456789abcdef";
    std::string s;
    for (unsigned char c : b) {
        s += d[c >> 4];
        s += d[c & 15];
    }
    return s;
}

struct Conn {
    uint32_t max_len = 0;
    std::string wire;
    std::unique_ptr<fpnn::StreamEncryptor> enc;
    fpnn::StreamReceiverBatch *rx = nullptr;
    int id = -1;
    size_t fed = 0;
    std::vector<std::string> msgs;
};

}  // namespace

int main(int argc, char **argv) {
    const size_t piece = argc > 1 ? (size_t)atol(argv[1]) : 7;
    std::vector<Conn> conns;
    std::string line;
    while (std::getline(std::cin, line)) {
        if (line.empty()) continue;
        std::istringstream ss(line);
        std::string key, iv, wire;
        Conn c;
        ss >> c.max_len >> key >> iv >> wire;
        if (wire == "-") wire.clear();
        std::string k = unhex(key), v = unhex(iv);
        c.wire = unhex(wire);
        c.enc.reset(new fpnn::StreamEncryptor((uint8_t *)&k[0], k.size(), (uint8_t *)&v[0]));
        conns.push_back(std::move(c));
    }
    // Config::_max_recv_package_length is process-wide: one batch per value in the input
    std::map<uint32_t, std::unique_ptr<fpnn::StreamReceiverBatch>> batches;
    for (Conn &c : conns) {
        auto &b = batches[c.max_len];
        if (!b) b.reset(new fpnn::StreamReceiverBatch(c.max_len, 4));  // 4: exercise max_frames passes
        c.rx = b.get();
        c.id = b->open(c.enc.get());
    }
    try {
        for (bool more = true; more;) {
            more = false;
            for (Conn &c : conns) {  // one read per readable connection
                if (c.fed >= c.wire.size() || c.rx->status(c.id) != 0) continue;
                const size_t n = std::min(piece, c.wire.size() - c.fed);
                c.rx->received(c.id, (const uint8_t *)c.wire.data() + c.fed, n);
                c.fed += n;
                more = true;
            }
            for (auto &b : batches) b.second->flush();
            for (Conn &c : conns)
                for (const std::string &m : c.rx->messages(c.id)) c.msgs.push_back(m);
        }
    } catch (const fpnn::EncryptorError &e) {
        fprintf(stderr, "EncryptorError: %s\n", e.what());
        return 2;
    }
    for (Conn &c : conns) {
        std::string iv((const char *)c.enc->iv(), 16);
        std::cout << c.rx->status(c.id) << " " << c.rx->pending(c.id) << " " << hex(iv) << " " << c.enc->pos() << " "
                  << c.fed;
        for (const std::string &m : c.msgs) std::cout << " " << hex(m);
        std::cout << "\n";
    }
    return 0;
}
