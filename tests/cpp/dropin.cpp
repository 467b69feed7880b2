// dropin.cpp -- uses the MI355X library exactly the way FPNN's own code uses the
// reference classes (core/IOBuffer.cpp:36-45, core/EncryptedPackageReceiver.cpp:110,
// core/EncryptedStreamReceiver.cpp:89,124, base/test/rijndaelDemo.cpp), compiled
// against include/Encryptor.h + include/rijndael.h and linked with libfpnn_aes.so.
//
// stdin, one case per line:
//   P <key> <iv> <data>            -> "<encrypt> <decrypt> <frame>"
//   S <E|D> <key> <iv> <f1> .. <fn> -> "<out1> .. <outn>"      (StreamEncryptor)
//   R <key> <iv> <data>            -> "<roundtrip-memcmp> <cipher>" (rijndael.h API)
//   BP / BS ...                    as P / S, but queued on one fpnn::EncryptorBatch
//                                  (BS E: a frame "s<hex>" / "s-" is queued as encrypt(std::string*))
//   F                              flush the batch, then print the queued cases' lines
// hex fields, "-" for an empty buffer.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "Encryptor.h"
#include "EncryptorBatch.h"
#include "rijndael.h"

static std::vector<uint8_t> unhex(const std::string &h) {
    std::vector<uint8_t> v;
    if (h == "-") return v;
    for (size_t i = 0; i + 1 < h.size(); i += 2) v.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
    return v;
}

static std::string hex(const uint8_t *p, size_t n) {
    static const char *d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; i++) {
        s += d[p[i] >> 4];
        s += d[p[i] & 15];
    }
    return n ? s : "-";
}

// Cases queued on the batch: the encryptors and buffers live until the flush.
struct Queued {
    std::vector<std::unique_ptr<fpnn::Encryptor>> encs;
    std::vector<std::unique_ptr<std::vector<uint8_t>>> bufs;
    std::vector<std::unique_ptr<std::string>> strs;
    // per case: a list of (buffer, length) or string outputs, printed space-separated
    struct Out {
        std::vector<uint8_t> *buf;
        size_t n;
        std::string *str;
    };
    std::vector<std::vector<Out>> lines;
    std::vector<uint8_t> *keep(const std::vector<uint8_t> &v) {
        bufs.emplace_back(new std::vector<uint8_t>(v));
        bufs.back()->push_back(0);  // never empty: data() is a valid pointer
        return bufs.back().get();
    }
};

int main() {
    std::string line;
    fpnn::EncryptorBatch batch;
    Queued q;
    // connections that live across flushes (the batch's persistent key table)
    std::map<std::string, std::unique_ptr<fpnn::Encryptor>> named;
    std::map<std::string, bool> named_dir;
    while (std::getline(std::cin, line)) {
        std::istringstream is(line);
        std::string kind;
        is >> kind;
        if (kind == "BP") {  // PackageEncryptor calls through the batch
            std::string k, v, d;
            is >> k >> v >> d;
            auto key = unhex(k), iv = unhex(v), data = unhex(d);
            q.encs.emplace_back(new fpnn::PackageEncryptor(key.data(), key.size(), iv.data()));
            fpnn::Encryptor *enc = q.encs.back().get();
            std::vector<uint8_t> *src = q.keep(data), *a = q.keep(data), *b = q.keep(data);
            batch.encrypt(enc, a->data(), src->data(), (int)data.size());
            batch.decrypt(enc, b->data(), src->data(), (int)data.size());
            q.strs.emplace_back(new std::string((const char *)data.data(), data.size()));
            batch.encrypt(enc, q.strs.back().get());
            q.lines.push_back({{a, data.size(), nullptr}, {b, data.size(), nullptr}, {nullptr, 0, q.strs.back().get()}});
        } else if (kind == "BS") {  // StreamEncryptor calls through the batch
            std::string dir, k, v, f;
            is >> dir >> k >> v;
            auto key = unhex(k), iv = unhex(v);
            q.encs.emplace_back(new fpnn::StreamEncryptor(key.data(), key.size(), iv.data()));
            fpnn::Encryptor *enc = q.encs.back().get();
            std::vector<Queued::Out> outs;
            while (is >> f) {
                if (dir == "E" && f.compare(0, 1, "s") == 0) {  // s<hex> / s-: encrypt(std::string*) (SendBuffer's form)
                    auto data = unhex(f.substr(1));
                    q.strs.emplace_back(new std::string((const char *)data.data(), data.size()));
                    batch.encrypt(enc, q.strs.back().get());
                    outs.push_back({nullptr, 0, q.strs.back().get()});
                    continue;
                }
                auto data = unhex(f);
                std::vector<uint8_t> *src = q.keep(data), *o = q.keep(data);
                if (dir == "E")
                    batch.encrypt(enc, o->data(), src->data(), (int)data.size());
                else
                    batch.decrypt(enc, o->data(), src->data(), (int)data.size());
                outs.push_back({o, data.size(), nullptr});
            }
            q.lines.push_back(outs);
        } else if (kind == "NS" || kind == "NP") {  // NS <name> <E|D> <key> <iv> / NP <name> - <key> <iv>
            std::string name, dir, k, v;
            is >> name >> dir >> k >> v;
            auto key = unhex(k), iv = unhex(v);
            if (kind == "NS")
                named[name].reset(new fpnn::StreamEncryptor(key.data(), key.size(), iv.data()));
            else
                named[name].reset(new fpnn::PackageEncryptor(key.data(), key.size(), iv.data()));
            named_dir[name] = dir != "D";
        } else if (kind == "NF") {  // NF <name> <frame>...: queue frames on a named connection
            std::string name, f;
            is >> name;
            fpnn::Encryptor *enc = named.at(name).get();
            std::vector<Queued::Out> outs;
            while (is >> f) {
                auto data = unhex(f);
                std::vector<uint8_t> *src = q.keep(data), *o = q.keep(data);
                if (named_dir[name])
                    batch.encrypt(enc, o->data(), src->data(), (int)data.size());
                else
                    batch.decrypt(enc, o->data(), src->data(), (int)data.size());
                outs.push_back({o, data.size(), nullptr});
            }
            q.lines.push_back(outs);
        } else if (kind == "F") {
            batch.flush();
            for (const auto &l : q.lines) {
                std::string sep;
                for (const auto &o : l) {
                    std::cout << sep
                              << (o.str ? hex((const uint8_t *)o.str->data(), o.str->size()) : hex(o.buf->data(), o.n));
                    sep = " ";
                }
                std::cout << "\n";
            }
            q = Queued();
        } else if (kind == "P") {
            std::string k, v, d;
            is >> k >> v >> d;
            auto key = unhex(k), iv = unhex(v), data = unhex(d);
            fpnn::PackageEncryptor enc(key.data(), key.size(), iv.data());
            std::vector<uint8_t> a(data.size() + 1), b(data.size() + 1);
            enc.encrypt(a.data(), data.data(), (int)data.size());
            enc.decrypt(b.data(), data.data(), (int)data.size());
            std::string s((const char *)data.data(), data.size());
            fpnn::Encryptor *base = &enc;  // SendBuffer holds an Encryptor* (core/IOBuffer.h:117)
            base->encrypt(&s);
            std::cout << hex(a.data(), data.size()) << " " << hex(b.data(), data.size()) << " "
                      << hex((const uint8_t *)s.data(), s.size()) << "\n";
        } else if (kind == "S") {
            std::string dir, k, v, f;
            is >> dir >> k >> v;
            auto key = unhex(k), iv = unhex(v);
            fpnn::StreamEncryptor enc(key.data(), key.size(), iv.data());
            std::string sep;
            while (is >> f) {
                auto data = unhex(f);
                std::vector<uint8_t> o(data.size() + 1);
                if (dir == "E")
                    enc.encrypt(o.data(), data.data(), (int)data.size());
                else
                    enc.decrypt(o.data(), data.data(), (int)data.size());
                std::cout << sep << hex(o.data(), data.size());
                sep = " ";
            }
            std::cout << "\n";
        } else if (kind == "R") {
            std::string k, v, d;
            is >> k >> v >> d;
            auto key = unhex(k), iv = unhex(v), data = unhex(d);
            rijndael_context enCtx, deCtx;
            rijndael_setup_encrypt(&enCtx, key.data(), key.size());
            rijndael_setup_encrypt(&deCtx, key.data(), key.size());
            std::vector<uint8_t> iva(iv), ivb(iv), buf(data.size() + 1), buf2(data.size() + 1);
            size_t pos = 0;
            rijndael_cfb_encrypt(&enCtx, true, data.data(), buf.data(), data.size(), iva.data(), &pos);
            pos = 0;
            rijndael_cfb_encrypt(&deCtx, false, buf.data(), buf2.data(), data.size(), ivb.data(), &pos);
            std::cout << memcmp(data.data(), buf2.data(), data.size()) << " " << hex(buf.data(), data.size()) << "\n";
        }
    }
    return 0;
}
