// TEST INFRASTRUCTURE ONLY -- see io_collect.h.  A CPU stand-in for the collector, built
// against the REFERENCE's core/Encryptor.h: a flush runs the queued calls on the reference
// Encryptor in queue order.  io_multi_cpucollect (oracle/Makefile) uses it to check, on any
// machine, that the patched IO plumbing (collect_patch.py) defers and orders every cipher
// call correctly -- its wire bytes must equal the unpatched reference build's.
#include <stdlib.h>

#include <functional>
#include <vector>

#include "Encryptor.h"
#include "io_collect.h"

namespace fpnn_io {
namespace {
struct CpuQueue : Queue {
    std::vector<std::function<void()>> ops;
    void encrypt(fpnn::Encryptor *enc, std::string *buffer) override {
        ops.push_back([=]() { enc->encrypt(buffer); });
    }
    void decrypt(fpnn::Encryptor *enc, uint8_t *dest, uint8_t *src, int len) override {
        ops.push_back([=]() { enc->decrypt(dest, src, len); });
    }
    size_t size() const override { return ops.size(); }
    void flush() override {
        for (auto &f : ops) f();
        ops.clear();
    }
};
}  // namespace
Queue *make_queue() { return new CpuQueue(); }
}  // namespace fpnn_io

#include "io_collect_common.inc"
