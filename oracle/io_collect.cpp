// TEST INFRASTRUCTURE ONLY -- see io_collect.h.  The product queue: fpnn::EncryptorBatch
// (include/EncryptorBatch.h), one GPU pass per (mode, direction, key length) per flush.
#include <stdlib.h>

#include <vector>

#include "EncryptorBatch.h"
#include "io_collect.h"

namespace fpnn_io {
namespace {
struct GpuQueue : Queue {
    fpnn::EncryptorBatch b;
    void encrypt(fpnn::Encryptor *enc, std::string *buffer) override { b.encrypt(enc, buffer); }
    void decrypt(fpnn::Encryptor *enc, uint8_t *dest, uint8_t *src, int len) override { b.decrypt(enc, dest, src, len); }
    size_t size() const override { return b.size(); }
    void flush() override { b.flush(); }
};
}  // namespace
Queue *make_queue() { return new GpuQueue(); }
}  // namespace fpnn_io

#include "io_collect_common.inc"
