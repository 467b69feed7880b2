// TEST INFRASTRUCTURE ONLY -- the collector hooks that oracle/collect_patch.py puts at the
// reference's two per-frame cipher call sites when it builds the patched scratch copy of
// FPNN's IO plumbing under oracle/_ref/co/ (applied):
//   SendBuffer::encryptData          core/IOBuffer.cpp:36-45   _encryptor->encrypt(_currBuffer)
//   EncryptedPackageReceiver::fetch  core/EncryptedPackageReceiver.cpp:110   _encryptor.decrypt(...)
// While an IO thread runs a collect phase (active() != nullptr) the calls are queued in that
// thread's Queue and take effect at its flush(); otherwise they run at once, exactly as the
// unpatched call would.  The product queue is fpnn::EncryptorBatch (include/EncryptorBatch.h,
// io_collect.cpp); io_collect_cpu.cpp is a CPU stand-in over the reference's own Encryptor
// that checks the patched call order on any machine (tests/test_oracle.py).
#ifndef FPNN_AMD_IO_COLLECT_H
#define FPNN_AMD_IO_COLLECT_H

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace fpnn {
class Encryptor;
}  // namespace fpnn

namespace fpnn_io {

struct Queue {
    virtual ~Queue() {}
    virtual void encrypt(fpnn::Encryptor *enc, std::string *buffer) = 0;
    virtual void decrypt(fpnn::Encryptor *enc, uint8_t *dest, uint8_t *src, int len) = 0;
    virtual size_t size() const = 0;
    virtual void flush() = 0;
};
Queue *make_queue();  // this build's queue (io_collect.cpp / io_collect_cpu.cpp)

// the calling thread's queue during a collect phase, else nullptr
Queue *&active();

// RAII: a collect phase on this thread
struct Collect {
    Queue *prev;
    explicit Collect(Queue *q) : prev(active()) { active() = q; }
    ~Collect() { active() = prev; }
};

void encrypt(fpnn::Encryptor *enc, std::string *buffer);
void decrypt(fpnn::Encryptor *enc, uint8_t *dest, uint8_t *src, int len);
// free() of a buffer a queued call still reads (fetch frees the received ciphertext right
// after its decrypt call, core/EncryptedPackageReceiver.cpp:112): deferred to
// release_deferred(), which the IO loop calls after the flush; immediate outside a phase
void release(void *p);
void release_deferred();

}  // namespace fpnn_io

#endif
