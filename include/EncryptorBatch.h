/*
 * EncryptorBatch.h -- cross-connection batch collector for the Encryptor classes
 * (SURVEY.md section 8f, row 1).
 *
 * FPNN encrypts one frame per call: SendBuffer::encryptData (core/IOBuffer.cpp:36-45)
 * per dequeued std::string, EncryptedPackageReceiver::fetch (core/EncryptedPackageReceiver.cpp:110)
 * and EncryptedStreamReceiver (core/EncryptedStreamReceiver.cpp:89,124) per received
 * frame.  On the GPU one round trip per 1 KiB frame costs more than the frame's CPU
 * cipher, so an IO loop queues the frames of all its connections for one epoll cycle
 * here and runs them in one pass (fpnn_aes_package_host / fpnn_aes_stream_host: a
 * parallel gather into pinned staging, pipelined H2D / kernel / D2H, scatter back).
 *
 * Semantics: after flush(), every queued call has had exactly the effect of calling
 * the same method on the same Encryptor at that point, in queue order per Encryptor
 * (the buffers must stay valid and untouched until flush returns).  A StreamEncryptor
 * carries state, so within one batch it must be used in a single direction (FPNN
 * gives each connection direction its own encryptor, core/IOBuffer.cpp:20-22,264-266).
 * Errors throw fpnn::EncryptorError; there is no CPU fallback.
 */
#ifndef FPNN_AMD_ENCRYPTOR_BATCH_H
#define FPNN_AMD_ENCRYPTOR_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "Encryptor.h"

namespace fpnn {

class EncryptorBatch {
public:
    EncryptorBatch() {}
    ~EncryptorBatch();
    EncryptorBatch(const EncryptorBatch &) = delete;
    EncryptorBatch &operator=(const EncryptorBatch &) = delete;

    /* enc->encrypt(buffer): package mode -> htole32(len) || ciphertext, stream mode ->
       ciphertext of the same length (core/Encryptor.cpp:34-51, 63-70). */
    void encrypt(Encryptor *enc, std::string *buffer);
    /* enc->encrypt(dest, src, len) / enc->decrypt(dest, src, len) */
    void encrypt(Encryptor *enc, uint8_t *dest, uint8_t *src, int len);
    void decrypt(Encryptor *enc, uint8_t *dest, uint8_t *src, int len);

    size_t size() const { return _ops.size(); }
    size_t bytes() const { return _bytes; }
    /* Run every queued call (one GPU pass per mode/direction/key length group); the
       batch is empty afterwards, also when it throws. */
    void flush();
    void clear() {
        _ops.clear();
        _bytes = 0;
    }

private:
    struct Op {
        Encryptor *enc;
        uint8_t *dest;
        const uint8_t *src;
        uint32_t len;
        bool encrypt;
        std::string *buffer;  // non-null: the std::string* form
    };
    std::vector<Op> _ops;
    size_t _bytes = 0;
    // Persistent device key tables, one per key length (AES-128/192/256): a slot per
    // Encryptor seen, uploaded once; a flush only adds its new connections.
    struct KeyTable;
    KeyTable *_tables[3] = {nullptr, nullptr, nullptr};
    void add(Encryptor *enc, bool encrypt, uint8_t *dest, const uint8_t *src, int len, std::string *buffer);
};

}  // namespace fpnn

#endif
