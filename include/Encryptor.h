/*
 * Encryptor.h -- source-compatible replacement for the reference's core/Encryptor.h
 * (core/Encryptor.h:11-61).  Same namespace, class names, constructors, protected
 * members and virtual methods, so EncryptedPackageReceiver / EncryptedStreamReceiver
 * (which embed these by value, core/Receiver.h:104,145) and SendBuffer (which owns
 * one through new/delete, core/IOBuffer.cpp:262-266) compile unchanged against it.
 *
 * Every call runs the CFB cipher on the MI355X through the C-ABI in fpnn_aes.h
 * (per calling thread: one engine, one HIP stream, pinned staging).  Results are
 * byte-identical to the reference's.  There is no CPU fallback.  A GPU failure aborts the
 * process with a message (FPNN_AES_ON_ERROR=abort, the default: the reference's callers
 * cannot fail, and an exception escaping them would leave the connection wedged with its
 * token held); FPNN_AES_ON_ERROR=throw raises fpnn::EncryptorError instead, for callers
 * that catch it.
 *
 * For throughput, frames should be submitted in batches (fpnn_aes_package_* /
 * fpnn_aes_stream_* in fpnn_aes.h): one GPU round trip per 1 KiB frame costs more
 * than the frame's CPU cipher time (hard part 6).
 */
#ifndef FPNN_AMD_ENCRYPTOR_H
#define FPNN_AMD_ENCRYPTOR_H

#include <stdint.h>
#include <string.h>

#include <atomic>
#include <stdexcept>
#include <string>

#include "rijndael.h"

namespace fpnn {

class EncryptorBatch;       // EncryptorBatch.h: runs queued calls of many encryptors in one GPU pass
class StreamReceiverBatch;  // StreamReceiverBatch.h: the stream receive side of many connections per pass

/* libfpnn_aes.so: a process-unique number per constructed Encryptor -- the key of its
   slot in an EncryptorBatch's persistent device key table (an address can be reused by
   a later Encryptor, a serial cannot).  A copy gets a serial of its own (its state then
   evolves apart from the original's); a destroyed or overwritten Encryptor retires its
   serial, which frees its slot in every key table at that table's next flush. */
uint64_t encryptor_serial();
void encryptor_retire(uint64_t serial);

class EncryptorError : public std::runtime_error {
public:
    explicit EncryptorError(const std::string &what) : std::runtime_error(what) {}
};

class Encryptor {
    friend class EncryptorBatch;
    friend class StreamReceiverBatch;

protected:
    uint8_t _iv[16];
    uint8_t _key[32];
    size_t _keyLen;
    uint64_t _serial;
    // EncryptorBatch bookkeeping: the subclass (1 package, 2 stream; 0 other), and this
    // encryptor's slot in the key table of one generation (tag), so a flush finds a known
    // connection's slot without a lookup: tag << 24 | slot in ONE atomic word, so two
    // batches flushing the same PackageEncryptor on two threads can never pair one table's
    // tag with the other's slot (0: none); _batchSeen = the last flush that listed it
    // (stream state hand-off; a StreamEncryptor belongs to one thread at a time anyway)
    uint8_t _kind = 0;
    std::atomic<uint64_t> _batchCache{0};
    uint64_t _batchSeen = 0;

public:
    Encryptor(uint8_t *key, size_t key_len, uint8_t *iv) {
        memcpy(_key, key, key_len);
        memcpy(_iv, iv, 16);
        _keyLen = key_len;
        _serial = encryptor_serial();
    }
    Encryptor(const Encryptor &o) : _keyLen(o._keyLen), _serial(encryptor_serial()), _kind(o._kind) {
        memcpy(_iv, o._iv, 16);
        memcpy(_key, o._key, sizeof _key);
    }
    Encryptor &operator=(const Encryptor &o) {
        if (this != &o) {
            memcpy(_iv, o._iv, 16);
            memcpy(_key, o._key, sizeof _key);
            _keyLen = o._keyLen;
            encryptor_retire(_serial);
            _serial = encryptor_serial();
            _batchCache.store(0, std::memory_order_relaxed);  // a new serial: no table slot yet
            _batchSeen = 0;
        }
        return *this;
    }
    virtual ~Encryptor() { encryptor_retire(_serial); }

    virtual void decrypt(uint8_t *dest, uint8_t *src, int len) = 0;
    virtual void encrypt(uint8_t *dest, uint8_t *src, int len) = 0;
    virtual void encrypt(std::string *buffer) = 0;
};

/* One fresh CFB chain per call from the connection IV (core/Encryptor.cpp:10-51). */
class PackageEncryptor : public Encryptor {
    friend class EncryptorBatch;
    rijndael_context _ctx;  // expanded once; the reference re-expands per call (same result)

public:
    PackageEncryptor(uint8_t *key, size_t key_len, uint8_t *iv) : Encryptor(key, key_len, iv) {
        rijndael_setup_encrypt(&_ctx, (const uint8_t *)_key, key_len);
        _kind = 1;
    }
    virtual ~PackageEncryptor() {}

    virtual void decrypt(uint8_t *dest, uint8_t *src, int len);
    virtual void encrypt(uint8_t *dest, uint8_t *src, int len);
    /* buffer := htole32(len) || CFB(buffer) */
    virtual void encrypt(std::string *buffer);
};

/* One CFB chain per connection direction, state (_iv, _pos) carried across calls
 * (core/Encryptor.cpp:53-70). */
class StreamEncryptor : public Encryptor {
    friend class EncryptorBatch;
    friend class StreamReceiverBatch;
    rijndael_context _ctx;
    size_t _pos;

public:
    StreamEncryptor(uint8_t *key, size_t key_len, uint8_t *iv) : Encryptor(key, key_len, iv), _pos(0) {
        rijndael_setup_encrypt(&_ctx, (const uint8_t *)_key, key_len);
        _kind = 2;
    }
    virtual ~StreamEncryptor() {}

    virtual void decrypt(uint8_t *dest, uint8_t *src, int len);
    virtual void encrypt(uint8_t *dest, uint8_t *src, int len);
    virtual void encrypt(std::string *buffer);

    /* state export/import (the only stream-mode state) */
    const uint8_t *iv() const { return _iv; }
    size_t pos() const { return _pos; }
};

}  // namespace fpnn

#endif
