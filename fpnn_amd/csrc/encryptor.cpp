// encryptor.cpp -- fpnn::PackageEncryptor / StreamEncryptor and the rijndael.h
// subset, implemented over the C-ABI (fpnn_aes.h).  Mirrors core/Encryptor.cpp:10-70
// call for call; the CFB work itself runs in the HIP kernels.
#include <endian.h>
#include <stdio.h>
#include <stdlib.h>

#include <memory>
#include <string>

#include "../../include/Encryptor.h"
#include "../../include/fpnn_aes.h"

namespace {

// One engine (HIP stream + pinned staging) per calling thread: an Encryptor is used
// by one thread at a time (core/IOBuffer.h:49-62, core/IOBuffer.cpp:219-245), and
// may migrate between IO and worker threads, which then use their own engines.
struct ThreadEngine {
    fpnn_aes_engine *e = nullptr;
    int status = FPNN_AES_OK;
    ThreadEngine() {
        const char *dev = getenv("FPNN_AES_DEVICE");
        status = fpnn_aes_engine_create(dev ? atoi(dev) : 0, FPNN_AES_OWN_STREAM, &e);
    }
    ~ThreadEngine() { fpnn_aes_engine_destroy(e); }
};

fpnn_aes_engine *thread_engine(int *status) {
    thread_local ThreadEngine te;
    *status = te.status;
    return te.e;
}

std::string describe(int rc) {
    std::string s = fpnn_aes_strerror(rc);
    const char *d = fpnn_aes_last_error();
    if (d && *d) s += std::string(": ") + d;
    return s;
}

int cfb(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16],
        size_t *p_num) {
    int rc;
    fpnn_aes_engine *e = thread_engine(&rc);
    if (!e) return rc ? rc : FPNN_AES_ERR_NODEV;
    static_assert(sizeof(rijndael_context) == sizeof(fpnn_aes_schedule), "context layout");
    return fpnn_aes_cfb_host(e, reinterpret_cast<const fpnn_aes_schedule *>(ctx), encrypt ? 1 : 0, in, out, len, ivec,
                             p_num);
}

void cfb_or_throw(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                  uint8_t ivec[16], size_t *p_num) {
    const int rc = cfb(ctx, encrypt, in, out, len, ivec, p_num);
    if (rc != FPNN_AES_OK) throw fpnn::EncryptorError("fpnn_aes GPU CFB failed: " + describe(rc));
}

}  // namespace

extern "C" {

bool rijndael_setup_encrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen) {
    return fpnn_aes_setup_encrypt(reinterpret_cast<fpnn_aes_schedule *>(ctx), key, keylen) == FPNN_AES_OK;
}

void rijndael_cfb_encrypt(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                          uint8_t ivec[16], size_t *p_num) {
    const int rc = cfb(ctx, encrypt, in, out, len, ivec, p_num);
    if (rc != FPNN_AES_OK) {
        fprintf(stderr, "rijndael_cfb_encrypt (fpnn_aes, MI355X): %s\n", describe(rc).c_str());
        abort();  // the reference has no error path; never fall back to a CPU cipher
    }
}

}  // extern "C"

namespace fpnn {

void PackageEncryptor::decrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:10-20
    if (len <= 0) return;
    uint8_t iv[16];
    memcpy(iv, _iv, 16);
    size_t pos = 0;
    cfb_or_throw(&_ctx, false, src, dest, (size_t)len, iv, &pos);
}

void PackageEncryptor::encrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:22-32
    if (len <= 0) return;
    uint8_t iv[16];
    memcpy(iv, _iv, 16);
    size_t pos = 0;
    cfb_or_throw(&_ctx, true, src, dest, (size_t)len, iv, &pos);
}

void PackageEncryptor::encrypt(std::string *buffer) {  // core/Encryptor.cpp:34-51
    const size_t n = buffer->length();
    std::string framed(n + sizeof(uint32_t), '\0');
    const uint32_t le = htole32((uint32_t)n);
    memcpy(&framed[0], &le, sizeof le);
    if (n) {
        uint8_t iv[16];
        memcpy(iv, _iv, 16);
        size_t pos = 0;
        cfb_or_throw(&_ctx, true, reinterpret_cast<const uint8_t *>(buffer->data()),
                     reinterpret_cast<uint8_t *>(&framed[sizeof(uint32_t)]), n, iv, &pos);
    }
    buffer->swap(framed);
}

void StreamEncryptor::decrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:53-56
    if (len <= 0) return;
    cfb_or_throw(&_ctx, false, src, dest, (size_t)len, _iv, &_pos);
}

void StreamEncryptor::encrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:58-61
    if (len <= 0) return;
    cfb_or_throw(&_ctx, true, src, dest, (size_t)len, _iv, &_pos);
}

void StreamEncryptor::encrypt(std::string *buffer) {  // core/Encryptor.cpp:63-70
    const size_t n = buffer->length();
    if (!n) return;
    std::string out(n, '\0');
    cfb_or_throw(&_ctx, true, reinterpret_cast<const uint8_t *>(buffer->data()), reinterpret_cast<uint8_t *>(&out[0]),
                 n, _iv, &_pos);
    buffer->swap(out);
}

}  // namespace fpnn
