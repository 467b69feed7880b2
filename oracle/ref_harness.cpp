/*
 * ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * C-linkage harness around the *reference's own* AES path, compiled by
 * oracle/Makefile together with /root/reference/base/rijndael.c and
 * /root/reference/core/Encryptor.cpp (nothing from the reference is copied
 * into this repository).  The resulting oracle/_ref/libfpnn_ref.so is used:
 *   - here, by oracle/gen_golden.py, to produce tests/golden/ fixtures and the
 *     full-size config digests;
 *   - on the GPU box (the .so travels with the snapshot, the sources do not),
 *     by bench.py's cpu_baseline leg (kind "reference") and by tests that find it.
 */
#include <stdint.h>
#include <string.h>
#include <string>
#include <thread>
#include <vector>
#include <chrono>

#include "rijndael.h"  /* /root/reference/base/rijndael.h */
#include "Encryptor.h" /* /root/reference/core/Encryptor.h */

using fpnn::PackageEncryptor;
using fpnn::StreamEncryptor;

extern "C" {

int ref_setup_encrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen)
{
    return rijndael_setup_encrypt(ctx, key, keylen) ? 1 : 0;
}

void ref_encrypt_block(const rijndael_context *ctx, const uint8_t *in, uint8_t *out)
{
    rijndael_encrypt(ctx, in, out);
}

int ref_setup_decrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen)
{
    return rijndael_setup_decrypt(ctx, key, keylen) ? 1 : 0;
}

void ref_decrypt_block(const rijndael_context *ctx, const uint8_t *in, uint8_t *out)
{
    rijndael_decrypt(ctx, in, out);
}

void ref_cbc(const rijndael_context *ctx, int encrypt, const uint8_t *in, uint8_t *out, size_t len, uint8_t *ivec)
{
    if (encrypt)
        rijndael_cbc_encrypt(ctx, in, out, len, ivec);
    else
        rijndael_cbc_decrypt(ctx, in, out, len, ivec);
}

void ref_ofb(const rijndael_context *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t *ivec, size_t *num)
{
    rijndael_ofb_encrypt(ctx, in, out, len, ivec, num);
}

void ref_cfb(const rijndael_context *ctx, int encrypt, const uint8_t *in, uint8_t *out, size_t len,
             uint8_t *ivec, size_t *num)
{
    rijndael_cfb_encrypt(ctx, encrypt != 0, in, out, len, ivec, num);
}

/* PackageEncryptor::encrypt / decrypt (dest, src, len) */
void ref_package_crypt(const uint8_t *key, size_t keylen, const uint8_t *iv, int encrypt,
                       const uint8_t *src, uint8_t *dst, size_t len)
{
    PackageEncryptor e(const_cast<uint8_t *>(key), keylen, const_cast<uint8_t *>(iv));
    if (encrypt)
        e.encrypt(dst, const_cast<uint8_t *>(src), (int)len);
    else
        e.decrypt(dst, const_cast<uint8_t *>(src), (int)len);
}

/* PackageEncryptor::encrypt(std::string*) -- wire frame with the LE length prefix */
size_t ref_package_encrypt_frame(const uint8_t *key, size_t keylen, const uint8_t *iv,
                                 const uint8_t *src, size_t len, uint8_t *dst)
{
    PackageEncryptor e(const_cast<uint8_t *>(key), keylen, const_cast<uint8_t *>(iv));
    std::string s((const char *)src, len);
    e.encrypt(&s);
    memcpy(dst, s.data(), s.size());
    return s.size();
}

void *ref_stream_new(const uint8_t *key, size_t keylen, const uint8_t *iv)
{
    return new StreamEncryptor(const_cast<uint8_t *>(key), keylen, const_cast<uint8_t *>(iv));
}

void ref_stream_crypt(void *h, int encrypt, const uint8_t *src, uint8_t *dst, size_t len)
{
    StreamEncryptor *e = static_cast<StreamEncryptor *>(h);
    if (encrypt)
        e->encrypt(dst, const_cast<uint8_t *>(src), (int)len);
    else
        e->decrypt(dst, const_cast<uint8_t *>(src), (int)len);
}

/* StreamEncryptor::encrypt(std::string*) -- no prefix, state carried */
void ref_stream_encrypt_string(void *h, const uint8_t *src, size_t len, uint8_t *dst)
{
    std::string s((const char *)src, len);
    static_cast<StreamEncryptor *>(h)->encrypt(&s);
    memcpy(dst, s.data(), s.size());
}

void ref_stream_free(void *h) { delete static_cast<StreamEncryptor *>(h); }

/* Package-mode batch over independent packets, one PackageEncryptor per worker
 * thread per key (a connection's encryptor), one call per packet as FPNN does. */
void ref_package_batch(int encrypt, const uint8_t *in, uint8_t *out, uint32_t count, uint64_t stride,
                       uint32_t uniform_len, const uint64_t *in_off, const uint64_t *out_off,
                       const uint32_t *len, const uint32_t *key_slot, const uint8_t *keys,
                       size_t keylen, const uint8_t *ivs, int threads)
{
    if (threads < 1) threads = 1;
    auto work = [&](uint32_t b, uint32_t e) {
        for (uint32_t i = b; i < e; i++) {
            uint64_t io = in_off ? in_off[i] : (uint64_t)i * stride;
            uint64_t oo = out_off ? out_off[i] : io;
            uint32_t l = len ? len[i] : uniform_len;
            uint32_t ks = key_slot ? key_slot[i] : 0;
            PackageEncryptor enc(const_cast<uint8_t *>(keys + (size_t)ks * keylen), keylen,
                                 const_cast<uint8_t *>(ivs + 16 * (size_t)ks));
            if (encrypt)
                enc.encrypt(out + oo, const_cast<uint8_t *>(in + io), (int)l);
            else
                enc.decrypt(out + oo, const_cast<uint8_t *>(in + io), (int)l);
        }
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads; t++)
        ts.emplace_back(work, (uint32_t)((uint64_t)count * t / threads), (uint32_t)((uint64_t)count * (t + 1) / threads));
    work(0, (uint32_t)((uint64_t)count / threads));
    for (auto &t : ts) t.join();
}

/* Stream-mode batch: segment i is one StreamEncryptor continued from (iv_state, pos_state). */
void ref_stream_batch(int encrypt, const uint8_t *in, uint8_t *out, uint32_t count,
                      const uint64_t *in_off, const uint64_t *out_off, const uint32_t *len,
                      const uint32_t *key_slot, const uint8_t *keys, size_t keylen,
                      uint8_t *iv_state, uint32_t *pos_state, int threads)
{
    if (threads < 1) threads = 1;
    auto work = [&](uint32_t b, uint32_t e) {
        for (uint32_t i = b; i < e; i++) {
            uint32_t ks = key_slot ? key_slot[i] : i;
            rijndael_context ctx;
            rijndael_setup_encrypt(&ctx, keys + (size_t)ks * keylen, keylen);
            size_t pos = pos_state[i];
            uint64_t oo = out_off ? out_off[i] : in_off[i];
            rijndael_cfb_encrypt(&ctx, encrypt != 0, in + in_off[i], out + oo, len[i], iv_state + 16 * (size_t)i, &pos);
            pos_state[i] = (uint32_t)pos;
        }
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads; t++)
        ts.emplace_back(work, (uint32_t)((uint64_t)count * t / threads), (uint32_t)((uint64_t)count * (t + 1) / threads));
    work(0, (uint32_t)((uint64_t)count / threads));
    for (auto &t : ts) t.join();
}

/* CPU baseline timing: encrypt then decrypt `count` uniform packets, `reps` times. */
double ref_time_package_roundtrip(const uint8_t *in, uint8_t *tmp, uint8_t *out, uint32_t count,
                                  uint32_t len, const uint8_t *key, size_t keylen, const uint8_t *iv,
                                  int threads, int reps)
{
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) {
        ref_package_batch(1, in, tmp, count, len, len, nullptr, nullptr, nullptr, nullptr, key, keylen, iv, threads);
        ref_package_batch(0, tmp, out, count, len, len, nullptr, nullptr, nullptr, nullptr, key, keylen, iv, threads);
    }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} /* extern "C" */
