/*
 * rijndael.h -- drop-in for the reference's base/rijndael.h (base/rijndael.h:13-60),
 * implemented by libfpnn_aes.so on the MI355X.  Every function the reference declares
 * is exported with the same signature and the same results, so a program links against
 * libfpnn_aes.so with rijndael.o removed from libfpbase:
 *
 *   rijndael_context        same layout                        (base/rijndael.h:13-16)
 *   rijndael_setup_encrypt  host key expansion, same rk[]      (base/rijndael.c:712-799)
 *   rijndael_setup_decrypt  host, same reversed/InvMixColumns rk[] (base/rijndael.c:805-850)
 *   rijndael_encrypt        one block on the GPU               (base/rijndael.c:852-959)
 *   rijndael_decrypt        one block on the GPU, inverse cipher (base/rijndael.c:961-1068)
 *   rijndael_cbc_encrypt    CBC on the GPU, zero-padded last block (base/rijndael.c:1070-1097)
 *   rijndael_cbc_decrypt    CBC on the GPU                     (base/rijndael.c:1099-1153)
 *   rijndael_cfb_encrypt    CFB-128 on the GPU, same (ivec, *p_num) semantics
 *                           (base/rijndael.c:1171-1201) -- FPNN's path
 *   rijndael_ofb_encrypt    OFB on the GPU, same (ivec, *p_num) semantics (base/rijndael.c:1155-1169)
 *
 * All calls are synchronous; in == out is allowed (base/rijndael.h:26-30).  For CBC the
 * cipher buffer is a multiple of 16 bytes, as the reference documents (:37-42).
 *
 * Failure policy: the reference functions are void and have no error path.  A GPU
 * failure here (no gfx950 device, HIP error) prints the reason and aborts -- there
 * is deliberately no CPU fallback.
 */
#ifndef FPNN_AMD_RIJNDAEL_H_
#define FPNN_AMD_RIJNDAEL_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int nrounds;
    uint32_t rk[60];
} rijndael_context;

bool rijndael_setup_encrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen);
bool rijndael_setup_decrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen);

void rijndael_encrypt(const rijndael_context *ctx, const uint8_t plain[16], uint8_t cipher[16]);
void rijndael_decrypt(const rijndael_context *ctx, const uint8_t cipher[16], uint8_t plain[16]);

void rijndael_cbc_encrypt(const rijndael_context *ctx, const uint8_t *plain, uint8_t *cipher, size_t len,
                          uint8_t ivec[16]);
void rijndael_cbc_decrypt(const rijndael_context *ctx, const uint8_t *cipher, uint8_t *plain, size_t len,
                          uint8_t ivec[16]);

void rijndael_cfb_encrypt(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                          uint8_t ivec[16], size_t *p_num);

void rijndael_ofb_encrypt(const rijndael_context *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16],
                          size_t *p_num);

#ifdef __cplusplus
}
#endif

#endif
