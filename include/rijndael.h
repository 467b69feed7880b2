/*
 * rijndael.h -- drop-in for the part of the reference's base/rijndael.h that is on
 * FPNN's encryption path (base/rijndael.h:13-16, 21, 50), implemented by
 * libfpnn_aes.so on the MI355X:
 *
 *   rijndael_context        same layout                   (base/rijndael.h:13-16)
 *   rijndael_setup_encrypt  host key expansion, same rk[] (base/rijndael.c:712-799)
 *   rijndael_cfb_encrypt    CFB-128 on the GPU, same (ivec, *p_num) semantics
 *                           (base/rijndael.c:1171-1201); synchronous; in == out allowed
 *
 * Not provided (unused by FPNN): setup_decrypt, the
 * single-block encrypt/decrypt entry points, CBC and OFB.
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

void rijndael_cfb_encrypt(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                          uint8_t ivec[16], size_t *p_num);

#ifdef __cplusplus
}
#endif

#endif
