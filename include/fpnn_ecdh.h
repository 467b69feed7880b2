/* fpnn_ecdh.h -- ECDH key derivation for many connections at once, on the GPU
 * (SURVEY.md §8f row 4).  Part of libfpnn_aes.so; C ABI, plain pointers, int status codes
 * (FPNN_AES_* from fpnn_aes.h).
 *
 * The reference derives each connection's AES key and IV when the connection is set up:
 *   ECCKeyExchange::init(curve, privateKey)           core/KeyExchange.cpp:49-85
 *   ECCKeyExchange::calcKey(key, iv, keylen, peer)    core/KeyExchange.cpp:87-127
 *     secret = uECC_shared_secret(peer, private)      core/micro-ecc/uECC.c:1034-1077
 *     key    = secret[0:16] (keylen 16), secret[0:32] (keylen 32, 32-byte secret),
 *              sha256(secret) (keylen 32, 28/24-byte secret);  iv = md5(secret)
 *   ECCKeysMaker::publicKey                           core/KeyExchange.cpp:161-187
 *     (uECC_make_key: the public key of a random private key)
 * These entry points compute the same bytes for a batch: one server private key and
 * `count` peer public keys (what the TCP/UDP servers do per accepted connection,
 * core/TCPEpollServer.h:380-383, core/UDP.v2/UDPCommon.v2.cpp:127-165), or the client
 * side.  Key formats are the reference's: private keys big-endian (private_len bytes),
 * public keys x || y big-endian (2 * secret_len bytes).
 *
 * ok[i] is calcKey's return value for connection i (0 when the shared secret is the
 * point at infinity, exactly where micro-ecc's ladder meets it).  The batch calls are
 * queued on the engine stream (no host wait); device pointers must be 4-byte aligned.
 */
#ifndef FPNN_ECDH_H
#define FPNN_ECDH_H

#include <stddef.h>
#include <stdint.h>

#include "fpnn_aes.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FPNN_ECDH_SECP256K1 0
#define FPNN_ECDH_SECP256R1 1
#define FPNN_ECDH_SECP224R1 2
#define FPNN_ECDH_SECP192R1 3

/* Curve by the reference's configuration name ("secp256k1", ...); -1 when unknown
 * (ECCKeyExchange::init returns false, core/KeyExchange.cpp:71-75). */
int fpnn_ecdh_curve(const char *name);
/* ECCKeyExchange::_secertLen: 32, 32, 28, 24 (public keys are twice as long); -1 unknown. */
int fpnn_ecdh_secret_len(int curve);
/* uECC_curve_private_key_size: 32, 32, 28, 24; -1 unknown. */
int fpnn_ecdh_private_len(int curve);
/* The reference's configuration name of a curve ("secp256k1", ...); NULL when unknown. */
const char *fpnn_ecdh_curve_name(int curve);
/* uECC_generate_random_int (core/micro-ecc/uECC.c:980-1002): a private key 0 < k < n from
 * the OS random source, big-endian private_len bytes.  1 on success, 0 when no random
 * bytes could be had. */
int fpnn_ecdh_random_private(int curve, uint8_t *out);

/* Server side: private_key (host, private_len bytes) against count peer public keys
 * (device, count * 2*secret_len bytes).  keys (device, count*keylen), ivs (device,
 * count*16), ok (device, count).  keylen must be 16 or 32 (FPNN_AES_ERR_KEYLEN otherwise:
 * calcKey's "key len error"). */
int fpnn_ecdh_calc_keys(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                        uint32_t count, int keylen, uint8_t *keys, uint8_t *ivs, uint8_t *ok);

/* Client side (ECCKeysMaker::calcKey): count private keys (device) against one server
 * public key (host, 2*secret_len bytes). */
int fpnn_ecdh_calc_keys_client(fpnn_aes_engine *e, int curve, const uint8_t *private_keys,
                               const uint8_t *server_public, uint32_t count, int keylen, uint8_t *keys,
                               uint8_t *ivs, uint8_t *ok);

/* Public keys of count private keys (device): EccPoint_compute_public_key
 * (core/micro-ecc/uECC.c:915-933).  public_keys: device, count * 2*secret_len. */
int fpnn_ecdh_public_keys(fpnn_aes_engine *e, int curve, const uint8_t *private_keys, uint32_t count,
                          uint8_t *public_keys, uint8_t *ok);

/* Server side straight into a key set: derive (key, iv) for every peer and expand the
 * keys on the device (fpnn_aes_keyset_create).  private_key: host; peer_public: DEVICE,
 * count * 2*secret_len bytes (as fpnn_ecdh_calc_keys); ok: DEVICE, count bytes, or NULL
 * (the kernel writes it; a host pointer here is a GPU memory fault).  Slot i is
 * connection i; where ok[i] == 0 the slot holds the zero-derived key and must not be
 * used (the reference refuses the connection).  Synchronous (returns a usable key set);
 * the derived keys pass through the engine's own scratch, which is kept between calls. */
int fpnn_ecdh_keyset(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                     uint32_t count, int keylen, uint8_t *ok, fpnn_aes_keyset **out);

/* fpnn_ecdh_calc_keys with host buffers (peer_public count * 2*secret_len, keys, ivs,
 * ok); synchronous. */
int fpnn_ecdh_calc_keys_host(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                             uint32_t count, int keylen, uint8_t *keys, uint8_t *ivs, uint8_t *ok);

/* One connection, host buffers, synchronous: exactly ECCKeyExchange::init(curve,
 * private_key) + calcKey(key, iv, keylen, peer).  Returns 1 (true) / 0 (false) like the
 * reference -- including its length checks -- or a negative FPNN_AES_ERR_* for a
 * device/runtime failure. */
int fpnn_ecdh_calc_key_host(fpnn_aes_engine *e, const char *curve, const uint8_t *private_key, size_t private_len,
                            const uint8_t *peer_public, size_t peer_len, int keylen, uint8_t *key, uint8_t *iv);

/* One key pair, host buffers, synchronous: public key (2*secret_len bytes) of a given
 * private key; 1 = valid, 0 = micro-ecc would reject this private key. */
int fpnn_ecdh_public_key_host(fpnn_aes_engine *e, int curve, const uint8_t *private_key, uint8_t *public_key);

#ifdef __cplusplus
}
#endif

#endif /* FPNN_ECDH_H */
