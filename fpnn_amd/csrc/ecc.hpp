// ecc.hpp -- prime-field and co-Z ladder arithmetic for the ECDH key derivation
// (§8f row 4: core/KeyExchange.cpp:87-127 over the vendored micro-ecc).
//
// One lane computes one scalar multiplication.  Field elements are NW little-endian
// 32-bit limbs in Montgomery form (R = 2^(32*NW)); the modulus and its constants are
// wave-uniform kernel arguments (SGPRs), so one instantiation per (NW, a) serves a curve.
// Add, subtract and halve commute with the Montgomery map, so micro-ecc's formula
// sequence -- including its halving in the doubling -- is followed operation for
// operation: degenerate inputs (ladder steps meeting the point at infinity, peer points
// off the curve) give the reference's results, not just valid ones.
// Every data-dependent choice is a select, never a branch: the scalar is the server's
// private key.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpnn_aes {

enum : int { ECC_SECP256K1 = 0, ECC_SECP256R1 = 1, ECC_SECP224R1 = 2, ECC_SECP192R1 = 3, ECC_NCURVES = 4 };

// Wave-uniform curve description (kernel argument).  All arrays are little-endian
// 32-bit limbs; entries past NW are zero.
struct EccConst {
    uint32_t p[8];      // field prime
    uint32_t n[8];      // group order
    uint32_t pm2[8];    // p - 2 (Fermat inversion exponent)
    uint32_t r1[8];     // R mod p   (Montgomery 1)
    uint32_t r2[8];     // R^2 mod p (to Montgomery form)
    uint32_t px[8];     // uniform point (normal form): G, or one peer's public key
    uint32_t py[8];
    uint32_t k[9];      // uniform effective scalar (regularized), num_n_bits + 1 bits
    uint32_t n0inv;     // -p^-1 mod 2^32
    int32_t nw;         // limbs
    int32_t num_bytes;  // coordinate bytes (KeyExchange _secertLen)
    int32_t num_n_bits;
    int32_t private_bytes;
};

struct EcdhJob {
    const uint8_t *priv;   // per-lane private keys, big-endian private_bytes each (NULL: k)
    const uint8_t *pub;    // per-lane points, x || y big-endian num_bytes each (NULL: px, py)
    uint32_t count;
    int32_t mode;          // ECDH_KEYS: (key, iv) from the shared secret; ECDH_PUBLIC: x || y out
    int32_t keylen;        // 16 or 32 (ECDH_KEYS)
    int32_t pad;
    uint8_t *key_out;      // count * keylen
    uint8_t *iv_out;       // count * 16
    uint8_t *pub_out;      // count * 2 * num_bytes (ECDH_PUBLIC)
    uint8_t *ok_out;       // count: 1 = the reference returns true
};
enum : int { ECDH_KEYS = 0, ECDH_PUBLIC = 1 };

// ---- host side: curve table and derived constants -----------------------------------
struct EccCurveInfo {
    const char *name;
    int nw, num_bytes, num_n_bits;
    bool a_minus3;
};
const EccCurveInfo &ecc_curve_info(int curve);
// Fill the constants of `curve` (px/py = G, k = 0).  Returns false for an unknown curve.
bool ecc_fill_const(int curve, EccConst &c);
// regularize_k (micro-ecc uECC.c:902-913) of a big-endian private key into c.k.
void ecc_set_uniform_scalar(EccConst &c, const uint8_t *priv_be);
// Load a big-endian x || y point into c.px / c.py (normal form, not reduced).
void ecc_set_uniform_point(EccConst &c, const uint8_t *pub_be);

hipError_t launch_ecdh(const EccConst &c, const EcdhJob &j, int curve, hipStream_t st);

}  // namespace fpnn_aes
