// aes_common.hpp -- host/device definitions shared by the HIP kernels and the C-ABI.
//
// The AES tables are generated at compile time from GF(2^8) arithmetic (FIPS-197
// section 5.1.1); they equal the reference's static Te0..Te4 (base/rijndael.c:8-346),
// which is checked by tests/test_abi.py through fpnn_aes_setup_encrypt and by every
// GPU parity test.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace fpnn_aes {

constexpr int kThreads = 1024;  // AES kernels: one workgroup of 16 waves per CU

// ---------------------------------------------------------------------------
// Device key record: one expanded key + the connection IV (package mode).
// Round keys are stored in *block byte order* (little-endian words of the state as
// it sits in memory), i.e. bswap() of rijndael_context.rk, so the kernels never
// byte-swap the 16-byte blocks they load from HBM.
struct DevKey {
    uint32_t rk[60];
    uint32_t nrounds;
    uint32_t keylen;
    uint32_t reserved[2];
    uint8_t iv[16];
};
static_assert(sizeof(DevKey) == 272, "DevKey must stay 16-byte aligned and 272 bytes");

// ---------------------------------------------------------------------------
// Compile-time S-box and T-table (little-endian form).
struct Tables {
    uint8_t sbox[256];
    uint32_t t0le[256];   // bswap(Te0[x]): bytes in memory = (2s, s, s, 3s)
    uint8_t isbox[256];   // inverse S-box (Td4's byte, base/rijndael.c:620-686)
    uint32_t td0le[256];  // bswap(Td0[x]): bytes in memory = (14i, 9i, 13i, 11i), i = isbox[x]

    static constexpr uint8_t mul2(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
    static constexpr uint8_t rotl8(uint8_t v, int n) { return (uint8_t)((v << n) | (v >> (8 - n))); }

    constexpr Tables() : sbox{}, t0le{}, isbox{}, td0le{} {
        uint8_t exp_t[255] = {};
        uint8_t log_t[256] = {};
        uint8_t a = 1;
        for (int i = 0; i < 255; i++) {  // powers of the generator 0x03
            exp_t[i] = a;
            log_t[a] = (uint8_t)i;
            a = (uint8_t)(a ^ mul2(a));
        }
        for (int x = 0; x < 256; x++) {
            uint8_t inv = x ? exp_t[(255 - log_t[x]) % 255] : 0;
            sbox[x] = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
        }
        for (int x = 0; x < 256; x++) {
            uint8_t s = sbox[x], s2 = mul2(s), s3 = (uint8_t)(s2 ^ s);
            t0le[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
            isbox[s] = (uint8_t)x;
        }
        for (int x = 0; x < 256; x++) {
            const uint8_t i1 = isbox[x], i2 = mul2(i1), i4 = mul2(i2), i8 = mul2(i4);
            const uint8_t i9 = (uint8_t)(i8 ^ i1), i11 = (uint8_t)(i8 ^ i2 ^ i1), i13 = (uint8_t)(i8 ^ i4 ^ i1),
                          i14 = (uint8_t)(i8 ^ i4 ^ i2);
            td0le[x] = (uint32_t)i14 | ((uint32_t)i9 << 8) | ((uint32_t)i13 << 16) | ((uint32_t)i11 << 24);
        }
    }
};

inline constexpr Tables kTables{};
static_assert(kTables.sbox[0] == 0x63 && kTables.sbox[1] == 0x7c && kTables.sbox[0x53] == 0xed, "S-box");
static_assert(kTables.t0le[0] == 0xa56363c6u, "T0 little-endian form of Te0[0] = 0xc66363a5");
static_assert(kTables.isbox[0] == 0x52 && kTables.isbox[0x63] == 0x00, "inverse S-box");
static_assert(kTables.td0le[0] == 0x50a7f451u, "Td0 little-endian form of Td0[0] = 0x51f4a750");

static inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// FIPS-197 key expansion in the reference's big-endian word form
// (rijndael_setup_encrypt, base/rijndael.c:712-799).  Returns nrounds or 0.
static inline int expand_key_be(uint32_t *w, const uint8_t *key, size_t keylen) {
    int nk, nr;
    switch (keylen) {
        case 16: nk = 4; nr = 10; break;
        case 24: nk = 6; nr = 12; break;
        case 32: nk = 8; nr = 14; break;
        default: return 0;
    }
    for (int i = 0; i < nk; i++)
        w[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
               ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
    auto sub = [](uint32_t t) {
        return ((uint32_t)kTables.sbox[t >> 24] << 24) | ((uint32_t)kTables.sbox[(t >> 16) & 0xff] << 16) |
               ((uint32_t)kTables.sbox[(t >> 8) & 0xff] << 8) | kTables.sbox[t & 0xff];
    };
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = sub((t << 8) | (t >> 24)) ^ ((uint32_t)rcon << 24);
            rcon = Tables::mul2(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = sub(t);
        }
        w[i] = w[i - nk] ^ t;
    }
    return nr;
}

// Decryption key schedule in the reference's form (rijndael_setup_decrypt,
// base/rijndael.c:805-850): the encryption schedule with the round keys in reverse
// order and InvMixColumns applied to all but the first and last.  Returns nrounds or 0.
static inline int expand_key_dec_be(uint32_t *rk, const uint8_t *key, size_t keylen) {
    const int nr = expand_key_be(rk, key, keylen);
    if (!nr) return 0;
    for (int i = 0, j = 4 * nr; i < j; i += 4, j -= 4)
        for (int k = 0; k < 4; k++) {
            const uint32_t t = rk[i + k];
            rk[i + k] = rk[j + k];
            rk[j + k] = t;
        }
    // InvMixColumns(w) for w in BE form: Td_k(S(byte k)), Td_k = bswap of td0le rotated
    auto td = [](int k, uint8_t x) {
        const uint32_t v = kTables.td0le[x];
        const uint32_t r = k ? (v << (8 * k)) | (v >> (32 - 8 * k)) : v;  // rotl: Td_k in LE form
        return bswap32(r);
    };
    for (int r = 1; r < nr; r++)
        for (int k = 0; k < 4; k++) {
            const uint32_t w = rk[4 * r + k];
            rk[4 * r + k] = td(0, kTables.sbox[w >> 24]) ^ td(1, kTables.sbox[(w >> 16) & 0xff]) ^
                            td(2, kTables.sbox[(w >> 8) & 0xff]) ^ td(3, kTables.sbox[w & 0xff]);
        }
    return nr;
}

}  // namespace fpnn_aes
