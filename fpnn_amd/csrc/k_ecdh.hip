// k_ecdh.hip -- batched ECDH key derivation on the device (§8f row 4).
//
// Reference: ECCKeyExchange::calcKey (core/KeyExchange.cpp:87-127) over the vendored
// micro-ecc: uECC_shared_secret (core/micro-ecc/uECC.c:1034-1077) = co-Z Montgomery ladder
// (uECC.c:857-900; Rivain, eprint 2011/338) on the regularized scalar (uECC.c:902-913),
// then key = secret[0:16] | secret[0:32] | sha256(secret), iv = md5(secret).  The public
// half of uECC_make_key (EccPoint_compute_public_key, uECC.c:915-933) is the same ladder
// from G.  One lane per connection; field arithmetic in ecc.hpp's Montgomery form.
#include <stdlib.h>
#include <string.h>

#include "ecc.hpp"

namespace fpnn_aes {

namespace {

template <int NW>
struct Fe {
    uint32_t v[NW];
};

#include "ecc_chains.hpp"

// Carry chains are written with clang's multiprecision builtins: each limb is one
// v_add_co / v_addc (v_sub_co / v_subb) with the carry in vcc.  (The 64-bit form
// `s = (uint64_t)a - b - borrow; borrow = s >> 63` costs 3-4 instructions per limb: 64-bit
// shifts, register-pair moves.)
__device__ __forceinline__ uint32_t addc(uint32_t x, uint32_t y, uint32_t &c) {
    unsigned co;
    const uint32_t r = __builtin_addc(x, y, c, &co);
    c = co;
    return r;
}

// t[0..NW] (t < 2p) -> t mod p (one borrow chain through top, one select; ecc_chains.hpp)
template <int NW>
__device__ __forceinline__ Fe<NW> reduce_once(const uint32_t *t, uint32_t top, const EccConst &c) {
    Fe<NW> r;
    reduce_n<NW>(r.v, t, top, c.p);
    return r;
}

// secp256k1 (p = 2^256 - 2^32 - 977) in normal form: the 512-bit product t = H*2^256 + L
// by product scanning (NW^2 partial products, half the Montgomery product's 2*NW^2), then
// t = L + H*(2^32 + 977) (mod p) folded twice and one conditional subtraction.  The host
// passes R = 1 (r1 = r2 = 1) for this form, so the Montgomery-form conversions around the
// ladder become identities and every field value is the same residue as micro-ecc's.
// Field kinds: normal form with a special-prime reduction of the full 2*NW-limb product
// per curve (R = 1 on the host side).  (Rounds 1-2 also built a generic Montgomery-form
// product for any curve; it was the A/B baseline and is gone since round 4.)
enum : int { FK_K1 = 1, FK_P256 = 2, FK_P224 = 3, FK_P192 = 4 };

// t (512 bits) mod p: t = L + H*(2^32 + 977) as three carry chains over the limbs --
// L + lo(H_i * 977), then + H << 32, then + hi(H_i * 977) << 32 -- leaving a top
// u8 + u9 * 2^32 < 2^34; that folds once more the same way into one chain
// (U + top * (2^32 + 977) < 2^256 + 2^67 < 2p, a carry-out of at most 1) and one
// conditional subtraction.
template <int NW>
__device__ __forceinline__ Fe<NW> k1_fold(const uint32_t (&t)[16], const EccConst &c) {
    uint32_t u[8], ml[8], mh[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t m = (uint64_t)t[8 + i] * 977u;
        ml[i] = (uint32_t)m;
        mh[i] = (uint32_t)(m >> 32);
    }
    const uint32_t c1 = add_n<8>(u, t, ml);
    uint32_t x[8], w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = i < 7 ? u[i + 1] : c1;
    const uint32_t c2 = add_n<8>(w, x, t + 8);  // + H << 32: limbs 1..8
    const uint32_t c3 = add_n<8>(x, w, mh);     // + hi(H * 977) << 32
#pragma unroll
    for (int i = 1; i < 8; i++) u[i] = x[i - 1];
    const uint32_t u8 = x[7], u9 = c2 + c3;  // top = u8 + u9 * 2^32
    const uint64_t a = (uint64_t)u8 * 977u;
    const uint32_t a1 = (uint32_t)(a >> 32) + u9 * 977u;  // < 2^11
    uint32_t k = 0;
    const uint32_t s1 = addc(a1, u8, k);  // limb 1: hi(u8 * 977) + u9 * 977 + u8 (top << 32)
    const uint32_t z[8] = {(uint32_t)a, s1, u9 + k, 0u, 0u, 0u, 0u, 0u};
    const uint32_t cy = add_n<8>(u, u, z);
    return reduce_once<NW>(u, cy, c);
}

// secp256r1 (p = 2^256 - 2^224 + 2^192 + 2^96 - 1): the NIST word-sum reduction (FIPS
// 186-4 D.2.3) t = s1 + 2 s2 + 2 s3 + s4 + s5 - s6 - s7 - s8 - s9, as nine 8-limb carry
// chains (ecc_chains.hpp; 2 (s2 + s3) as one sum doubled) whose carries and borrows add up
// to a signed top k in [-4, 6]; k * 2^256 is folded back as k * (2^224 - 2^192 - 2^96 + 1)
// in one add and one subtract chain ([kp,0,0,kn,0,0,kn,kp] and [kn,0,0,kp,0,0,kp,kn] with
// kp = max(k, 0), kn = max(-k, 0)); their carry minus borrow (-1, 0 or 1) is settled by
// one add or subtract of p (selects).  (Round 2 summed the words as signed 64-bit column
// sums: ~50 more instructions per fold.)
template <int NW>
__device__ __forceinline__ Fe<NW> p256_fold(const uint32_t (&t)[16], const EccConst &c) {
    const uint32_t z = 0;
    const uint32_t s2[8] = {z, z, z, t[11], t[12], t[13], t[14], t[15]};
    const uint32_t s3[8] = {z, z, z, t[12], t[13], t[14], t[15], z};
    const uint32_t s4[8] = {t[8], t[9], t[10], z, z, z, t[14], t[15]};
    const uint32_t s5[8] = {t[9], t[10], t[11], t[13], t[14], t[15], t[13], t[8]};
    const uint32_t s6[8] = {t[11], t[12], t[13], z, z, z, t[8], t[10]};
    const uint32_t s7[8] = {t[12], t[13], t[14], t[15], z, z, t[9], t[11]};
    const uint32_t s8[8] = {t[13], t[14], t[15], t[8], t[9], t[10], z, t[12]};
    const uint32_t s9[8] = {t[14], t[15], z, t[9], t[10], t[11], z, t[13]};
    uint32_t v[8], w[8], u[8];
    const uint32_t cv = add_n<8>(v, s2, s3);
    const uint32_t cw = add_n<8>(w, v, v);  // 2 (s2 + s3) = w + (2 cv + cw) 2^256
    int32_t k = (int32_t)(2 * cv + cw);
    k += (int32_t)add_n<8>(u, t, w);  // s1 = t[0..7]
    k += (int32_t)add_n<8>(v, u, s4);
    k += (int32_t)add_n<8>(u, v, s5);
    k -= (int32_t)sub_n<8>(v, u, s6);
    k -= (int32_t)sub_n<8>(u, v, s7);
    k -= (int32_t)sub_n<8>(v, u, s8);
    k -= (int32_t)sub_n<8>(u, v, s9);
    const uint32_t kp = k > 0 ? (uint32_t)k : 0u, kn = k < 0 ? (uint32_t)-k : 0u;
    const uint32_t fa[8] = {kp, z, z, kn, z, z, kn, kp};
    const uint32_t fb[8] = {kn, z, z, kp, z, z, kp, kn};
    const int32_t cr = (int32_t)add_n<8>(v, u, fa) - (int32_t)sub_n<8>(u, v, fb);  // value = U + cr 2^256
    uint32_t d[8], e[8];
    const uint32_t borrow = sub_n<8>(d, u, c.p);
    add_n<8>(e, u, c.p);
    const bool use_e = cr < 0, use_d = cr > 0 || (cr == 0 && borrow == 0);
    Fe<NW> r;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = use_e ? e[j] : (use_d ? d[j] : u[j]);
    return r;
}

// column i of a product scan: partial products a[j] * b[i - j] for j in [col_first, col_last]
// (a square's cross products: j < i - j only)
template <int NW>
__device__ constexpr int col_first(int i) { return i > NW - 1 ? i - (NW - 1) : 0; }
template <int NW, bool SQ>
__device__ constexpr int col_last(int i) { return SQ ? (i + 1) / 2 - 1 : (i < NW - 1 ? i : NW - 1); }

// Product scanning: one 96-bit column accumulator (lo 64 + hi 32); each column's partial
// products are one asm block (mac_col, ecc_chains.hpp: hi from the carries alone), the carried
// value of the next column is (lo >> 32 | hi << 32).  SQ: the square's cross products only
// (finished by sqr_finish).  Columns by template recursion: a column's length is a template
// argument of mac_col.
template <int NW, bool SQ, int I>
__device__ __forceinline__ void scan_col(const uint32_t *a, const uint32_t *b, uint32_t (&t)[2 * NW], uint64_t &lo) {
    if constexpr (I < 2 * NW - 1) {
        constexpr int f = col_first<NW>(I), n = col_last<NW, SQ>(I) - f + 1;
        uint32_t hi = 0;
        if constexpr (n > 0) {
            uint32_t x[n], y[n];
#pragma unroll
            for (int k = 0; k < n; k++) {
                x[k] = a[f + k];
                y[k] = b[I - f - k];
            }
            mac_col<n>(lo, hi, x, y);
        }
        t[I] = (uint32_t)lo;
        lo = (lo >> 32) | ((uint64_t)hi << 32);
        scan_col<NW, SQ, I + 1>(a, b, t, lo);
    }
}

template <int NW, bool SQ>
__device__ __forceinline__ void prod_scan(const uint32_t *a, const uint32_t *b, uint32_t (&t)[2 * NW]) {
    uint64_t lo = 0;
    scan_col<NW, SQ, 0>(a, b, t, lo);
    t[2 * NW - 1] = (uint32_t)lo;
}

// 2*NW-limb product of two NW-limb values
template <int NW>
__device__ __forceinline__ void prodN(const uint32_t *a, const uint32_t *b, uint32_t (&t)[2 * NW]) {
    prod_scan<NW, false>(a, b, t);
}

// the square's second half: the cross-product sum t doubled by a one-bit shift, plus the
// NW squares a_i^2 on the diagonal in one carry chain (the total a^2 < 2^(64 NW): no carry out)
template <int NW>
__device__ __forceinline__ void sqr_finish(const uint32_t *a, uint32_t (&t)[2 * NW]) {
    uint32_t d[2 * NW];
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint64_t q = (uint64_t)a[i] * a[i];
        d[2 * i] = (uint32_t)q;
        d[2 * i + 1] = (uint32_t)(q >> 32);
    }
#pragma unroll
    for (int i = 2 * NW - 1; i > 0; i--) t[i] = __builtin_amdgcn_alignbit(t[i], t[i - 1], 31);
    t[0] = 0;  // (the cross sum has no limb-0 term)
    add_n<2 * NW>(t, t, d);
}

// a^2: the NW(NW-1)/2 cross products once, doubled, plus the NW squares (36 partial
// products instead of 64 at NW = 8)
template <int NW>
__device__ __forceinline__ void sqrN(const uint32_t *a, uint32_t (&t)[2 * NW]) {
    prod_scan<NW, true>(a, a, t);
    sqr_finish<NW>(a, t);
}

// Two independent 2*NW-limb products (SQ: a square's cross-product half).  The ladder's
// field products come in independent pairs (xycz_add / xycz_addc below); the two scans are
// independent instruction streams the scheduler may interleave.
template <int NW, bool SQ1, bool SQ2>
__device__ __forceinline__ void prod_dual(const uint32_t *a1, const uint32_t *b1, uint32_t (&t1)[2 * NW],
                                          const uint32_t *a2, const uint32_t *b2, uint32_t (&t2)[2 * NW]) {
    prod_scan<NW, SQ1>(a1, b1, t1);
    prod_scan<NW, SQ2>(a2, b2, t2);
}

// secp192r1 (p = 2^192 - 2^64 - 1): the NIST word-sum reduction (FIPS 186-4 D.2.1)
// t = s1 + s2 + s3 + s4 as three 6-limb carry chains, the top k in [0, 3] folded back as
// k * (2^64 + 1) in one chain, and one conditional subtraction through its carry
// (U + c 2^192 < 2p: c = 1 only when U < 2^66)
template <int NW>
__device__ __forceinline__ Fe<NW> p192_fold(const uint32_t (&t)[12], const EccConst &c) {
    const uint32_t z = 0;
    const uint32_t s2[6] = {t[6], t[7], t[6], t[7], z, z};
    const uint32_t s3[6] = {z, z, t[8], t[9], t[8], t[9]};
    const uint32_t s4[6] = {t[10], t[11], t[10], t[11], t[10], t[11]};
    uint32_t u[6], v[6];
    uint32_t k = add_n<6>(u, t, s2);  // s1 = t[0..5]
    k += add_n<6>(v, u, s3);
    k += add_n<6>(u, v, s4);
    const uint32_t fk[6] = {k, z, k, z, z, z};
    const uint32_t cy = add_n<6>(v, u, fk);
    return reduce_once<NW>(v, cy, c);
}

// secp224r1 (p = 2^224 - 2^96 + 1): the NIST word-sum reduction (FIPS 186-4 D.2.2)
// t = s1 + s2 + s3 - s4 - s5 as four 7-limb carry chains whose carries and borrows sum to a
// signed top k in [-2, 2]; k * 2^224 is folded back as k * (2^96 - 1) in one add and one
// subtract chain ([kn,0,0,kp,0,0,0] and [kp,0,0,kn,0,0,0]); their carry minus borrow
// (-1, 0 or 1) is settled by one add or subtract of p (selects), as p256_fold.
template <int NW>
__device__ __forceinline__ Fe<NW> p224_fold(const uint32_t (&t)[14], const EccConst &c) {
    const uint32_t z = 0;
    const uint32_t s2[7] = {z, z, z, t[7], t[8], t[9], t[10]};
    const uint32_t s3[7] = {z, z, z, t[11], t[12], t[13], z};
    const uint32_t s4[7] = {t[7], t[8], t[9], t[10], t[11], t[12], t[13]};
    const uint32_t s5[7] = {t[11], t[12], t[13], z, z, z, z};
    uint32_t u[7], v[7];
    int32_t k = (int32_t)add_n<7>(u, t, s2);  // s1 = t[0..6]
    k += (int32_t)add_n<7>(v, u, s3);
    k -= (int32_t)sub_n<7>(u, v, s4);
    k -= (int32_t)sub_n<7>(v, u, s5);
    const uint32_t kp = k > 0 ? (uint32_t)k : 0u, kn = k < 0 ? (uint32_t)-k : 0u;
    const uint32_t fa[7] = {kn, z, z, kp, z, z, z};
    const uint32_t fb[7] = {kp, z, z, kn, z, z, z};
    const int32_t cr = (int32_t)add_n<7>(u, v, fa) - (int32_t)sub_n<7>(v, u, fb);  // value = V + cr 2^224
    uint32_t d[7], e[7];
    const uint32_t borrow = sub_n<7>(d, v, c.p);
    add_n<7>(e, v, c.p);
    const bool use_e = cr < 0, use_d = cr > 0 || (cr == 0 && borrow == 0);
    Fe<NW> r;
#pragma unroll
    for (int j = 0; j < 7; j++) r.v[j] = use_e ? e[j] : (use_d ? d[j] : v[j]);
    return r;
}

template <int NW, int FK>
__device__ __forceinline__ Fe<NW> fold_nf(const uint32_t (&t)[2 * NW], const EccConst &c) {
    if constexpr (FK == FK_K1) {
        static_assert(NW == 8, "secp256k1 has 8 limbs");
        return k1_fold<NW>(t, c);
    } else if constexpr (FK == FK_P256) {
        static_assert(NW == 8, "secp256r1 has 8 limbs");
        return p256_fold<NW>(t, c);
    } else if constexpr (FK == FK_P224) {
        static_assert(NW == 7, "secp224r1 has 7 limbs");
        return p224_fold<NW>(t, c);
    } else {
        static_assert(NW == 6 && FK == FK_P192, "secp192r1 has 6 limbs");
        return p192_fold<NW>(t, c);
    }
}

template <int NW, int FK>
__device__ __forceinline__ Fe<NW> fmul(const Fe<NW> &a, const Fe<NW> &b, const EccConst &c) {
    uint32_t t[2 * NW];
    prodN<NW>(a.v, b.v, t);
    return fold_nf<NW, FK>(t, c);
}

template <int NW, int FK>
__device__ __forceinline__ Fe<NW> fsqr(const Fe<NW> &a, const EccConst &c) {
    uint32_t t[2 * NW];
    sqrN<NW>(a.v, t);
    return fold_nf<NW, FK>(t, c);
}

// r1 = a1 * b1 (a1^2 if SQ1), r2 = a2 * b2 (a2^2 if SQ2) -- two independent field products
// computed together (prod_dual); every operand is read before either result is written, so
// r1 / r2 may alias any input.
template <int NW, int FK, bool SQ1, bool SQ2>
__device__ __forceinline__ void fdual(Fe<NW> &r1, const Fe<NW> &a1, const Fe<NW> &b1, Fe<NW> &r2, const Fe<NW> &a2,
                                      const Fe<NW> &b2, const EccConst &c) {
    uint32_t t1[2 * NW], t2[2 * NW];
    prod_dual<NW, SQ1, SQ2>(a1.v, SQ1 ? a1.v : b1.v, t1, a2.v, SQ2 ? a2.v : b2.v, t2);
    if (SQ1) sqr_finish<NW>(a1.v, t1);
    if (SQ2) sqr_finish<NW>(a2.v, t2);
    r1 = fold_nf<NW, FK>(t1, c);
    r2 = fold_nf<NW, FK>(t2, c);
}

template <int NW>
__device__ __forceinline__ Fe<NW> fadd(const Fe<NW> &a, const Fe<NW> &b, const EccConst &c) {
    uint32_t t[NW];
    const uint32_t carry = add_n<NW>(t, a.v, b.v);
    return reduce_once<NW>(t, carry, c);
}

template <int NW>
__device__ __forceinline__ Fe<NW> fsub(const Fe<NW> &a, const Fe<NW> &b, const EccConst &c) {
    Fe<NW> r;
    fsub_n<NW>(r.v, a.v, b.v, c.p);  // a - b, plus p where that borrowed
    return r;
}

// a/2 mod p: (a + p)/2 when a is odd (curve-specific.inc:76-82 / 1130-1136)
template <int NW>
__device__ __forceinline__ Fe<NW> fhalf(const Fe<NW> &a, const EccConst &c) {
    const uint32_t mask = 0u - (a.v[0] & 1u);
    uint32_t t[NW];
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < NW; j++) t[j] = addc(a.v[j], c.p[j] & mask, carry);
    Fe<NW> r;
#pragma unroll
    for (int j = 0; j < NW - 1; j++) r.v[j] = __builtin_amdgcn_alignbit(t[j + 1], t[j], 1);
    r.v[NW - 1] = __builtin_amdgcn_alignbit(carry, t[NW - 1], 1);
    return r;
}

template <int NW>
__device__ __forceinline__ Fe<NW> fsel(bool s, const Fe<NW> &a, const Fe<NW> &b) {
    Fe<NW> r;
#pragma unroll
    for (int j = 0; j < NW; j++) r.v[j] = s ? a.v[j] : b.v[j];
    return r;
}

template <int NW>
__device__ __forceinline__ Fe<NW> fconst(const uint32_t *k) {
    Fe<NW> r;
#pragma unroll
    for (int j = 0; j < NW; j++) r.v[j] = k[j];
    return r;
}

// x^(2^n): n squarings (a loop: the square is too large to unroll hundreds of times)
template <int NW, int FK>
__device__ __forceinline__ Fe<NW> fsqr_n(Fe<NW> x, int n, const EccConst &c) {
#pragma unroll 1
    for (int i = 0; i < n; i++) x = fsqr<NW, FK>(x, c);
    return x;
}

// a^(p-2) = 1/a (0 -> 0, as uECC_vli_modInv); the exponent is public: uniform branches.
// Special forms: addition chains for p - 2 (blocks of ones x_k = a^(2^k - 1)) -- the same
// power with far fewer products, so the same result (chains checked in Python against
// pow(a, p - 2, p)).  secp256k1: 255 squarings and 15 products instead of ~248.
template <int NW, int FK>
__device__ Fe<NW> finv(const Fe<NW> &a, const EccConst &c) {
    if constexpr (FK == FK_K1) {
        const Fe<NW> x2 = fmul<NW, FK>(fsqr<NW, FK>(a, c), a, c);
        const Fe<NW> x3 = fmul<NW, FK>(fsqr<NW, FK>(x2, c), a, c);
        const Fe<NW> x6 = fmul<NW, FK>(fsqr_n<NW, FK>(x3, 3, c), x3, c);
        const Fe<NW> x9 = fmul<NW, FK>(fsqr_n<NW, FK>(x6, 3, c), x3, c);
        const Fe<NW> x11 = fmul<NW, FK>(fsqr_n<NW, FK>(x9, 2, c), x2, c);
        const Fe<NW> x22 = fmul<NW, FK>(fsqr_n<NW, FK>(x11, 11, c), x11, c);
        const Fe<NW> x44 = fmul<NW, FK>(fsqr_n<NW, FK>(x22, 22, c), x22, c);
        const Fe<NW> x88 = fmul<NW, FK>(fsqr_n<NW, FK>(x44, 44, c), x44, c);
        const Fe<NW> x176 = fmul<NW, FK>(fsqr_n<NW, FK>(x88, 88, c), x88, c);
        const Fe<NW> x220 = fmul<NW, FK>(fsqr_n<NW, FK>(x176, 44, c), x44, c);
        const Fe<NW> x223 = fmul<NW, FK>(fsqr_n<NW, FK>(x220, 3, c), x3, c);
        Fe<NW> t = fmul<NW, FK>(fsqr_n<NW, FK>(x223, 23, c), x22, c);
        t = fmul<NW, FK>(fsqr_n<NW, FK>(t, 5, c), a, c);
        t = fmul<NW, FK>(fsqr_n<NW, FK>(t, 3, c), x2, c);
        return fmul<NW, FK>(fsqr_n<NW, FK>(t, 2, c), a, c);
    } else if constexpr (FK == FK_P256) {
        // p - 2 = 1^32 0^31 1 0^96 1^94 0 1: 255 squarings and 13 products (Fermat: ~127)
        const Fe<NW> x2 = fmul<NW, FK>(fsqr<NW, FK>(a, c), a, c);
        const Fe<NW> x3 = fmul<NW, FK>(fsqr<NW, FK>(x2, c), a, c);
        const Fe<NW> x6 = fmul<NW, FK>(fsqr_n<NW, FK>(x3, 3, c), x3, c);
        const Fe<NW> x12 = fmul<NW, FK>(fsqr_n<NW, FK>(x6, 6, c), x6, c);
        const Fe<NW> x15 = fmul<NW, FK>(fsqr_n<NW, FK>(x12, 3, c), x3, c);
        const Fe<NW> x30 = fmul<NW, FK>(fsqr_n<NW, FK>(x15, 15, c), x15, c);
        const Fe<NW> x32 = fmul<NW, FK>(fsqr_n<NW, FK>(x30, 2, c), x2, c);
        Fe<NW> t = fmul<NW, FK>(fsqr_n<NW, FK>(x32, 32, c), a, c);
        t = fsqr_n<NW, FK>(t, 96, c);
        t = fmul<NW, FK>(fsqr_n<NW, FK>(t, 32, c), x32, c);
        t = fmul<NW, FK>(fsqr_n<NW, FK>(t, 32, c), x32, c);
        t = fmul<NW, FK>(fsqr_n<NW, FK>(t, 30, c), x30, c);
        return fmul<NW, FK>(fsqr_n<NW, FK>(t, 2, c), a, c);
    } else if constexpr (FK == FK_P224 || FK == FK_P192) {
        // common head: x127 (126 squarings, 10 products)
        const Fe<NW> x2 = fmul<NW, FK>(fsqr<NW, FK>(a, c), a, c);
        const Fe<NW> x3 = fmul<NW, FK>(fsqr<NW, FK>(x2, c), a, c);
        const Fe<NW> x6 = fmul<NW, FK>(fsqr_n<NW, FK>(x3, 3, c), x3, c);
        const Fe<NW> x12 = fmul<NW, FK>(fsqr_n<NW, FK>(x6, 6, c), x6, c);
        const Fe<NW> x24 = fmul<NW, FK>(fsqr_n<NW, FK>(x12, 12, c), x12, c);
        const Fe<NW> x48 = fmul<NW, FK>(fsqr_n<NW, FK>(x24, 24, c), x24, c);
        const Fe<NW> x96 = fmul<NW, FK>(fsqr_n<NW, FK>(x48, 48, c), x48, c);
        const Fe<NW> x120 = fmul<NW, FK>(fsqr_n<NW, FK>(x96, 24, c), x24, c);
        const Fe<NW> x126 = fmul<NW, FK>(fsqr_n<NW, FK>(x120, 6, c), x6, c);
        const Fe<NW> x127 = fmul<NW, FK>(fsqr<NW, FK>(x126, c), a, c);
        if constexpr (FK == FK_P224) {  // p - 2 = 1^127 0 1^96: 223 squarings, 11 products
            return fmul<NW, FK>(fsqr_n<NW, FK>(x127, 97, c), x96, c);
        } else {  // p - 2 = 1^127 0 1^62 0 1: 205 squarings, 14 products (Fermat ~189)
            const Fe<NW> x62 = fmul<NW, FK>(fsqr_n<NW, FK>(fmul<NW, FK>(fsqr_n<NW, FK>(x48, 12, c), x12, c), 2, c), x2, c);
            const Fe<NW> t = fmul<NW, FK>(fsqr_n<NW, FK>(x127, 63, c), x62, c);
            return fmul<NW, FK>(fsqr_n<NW, FK>(t, 2, c), a, c);
        }
    }
}

// double_jacobian (curve-specific.inc:50-95 a = -3; :1110-1141 secp256k1, a = 0), z != 0
template <int NW, bool AM3, int FK>
__device__ __forceinline__ void dbl_jacobian(Fe<NW> &X1, Fe<NW> &Y1, Fe<NW> &Z1, const EccConst &c) {
    if (AM3) {
        Fe<NW> t4 = fsqr<NW, FK>(Y1, c);
        Fe<NW> t5 = fmul<NW, FK>(X1, t4, c);
        t4 = fsqr<NW, FK>(t4, c);
        Y1 = fmul<NW, FK>(Y1, Z1, c);
        Z1 = fsqr<NW, FK>(Z1, c);
        X1 = fadd<NW>(X1, Z1, c);
        Z1 = fadd<NW>(Z1, Z1, c);
        Z1 = fsub<NW>(X1, Z1, c);
        X1 = fmul<NW, FK>(X1, Z1, c);
        Z1 = fadd<NW>(X1, X1, c);
        X1 = fadd<NW>(X1, Z1, c);
        X1 = fhalf<NW>(X1, c);
        Z1 = fsqr<NW, FK>(X1, c);
        Z1 = fsub<NW>(Z1, t5, c);
        Z1 = fsub<NW>(Z1, t5, c);
        t5 = fsub<NW>(t5, Z1, c);
        X1 = fmul<NW, FK>(X1, t5, c);
        t4 = fsub<NW>(X1, t4, c);
        X1 = Z1;
        Z1 = Y1;
        Y1 = t4;
    } else {
        Fe<NW> t5 = fsqr<NW, FK>(Y1, c);
        Fe<NW> t4 = fmul<NW, FK>(X1, t5, c);
        X1 = fsqr<NW, FK>(X1, c);
        t5 = fsqr<NW, FK>(t5, c);
        Z1 = fmul<NW, FK>(Y1, Z1, c);
        Y1 = fadd<NW>(X1, X1, c);
        Y1 = fadd<NW>(Y1, X1, c);
        Y1 = fhalf<NW>(Y1, c);
        X1 = fsqr<NW, FK>(Y1, c);
        X1 = fsub<NW>(X1, t4, c);
        X1 = fsub<NW>(X1, t4, c);
        t4 = fsub<NW>(t4, X1, c);
        Y1 = fmul<NW, FK>(Y1, t4, c);
        Y1 = fsub<NW>(Y1, t5, c);
    }
}

// (x, y) -> (x z^2, y z^3)  (uECC.c:748-758)
template <int NW, int FK>
__device__ __forceinline__ void apply_z(Fe<NW> &X, Fe<NW> &Y, const Fe<NW> &Z, const EccConst &c) {
    Fe<NW> t = fsqr<NW, FK>(Z, c);
    X = fmul<NW, FK>(X, t, c);
    t = fmul<NW, FK>(t, Z, c);
    Y = fmul<NW, FK>(Y, t, c);
}

// XYcZ_add (uECC.c:788-813): (P, Q) co-Z -> P into P', Q into P + Q
template <int NW, int FK>
// The same operation sequence, its six field products taken in three independent pairs
// (fdual): (X2 - X1)^2 with (Y2 - Y1)^2, X1 * t5 with X2 * t5, Y1 * (X2 - X1) with
// Y2 * (X1 - t5).
__device__ __forceinline__ void xycz_add(Fe<NW> &X1, Fe<NW> &Y1, Fe<NW> &X2, Fe<NW> &Y2, const EccConst &c) {
    Fe<NW> t5 = fsub<NW>(X2, X1, c), s2;
    Y2 = fsub<NW>(Y2, Y1, c);
    fdual<NW, FK, true, true>(t5, t5, t5, s2, Y2, Y2, c);  // t5 = (X2 - X1)^2, s2 = Y2^2
    fdual<NW, FK, false, false>(X1, X1, t5, X2, X2, t5, c);
    t5 = fsub<NW>(s2, X1, c);
    t5 = fsub<NW>(t5, X2, c);
    X2 = fsub<NW>(X2, X1, c);
    const Fe<NW> x2b = fsub<NW>(X1, t5, c);
    fdual<NW, FK, false, false>(Y1, Y1, X2, Y2, Y2, x2b, c);
    Y2 = fsub<NW>(Y2, Y1, c);
    X2 = t5;
}

// XYcZ_addC (uECC.c:819-854): (P, Q) co-Z -> P into P - Q, Q into P + Q
template <int NW, int FK>
// Its eight field products in four independent pairs: (X2 - X1)^2 with (Y2 - Y1)^2,
// X1 * t5 with X2 * t5, Y1 * (X2 - X1) with (Y2 + Y1)^2, Y2 * t7 with t6 * (Y2 + Y1).
__device__ __forceinline__ void xycz_addc(Fe<NW> &X1, Fe<NW> &Y1, Fe<NW> &X2, Fe<NW> &Y2, const EccConst &c) {
    Fe<NW> t5 = fsub<NW>(X2, X1, c), sy, t7s;
    const Fe<NW> yp = fadd<NW>(Y2, Y1, c);  // uECC's t5 = Y2 + Y1
    Y2 = fsub<NW>(Y2, Y1, c);
    fdual<NW, FK, true, true>(t5, t5, t5, sy, Y2, Y2, c);  // t5 = (X2 - X1)^2, sy = Y2^2
    fdual<NW, FK, false, false>(X1, X1, t5, X2, X2, t5, c);
    Fe<NW> t6 = fsub<NW>(X2, X1, c);
    fdual<NW, FK, false, true>(Y1, Y1, t6, t7s, yp, yp, c);  // Y1 *= X2 - X1, t7s = (Y2 + Y1)^2
    t6 = fadd<NW>(X1, X2, c);
    X2 = fsub<NW>(sy, t6, c);
    const Fe<NW> t7 = fsub<NW>(X1, X2, c);
    const Fe<NW> t7b = fsub<NW>(t7s, t6, c);
    t6 = fsub<NW>(t7b, X1, c);
    fdual<NW, FK, false, false>(Y2, Y2, t7, t6, t6, yp, c);
    Y2 = fsub<NW>(Y2, Y1, c);
    Y1 = fsub<NW>(t6, Y1, c);
    X1 = t7b;
}

template <int NW>
__device__ __forceinline__ void cswap(bool s, Fe<NW> &a, Fe<NW> &b) {
#pragma unroll
    for (int j = 0; j < NW; j++) {
        const uint32_t x = (a.v[j] ^ b.v[j]) & (0u - (uint32_t)s);
        a.v[j] ^= x;
        b.v[j] ^= x;
    }
}

// EccPoint_mult (uECC.c:857-900): P (Montgomery form), scalar of nbits bits (top bit 1)
// -> affine result (Montgomery form).  Registers (A, B) hold (R[bit], R[!bit]) of the
// step; `sw` records whether they currently hold (R0, R1) so that swaps happen only
// when consecutive bits differ.
template <int NW, bool AM3, int FK>
__device__ __forceinline__ void ladder(Fe<NW> &rx, Fe<NW> &ry, const Fe<NW> &xp, const Fe<NW> &yp, const uint32_t *s, int nbits,
                       const EccConst &c) {
    Fe<NW> ax = xp, ay = yp;  // R1
    Fe<NW> bx = xp, by = yp;  // R0
    Fe<NW> z = fconst<NW>(c.r1);
    dbl_jacobian<NW, AM3, FK>(ax, ay, z, c);  // XYcZ_initial_double: R1 = 2P, R0 = P co-Z
    apply_z<NW, FK>(bx, by, z, c);
    bool sw = false;  // (A, B) == (R1, R0)
    uint32_t word = 0;
    for (int i = nbits - 2; i >= 0; --i) {
        if (i == nbits - 2 || (i & 31) == 31) {
            word = s[0];
#pragma unroll
            for (int j = 1; j <= NW; j++) word = (i >> 5) == j ? s[j] : word;
        }
        const bool bit = (word >> (i & 31)) & 1u;
        const bool want = !bit;  // A must be R[bit]: R0 when the bit is 0
        cswap<NW>(want != sw, ax, bx);
        cswap<NW>(want != sw, ay, by);
        sw = want;
        xycz_addc<NW, FK>(ax, ay, bx, by, c);  // R[bit] - R[!bit], R[bit] + R[!bit]
        if (i == 0) break;
        xycz_add<NW, FK>(bx, by, ax, ay, c);
    }
    // 1/Z = yP * Xb / (xP * Yb * (X1 - X0)), b = bit 0 (A holds R[b])
    const Fe<NW> x1 = fsel<NW>(sw, bx, ax), x0 = fsel<NW>(sw, ax, bx);
    Fe<NW> zi = fsub<NW>(x1, x0, c);
    zi = fmul<NW, FK>(zi, ay, c);
    zi = fmul<NW, FK>(zi, xp, c);
    zi = finv<NW, FK>(zi, c);
    zi = fmul<NW, FK>(zi, yp, c);
    zi = fmul<NW, FK>(zi, ax, c);
    xycz_add<NW, FK>(bx, by, ax, ay, c);
    rx = fsel<NW>(sw, ax, bx);  // R0
    ry = fsel<NW>(sw, ay, by);
    apply_z<NW, FK>(rx, ry, zi, c);
}

// big-endian bytes (4-byte aligned, nbytes = 4*NW) -> limbs
template <int NW>
__device__ __forceinline__ Fe<NW> load_be(const uint8_t *p) {
    Fe<NW> r;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(p);
#pragma unroll
    for (int j = 0; j < NW; j++) r.v[j] = __builtin_bswap32(w[NW - 1 - j]);
    return r;
}

template <int NW>
__device__ __forceinline__ void store_be(uint8_t *p, const Fe<NW> &a) {
    uint32_t *w = reinterpret_cast<uint32_t *>(p);
#pragma unroll
    for (int j = 0; j < NW; j++) w[NW - 1 - j] = __builtin_bswap32(a.v[j]);
}

// ---- MD5 (RFC 1321) and SHA-256 (FIPS 180-4) of one short message (< 56 bytes) ----
__constant__ uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// msg: nw32 words as they sit in memory (little-endian loads of the bytes), 4*nw32 bytes
__device__ void md5_short(const uint32_t *mem, int nw32, uint32_t out[4]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = 0;
    for (int i = 0; i < nw32; i++) m[i] = mem[i];
    m[nw32] = 0x80u;
    m[14] = (uint32_t)(nw32 * 32);
    uint32_t a = 0x67452301, b = 0xefcdab89, c = 0x98badcfe, d = 0x10325476;
    const int sh[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl(a + f + kMd5K[i] + m[g], sh[i >> 4][i & 3]);
        a = t;
    }
    out[0] = 0x67452301 + a;
    out[1] = 0xefcdab89 + b;
    out[2] = 0x98badcfe + c;
    out[3] = 0x10325476 + d;  // little-endian words = digest bytes in order
}

__device__ void sha256_short(const uint32_t *mem, int nw32, uint32_t out[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = 0;
    for (int i = 0; i < nw32; i++) w[i] = __builtin_bswap32(mem[i]);  // big-endian message words
    w[nw32] = 0x80000000u;
    w[15] = (uint32_t)(nw32 * 32);
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
        }
        const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = hh + S1 + ch + kSha256K[i] + wi;
        const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
        const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + mj;
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    out[0] = h[0] + a;
    out[1] = h[1] + b;
    out[2] = h[2] + c;
    out[3] = h[3] + d;
    out[4] = h[4] + e;
    out[5] = h[5] + f;
    out[6] = h[6] + g;
    out[7] = h[7] + hh;  // big-endian words of the digest
}

template <int NW, bool AM3, int FK>
__global__ __launch_bounds__(256) void k_ecdh(EccConst c, EcdhJob j) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= j.count) return;  // lanes never exchange data: an early exit is safe
    // the point (reduced once: every coordinate < 2^(32*NW) < 2p), to Montgomery form
    Fe<NW> x, y;
    if (j.pub) {
        x = load_be<NW>(j.pub + (size_t)i * 8 * NW);
        y = load_be<NW>(j.pub + (size_t)i * 8 * NW + 4 * NW);
    } else {
        x = fconst<NW>(c.px);
        y = fconst<NW>(c.py);
    }
    x = reduce_once<NW>(x.v, 0, c);
    y = reduce_once<NW>(y.v, 0, c);
    const Fe<NW> r2 = fconst<NW>(c.r2);
    const Fe<NW> xp = fmul<NW, FK>(x, r2, c), yp = fmul<NW, FK>(y, r2, c);
    // the scalar: regularize_k (uECC.c:902-913) -> k + n if that reaches 2^num_n_bits, else k + 2n
    uint32_t s[NW + 1];
    if (j.priv) {
        const Fe<NW> k = load_be<NW>(j.priv + (size_t)i * 4 * NW);
        uint32_t k0[NW + 1], k1[NW + 1], carry = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint64_t t = (uint64_t)k.v[w] + c.n[w] + carry;
            k0[w] = (uint32_t)t;
            carry = (uint32_t)(t >> 32);
        }
        k0[NW] = carry;
        carry = 0;
#pragma unroll
        for (int w = 0; w <= NW; w++) {
            const uint64_t t = (uint64_t)k0[w] + (w < NW ? c.n[w] : 0u) + carry;
            k1[w] = (uint32_t)t;
            carry = (uint32_t)(t >> 32);
        }
        const bool hi = k0[NW] & 1u;  // bit num_n_bits: num_n_bits == 32 * NW on all four curves
#pragma unroll
        for (int w = 0; w <= NW; w++) s[w] = hi ? k0[w] : k1[w];
    } else {
#pragma unroll
        for (int w = 0; w <= NW; w++) s[w] = c.k[w];
    }
    Fe<NW> rx, ry;
    ladder<NW, AM3, FK>(rx, ry, xp, yp, s, c.num_n_bits + 1, c);
    Fe<NW> one;
#pragma unroll
    for (int w = 0; w < NW; w++) one.v[w] = w == 0;
    rx = fmul<NW, FK>(rx, one, c);  // out of Montgomery form
    ry = fmul<NW, FK>(ry, one, c);
    uint32_t nz = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) nz |= rx.v[w] | ry.v[w];
    j.ok_out[i] = nz != 0;
    if (j.mode == ECDH_PUBLIC) {
        store_be<NW>(j.pub_out + (size_t)i * 8 * NW, rx);
        store_be<NW>(j.pub_out + (size_t)i * 8 * NW + 4 * NW, ry);
        return;
    }
    // secret = x, big-endian; key / iv as ECCKeyExchange::calcKey
    uint32_t sec[NW];  // the secret bytes as little-endian words (memory order)
#pragma unroll
    for (int w = 0; w < NW; w++) sec[w] = __builtin_bswap32(rx.v[NW - 1 - w]);
    uint32_t iv[4];
    md5_short(sec, NW, iv);
    uint32_t *ivo = reinterpret_cast<uint32_t *>(j.iv_out + (size_t)i * 16);
#pragma unroll
    for (int w = 0; w < 4; w++) ivo[w] = iv[w];
    uint32_t *ko = reinterpret_cast<uint32_t *>(j.key_out + (size_t)i * j.keylen);
    if (j.keylen == 16 || NW == 8) {
        for (int w = 0; w < j.keylen / 4; w++) ko[w] = sec[w];
    } else {
        uint32_t h[8];
        sha256_short(sec, NW, h);
#pragma unroll
        for (int w = 0; w < 8; w++) ko[w] = __builtin_bswap32(h[w]);
    }
}

// ---- host: curve table -----------------------------------------------------------------
// SEC 2 v2 domain parameters (big-endian hex).
struct CurveHex {
    EccCurveInfo info;
    const char *p, *n, *gx, *gy;
};
const CurveHex kCurves[ECC_NCURVES] = {
    {{"secp256k1", 8, 32, 256, false},
     "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F",
     "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141",
     "79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798",
     "483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8"},
    {{"secp256r1", 8, 32, 256, true},
     "FFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF",
     "FFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551",
     "6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296",
     "4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5"},
    {{"secp224r1", 7, 28, 224, true},
     "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF000000000000000000000001",
     "FFFFFFFFFFFFFFFFFFFFFFFFFFFF16A2E0B8F03E13DD29455C5C2A3D",
     "B70E0CBD6BB4BF7F321390B94A03C1D356C21122343280D6115C1D21",
     "BD376388B5F723FB4C22DFE6CD4375A05A07476444D5819985007E34"},
    {{"secp192r1", 6, 24, 192, true},
     "FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFFFFFFFFFFFF",
     "FFFFFFFFFFFFFFFFFFFFFFFF99DEF836146BC9B1B4D22831",
     "188DA80EB03090F67CBF20EB43A18800F4FF0AFD82FF1012",
     "07192B95FFC8DA78631011ED6B24CDD573F977A11E794811"},
};

void hex_limbs(const char *h, uint32_t out[8]) {
    memset(out, 0, 8 * sizeof(uint32_t));
    const int n = (int)strlen(h);
    for (int i = 0; i < n; i++) {
        const char ch = h[n - 1 - i];
        const uint32_t d = ch <= '9' ? (uint32_t)(ch - '0') : (uint32_t)((ch | 0x20) - 'a' + 10);
        out[i / 8] |= d << (4 * (i % 8));
    }
}

void be_to_limbs(const uint8_t *be, int nbytes, uint32_t *out, int nlimbs) {
    memset(out, 0, nlimbs * sizeof(uint32_t));
    for (int i = 0; i < nbytes; i++) out[i / 4] |= (uint32_t)be[nbytes - 1 - i] << (8 * (i % 4));
}

template <int NW, bool AM3, int FK>
void launch_nw(const EccConst &c, const EcdhJob &j, hipStream_t st) {
    hipLaunchKernelGGL((k_ecdh<NW, AM3, FK>), dim3((j.count + 255) / 256), dim3(256), 0, st, c, j);
}

}  // namespace

const EccCurveInfo &ecc_curve_info(int curve) { return kCurves[curve].info; }

bool ecc_fill_const(int curve, EccConst &c) {
    if (curve < 0 || curve >= ECC_NCURVES) return false;
    const CurveHex &h = kCurves[curve];
    memset(&c, 0, sizeof c);
    const int nw = h.info.nw;
    c.nw = nw;
    c.num_bytes = h.info.num_bytes;
    c.num_n_bits = h.info.num_n_bits;
    c.private_bytes = (h.info.num_n_bits + 7) / 8;
    if (c.num_n_bits != 32 * nw || c.num_bytes != 4 * nw) return false;  // the kernel relies on both
    hex_limbs(h.p, c.p);
    hex_limbs(h.n, c.n);
    hex_limbs(h.gx, c.px);
    hex_limbs(h.gy, c.py);
    uint32_t borrow = 2;  // pm2 = p - 2 (secp224r1's low limb is 1: the borrow runs on)
    for (int j = 0; j < 8; j++) {
        const uint64_t s = (uint64_t)c.p[j] - borrow;
        c.pm2[j] = (uint32_t)s;
        borrow = (uint32_t)(s >> 63);
    }
    uint32_t inv = 1;  // p^-1 mod 2^32 by Newton iteration
    for (int i = 0; i < 5; i++) inv *= 2u - c.p[0] * inv;
    c.n0inv = 0u - inv;
    // every kernel works in normal form (special-prime reduction): R = 1, so the Montgomery
    // conversions around the ladder are identities
    memset(c.r1, 0, sizeof c.r1);
    memset(c.r2, 0, sizeof c.r2);
    c.r1[0] = c.r2[0] = 1;
    return true;
}

void ecc_set_uniform_scalar(EccConst &c, const uint8_t *priv_be) {
    uint32_t k[9];
    be_to_limbs(priv_be, c.private_bytes, k, 9);
    uint32_t k0[9], k1[9], carry = 0;
    for (int w = 0; w < 9; w++) {
        const uint64_t t = (uint64_t)k[w] + (w < 8 ? c.n[w] : 0u) + carry;
        k0[w] = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
    }
    carry = 0;
    for (int w = 0; w < 9; w++) {
        const uint64_t t = (uint64_t)k0[w] + (w < 8 ? c.n[w] : 0u) + carry;
        k1[w] = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
    }
    const bool hi = (k0[c.num_n_bits >> 5] >> (c.num_n_bits & 31)) & 1u;
    memcpy(c.k, hi ? k0 : k1, sizeof c.k);
}

void ecc_set_uniform_point(EccConst &c, const uint8_t *pub_be) {
    be_to_limbs(pub_be, c.num_bytes, c.px, 8);
    be_to_limbs(pub_be + c.num_bytes, c.num_bytes, c.py, 8);
}

hipError_t launch_ecdh(const EccConst &c, const EcdhJob &j, int curve, hipStream_t st) {
    if (j.count == 0) return hipSuccess;
    // every curve in normal form with its special-prime reduction (round 2/3; the generic
    // Montgomery-form kernel was the A/B baseline and is no longer built)
    switch (curve) {
        case ECC_SECP256K1: launch_nw<8, false, FK_K1>(c, j, st); break;
        case ECC_SECP256R1: launch_nw<8, true, FK_P256>(c, j, st); break;
        case ECC_SECP224R1: launch_nw<7, true, FK_P224>(c, j, st); break;
        case ECC_SECP192R1: launch_nw<6, true, FK_P192>(c, j, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
