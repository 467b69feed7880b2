// coop.hpp -- the quad-per-chain CFB round (K2c / K2q / K2h's quad session): lane q of
// a 4-lane quad owns state column q and the quad sums the T-table contributions with
// DPP quad_perm XORs; plus the per-lane word byte helpers those kernels use.
#pragma once

#include "segments.hpp"

namespace fpnn_aes {

// value held by lane (q + SHIFT) & 3 of this lane's quad.  bound_ctrl: every lane has a
// source under quad_perm, so no "old" value is needed (update_dpp with old = 0 costs a
// v_mov per call to materialise it -- 3 of the 12 VALU of a K2c round).
template <int SHIFT>
__device__ __forceinline__ uint32_t quad_from(uint32_t v) {
    constexpr int ctl = ((0 + SHIFT) & 3) | (((1 + SHIFT) & 3) << 2) | (((2 + SHIFT) & 3) << 4) | (((3 + SHIFT) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctl, 0xf, 0xf, true);
}

// XOR of a and the value b holds in lane (q + SHIFT) & 3: one v_xor_b32 with a DPP
// quad_perm source (the mov_dpp folds into the xor).
template <int SHIFT>
__device__ __forceinline__ uint32_t xor_quad_from(uint32_t a, uint32_t b) {
    return a ^ quad_from<SHIFT>(b);
}

// Round structure: lane q looks up ITS OWN four bytes -- T0[b0] feeds output column q,
// T1[b1] column q-1, T2[b2] column q-2, T3[b3] column q-3 -- and the quad then sums
// the contributions with DPP-sourced XORs.  Per lane and round: 4 v_perm + 4 ds_read
// + 3 DPP ops + 1 v_bitop3 = 8 VALU, and every DPP operand is an LDS result or a round
// key, never a fresh VALU result, so no hazard wait states (moving the state words to
// the neighbours first costs 9 VALU plus an s_nop per round).
template <int NR, int NT>
__device__ __forceinline__ uint32_t aes_encrypt_column(uint32_t sq, const uint32_t *rkq, const Tables4<NT> &T) {
    uint32_t s0 = sq ^ rkq[0];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = T.template t<0>(s0), t1 = T.template t<1>(s0), t2 = T.template t<2>(s0),
                       t3 = T.template t<3>(s0);
        // three independent DPP ops whose other operand is an LDS result or a round key
        // (a chain of DPP xors would need 2 wait states between them), then one xor3
        s0 = xor3(xor_quad_from<1>(t0, t1), xor_quad_from<2>(rkq[r], t2), quad_from<3>(t3));
    }
    // final round: S(byte j) of the own word, masked to byte j, summed the same way
    const uint32_t m0 = T.template sraw<0>(s0) & 0x000000ffu, m1 = T.template sraw<1>(s0) & 0x0000ff00u,
                   m2 = T.template sraw<2>(s0) & 0x00ff0000u, m3 = T.template sraw<3>(s0) & 0xff000000u;
    return xor3(xor_quad_from<1>(m0, m1), xor_quad_from<2>(rkq[NR], m2), quad_from<3>(m3));
}

// The same rounds for a serial CFB chain with the chain's two XORs folded into the round
// keys: sw = C_{i-1} ^ rk[0] (the whitened state, already), fin = rk[NR] ^ P_i ^ rk[0];
// returns C_i ^ rk[0], the next block's whitened state -- the ciphertext C_i = result ^
// rk[0] and the keystream E(C_{i-1}) = C_i ^ P_i are side computations off the chain.  Two
// dependent VALU ops fewer per block than aes_encrypt_column + (k ^ P) + (C ^ rk[0]).
template <int NR, int NT>
__device__ __forceinline__ uint32_t aes_chain_column(uint32_t sw, const uint32_t *rkq, uint32_t fin,
                                                     const Tables4<NT> &T) {
    uint32_t s0 = sw;
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = T.template t<0>(s0), t1 = T.template t<1>(s0), t2 = T.template t<2>(s0),
                       t3 = T.template t<3>(s0);
        s0 = xor3(xor_quad_from<1>(t0, t1), xor_quad_from<2>(rkq[r], t2), quad_from<3>(t3));
    }
    const uint32_t m0 = T.template sraw<0>(s0) & 0x000000ffu, m1 = T.template sraw<1>(s0) & 0x0000ff00u,
                   m2 = T.template sraw<2>(s0) & 0x00ff0000u, m3 = T.template sraw<3>(s0) & 0xff000000u;
    return xor3(xor_quad_from<1>(m0, m1), xor_quad_from<2>(fin, m2), quad_from<3>(m3));
}

typedef uint32_t __attribute__((aligned(1))) uint32_u;

// bytes [lo, hi) of this lane's word (word covers block bytes [4q, 4q+4))
__device__ __forceinline__ uint32_t load_word_bytes(const uint8_t *p, int lo, int hi) {
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (j >= lo && j < hi) w |= (uint32_t)p[j] << (8 * j);
    return w;
}

__device__ __forceinline__ void store_word_bytes(uint8_t *p, uint32_t w, int lo, int hi) {
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (j >= lo && j < hi) p[j] = (uint8_t)(w >> (8 * j));
}

__device__ __forceinline__ uint32_t word_mask(int lo, int hi) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) m |= (j >= lo && j < hi) ? (0xffu << (8 * j)) : 0u;
    return m;
}

}  // namespace fpnn_aes
