// bs_aes.hpp -- bitsliced AES forward cipher for gfx950 (32 blocks per lane, no LDS).
//
// The T-table kernels are bound by LDS lookup issue (224 ds_read_b32 per AES-256
// block) while two thirds of VALU issue stays idle.  This cipher uses VALU only: the
// state of 32 blocks is held as 128 words, S[32*d + p] = bit p of state word d of
// each of the 32 blocks (bit j of the word = block j).  Word d, bit p is byte
// 4d + p/8, bit p%8 of the block, i.e. byte (row p/8, column d) of the FIPS-197 state.
//
//   SubBytes   : generated tower-field circuit (bs_sbox.inc, 111 v_bitop3 ops / byte)
//   ShiftRows  : register renaming (output bytes written to their shifted slots)
//   MixColumns : b_i = a_i ^ t ^ xtime(a_i ^ a_{i+1}), t = a0^a1^a2^a3, with the round
//                key folded into the last 3-input XOR
//   AddRoundKey: masks -(bit p of rk word d), from SGPR round keys
//
// Output is bit-identical to aes_encrypt_block / base/rijndael.c:852-959 (tests).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aes_common.hpp"

namespace fpnn_aes {

#define BOP3(a, b, c, t) __builtin_amdgcn_bitop3_b32((a), (b), (c), (t))
#include "bs_sbox.inc"

// One bit-level stage of the 32x32 transpose: swap the off-diagonal SxS sub-blocks.
template <int SH, uint32_t MLO>
__device__ __forceinline__ void bs_transpose_stage(uint32_t *a) {
#pragma unroll
    for (int j = 0; j < 32; j++) {
        if (j & SH) continue;
        const uint32_t x = a[j], y = a[j + SH];
        a[j] = BOP3(MLO, x, y << SH, 0xca);       // MLO ? x : y<<SH
        a[j + SH] = BOP3(MLO, x >> SH, y, 0xca);  // MLO ? x>>SH : y
    }
}

// In-place transpose of the 32x32 bit matrix a[j] (row j = word j).  Involution.
__device__ __forceinline__ void bs_transpose32(uint32_t *a) {
#pragma unroll
    for (int j = 0; j < 16; j++) {  // 16-bit blocks: one v_perm per output word
        const uint32_t x = a[j], y = a[j + 16];
        a[j] = __builtin_amdgcn_perm(y, x, 0x05040100u);
        a[j + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
    }
#pragma unroll
    for (int j = 0; j < 32; j++) {  // 8-bit blocks
        if (j & 8) continue;
        const uint32_t x = a[j], y = a[j + 8];
        a[j] = __builtin_amdgcn_perm(y, x, 0x06020400u);
        a[j + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    }
    bs_transpose_stage<4, 0x0F0F0F0Fu>(a);
    bs_transpose_stage<2, 0x33333333u>(a);
    bs_transpose_stage<1, 0x55555555u>(a);
}

// AddRoundKey with the 4 round-key words of one round (block byte order).
__device__ __forceinline__ void bs_add_round_key(uint32_t *S, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
#pragma unroll
    for (int p = 0; p < 32; p++) {
        S[p] ^= 0u - ((k0 >> p) & 1u);
        S[32 + p] ^= 0u - ((k1 >> p) & 1u);
        S[64 + p] ^= 0u - ((k2 >> p) & 1u);
        S[96 + p] ^= 0u - ((k3 >> p) & 1u);
    }
}

// byte (row r, column c) of the state, bit k
#define BS_IDX(r, c, k) (32 * (c) + 8 * (r) + (k))

// SubBytes + ShiftRows: new[r][c] = S(old[r][(c + r) & 3]).
__device__ __forceinline__ void bs_sub_shift(uint32_t *S) {
    uint32_t T[128];
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t x[8], y[8];
#pragma unroll
            for (int k = 0; k < 8; k++) x[k] = S[BS_IDX(r, (c + r) & 3, k)];
            bs_sbox(x, y);
#pragma unroll
            for (int k = 0; k < 8; k++) T[BS_IDX(r, c, k)] = y[k];
        }
    }
#pragma unroll
    for (int i = 0; i < 128; i++) S[i] = T[i];
}

// MixColumns fused with AddRoundKey (round key words k[c]).
__device__ __forceinline__ void bs_mix_add(uint32_t *S, const uint32_t k[4]) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a[4][8], t[8], u[4][8];
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int b = 0; b < 8; b++) a[r][b] = S[BS_IDX(r, c, b)];
#pragma unroll
        for (int b = 0; b < 8; b++) t[b] = BOP3(a[0][b], a[1][b], a[2][b], 0x96) ^ a[3][b];
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int b = 0; b < 8; b++) u[r][b] = a[r][b] ^ a[(r + 1) & 3][b];
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint32_t key = 0u - ((k[c] >> (8 * r + b)) & 1u);
                // xtime(u)[b] = u[b-1] (u[7] for b = 0), plus u[7] for b in {1, 3, 4}
                const uint32_t xt = b == 0 ? u[r][7] : u[r][b - 1];
                const uint32_t v = BOP3(a[r][b], t[b], xt, 0x96);
                S[BS_IDX(r, c, b)] = (b == 1 || b == 3 || b == 4) ? BOP3(v, u[r][7], key, 0x96) : (v ^ key);
            }
        }
    }
}

// Bitsliced AES encryption of 32 blocks in place.  rk: round keys in block byte order
// (DevKey::rk, uniform across the wave -> scalar loads inside the round loop).
template <int NR>
__device__ __forceinline__ void bs_aes_encrypt(uint32_t *S, const uint32_t *__restrict__ rk) {
    bs_add_round_key(S, rk[0], rk[1], rk[2], rk[3]);
#pragma unroll 1
    for (int r = 1; r < NR; r++) {
        bs_sub_shift(S);
        const uint32_t k[4] = {rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3]};
        bs_mix_add(S, k);
    }
    bs_sub_shift(S);
    bs_add_round_key(S, rk[4 * NR], rk[4 * NR + 1], rk[4 * NR + 2], rk[4 * NR + 3]);
}

}  // namespace fpnn_aes
