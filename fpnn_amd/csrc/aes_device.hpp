// aes_device.hpp -- CDNA4 (gfx950) device building blocks for the AES-CFB kernels.
//
// LDS table image (128 KiB per workgroup, one workgroup per CU):
//   The four forward T-tables T0..T3 (little-endian form of the reference's
//   Te0..Te3, base/rijndael.c:8-278) are replicated 32 times so that lane l reads
//   copy (l & 31), which lives in bank (l & 31): every ds_read_b32 of a wave is
//   bank-conflict free whatever the table indices are.
//     table k = 2*r + h  (region r in {0,1}, half h in {0,1})
//     entry (x, copy c) at byte  r*65536 + x*256 + h*128 + c*4
//   The byte address of a lookup is then a single v_perm_b32:
//     addr = { lanebase.b0, state.byte_j, lanebase.b2, 0 }   (lanebase = c*4 | r<<16)
//   and the table half is the ds_read immediate offset (0 or 128).
//
// Round function (T-table form of FIPS-197, as base/rijndael.c:871-925): per output
// column 4 lookups + round key, folded with two v_bitop3_b32 (3-input xor).  Per
// 16-byte block and round: 16 v_perm + 16 ds_read_b32 + 8 v_bitop3.  The final round
// takes the S-box byte out of T0/T2 entries (the reference uses Te4, :931-958).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aes_common.hpp"

namespace fpnn_aes {

constexpr uint32_t kLdsBytes = 131072;  // 4 tables x 256 entries x 32 copies x 4 B

__device__ __forceinline__ uint32_t rotl32(uint32_t v, uint32_t n) { return __builtin_rotateleft32(v, n); }

// Fill the replicated table image from the 1 KiB T0 (little-endian) source.
__device__ __forceinline__ void lds_fill_tables(uint4 *lds4, const uint32_t *__restrict__ t0le) {
    for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += blockDim.x) {
        // uint4 index i covers copies c = 4*(i&7) .. +3 of entry (r, x, h)
        const uint32_t r = i >> 12, x = (i >> 4) & 255, h = (i >> 3) & 1;
        const uint32_t v = rotl32(__ldg(t0le + x), 8u * (2u * r + h));
        lds4[i] = make_uint4(v, v, v, v);
    }
}

constexpr uint32_t sel(uint32_t j) { return 0x0c060004u | (j << 8); }

struct LaneBase {
    uint32_t lb0, lb1;
    __device__ __forceinline__ LaneBase() {
        lb0 = (threadIdx.x & 31u) << 2;
        lb1 = lb0 | 0x10000u;
    }
};

__device__ __forceinline__ uint32_t lds_word(const char *lds, uint32_t addr, uint32_t imm) {
    return *reinterpret_cast<const uint32_t *>(lds + addr + imm);
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Round keys for NR rounds (block byte order).  Loaded from a uniform pointer they
// live in SGPRs; from a per-lane pointer in VGPRs.
template <int NR>
struct RoundKeys {
    uint32_t k[4 * (NR + 1)];
};

template <int NR>
__device__ __forceinline__ RoundKeys<NR> load_round_keys(const DevKey *key) {
    RoundKeys<NR> r;
    const uint4 *p = reinterpret_cast<const uint4 *>(key->rk);
#pragma unroll
    for (int i = 0; i <= NR; i++) {
        const uint4 v = p[i];
        r.k[4 * i + 0] = v.x;
        r.k[4 * i + 1] = v.y;
        r.k[4 * i + 2] = v.z;
        r.k[4 * i + 3] = v.w;
    }
    return r;
}

template <int NR>
__device__ __forceinline__ uint4 aes_encrypt_block(uint4 in, const RoundKeys<NR> &rk, const char *lds,
                                                   const LaneBase &lb) {
    uint32_t s0 = in.x ^ rk.k[0], s1 = in.y ^ rk.k[1], s2 = in.z ^ rk.k[2], s3 = in.w ^ rk.k[3];
#define FPNN_T0(w) lds_word(lds, __builtin_amdgcn_perm(lb.lb0, (w), sel(0)), 0)
#define FPNN_T1(w) lds_word(lds, __builtin_amdgcn_perm(lb.lb0, (w), sel(1)), 128)
#define FPNN_T2(w) lds_word(lds, __builtin_amdgcn_perm(lb.lb1, (w), sel(2)), 0)
#define FPNN_T3(w) lds_word(lds, __builtin_amdgcn_perm(lb.lb1, (w), sel(3)), 128)
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = xor3(xor3(FPNN_T0(s0), FPNN_T1(s1), FPNN_T2(s2)), FPNN_T3(s3), rk.k[4 * r + 0]);
        const uint32_t t1 = xor3(xor3(FPNN_T0(s1), FPNN_T1(s2), FPNN_T2(s3)), FPNN_T3(s0), rk.k[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(FPNN_T0(s2), FPNN_T1(s3), FPNN_T2(s0)), FPNN_T3(s1), rk.k[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(FPNN_T0(s3), FPNN_T1(s0), FPNN_T2(s1)), FPNN_T3(s2), rk.k[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
#undef FPNN_T0
#undef FPNN_T1
#undef FPNN_T2
#undef FPNN_T3
    // Final round: S(x) sits in bytes 1,2 of T0 entries and bytes 0,3 of T2 entries.
#define FPNN_S0(w) (lds_word(lds, __builtin_amdgcn_perm(lb.lb1, (w), sel(0)), 0) & 0x000000ffu)
#define FPNN_S1(w) (lds_word(lds, __builtin_amdgcn_perm(lb.lb0, (w), sel(1)), 0) & 0x0000ff00u)
#define FPNN_S2(w) (lds_word(lds, __builtin_amdgcn_perm(lb.lb0, (w), sel(2)), 0) & 0x00ff0000u)
#define FPNN_S3(w) (lds_word(lds, __builtin_amdgcn_perm(lb.lb1, (w), sel(3)), 0) & 0xff000000u)
    uint4 o;
    o.x = (FPNN_S0(s0) | FPNN_S1(s1) | FPNN_S2(s2) | FPNN_S3(s3)) ^ rk.k[4 * NR + 0];
    o.y = (FPNN_S0(s1) | FPNN_S1(s2) | FPNN_S2(s3) | FPNN_S3(s0)) ^ rk.k[4 * NR + 1];
    o.z = (FPNN_S0(s2) | FPNN_S1(s3) | FPNN_S2(s0) | FPNN_S3(s1)) ^ rk.k[4 * NR + 2];
    o.w = (FPNN_S0(s3) | FPNN_S1(s0) | FPNN_S2(s1) | FPNN_S3(s2)) ^ rk.k[4 * NR + 3];
#undef FPNN_S0
#undef FPNN_S1
#undef FPNN_S2
#undef FPNN_S3
    return o;
}

// ---------------------------------------------------------------------------
// 16-byte block helpers.  Interior blocks use (possibly unaligned) dwordx4 accesses;
// edge blocks of a segment use byte accesses restricted to the segment so that no
// byte outside [in, in+len) is read and none outside [out, out+len) is written.

typedef uint4 __attribute__((aligned(1))) uint4_u;

// gfx950 global dwordx4 accesses tolerate any byte alignment (unaligned-access mode);
// the type above makes hipcc emit one global_load/store_dwordx4 regardless.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Walign-mismatch"
__device__ __forceinline__ uint4 load16(const uint8_t *p) { return *reinterpret_cast<const uint4_u *>(p); }
__device__ __forceinline__ void store16(uint8_t *p, uint4 v) { *reinterpret_cast<uint4_u *>(p) = v; }
#pragma clang diagnostic pop

__device__ __forceinline__ uint4 operator^(uint4 a, uint4 b) {
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__device__ __forceinline__ uint32_t word_of(const uint4 &v, int d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// byte j (0..15) of a block
__device__ __forceinline__ uint32_t byte_of(const uint4 &v, int j) { return (word_of(v, j >> 2) >> (8 * (j & 3))) & 0xffu; }

// mask with bytes [lo, hi) set; lo, hi in [0, 16]
__device__ __forceinline__ uint4 byte_mask(int lo, int hi) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++)
        w[j >> 2] |= (j >= lo && j < hi) ? (0xffu << (8 * (j & 3))) : 0u;
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint4 select_bytes(uint4 m, uint4 a, uint4 b) {  // (a & m) | (b & ~m)
    return make_uint4((a.x & m.x) | (b.x & ~m.x), (a.y & m.y) | (b.y & ~m.y), (a.z & m.z) | (b.z & ~m.z),
                      (a.w & m.w) | (b.w & ~m.w));
}

// block whose byte j = base[j] for j in [lo, hi), 0 elsewhere (base may point outside
// the buffer; only bytes inside [lo, hi) are dereferenced)
__device__ __forceinline__ uint4 load_bytes(const uint8_t *base, int lo, int hi) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (j >= lo && j < hi) w[j >> 2] |= (uint32_t)base[j] << (8 * (j & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_bytes(uint8_t *base, const uint4 &v, int lo, int hi) {
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (j >= lo && j < hi) base[j] = (uint8_t)byte_of(v, j);
}

// Lane l receives lane (l-1)'s value (lane 0 receives `fill`): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}

__device__ __forceinline__ uint4 wave_shr1(const uint4 &v) {
    return make_uint4(wave_shr1(v.x, 0u), wave_shr1(v.y, 0u), wave_shr1(v.z, 0u), wave_shr1(v.w, 0u));
}

// floor(g / d) for g, d < 2^32 with magic = ceil(2^64 / d)
__device__ __forceinline__ uint32_t fast_div(uint32_t g, uint64_t magic) {
    return (uint32_t)__umul64hi((uint64_t)g, magic);
}

}  // namespace fpnn_aes
