// aes_device.hpp -- CDNA4 (gfx950) device building blocks for the AES-CFB kernels.
//
// LDS table image:
//   The forward T-tables (little-endian form of the reference's Te0..Te3,
//   base/rijndael.c:8-278) are replicated 32 times so that lane l reads copy
//   (l & 31), which lives in bank (l & 31): every ds_read_b32 of a wave is
//   bank-conflict free whatever the table indices are.
//     table k = 2*r + h  (region r in {0,1}, half h in {0,1}; NT = 4 layout)
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

// Two LDS layouts (template parameter NT = number of distinct tables in LDS):
//   NT = 4: T0..T3, 128 KiB -> one 1024-thread workgroup per CU (4 waves/SIMD).
//   NT = 2: T0 and T2 only, 64 KiB -> two workgroups per CU (8 waves/SIMD);
//           T1 = rotl8(T0) and T3 = rotl8(T2) cost one v_alignbit each.
template <int NT>
struct Lds {
    static constexpr uint32_t kBytes = NT == 4 ? 131072u : 65536u;
    static constexpr int kBlocksPerCU = NT == 4 ? 1 : 2;
};

__device__ __forceinline__ uint32_t rotl32(uint32_t v, uint32_t n) { return __builtin_rotateleft32(v, n); }

// Fill the replicated table image from the 1 KiB T0 (little-endian) source.
template <int NT>
__device__ __forceinline__ void lds_fill_tables(uint4 *lds4, const uint32_t *__restrict__ t0le) {
    for (uint32_t i = threadIdx.x; i < Lds<NT>::kBytes / 16; i += blockDim.x) {
        // uint4 index i covers copies c = 4*(i&7) .. +3 of entry (r, x, h)
        const uint32_t r = i >> 12, x = (i >> 4) & 255, h = (i >> 3) & 1;
        const uint32_t k = NT == 4 ? 2u * r + h : 2u * h;  // which T_k this half holds
        const uint32_t v = rotl32(__ldg(t0le + x), 8u * k);
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

// T_j lookup of byte j of w (j = 0..3) and the final-round S-box byte placed at byte j.
template <int NT>
struct Tables4 {
    const char *lds;
    LaneBase lb;
    template <int J>
    __device__ __forceinline__ uint32_t t(uint32_t w) const {
        if (NT == 4) {
            const uint32_t base = (J < 2) ? lb.lb0 : lb.lb1;
            return lds_word(lds, __builtin_amdgcn_perm(base, w, sel(J)), (J & 1) ? 128 : 0);
        } else {  // T0 at +0, T2 at +128; odd tables by rotation
            const uint32_t v = lds_word(lds, __builtin_amdgcn_perm(lb.lb0, w, sel(J)), (J >= 2) ? 128 : 0);
            return (J & 1) ? rotl32(v, 8) : v;
        }
    }
    // Raw final-round entry for byte j of w: S(byte j) sits at byte j of it (T0 entries
    // hold S in bytes 1,2; T2 entries in bytes 0,3), the other bytes are junk.
    template <int J>
    __device__ __forceinline__ uint32_t sraw(uint32_t w) const {
        constexpr bool from_t2 = (J == 0 || J == 3);
        if (NT == 4) {
            const uint32_t base = from_t2 ? lb.lb1 : lb.lb0;
            return lds_word(lds, __builtin_amdgcn_perm(base, w, sel(J)), 0);
        } else {
            return lds_word(lds, __builtin_amdgcn_perm(lb.lb0, w, sel(J)), from_t2 ? 128 : 0);
        }
    }
    // S(byte j of w) at byte j, zero elsewhere
    template <int J>
    __device__ __forceinline__ uint32_t s(uint32_t w) const {
        return sraw<J>(w) & (0xffu << (8 * J));
    }
    // Final-round output word: S(a.b0) | S(b.b1) << 8 | S(c.b2) << 16 | S(d.b3) << 24, ^ k.
    // Two v_perm gather the four S bytes into disjoint halves, one v_bitop3 XORs them
    // with the round key (3 VALU instead of 4 masks, 3 ORs and an XOR).
    __device__ __forceinline__ uint32_t last(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        const uint32_t lo = __builtin_amdgcn_perm(sraw<1>(b), sraw<0>(a), 0x0c0c0500u);
        const uint32_t hi = __builtin_amdgcn_perm(sraw<3>(d), sraw<2>(c), 0x07020c0cu);
        return xor3(lo, hi, k);
    }
};

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

template <int NR, int NT>
__device__ __forceinline__ uint4 aes_encrypt_block(uint4 in, const RoundKeys<NR> &rk, const Tables4<NT> &T) {
    uint32_t s0 = in.x ^ rk.k[0], s1 = in.y ^ rk.k[1], s2 = in.z ^ rk.k[2], s3 = in.w ^ rk.k[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t t0 = xor3(xor3(T.template t<0>(s0), T.template t<1>(s1), T.template t<2>(s2)),
                                 T.template t<3>(s3), rk.k[4 * r + 0]);
        const uint32_t t1 = xor3(xor3(T.template t<0>(s1), T.template t<1>(s2), T.template t<2>(s3)),
                                 T.template t<3>(s0), rk.k[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(T.template t<0>(s2), T.template t<1>(s3), T.template t<2>(s0)),
                                 T.template t<3>(s1), rk.k[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(T.template t<0>(s3), T.template t<1>(s0), T.template t<2>(s1)),
                                 T.template t<3>(s2), rk.k[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    uint4 o;
    o.x = T.last(s0, s1, s2, s3, rk.k[4 * NR + 0]);
    o.y = T.last(s1, s2, s3, s0, rk.k[4 * NR + 1]);
    o.z = T.last(s2, s3, s0, s1, rk.k[4 * NR + 2]);
    o.w = T.last(s3, s0, s1, s2, rk.k[4 * NR + 3]);
    return o;
}

// aes_encrypt_block with each round's 16 lookups issued before any of them is folded
// (a scheduling fence after the loads): where the surrounding kernel holds many live
// registers the compiler otherwise interleaves loads and XORs two or three at a time,
// leaving the LDS pipe nearly empty per wave.
template <int NR, int NT>
__device__ __forceinline__ uint4 aes_encrypt_block_fenced(uint4 in, const RoundKeys<NR> &rk, const Tables4<NT> &T) {
    uint32_t s0 = in.x ^ rk.k[0], s1 = in.y ^ rk.k[1], s2 = in.z ^ rk.k[2], s3 = in.w ^ rk.k[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t a0 = T.template t<0>(s0), a1 = T.template t<1>(s1), a2 = T.template t<2>(s2), a3 = T.template t<3>(s3);
        const uint32_t b0 = T.template t<0>(s1), b1 = T.template t<1>(s2), b2 = T.template t<2>(s3), b3 = T.template t<3>(s0);
        const uint32_t c0 = T.template t<0>(s2), c1 = T.template t<1>(s3), c2 = T.template t<2>(s0), c3 = T.template t<3>(s1);
        const uint32_t d0 = T.template t<0>(s3), d1 = T.template t<1>(s0), d2 = T.template t<2>(s1), d3 = T.template t<3>(s2);
        __builtin_amdgcn_sched_barrier(0);
        s0 = xor3(xor3(a0, a1, a2), a3, rk.k[4 * r + 0]);
        s1 = xor3(xor3(b0, b1, b2), b3, rk.k[4 * r + 1]);
        s2 = xor3(xor3(c0, c1, c2), c3, rk.k[4 * r + 2]);
        s3 = xor3(xor3(d0, d1, d2), d3, rk.k[4 * r + 3]);
    }
    uint4 o;
    o.x = T.last(s0, s1, s2, s3, rk.k[4 * NR + 0]);
    o.y = T.last(s1, s2, s3, s0, rk.k[4 * NR + 1]);
    o.z = T.last(s2, s3, s0, s1, rk.k[4 * NR + 2]);
    o.w = T.last(s3, s0, s1, s2, rk.k[4 * NR + 3]);
    return o;
}

// aes_encrypt_block with per-lane round keys read from LDS, one 16-byte row per round
// (krow[r] = round key r): lanes of a wave that use different keys (K1r chunks spanning
// several connections' frames) run one pass instead of one pass per key.  A row read is
// one ds_read_b128 per round beside the round's 16 lookups.
template <int NR, int NT, bool FENCE>
__device__ __forceinline__ uint4 aes_encrypt_block_ldsk(uint4 in, const uint4 *krow, const Tables4<NT> &T) {
    const uint4 k0 = krow[0];
    uint32_t s0 = in.x ^ k0.x, s1 = in.y ^ k0.y, s2 = in.z ^ k0.z, s3 = in.w ^ k0.w;
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t a0 = T.template t<0>(s0), a1 = T.template t<1>(s1), a2 = T.template t<2>(s2), a3 = T.template t<3>(s3);
        const uint32_t b0 = T.template t<0>(s1), b1 = T.template t<1>(s2), b2 = T.template t<2>(s3), b3 = T.template t<3>(s0);
        const uint32_t c0 = T.template t<0>(s2), c1 = T.template t<1>(s3), c2 = T.template t<2>(s0), c3 = T.template t<3>(s1);
        const uint32_t d0 = T.template t<0>(s3), d1 = T.template t<1>(s0), d2 = T.template t<2>(s1), d3 = T.template t<3>(s2);
        const uint4 kr = krow[r];
        if (FENCE) __builtin_amdgcn_sched_barrier(0);
        s0 = xor3(xor3(a0, a1, a2), a3, kr.x);
        s1 = xor3(xor3(b0, b1, b2), b3, kr.y);
        s2 = xor3(xor3(c0, c1, c2), c3, kr.z);
        s3 = xor3(xor3(d0, d1, d2), d3, kr.w);
    }
    const uint4 kn = krow[NR];
    uint4 o;
    o.x = T.last(s0, s1, s2, s3, kn.x);
    o.y = T.last(s1, s2, s3, s0, kn.y);
    o.z = T.last(s2, s3, s0, s1, kn.z);
    o.w = T.last(s3, s0, s1, s2, kn.w);
    return o;
}

template <bool FENCE, int NR, int NT>
__device__ __forceinline__ uint4 aes_encrypt_block_sel(uint4 in, const RoundKeys<NR> &rk, const Tables4<NT> &T) {
    return FENCE ? aes_encrypt_block_fenced<NR, NT>(in, rk, T) : aes_encrypt_block<NR, NT>(in, rk, T);
}

// M independent blocks under one key, round-interleaved: round r of every block is
// issued before round r+1 of any, in ONE basic block, so a wave has 16*M LDS lookups
// in flight per round instead of 16 and the LDS pipe is fed while the VALU folds the
// previous block's lookups.  (Separate aes_encrypt_block calls end up serialized by
// the compiler when control flow sits between them.)
template <int NR, int NT, int M, bool FENCE = false>
__device__ __forceinline__ void aes_encrypt_blocks(uint4 (&st)[M], const RoundKeys<NR> &rk, const Tables4<NT> &T) {
    uint32_t s[M][4];
#pragma unroll
    for (int m = 0; m < M; m++) {
        s[m][0] = st[m].x ^ rk.k[0];
        s[m][1] = st[m].y ^ rk.k[1];
        s[m][2] = st[m].z ^ rk.k[2];
        s[m][3] = st[m].w ^ rk.k[3];
    }
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t[M][4];
        if (FENCE) {  // every lookup of the round issued before any fold (see aes_encrypt_block_fenced)
            uint32_t l[M][4][4];
#pragma unroll
            for (int m = 0; m < M; m++)
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    l[m][c][0] = T.template t<0>(s[m][c]);
                    l[m][c][1] = T.template t<1>(s[m][(c + 1) & 3]);
                    l[m][c][2] = T.template t<2>(s[m][(c + 2) & 3]);
                    l[m][c][3] = T.template t<3>(s[m][(c + 3) & 3]);
                }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < M; m++)
#pragma unroll
                for (int c = 0; c < 4; c++)
                    t[m][c] = xor3(xor3(l[m][c][0], l[m][c][1], l[m][c][2]), l[m][c][3], rk.k[4 * r + c]);
        } else {
#pragma unroll
            for (int m = 0; m < M; m++) {
#pragma unroll
                for (int c = 0; c < 4; c++)
                    t[m][c] = xor3(xor3(T.template t<0>(s[m][c]), T.template t<1>(s[m][(c + 1) & 3]),
                                        T.template t<2>(s[m][(c + 2) & 3])),
                                   T.template t<3>(s[m][(c + 3) & 3]), rk.k[4 * r + c]);
            }
        }
#pragma unroll
        for (int m = 0; m < M; m++)
#pragma unroll
            for (int c = 0; c < 4; c++) s[m][c] = t[m][c];
    }
#pragma unroll
    for (int m = 0; m < M; m++) {
        st[m].x = T.last(s[m][0], s[m][1], s[m][2], s[m][3], rk.k[4 * NR + 0]);
        st[m].y = T.last(s[m][1], s[m][2], s[m][3], s[m][0], rk.k[4 * NR + 1]);
        st[m].z = T.last(s[m][2], s[m][3], s[m][0], s[m][1], rk.k[4 * NR + 2]);
        st[m].w = T.last(s[m][3], s[m][0], s[m][1], s[m][2], rk.k[4 * NR + 3]);
    }
}

// ---------------------------------------------------------------------------
// Inverse cipher (base/rijndael.c:961-1068, rijndael_decrypt) for the rest of the
// rijndael.h surface (ECB / CBC decrypt).  The LDS image is the same layout filled from
// Td0 (td0le) instead of Te0, followed by the inverse S-box packed four entries per word
// and replicated 32x: entry x of copy c at byte kIsboxBase + (x & ~3) * 32 + c * 4 + (x & 3),
// so lane l reads bank l & 31 -- conflict-free -- for 8 KiB instead of 32.
constexpr uint32_t kIsboxBase = 131072u;
constexpr uint32_t kIsboxBytes = 8192u;

__device__ __forceinline__ void lds_fill_isbox(uint32_t *lds_words, const uint8_t *__restrict__ isbox) {
    for (uint32_t i = threadIdx.x; i < kIsboxBytes / 4; i += blockDim.x) {
        const uint32_t q = i >> 5;  // group of four entries; copy = i & 31
        lds_words[(kIsboxBase >> 2) + i] = (uint32_t)isbox[4 * q] | ((uint32_t)isbox[4 * q + 1] << 8) |
                                           ((uint32_t)isbox[4 * q + 2] << 16) | ((uint32_t)isbox[4 * q + 3] << 24);
    }
}

// inverse S-box of byte j of w, placed at byte k of the result
template <int J, int K>
__device__ __forceinline__ uint32_t isb(const char *lds, uint32_t lb0, uint32_t w) {
    const uint32_t x = (w >> (8 * J)) & 0xffu;
    const uint32_t v = *reinterpret_cast<const uint8_t *>(lds + kIsboxBase + ((x & ~3u) << 5) + (x & 3u) + lb0);
    return v << (8 * K);
}

// One block through the inverse cipher with the decryption schedule rk (block byte
// order, the reference's setup_decrypt rk[] byte-swapped).  T holds Td0..Td3.
template <int NR, int NT>
__device__ __forceinline__ uint4 aes_decrypt_block(uint4 in, const RoundKeys<NR> &rk, const Tables4<NT> &T) {
    uint32_t s0 = in.x ^ rk.k[0], s1 = in.y ^ rk.k[1], s2 = in.z ^ rk.k[2], s3 = in.w ^ rk.k[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {  // column c takes rows 0..3 from columns c, c-1, c-2, c-3
        const uint32_t t0 = xor3(xor3(T.template t<0>(s0), T.template t<1>(s3), T.template t<2>(s2)),
                                 T.template t<3>(s1), rk.k[4 * r + 0]);
        const uint32_t t1 = xor3(xor3(T.template t<0>(s1), T.template t<1>(s0), T.template t<2>(s3)),
                                 T.template t<3>(s2), rk.k[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(T.template t<0>(s2), T.template t<1>(s1), T.template t<2>(s0)),
                                 T.template t<3>(s3), rk.k[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(T.template t<0>(s3), T.template t<1>(s2), T.template t<2>(s1)),
                                 T.template t<3>(s0), rk.k[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t lb = T.lb.lb0;
    auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return (isb<0, 0>(T.lds, lb, a) | isb<1, 1>(T.lds, lb, b) | isb<2, 2>(T.lds, lb, c) | isb<3, 3>(T.lds, lb, d)) ^ k;
    };
    uint4 o;
    o.x = last(s0, s3, s2, s1, rk.k[4 * NR + 0]);
    o.y = last(s1, s0, s3, s2, rk.k[4 * NR + 1]);
    o.z = last(s2, s1, s0, s3, rk.k[4 * NR + 2]);
    o.w = last(s3, s2, s1, s0, rk.k[4 * NR + 3]);
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
// the buffer; only bytes inside [lo, hi) are dereferenced).  The byte loads are
// unconditional -- byte j reads base[clamp(j, lo, hi - 1)] and is masked afterwards -- so
// each word's four loads go out together (one wait per word, not per byte).
__device__ __forceinline__ uint4 load_bytes(const uint8_t *base, int lo, int hi) {
    uint32_t w[4] = {0, 0, 0, 0};
    if (lo >= hi) return make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t v[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int j = 4 * q + t;
            v[t] = base[j < lo ? lo : j >= hi ? hi - 1 : j];
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int j = 4 * q + t;
            w[q] |= (j >= lo && j < hi ? v[t] : 0u) << (8 * t);
        }
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Byte shifts of a 16-byte block by a per-lane count n in [0, 16]: shr_bytes gives
// byte j = v byte (j + n), shl_bytes byte j = v byte (j - n); zeros shifted in.
__device__ __forceinline__ uint4 shr_bytes(const uint4 &v, int n) {
    uint64_t lo = v.x | ((uint64_t)v.y << 32), hi = v.z | ((uint64_t)v.w << 32);
    if (n >= 8) {
        lo = n >= 16 ? 0ull : hi >> (8 * (n - 8));
        hi = 0;
    } else if (n > 0) {
        lo = (lo >> (8 * n)) | (hi << (64 - 8 * n));
        hi >>= 8 * n;
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

__device__ __forceinline__ uint4 shl_bytes(const uint4 &v, int n) {
    uint64_t lo = v.x | ((uint64_t)v.y << 32), hi = v.z | ((uint64_t)v.w << 32);
    if (n >= 8) {
        hi = n >= 16 ? 0ull : lo << (8 * (n - 8));
        lo = 0;
    } else if (n > 0) {
        hi = (hi << (8 * n)) | (lo >> (64 - 8 * n));
        lo <<= 8 * n;
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

typedef uint2 __attribute__((aligned(1))) uint2_ua;
typedef uint32_t __attribute__((aligned(1))) uint32_ua;
typedef uint16_t __attribute__((aligned(1))) uint16_ua;

// Bytes [lo, hi) of v to base + lo .. base + hi - 1, nothing else written: the range goes
// out as 8-, 4-, 2- and 1-byte stores (at most four instead of up to sixteen byte stores;
// gfx950 global stores tolerate any alignment).
__device__ __forceinline__ void store_bytes(uint8_t *base, const uint4 &v, int lo, int hi) {
    if (lo >= hi) return;
    uint4 s = shr_bytes(v, lo);  // byte 0 = v byte lo
    uint8_t *p = base + lo;
    const int n = hi - lo;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Walign-mismatch"
    if (n == 16) {
        store16(p, s);
        return;
    }
    if (n & 8) {
        *reinterpret_cast<uint2_ua *>(p) = make_uint2(s.x, s.y);
        p += 8;
        s = make_uint4(s.z, s.w, 0u, 0u);
    }
    if (n & 4) {
        *reinterpret_cast<uint32_ua *>(p) = s.x;
        p += 4;
        s = make_uint4(s.y, s.z, s.w, 0u);
    }
    if (n & 2) {
        *reinterpret_cast<uint16_ua *>(p) = (uint16_t)s.x;
        p += 2;
        s.x >>= 16;
    }
    if (n & 1) *p = (uint8_t)s.x;
#pragma clang diagnostic pop
}

// Lane l receives lane (l-1)'s value (lane 0 receives `fill`): DPP wave_shr:1.
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, 0x138, 0xf, 0xf, false);
}

// Lane l receives lane (l-1)'s value, lane 0 lane 63's: DPP wave_ror:1.
__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xf, 0xf, true);
}

// Same with 0 into lane 0 (bound_ctrl: no "old" register to materialise).
__device__ __forceinline__ uint32_t wave_shr1_zero(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}

__device__ __forceinline__ uint4 wave_shr1(const uint4 &v) {
    return make_uint4(wave_shr1_zero(v.x), wave_shr1_zero(v.y), wave_shr1_zero(v.z), wave_shr1_zero(v.w));
}

// floor(g / d) for g, d < 2^32 with magic = ceil(2^64 / d)
__device__ __forceinline__ uint32_t fast_div(uint32_t g, uint64_t magic) {
    return (uint32_t)__umul64hi((uint64_t)g, magic);
}

}  // namespace fpnn_aes
