// kernels.hip -- hand-written CDNA4 (gfx950) kernels for FPNN's AES-CFB path.
//
//   K1 k_cfb_decrypt_blocks : CFB-128 decryption, one lane per 16-byte block.
//        P_i = C_i ^ E(C_{i-1}), C_{-1} = IV (base/rijndael.c:1189-1197).  Every
//        C is known up front, so all blocks of all packets run in parallel; lane l
//        gets C_{i-1} from lane l-1 by DPP wave_shr:1, only lane 0 reloads it.
//   K2 k_cfb_encrypt_chains : CFB-128 encryption, one lane per packet / stream chain.
//        C_i = P_i ^ E(C_{i-1}) is serial inside a chain (base/rijndael.c:1176-1185),
//        so parallelism is across packets (package mode) or streams (stream mode).
//   Both keep the T-table image in LDS (aes_device.hpp) and are persistent: one
//   1024-thread workgroup per CU walks the work with a grid stride.
//
//   Segments follow the reference's exact byte semantics (rijndael_cfb_encrypt's
//   (ivec, pos) carry): a stream segment that starts at CFB position n0 != 0 first
//   consumes the keystream bytes ivec[n0..15]; block alignment is relative to the
//   stream, not to memory; partial final blocks leave (ivec, pos) exactly as the
//   reference's byte loop does.  Package mode is the special case n0 = 0,
//   ivec = connection IV, state discarded (core/Encryptor.cpp:10-32).
#include <type_traits>

#include "aes_device.hpp"
#include "kernels.hpp"

namespace fpnn_aes {

struct Seg {
    const uint8_t *in;
    uint8_t *out;
    uint32_t len;
    uint32_t slot;
};

template <int LAYOUT>
__device__ __forceinline__ Seg get_seg(const KBatch &b, uint64_t s) {
    Seg g;
    if (LAYOUT != LAYOUT_GENERAL) {
        const uint64_t o = s * b.stride;
        g.in = b.in + o;
        g.out = b.out + o;
        g.len = b.uniform_len;
        g.slot = 0;
    } else {
        const uint64_t io = b.in_off ? b.in_off[s] : s * b.stride;
        const uint64_t oo = b.out_off ? b.out_off[s] : io;
        g.in = b.in + io;
        g.out = b.out + oo;
        g.len = b.len ? b.len[s] : b.uniform_len;
        g.slot = b.key_slot ? b.key_slot[s] : 0u;
    }
    return g;
}

__device__ __forceinline__ uint4 ld_state_iv(const uint8_t *p) { return *reinterpret_cast<const uint4 *>(p); }

// Virtual (stream-aligned) block `bi` of a segment that starts at CFB position n0:
// bytes j < n0 of block 0 come from the carried ivec (they are the ciphertext bytes
// already consumed, base/rijndael.c:1182,1195), data bytes from the segment.
__device__ __forceinline__ uint4 load_cx(const Seg &g, uint32_t n0, uint32_t bi, const uint4 &ivs) {
    const int64_t vlo = 16 * (int64_t)bi;
    const int lo = bi == 0 ? (int)n0 : 0;
    const int64_t hi64 = (int64_t)n0 + g.len - vlo;
    const int hi = hi64 > 16 ? 16 : (int)hi64;
    const uint8_t *base = g.in + (vlo - (int64_t)n0);
    if (lo == 0 && hi == 16) return load16(base);
    uint4 d = load_bytes(base, lo, hi);
    if (lo != 0) d = select_bytes(byte_mask(0, lo), ivs, d);
    return d;
}

__device__ __forceinline__ void store_cx(const Seg &g, uint32_t n0, uint32_t bi, const uint4 &v) {
    const int64_t vlo = 16 * (int64_t)bi;
    const int lo = bi == 0 ? (int)n0 : 0;
    const int64_t hi64 = (int64_t)n0 + g.len - vlo;
    const int hi = hi64 > 16 ? 16 : (int)hi64;
    uint8_t *base = g.out + (vlo - (int64_t)n0);
    if (lo == 0 && hi == 16)
        store16(base, v);
    else
        store_bytes(base, v, lo, hi);
}

__device__ __forceinline__ uint64_t seg_blocks(uint32_t len, uint32_t n0) {
    return len ? ((uint64_t)n0 + len + 15) >> 4 : 0;
}

// ---------------------------------------------------------------------------
// K2: encryption, one lane per chain.

template <int NR, int LAYOUT, int KM, bool STREAM, int NT, int CH>
__global__ __launch_bounds__(kThreads, 4 * Lds<NT>::kBlocksPerCU) void k_cfb_encrypt_chains(KBatch b) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};

    RoundKeys<NR> rku;
    if (KM == KEY_UNIFORM) rku = load_round_keys<NR>(b.keys);

    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < b.count; s += nthreads) {
        const Seg g = get_seg<LAYOUT>(b, s);
        const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
        RoundKeys<NR> rk;
        if (KM == KEY_UNIFORM)
            rk = rku;
        else
            rk = load_round_keys<NR>(key);

        uint4 iv;
        uint32_t n = 0;
        if (STREAM) {
            iv = ld_state_iv(b.iv_state + 16 * s);
            n = b.pos_state[s];
        } else {
            iv = *reinterpret_cast<const uint4 *>(key->iv);
        }
        const uint8_t *p = g.in;
        uint8_t *q = g.out;
        uint32_t rem = g.len;

        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {  // htole32(len) ‖ ciphertext (core/Encryptor.cpp:47-48)
            q[0] = (uint8_t)rem;
            q[1] = (uint8_t)(rem >> 8);
            q[2] = (uint8_t)(rem >> 16);
            q[3] = (uint8_t)(rem >> 24);
            q += 4;
        }

        if (STREAM && n != 0 && rem != 0) {  // finish the partially consumed keystream block
            const uint32_t take = rem < 16 - n ? rem : 16 - n;
            const int lo = (int)n, hi = (int)(n + take);
            const uint4 o = load_bytes(p - n, lo, hi) ^ iv;
            store_bytes(q - n, o, lo, hi);
            iv = select_bytes(byte_mask(lo, hi), o, iv);
            p += take;
            q += take;
            rem -= take;
            n = (n + take) & 15u;
        }

        const uint32_t nfull = rem >> 4;
        uint32_t i = 0;
        if (CH > 1 && nfull >= CH) {
            // CH-block chunks (CH*16 = 64 or 128 bytes): a chunk's loads and its stores
            // each go out back to back, so every cache line is read and written whole
            // while it is in L2; the next chunk's loads are in flight during this
            // chunk's rounds.  (Two alternating buffers with unconditional loads, which
            // avoid the copy and the conservative waits below, measured 1.3 % slower.)
            uint4 a[CH], c[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) a[j] = load16(p + 16 * j);
            for (; i + CH <= nfull; i += CH) {
                const bool more = i + 2 * CH <= nfull;
                uint4 nx[CH];
#pragma unroll
                for (int j = 0; j < CH; j++) nx[j] = more ? load16(p + 16 * (CH + j)) : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    iv = aes_encrypt_block<NR, NT>(iv, rk, T) ^ a[j];
                    c[j] = iv;
                }
#pragma unroll
                for (int j = 0; j < CH; j++) store16(q + 16 * j, c[j]);
#pragma unroll
                for (int j = 0; j < CH; j++) a[j] = nx[j];
                p += 16 * CH;
                q += 16 * CH;
            }
        }
        uint4 pt = i < nfull ? load16(p) : make_uint4(0, 0, 0, 0);
        for (; i < nfull; i++) {
            const uint4 pn = (i + 1 < nfull) ? load16(p + 16) : make_uint4(0, 0, 0, 0);  // prefetch
            iv = aes_encrypt_block<NR, NT>(iv, rk, T) ^ pt;  // C_i = P_i ^ E(C_{i-1})
            store16(q, iv);
            pt = pn;
            p += 16;
            q += 16;
        }
        rem &= 15u;
        if (rem) {  // partial final block: ivec = E(C) with the first rem bytes replaced
            const uint4 ks = aes_encrypt_block<NR, NT>(iv, rk, T);
            const uint4 o = load_bytes(p, 0, (int)rem) ^ ks;
            store_bytes(q, o, 0, (int)rem);
            iv = select_bytes(byte_mask(0, (int)rem), o, ks);
            n = rem;
        }
        if (STREAM) {
            *reinterpret_cast<uint4 *>(b.iv_state + 16 * s) = iv;
            b.pos_state[s] = n;
        }
    }
}

// ---------------------------------------------------------------------------
// K2c: encryption, one lane QUAD per chain.  Lane q of the quad owns state column q:
// per round it fetches the other three columns from its quad neighbours with DPP
// quad_perm (VALU only), then does the 4 T-table lookups of its output column.  A
// chain therefore issues 4 LDS reads per round instead of 16 -- 4x the lanes per
// chain and ~4x shorter per-chain critical path -- and holds 15 round-key words per
// lane instead of 60.  Used when chains are few (streams) or long/ragged.

template <int SHIFT>  // value held by lane (q + SHIFT) & 3 of this lane's quad
__device__ __forceinline__ uint32_t quad_from(uint32_t v) {
    constexpr int ctl = ((0 + SHIFT) & 3) | (((1 + SHIFT) & 3) << 2) | (((2 + SHIFT) & 3) << 4) | (((3 + SHIFT) & 3) << 6);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctl, 0xf, 0xf, false);
}

template <int NR, int NT>
__device__ __forceinline__ uint32_t aes_encrypt_column(uint32_t sq, const uint32_t *rkq, const Tables4<NT> &T) {
    uint32_t s0 = sq ^ rkq[0];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t s1 = quad_from<1>(s0), s2 = quad_from<2>(s0), s3 = quad_from<3>(s0);
        s0 = xor3(xor3(T.template t<0>(s0), T.template t<1>(s1), T.template t<2>(s2)), T.template t<3>(s3), rkq[r]);
    }
    const uint32_t s1 = quad_from<1>(s0), s2 = quad_from<2>(s0), s3 = quad_from<3>(s0);
    return T.last(s0, s1, s2, s3, rkq[NR]);
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

template <int NR, int LAYOUT, int KM, bool STREAM, int NT>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_encrypt_coop(KBatch b) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = (int)(threadIdx.x & 3u);
    constexpr int CH = 8;

    const uint64_t nquads = ((uint64_t)gridDim.x * blockDim.x) >> 2;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; t < b.count; t += nquads) {
        const uint64_t s = b.perm ? b.perm[t] : t;  // longest chains first (ragged batches)
        const Seg g = get_seg<LAYOUT>(b, s);
        const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
        uint32_t rkq[NR + 1];
#pragma unroll
        for (int r = 0; r <= NR; r++) rkq[r] = key->rk[4 * r + q];

        uint32_t iv;  // this lane's word of the 16-byte feedback register
        uint32_t n = 0;
        if (STREAM) {
            iv = reinterpret_cast<const uint32_t *>(b.iv_state + 16 * s)[q];
            n = b.pos_state[s];
        } else {
            iv = reinterpret_cast<const uint32_t *>(key->iv)[q];
        }
        const uint8_t *p = g.in;
        uint8_t *o = g.out;
        uint32_t rem = g.len;
        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
            if (q == 0) store_word_bytes(o, rem, 0, 4);
            o += 4;
        }
        const int wlo = 4 * q;  // block bytes [wlo, wlo + 4) belong to this lane
        if (STREAM && n != 0 && rem != 0) {  // rest of the partially used keystream block
            const uint32_t take = rem < 16 - n ? rem : 16 - n;
            const int lo = max((int)n, wlo) - wlo, hi = min((int)(n + take), wlo + 4) - wlo;
            if (lo < hi) {
                const uint32_t c = load_word_bytes(p - n + wlo, lo, hi) ^ iv;
                store_word_bytes(o - n + wlo, c, lo, hi);
                const uint32_t m = word_mask(lo, hi);
                iv = (c & m) | (iv & ~m);
            }
            p += take;
            o += take;
            rem -= take;
            n = (n + take) & 15u;
        }
        const uint32_t nfull = rem >> 4;
        uint32_t i = 0;
        if (nfull >= CH) {
            uint32_t a[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) a[j] = *reinterpret_cast<const uint32_u *>(p + 16 * j + wlo);
            for (; i + CH <= nfull; i += CH) {
                const bool more = i + 2 * CH <= nfull;
                uint32_t nx[CH], c[CH];
#pragma unroll
                for (int j = 0; j < CH; j++) nx[j] = more ? *reinterpret_cast<const uint32_u *>(p + 16 * (CH + j) + wlo) : 0u;
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    iv = aes_encrypt_column<NR, NT>(iv, rkq, T) ^ a[j];
                    c[j] = iv;
                }
#pragma unroll
                for (int j = 0; j < CH; j++) *reinterpret_cast<uint32_u *>(o + 16 * j + wlo) = c[j];
#pragma unroll
                for (int j = 0; j < CH; j++) a[j] = nx[j];
                p += 16 * CH;
                o += 16 * CH;
            }
        }
        for (; i < nfull; i++) {
            const uint32_t pt = *reinterpret_cast<const uint32_u *>(p + wlo);
            iv = aes_encrypt_column<NR, NT>(iv, rkq, T) ^ pt;
            *reinterpret_cast<uint32_u *>(o + wlo) = iv;
            p += 16;
            o += 16;
        }
        rem &= 15u;
        if (rem) {  // partial final block
            const uint32_t ks = aes_encrypt_column<NR, NT>(iv, rkq, T);
            const int lo = 0, hi = min((int)rem, wlo + 4) - wlo;
            if (hi > lo) {
                const uint32_t c = load_word_bytes(p + wlo, lo, hi) ^ ks;
                store_word_bytes(o + wlo, c, lo, hi);
                const uint32_t m = word_mask(lo, hi);
                iv = (c & m) | (ks & ~m);
            } else {
                iv = ks;
            }
            n = rem;
        }
        if (STREAM) {
            reinterpret_cast<uint32_t *>(b.iv_state + 16 * s)[q] = iv;
            if (q == 0) b.pos_state[s] = n;
        }
    }
}

// ---------------------------------------------------------------------------
// K1: decryption, one lane per virtual block, 64 consecutive blocks per wave step.

template <int LAYOUT>
__device__ __forceinline__ void locate_block(const KBatch &b, uint64_t c, uint64_t gblk, uint64_t total, uint64_t &s,
                                             uint32_t &bi) {
    if (LAYOUT != LAYOUT_GENERAL) {
        const uint32_t g32 = (uint32_t)(gblk < total ? gblk : total - 1);
        const uint32_t q = fast_div(g32, b.magic);
        s = q;
        bi = g32 - q * b.nb_uniform;
    } else {
        const uint64_t gg = gblk < total ? gblk : total - 1;
        uint64_t lo = b.tile_first[c], hi = b.tile_first[c + 1];
        while (lo < hi) {  // largest s in [lo, hi] with bstart[s] <= gg
            const uint64_t mid = (lo + hi + 1) >> 1;
            if (b.bstart[mid] <= gg)
                lo = mid;
            else
                hi = mid - 1;
        }
        s = lo;
        bi = (uint32_t)(gg - b.bstart[lo]);
    }
}

// Everything one lane needs for one 64-block chunk; fetch_chunk() only issues the
// loads, so the next chunk's HBM latency overlaps the current chunk's rounds.
struct ChunkIn {
    Seg g;
    uint64_t s;
    uint32_t n0, bi, slot;
    bool valid;
    uint4 ivs, x, xp0;  // ivs: chunk's carried/connection IV; x: C_i; xp0: lane 0's C_{i-1}
};

template <int LAYOUT, int KM, bool STREAM, bool INPLACE>
__device__ __forceinline__ void fetch_chunk(const KBatch &b, uint64_t c, uint64_t total, uint32_t lane, ChunkIn &ci) {
    const uint64_t nchunks = (total + 63) >> 6;
    const uint64_t cc = c < nchunks ? c : nchunks - 1;  // steps may overhang the last chunk
    const uint64_t gblk = (c << 6) + lane;
    ci.valid = gblk < total;
    locate_block<LAYOUT>(b, cc, gblk, total, ci.s, ci.bi);
    ci.g = get_seg<LAYOUT>(b, ci.s);
    ci.n0 = STREAM ? b.pos_snap[ci.s] : 0u;
    ci.slot = KM == KEY_UNIFORM ? 0u : ci.g.slot;
    ci.ivs = STREAM ? b.iv_snap[ci.s] : *reinterpret_cast<const uint4 *>(b.keys[ci.slot].iv);
    ci.xp0 = make_uint4(0, 0, 0, 0);
    if (LAYOUT == LAYOUT_FULL) {  // whole blocks only: plain 16-B loads
        ci.x = ci.valid ? load16(ci.g.in + 16ull * ci.bi) : make_uint4(0, 0, 0, 0);
        if (lane == 0 && ci.bi != 0 && ci.valid)
            ci.xp0 = INPLACE ? b.boundary[cc] : load16(ci.g.in + 16ull * (ci.bi - 1));
        return;
    }
    ci.x = ci.valid ? load_cx(ci.g, ci.n0, ci.bi, ci.ivs) : make_uint4(0, 0, 0, 0);
    if (lane == 0 && ci.bi != 0 && ci.valid)
        ci.xp0 = INPLACE ? b.boundary[cc] : load_cx(ci.g, ci.n0, ci.bi - 1, ci.ivs);
}

__device__ __forceinline__ uint4 readlane63(const uint4 &v) {
    return make_uint4(__builtin_amdgcn_readlane(v.x, 63), __builtin_amdgcn_readlane(v.y, 63),
                      __builtin_amdgcn_readlane(v.z, 63), __builtin_amdgcn_readlane(v.w, 63));
}

// One wave step covers U consecutive 64-block chunks (U blocks per lane): the U loads go
// out together, the U ciphers are independent (ILP for the LDS pipe), and a lane-0 block
// whose predecessor sits in the previous chunk gets it from lane 63 by readlane.
template <int NR, int LAYOUT, int KM, bool STREAM, bool INPLACE, int NT, int U, int IL>
__global__ __launch_bounds__(kThreads, 4 * Lds<NT>::kBlocksPerCU) void k_cfb_decrypt_blocks(KBatch b) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u;

    RoundKeys<NR> rku;
    if (KM == KEY_UNIFORM) rku = load_round_keys<NR>(b.keys);

    const uint64_t total = b.total_blocks;
    const uint64_t nchunks = (total + 63) >> 6;
    const uint64_t nsteps = (nchunks + U - 1) / U;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t st = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nsteps; st += nwaves) {
        ChunkIn ci[U];
#pragma unroll
        for (int j = 0; j < U; j++) fetch_chunk<LAYOUT, KM, STREAM, INPLACE>(b, st * U + j, total, lane, ci[j]);
        uint4 ks[U];
        if (KM == KEY_UNIFORM) {
            // All cipher inputs first (selects only, no lane-divergent branches), then
            // the U ciphers round-interleaved in groups of IL in one basic block.
#pragma unroll
            for (int j = 0; j < U; j++) {
                const uint4 shr = wave_shr1(ci[j].x);  // C_{i-1} from the neighbouring lane
                const uint4 l0 = j == 0 ? ci[0].xp0 : readlane63(ci[j - 1].x);
                const uint4 xp = lane == 0 ? l0 : shr;
                ks[j] = ci[j].bi == 0 ? ci[j].ivs : xp;
            }
#pragma unroll
            for (int j = 0; j < U; j += IL) {
                uint4 grp[IL];
#pragma unroll
                for (int m = 0; m < IL; m++) grp[m] = ks[j + m];
                aes_encrypt_blocks<NR, NT, IL>(grp, rku, T);
#pragma unroll
                for (int m = 0; m < IL; m++) ks[j + m] = grp[m];
            }
#pragma unroll
            for (int j = 0; j < U; j++)
                if (STREAM && ci[j].bi == 0 && ci[j].n0 != 0) ks[j] = ci[j].ivs;  // keystream already in the state
        } else
#pragma unroll
        for (int j = 0; j < U; j++) {
            uint4 xp = wave_shr1(ci[j].x);  // C_{i-1} from the neighbouring lane (all 64 lanes active)
            if (lane == 0) xp = j == 0 ? ci[0].xp0 : readlane63(ci[j - 1].x);
            const uint4 kin = ci[j].bi == 0 ? ci[j].ivs : xp;
            {
                const uint32_t slot0 = __builtin_amdgcn_readfirstlane(ci[j].slot);
                const uint32_t my = ci[j].valid ? ci[j].slot : slot0;
                if (__builtin_amdgcn_ballot_w64(my != slot0) == 0) {  // wave-uniform key: SGPR round keys
                    const RoundKeys<NR> rk = load_round_keys<NR>(b.keys + slot0);
                    ks[j] = aes_encrypt_block<NR, NT>(kin, rk, T);
                } else {
                    const RoundKeys<NR> rk = load_round_keys<NR>(b.keys + ci[j].slot);
                    ks[j] = aes_encrypt_block<NR, NT>(kin, rk, T);
                }
            }
            if (STREAM && ci[j].bi == 0 && ci[j].n0 != 0) ks[j] = ci[j].ivs;  // keystream already in the state
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const ChunkIn &c = ci[j];
            if (!c.valid) continue;
            if (LAYOUT == LAYOUT_FULL) {
                store16(c.g.out + 16ull * c.bi, c.x ^ ks[j]);
                continue;
            }
            store_cx(c.g, c.n0, c.bi, c.x ^ ks[j]);
            if (STREAM && (uint64_t)c.bi + 1 == seg_blocks(c.g.len, c.n0)) {  // last block: export (ivec, pos)
                const uint32_t pos = (c.n0 + c.g.len) & 15u;
                const uint4 nv = pos ? select_bytes(byte_mask(0, (int)pos), c.x, ks[j]) : c.x;
                *reinterpret_cast<uint4 *>(b.iv_state + 16 * c.s) = nv;
                b.pos_state[c.s] = pos;
            }
        }
    }
}

// K1d: K1 for DENSE whole-block uniform package batches -- packet i is the nb blocks
// at in + i*16*nb (stride == length, length % 16 == 0, one key): the C2 shape and any
// contiguous array of equal-size packets.  Block g then sits at in + 16*g, so a
// 64-block chunk is one wave-uniform base address plus lane*16 (global_load saddr
// form: no per-lane address arithmetic), and the CFB predecessor of lane 0 is a
// wave-uniform value (the connection IV, lane 63 of the previous chunk by readlane,
// or one scalar load).  C_{i-1} for lanes 1..63 is one DPP wave_shr:1 whose "old"
// operand already holds lane 0's value.  Per 16-byte block this leaves ~16 VALU
// besides the 340 of the cipher (K1: ~60).
//   ALIGNED (nb % 64 == 0): packet starts fall only on lane 0, everything above is
//   scalar.  Otherwise a lane whose block opens a packet (bi == 0) takes the IV by a
//   per-lane select.
template <bool ALIGNED>
__device__ __forceinline__ uint32_t chunk_bi0(uint64_t c, uint32_t nb, uint64_t magic) {
    // block-in-packet index of the chunk's first block (wave-uniform)
    const uint32_t g = (uint32_t)(c << 6);  // total blocks < 2^32 (checked by the engine)
    return g - nb * fast_div(g, magic);
}

// Key table and key slots read through the constant address space: they do not change
// during a launch, so a wave-uniform index becomes scalar loads into SGPRs.
typedef __attribute__((address_space(4))) const DevKey ConstDevKey;
typedef __attribute__((address_space(4))) const uint32_t ConstU32;

//   KEYED: one key per packet (key_slot[] with the dense layout, chunk-aligned packets:
//   the C5 shape).  A step's U chunks never straddle two packets (U divides nb/64), so
//   the step's key is wave-uniform: slot and round keys are scalar loads per step.
template <int NR, bool INPLACE, int NT, bool ALIGNED, int U, int IL, bool PF, bool KEYED>
__global__ __launch_bounds__(kThreads, 4 * Lds<NT>::kBlocksPerCU) void k_cfb_decrypt_dense(KBatch b) {
    static_assert(U % IL == 0, "IL-way interleave of U chunks");
    static_assert(!KEYED || ALIGNED, "per-packet keys need chunk-aligned packets");
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u;
    RoundKeys<NR> rk;
    uint4 iv;
    auto set_key = [&](uint32_t slot) {
        ConstDevKey *kp = (ConstDevKey *)b.keys + slot;
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) rk.k[i] = kp->rk[i];
        ConstU32 *ivp = (ConstU32 *)kp->iv;
        iv = make_uint4(ivp[0], ivp[1], ivp[2], ivp[3]);
    };
    if (!KEYED) set_key(0);
    const uint64_t total = b.total_blocks;
    const uint64_t nchunks = (total + 63) >> 6;
    const uint64_t nsteps = (nchunks + U - 1) / U;
    const uint32_t nb = b.nb_uniform;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w0 = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t lane16 = lane * 16u;

    // One step = U consecutive chunks.  FULL: all U chunks hold 64 valid blocks (no
    // clamping, unconditional stores).  A StepBuf holds the step's ciphertext and lane
    // 0's predecessor of its first chunk (the only fill that may need a load), loaded
    // together.  With PF the step st + nwaves is loaded into the other buffer before
    // this step's rounds (ping-pong, no register copies).
    struct StepBuf {
        uint4 x[U];
        uint4 f;
    };
    auto load = [&](uint64_t st, StepBuf &D, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        // the fill first: the x loads are the newest, so a wait for them never covers
        // more stores than necessary
        const uint64_t c0 = FULL || st * U < nchunks ? st * U : nchunks - 1;
        if (chunk_bi0<ALIGNED>(c0, nb, b.magic) != 0)  // wave-uniform; at a packet start the IV is used
            D.f = INPLACE ? b.boundary[c0] : *reinterpret_cast<const uint4 *>(b.in + (c0 << 10) - 16);
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t c = st * U + j;
            const uint64_t cl = FULL || c < nchunks ? c : nchunks - 1;  // overhang: recompute the last chunk
            uint32_t lo = lane16;
            if (!FULL && !ALIGNED) {  // partial last chunk: clamp to the last block
                const uint64_t left = total - (cl << 6);
                if (left < 64) lo = min(lane, (uint32_t)left - 1u) * 16u;
            }
            D.x[j] = load16(b.in + (cl << 10) + lo);
        }
    };
    auto step = [&](uint64_t st, StepBuf &X, StepBuf &NX, bool pref, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        if (KEYED) set_key(((ConstU32 *)b.key_slot)[fast_div((uint32_t)((st * U) << 6), b.magic)]);
        if (!PF || !FULL) load(st, X, full_tag);
        uint4 ks[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t c = st * U + j;
            const uint64_t cl = FULL || c < nchunks ? c : nchunks - 1;
            const uint32_t bi0 = chunk_bi0<ALIGNED>(cl, nb, b.magic);
            // C_{i-1} of lane 0 (wave-uniform): IV at a packet start, else the block
            // before the chunk (lane 63 of chunk j-1; for j = 0 loaded with the step)
            const uint4 fill = bi0 == 0 ? iv : j == 0 ? X.f : readlane63(X.x[j - 1]);
            uint4 kin = make_uint4(wave_shr1(X.x[j].x, fill.x), wave_shr1(X.x[j].y, fill.y),
                                   wave_shr1(X.x[j].z, fill.z), wave_shr1(X.x[j].w, fill.w));
            if (!ALIGNED) {  // lanes 1..63 that open a packet take the IV
                const uint32_t r = bi0 + lane;
                const uint32_t q = fast_div(r, b.magic);
                if (lane != 0 && r == q * nb) kin = iv;
            }
            ks[j] = kin;
        }
        if (PF && FULL && pref) load(st + nwaves, NX, std::true_type{});
#pragma unroll
        for (int j = 0; j < U; j += IL) {
            uint4 grp[IL];
#pragma unroll
            for (int m = 0; m < IL; m++) grp[m] = ks[j + m];
            aes_encrypt_blocks<NR, NT, IL>(grp, rk, T);
#pragma unroll
            for (int m = 0; m < IL; m++) ks[j + m] = grp[m];
        }
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t c = st * U + j;
            if (!FULL) {
                if (c >= nchunks) break;  // wave-uniform
                if (!ALIGNED && (c << 6) + lane >= total) continue;
            }
            store16(b.out + (c << 10) + lane16, X.x[j] ^ ks[j]);
        }
    };
    const uint64_t nfull = (total >> 6) / U;  // steps made of U whole chunks
    uint64_t st = w0;
    StepBuf ba, bb;
    if (PF && st < nfull) {
        load(st, ba, std::true_type{});
        // Drain here: the loop header then only sees the back-edge state (prefetch
        // loads followed by 4 stores) and waits with vmcnt(4), not vmcnt(0).
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        while (true) {
            step(st, ba, bb, st + nwaves < nfull, std::true_type{});
            st += nwaves;
            if (st >= nfull) break;
            step(st, bb, ba, st + nwaves < nfull, std::true_type{});
            st += nwaves;
            if (st >= nfull) break;
        }
    }
    for (; st < nsteps; st += nwaves) step(st, ba, bb, false, std::false_type{});
}

// In-place decryption: save the ciphertext block that precedes every 64-block chunk
// before any wave overwrites it.
template <int LAYOUT, bool STREAM>
__global__ __launch_bounds__(256) void k_boundary_save(KBatch b, uint4 *boundary, uint64_t nchunks) {
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
         c += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t s;
        uint32_t bi;
        locate_block<LAYOUT>(b, c, c << 6, b.total_blocks, s, bi);
        if (bi == 0) continue;
        const Seg g = get_seg<LAYOUT>(b, s);
        const uint32_t n0 = STREAM ? b.pos_snap[s] : 0u;
        const DevKey *key = b.keys + g.slot;
        const uint4 ivs = STREAM ? b.iv_snap[s] : *reinterpret_cast<const uint4 *>(key->iv);
        boundary[c] = load_cx(g, n0, bi - 1, ivs);
    }
}

// ---------------------------------------------------------------------------
// General-layout block map: exclusive scan of per-segment block counts.

constexpr int kScanThreads = 256;
constexpr int kScanItems = 4;
constexpr int kScanTile = kScanThreads * kScanItems;

template <bool STREAM>
__device__ __forceinline__ uint64_t nblocks_of(const KBatch &b, uint64_t s) {
    if (s >= b.count) return 0;
    const uint32_t len = b.len ? b.len[s] : b.uniform_len;
    return seg_blocks(len, STREAM ? b.pos_snap[s] : 0u);
}

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *sh, uint64_t &total) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {
        const uint64_t add = t >= off ? sh[t - off] : 0;
        __syncthreads();
        sh[t] += add;
        __syncthreads();
    }
    total = sh[kScanThreads - 1];
    const uint64_t incl = sh[t];
    __syncthreads();
    return incl - v;
}

template <bool STREAM>
__global__ __launch_bounds__(kScanThreads) void k_scan_local(KBatch b, uint64_t *bstart, uint64_t *wg_sums) {
    __shared__ uint64_t sh[kScanThreads];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint64_t v[kScanItems], sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        v[k] = nblocks_of<STREAM>(b, base + k);
        sum += v[k];
    }
    uint64_t total;
    uint64_t run = block_exclusive_scan(sum, sh, total);
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        if (base + k < b.count) bstart[base + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 0) wg_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_sums(uint64_t *wg_sums, uint64_t nwg, uint64_t *bstart,
                                                            uint64_t count, uint64_t *total_out) {
    __shared__ uint64_t sh[kScanThreads];
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nwg; base += kScanThreads) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t v = i < nwg ? wg_sums[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(v, sh, tot);
        if (i < nwg) wg_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        bstart[count] = carry;
        *total_out = carry;
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_add(uint64_t *bstart, const uint64_t *wg_sums, uint64_t count) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) bstart[i] += wg_sums[i / kScanTile];
}

template <bool STREAM>
__global__ __launch_bounds__(kScanThreads) void k_tile_map(KBatch b, const uint64_t *bstart, uint64_t *tile_first,
                                                           uint64_t nchunks) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s == 0) tile_first[nchunks] = b.count ? b.count - 1 : 0;
    if (s >= b.count) return;
    const uint64_t nb = nblocks_of<STREAM>(b, s);
    if (!nb) return;
    const uint64_t first = bstart[s], last = first + nb - 1;
    for (uint64_t t = (first + 63) >> 6; (t << 6) <= last; t++) tile_first[t] = s;
}

// ---------------------------------------------------------------------------
// Length ordering for ragged encrypt batches: counting sort into 128 descending
// quarter-octave buckets of the block count (order inside a bucket is arbitrary; it
// only affects speed, never results).

constexpr int kBuckets = 128;

template <bool STREAM>
__device__ __forceinline__ uint32_t length_bucket(const KBatch &b, uint64_t s) {
    const uint64_t nb = nblocks_of<STREAM>(b, s) + 1;  // >= 1
    const uint32_t x = nb > 0xffffffffull ? 0xffffffffu : (uint32_t)nb;
    const int lz = 31 - __builtin_clz(x);
    const uint32_t frac = lz >= 2 ? (x >> (lz - 2)) & 3u : (x << (2 - lz)) & 3u;
    return (uint32_t)(kBuckets - 1) - (uint32_t)(4 * lz + frac);  // descending length
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_bucket_count(KBatch b, uint32_t *counts) {
    __shared__ uint32_t h[kBuckets];
    if (threadIdx.x < kBuckets) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < b.count; s += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[length_bucket<STREAM>(b, s)], 1u);
    __syncthreads();
    if (threadIdx.x < kBuckets && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

__global__ __launch_bounds__(kBuckets) void k_bucket_scan(uint32_t *counts, uint32_t *cursor) {
    __shared__ uint32_t sh[kBuckets];
    const int t = threadIdx.x;
    sh[t] = counts[t];
    __syncthreads();
    for (int off = 1; off < kBuckets; off <<= 1) {
        const uint32_t add = t >= off ? sh[t - off] : 0u;
        __syncthreads();
        sh[t] += add;
        __syncthreads();
    }
    cursor[t] = sh[t] - counts[t];  // exclusive
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_bucket_scatter(KBatch b, uint32_t *cursor, uint32_t *perm, uint64_t per_wg) {
    __shared__ uint32_t cnt[kBuckets], base[kBuckets];
    if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * per_wg;
    const uint64_t hi = lo + per_wg < b.count ? lo + per_wg : b.count;
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) atomicAdd(&cnt[length_bucket<STREAM>(b, s)], 1u);
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]) : 0u;
        cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    for (uint64_t s = lo + threadIdx.x; s < hi; s += blockDim.x) {
        const uint32_t k = length_bucket<STREAM>(b, s);
        perm[base[k] + atomicAdd(&cnt[k], 1u)] = (uint32_t)s;
    }
}

hipError_t launch_length_order(const KBatch &b, bool stream, uint32_t *perm, uint32_t *counts, hipStream_t st) {
    uint32_t *cursor = counts + kBuckets;
    hipError_t e = hipMemsetAsync(counts, 0, kBuckets * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)((b.count + 255) / 256 < 1024 ? (b.count + 255) / 256 : 1024);
    if (stream)
        hipLaunchKernelGGL((k_bucket_count<true>), dim3(grid ? grid : 1), dim3(256), 0, st, b, counts);
    else
        hipLaunchKernelGGL((k_bucket_count<false>), dim3(grid ? grid : 1), dim3(256), 0, st, b, counts);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(kBuckets), 0, st, counts, cursor);
    const uint64_t per_wg = 4096;
    const unsigned sgrid = (unsigned)((b.count + per_wg - 1) / per_wg);
    if (stream)
        hipLaunchKernelGGL((k_bucket_scatter<true>), dim3(sgrid ? sgrid : 1), dim3(256), 0, st, b, cursor, perm, per_wg);
    else
        hipLaunchKernelGGL((k_bucket_scatter<false>), dim3(sgrid ? sgrid : 1), dim3(256), 0, st, b, cursor, perm, per_wg);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Key expansion on the device (one lane per key; base/rijndael.c:712-799).

__global__ __launch_bounds__(256) void k_expand_keys(const uint8_t *keys, uint32_t keylen, const uint8_t *ivs,
                                                     uint32_t count, const uint8_t *sbox_g, DevKey *out) {
    __shared__ uint8_t sbox[256];
    sbox[threadIdx.x] = sbox_g[threadIdx.x];
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint8_t *key = keys + (uint64_t)i * keylen;
    const int nk = (int)keylen / 4, nr = nk + 6;
    uint32_t w[60];
    for (int k = 0; k < nk; k++)
        w[k] = ((uint32_t)key[4 * k] << 24) | ((uint32_t)key[4 * k + 1] << 16) | ((uint32_t)key[4 * k + 2] << 8) |
               key[4 * k + 3];
    auto sub = [&](uint32_t t) {
        return ((uint32_t)sbox[t >> 24] << 24) | ((uint32_t)sbox[(t >> 16) & 0xff] << 16) |
               ((uint32_t)sbox[(t >> 8) & 0xff] << 8) | sbox[t & 0xff];
    };
    uint32_t rcon = 1;
    for (int k = nk; k < 4 * (nr + 1); k++) {
        uint32_t t = w[k - 1];
        if (k % nk == 0) {
            t = sub((t << 8) | (t >> 24)) ^ (rcon << 24);
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0)) & 0xff;
        } else if (nk > 6 && k % nk == 4) {
            t = sub(t);
        }
        w[k] = w[k - nk] ^ t;
    }
    DevKey *d = out + i;
    for (int k = 0; k < 60; k++) d->rk[k] = k < 4 * (nr + 1) ? __builtin_bswap32(w[k]) : 0u;
    d->nrounds = (uint32_t)nr;
    d->keylen = keylen;
    d->reserved[0] = d->reserved[1] = 0;
    for (int k = 0; k < 16; k++) d->iv[k] = ivs ? ivs[16 * (uint64_t)i + k] : 0;
}

// ---------------------------------------------------------------------------
// Synthetic payload: counter-based splitmix64 (same definition as oracle/aes_oracle.c).

__device__ __forceinline__ uint64_t synth_word(uint64_t seed, uint64_t i) {
    uint64_t z = i + seed * 0xD1B54A32D192ED03ULL;
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill_synthetic(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t off) {
    const uint64_t w0 = off >> 3, w1 = (off + nbytes + 7) >> 3;
    const bool aligned = (((uintptr_t)dst - off) & 7) == 0;
    for (uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < w1;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t v = synth_word(seed, w);
        const uint64_t lo = w << 3;
        if (aligned && lo >= off && lo + 8 <= off + nbytes) {
            *reinterpret_cast<uint64_t *>(dst + (lo - off)) = v;
        } else {
            for (int k = 0; k < 8; k++) {
                const uint64_t a = lo + k;
                if (a >= off && a < off + nbytes) dst[a - off] = (uint8_t)(v >> (8 * k));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Launchers (runtime -> template dispatch)

// Variant selection.  Per-packet keys need ~100 VGPRs of round keys, so they always
// use the 4-table layout (one workgroup per CU); uniform-key variants take the
// layout the engine asks for.
template <int NR, int NT, int CH>
static void enc_launch(const KBatch &b, Layout layout, KeyMode km, bool stream, int grid, int threads,
                       hipStream_t st) {
#define FPNN_ENC(L, K, S, NTX) \
    hipLaunchKernelGGL((k_cfb_encrypt_chains<NR, L, K, S, NTX, CH>), dim3(grid), dim3(threads), 0, st, b)
    if (layout == LAYOUT_UNIFORM) {
        if (stream) FPNN_ENC(LAYOUT_UNIFORM, KEY_UNIFORM, true, NT); else FPNN_ENC(LAYOUT_UNIFORM, KEY_UNIFORM, false, NT);
    } else if (km == KEY_UNIFORM) {
        if (stream) FPNN_ENC(LAYOUT_GENERAL, KEY_UNIFORM, true, NT); else FPNN_ENC(LAYOUT_GENERAL, KEY_UNIFORM, false, NT);
    } else {
        if (stream) FPNN_ENC(LAYOUT_GENERAL, KEY_LANE, true, 4); else FPNN_ENC(LAYOUT_GENERAL, KEY_LANE, false, 4);
    }
#undef FPNN_ENC
}

template <int NR>
static void enc_nr(const KBatch &b, const Variant &v, Layout layout, KeyMode km, bool stream, int grid, int threads,
                   hipStream_t st) {
    if (v.tables == 2) {
        if (v.enc_chunk == 4) enc_launch<NR, 2, 4>(b, layout, km, stream, grid, threads, st);
        else enc_launch<NR, 2, 1>(b, layout, km, stream, grid, threads, st);
    } else {
        if (v.enc_chunk == 8) enc_launch<NR, 4, 8>(b, layout, km, stream, grid, threads, st);
        else if (v.enc_chunk == 4) enc_launch<NR, 4, 4>(b, layout, km, stream, grid, threads, st);
        else enc_launch<NR, 4, 1>(b, layout, km, stream, grid, threads, st);
    }
}

template <int NR>
static void coop_nr(const KBatch &b, Layout layout, KeyMode km, bool stream, int grid, int threads, hipStream_t st) {
#define FPNN_COOP(L, K, S) \
    hipLaunchKernelGGL((k_cfb_encrypt_coop<NR, L, K, S, 4>), dim3(grid), dim3(threads), 0, st, b)
    if (layout == LAYOUT_UNIFORM) {
        if (stream) FPNN_COOP(LAYOUT_UNIFORM, KEY_UNIFORM, true); else FPNN_COOP(LAYOUT_UNIFORM, KEY_UNIFORM, false);
    } else if (km == KEY_UNIFORM) {
        if (stream) FPNN_COOP(LAYOUT_GENERAL, KEY_UNIFORM, true); else FPNN_COOP(LAYOUT_GENERAL, KEY_UNIFORM, false);
    } else {
        if (stream) FPNN_COOP(LAYOUT_GENERAL, KEY_LANE, true); else FPNN_COOP(LAYOUT_GENERAL, KEY_LANE, false);
    }
#undef FPNN_COOP
}

hipError_t launch_encrypt_coop(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool stream, int grid,
                               int threads, hipStream_t st) {
    switch (nrounds) {
        case 10: coop_nr<10>(b, layout, km, stream, grid, threads, st); break;
        case 12: coop_nr<12>(b, layout, km, stream, grid, threads, st); break;
        case 14: coop_nr<14>(b, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int blocks_per_cu(const Variant &v, KeyMode km) { return (km == KEY_UNIFORM && v.tables == 2) ? 2 : 1; }

hipError_t launch_encrypt_chains(const KBatch &b, int nrounds, const Variant &v, Layout layout, KeyMode km,
                                 bool stream, int grid, int threads, hipStream_t st) {
    switch (nrounds) {
        case 10: enc_nr<10>(b, v, layout, km, stream, grid, threads, st); break;
        case 12: enc_nr<12>(b, v, layout, km, stream, grid, threads, st); break;
        case 14: enc_nr<14>(b, v, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// 64-block chunks per wave step in K1: 4 where the extra state fits in registers
// (package mode, one key), 1 for stream / per-packet-key variants (they would spill).
constexpr int dec_u(bool stream, int km) { return (!stream && km == KEY_UNIFORM) ? 4 : 1; }

template <int NR, bool INPLACE, int NT>
static void dec_launch(const KBatch &b, Layout layout, KeyMode km, bool stream, int dense, int grid, hipStream_t st) {
#define FPNN_DEC(L, K, S, NTX) \
    hipLaunchKernelGGL((k_cfb_decrypt_blocks<NR, L, K, S, INPLACE, NTX, dec_u(S, K), 1>), dim3(grid), dim3(kThreads), \
                       0, st, b)
#define FPNN_DENSE(AL, U, PF, KEYED) \
    hipLaunchKernelGGL((k_cfb_decrypt_dense<NR, INPLACE, NT, AL, U, 1, PF, KEYED>), dim3(grid), dim3(kThreads), 0, st, b)
    const bool aligned = b.nb_uniform % 64 == 0;
    if (layout == LAYOUT_FULL && km == KEY_LANE) {  // dense, chunk-aligned, one key per packet
        const uint32_t nbc = b.nb_uniform / 64;
        if (nbc % 4 == 0) FPNN_DENSE(true, 4, true, true);
        else if (nbc % 2 == 0) FPNN_DENSE(true, 2, true, true);
        else FPNN_DENSE(true, 1, true, true);
    } else if (layout == LAYOUT_FULL && dense == 2) {
        if (aligned) FPNN_DENSE(true, 4, true, false); else FPNN_DENSE(false, 4, true, false);
    } else if (layout == LAYOUT_FULL && dense) {
        if (aligned) FPNN_DENSE(true, 4, false, false); else FPNN_DENSE(false, 4, false, false);
    } else if (layout == LAYOUT_FULL) {
        FPNN_DEC(LAYOUT_FULL, KEY_UNIFORM, false, NT);
    } else if (layout == LAYOUT_UNIFORM) {
        if (stream) FPNN_DEC(LAYOUT_UNIFORM, KEY_UNIFORM, true, NT); else FPNN_DEC(LAYOUT_UNIFORM, KEY_UNIFORM, false, NT);
    } else if (km == KEY_UNIFORM) {
        if (stream) FPNN_DEC(LAYOUT_GENERAL, KEY_UNIFORM, true, NT); else FPNN_DEC(LAYOUT_GENERAL, KEY_UNIFORM, false, NT);
    } else {
        if (stream) FPNN_DEC(LAYOUT_GENERAL, KEY_LANE, true, 4); else FPNN_DEC(LAYOUT_GENERAL, KEY_LANE, false, 4);
    }
#undef FPNN_DENSE
#undef FPNN_DEC
}

template <int NR>
static void dec_nr(const KBatch &b, const Variant &v, Layout layout, KeyMode km, bool stream, bool inplace, int grid,
                   hipStream_t st) {
    const int dense = b.stride == 16ull * b.nb_uniform ? v.dec_dense : 0;
    if (v.tables == 2 && km == KEY_UNIFORM) {
        if (inplace) dec_launch<NR, true, 2>(b, layout, km, stream, dense, grid, st);
        else dec_launch<NR, false, 2>(b, layout, km, stream, dense, grid, st);
    } else {
        if (inplace) dec_launch<NR, true, 4>(b, layout, km, stream, dense, grid, st);
        else dec_launch<NR, false, 4>(b, layout, km, stream, dense, grid, st);
    }
}

hipError_t launch_decrypt_blocks(const KBatch &b, int nrounds, const Variant &v, Layout layout, KeyMode km,
                                 bool stream, bool inplace, int grid, hipStream_t st) {
    switch (nrounds) {
        case 10: dec_nr<10>(b, v, layout, km, stream, inplace, grid, st); break;
        case 12: dec_nr<12>(b, v, layout, km, stream, inplace, grid, st); break;
        case 14: dec_nr<14>(b, v, layout, km, stream, inplace, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

static int grid_for(uint64_t items, int threads, int cap) {
    uint64_t g = (items + threads - 1) / threads;
    if (g < 1) g = 1;
    return (int)(g > (uint64_t)cap ? cap : g);
}

hipError_t launch_boundary_save(const KBatch &b, Layout layout, bool stream, uint4 *boundary, uint64_t nchunks,
                                hipStream_t st) {
    const int grid = grid_for(nchunks, 256, 4096);
    if (layout != LAYOUT_GENERAL) {
        if (stream)
            hipLaunchKernelGGL((k_boundary_save<LAYOUT_UNIFORM, true>), dim3(grid), dim3(256), 0, st, b, boundary, nchunks);
        else
            hipLaunchKernelGGL((k_boundary_save<LAYOUT_UNIFORM, false>), dim3(grid), dim3(256), 0, st, b, boundary, nchunks);
    } else {
        if (stream)
            hipLaunchKernelGGL((k_boundary_save<LAYOUT_GENERAL, true>), dim3(grid), dim3(256), 0, st, b, boundary, nchunks);
        else
            hipLaunchKernelGGL((k_boundary_save<LAYOUT_GENERAL, false>), dim3(grid), dim3(256), 0, st, b, boundary, nchunks);
    }
    return hipGetLastError();
}

hipError_t launch_block_map_scan(const KBatch &b, bool stream, uint64_t *bstart, uint64_t *wg_sums, uint64_t *total,
                                 hipStream_t st) {
    const uint64_t nwg = (b.count + kScanTile - 1) / kScanTile;
    if (nwg) {
        if (stream)
            hipLaunchKernelGGL((k_scan_local<true>), dim3((unsigned)nwg), dim3(kScanThreads), 0, st, b, bstart, wg_sums);
        else
            hipLaunchKernelGGL((k_scan_local<false>), dim3((unsigned)nwg), dim3(kScanThreads), 0, st, b, bstart, wg_sums);
    }
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanThreads), 0, st, wg_sums, nwg, bstart, b.count, total);
    if (b.count)
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((b.count + kScanThreads - 1) / kScanThreads)),
                           dim3(kScanThreads), 0, st, bstart, wg_sums, b.count);
    return hipGetLastError();
}

hipError_t launch_tile_map(const KBatch &b, bool stream, const uint64_t *bstart, uint64_t *tile_first, uint64_t nchunks,
                           hipStream_t st) {
    const unsigned grid = (unsigned)((b.count + kScanThreads) / kScanThreads);
    if (stream)
        hipLaunchKernelGGL((k_tile_map<true>), dim3(grid), dim3(kScanThreads), 0, st, b, bstart, tile_first, nchunks);
    else
        hipLaunchKernelGGL((k_tile_map<false>), dim3(grid), dim3(kScanThreads), 0, st, b, bstart, tile_first, nchunks);
    return hipGetLastError();
}

hipError_t launch_expand_keys(const uint8_t *keys, uint32_t keylen, const uint8_t *ivs, uint32_t count,
                              const uint8_t *sbox, DevKey *out, hipStream_t st) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(k_expand_keys, dim3((count + 255) / 256), dim3(256), 0, st, keys, keylen, ivs, count, sbox, out);
    return hipGetLastError();
}

hipError_t launch_fill_synthetic(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, int grid,
                                 hipStream_t st) {
    if (!nbytes) return hipSuccess;
    hipLaunchKernelGGL(k_fill_synthetic, dim3(grid), dim3(256), 0, st, dst, nbytes, seed, byte_offset);
    return hipGetLastError();
}

}  // namespace fpnn_aes
