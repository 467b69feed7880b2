// PROBE (not built into the product): k_encrypt.hip with K2c/K2q generalised to G lanes per chain
// (G = 2 "pair" rounds).  Measured slower than quads -- profiles/r02/ab_pair_group.json.
// k_encrypt.hip -- CFB-128 encryption kernels for gfx950 (see segments.hpp for the
// segment semantics and aes_device.hpp for the LDS T-table round function).
//   K2  k_cfb_encrypt_chains : one lane per packet / stream chain.
//        C_i = P_i ^ E(C_{i-1}) is serial inside a chain (base/rijndael.c:1176-1185),
//        so parallelism is across packets (package mode) or streams (stream mode).
//   K2c k_cfb_encrypt_coop   : one lane quad per chain (few / long chains).
//   K2q k_cfb_encrypt_queue  : K2c with a work queue (many ragged chains).
//   All are persistent: workgroups walk the chains with a grid stride or the queue.
#include "segments.hpp"

namespace fpnn_aes {

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
        // Per-lane AES-256 round keys (60 VGPRs) leave room for 4-block chunks only.
        constexpr int C = (KM == KEY_LANE && NR == 14 && CH > 4) ? 4 : CH;
        if (C > 1 && nfull >= C) {
            // C-block chunks (C*16 = 64 or 128 bytes): a chunk's loads and its stores
            // each go out back to back, so every cache line is read and written whole
            // while it is in L2; the next chunk's loads are in flight during this
            // chunk's rounds.  Ciphertext overwrites the chunk's plaintext registers.
            // (Two alternating buffers with unconditional loads, which avoid the copy
            // and the conservative waits below, measured 1.3 % slower.)
            uint4 a[C];
#pragma unroll
            for (int j = 0; j < C; j++) a[j] = load16(p + 16 * j);
            for (; i + C <= nfull; i += C) {
                const bool more = i + 2 * C <= nfull;
                uint4 nx[C];
#pragma unroll
                for (int j = 0; j < C; j++) nx[j] = more ? load16(p + 16 * (C + j)) : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < C; j++) {
                    iv = aes_encrypt_block<NR, NT>(iv, rk, T) ^ a[j];
                    a[j] = iv;
                }
#pragma unroll
                for (int j = 0; j < C; j++) store16(q + 16 * j, a[j]);
#pragma unroll
                for (int j = 0; j < C; j++) a[j] = nx[j];
                p += 16 * C;
                q += 16 * C;
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
// K2c: encryption, one lane GROUP per chain.  G lanes share one chain's block:
//   G = 4 (quad): lane q owns state column q; per round it does the 4 T-table lookups
//          of its own 4 bytes and the quad sums the contributions with DPP quad_perm
//          (aes_encrypt_column below): 4 LDS reads + 8 VALU per lane and round.
//   G = 2 (pair): lane p owns columns 2p and 2p+1; 8 LDS reads + 14 VALU per lane and
//          round (aes_encrypt_pair): 1.75 VALU per lookup instead of the quad's 2.0, and
//          8 lookups in flight per lane.
// Either way a chain's critical path is ~G times shorter than one lane's and it holds
// (NR+1)*4/G round-key words per lane.  Used when chains are few (streams) or
// long/ragged.

// DPP quad_perm control: lane i of every quad reads lane src(i) -- within its group of G
// lanes, the lane SHIFT places further on (mod G).
constexpr int group_src(int G, int i, int shift) { return G == 4 ? ((i + shift) & 3) : ((i & 2) | ((i + shift) & 1)); }
constexpr int group_ctl(int G, int shift) {
    return group_src(G, 0, shift) | (group_src(G, 1, shift) << 2) | (group_src(G, 2, shift) << 4) |
           (group_src(G, 3, shift) << 6);
}

// value held by lane (g + SHIFT) mod G of this lane's group.  bound_ctrl: every lane has
// a source under quad_perm, so no "old" value is needed (update_dpp with old = 0 costs a
// v_mov per call to materialise it -- 3 of the 12 VALU of a K2c round).
template <int SHIFT, int G = 4>
__device__ __forceinline__ uint32_t quad_from(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, group_ctl(G, SHIFT), 0xf, 0xf, true);
}

// XOR of a and the value b holds in lane (g + SHIFT) mod G: one v_xor_b32 with a DPP
// quad_perm source (the mov_dpp folds into the xor).
template <int SHIFT, int G = 4>
__device__ __forceinline__ uint32_t xor_quad_from(uint32_t a, uint32_t b) {
    return a ^ quad_from<SHIFT, G>(b);
}

// Quad round structure: lane q looks up ITS OWN four bytes -- T0[b0] feeds output
// column q, T1[b1] column q-1, T2[b2] column q-2, T3[b3] column q-3 -- and the quad then
// sums the contributions with DPP-sourced XORs.  Per lane and round: 4 v_perm + 4
// ds_read + 3 DPP ops + 1 v_bitop3 = 8 VALU, and every DPP operand is an LDS result or
// a round key, never a fresh VALU result, so no hazard wait states (moving the state
// words to the neighbours first costs 9 VALU plus an s_nop per round).
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

// Pair round structure (FIPS-197 T-table round, base/rijndael.c:871-925, split over two
// lanes).  Lane p holds u = column 2p and v = column 2p+1; its partner holds u', v'.
//   out(2p)   = T0[u.b0] ^ T1[v.b1]  ^ T2[u'.b2] ^ T3[v'.b3] ^ rk
//   out(2p+1) = T0[v.b0] ^ T1[u'.b1] ^ T2[v'.b2] ^ T3[u.b3]  ^ rk
// so each lane looks up all 8 of its bytes once; the partner's two terms per output
// come over DPP (pair swap) straight from its LDS results: 8 v_perm + 8 ds_read + 4 DPP
// xors + 2 v_bitop3 per lane and round.
template <int NR, int NT>
__device__ __forceinline__ void aes_encrypt_pair(uint32_t &u, uint32_t &v, const uint32_t (*rk)[2],
                                                 const Tables4<NT> &T) {
    uint32_t su = u ^ rk[0][0], sv = v ^ rk[0][1];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        const uint32_t tu0 = T.template t<0>(su), tu1 = T.template t<1>(su), tu2 = T.template t<2>(su),
                       tu3 = T.template t<3>(su);
        const uint32_t tv0 = T.template t<0>(sv), tv1 = T.template t<1>(sv), tv2 = T.template t<2>(sv),
                       tv3 = T.template t<3>(sv);
        const uint32_t a = xor3(xor_quad_from<1, 2>(tu0, tu2), xor_quad_from<1, 2>(rk[r][0], tv3), tv1);
        const uint32_t c = xor3(xor_quad_from<1, 2>(tv0, tu1), xor_quad_from<1, 2>(rk[r][1], tv2), tu3);
        su = a;
        sv = c;
    }
    // final round: S-box bytes gathered by v_perm into the own half (lo) and the
    // partner's half (hi) of each output word
    const uint32_t loA = __builtin_amdgcn_perm(T.template sraw<1>(sv), T.template sraw<0>(su), 0x0c0c0500u);
    const uint32_t hiA = __builtin_amdgcn_perm(T.template sraw<3>(sv), T.template sraw<2>(su), 0x07020c0cu);
    const uint32_t loB = __builtin_amdgcn_perm(T.template sraw<3>(su), T.template sraw<0>(sv), 0x070c0c00u);
    const uint32_t hiB = __builtin_amdgcn_perm(T.template sraw<2>(sv), T.template sraw<1>(su), 0x0c06010cu);
    u = xor3(loA, rk[NR][0], quad_from<1, 2>(hiA));
    v = xor3(loB, rk[NR][1], quad_from<1, 2>(hiB));
}

// E(s) for the group's share of one block: W = 4 / G words per lane
template <int NR, int NT, int G>
__device__ __forceinline__ void aes_encrypt_group(uint32_t (&s)[4 / G], const uint32_t (&rk)[NR + 1][4 / G],
                                                  const Tables4<NT> &T) {
    if constexpr (G == 4)
        s[0] = aes_encrypt_column<NR, NT>(s[0], &rk[0][0], T);
    else
        aes_encrypt_pair<NR, NT>(s[0], s[1], rk, T);
}

typedef uint32_t __attribute__((aligned(1))) uint32_u;
typedef uint2 __attribute__((aligned(1))) uint2_u;

// bytes [lo, hi) of this lane's word (word covers block bytes [4q, 4q+4)); lo may be
// negative and hi above 4 (clipped)
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

// the lane's 4W whole bytes at p
template <int W>
__device__ __forceinline__ void load_lane(const uint8_t *p, uint32_t (&d)[W]) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Walign-mismatch"
    if constexpr (W == 1) {
        d[0] = *reinterpret_cast<const uint32_u *>(p);
    } else {
        const uint2 x = *reinterpret_cast<const uint2_u *>(p);
        d[0] = x.x;
        d[1] = x.y;
    }
#pragma clang diagnostic pop
}

template <int W>
__device__ __forceinline__ void store_lane(uint8_t *p, const uint32_t (&d)[W]) {
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Walign-mismatch"
    if constexpr (W == 1)
        *reinterpret_cast<uint32_u *>(p) = d[0];
    else
        *reinterpret_cast<uint2_u *>(p) = make_uint2(d[0], d[1]);
#pragma clang diagnostic pop
}

// CFB over bytes [lo, hi) of the lane's 4W bytes (relative to the lane's first byte):
// c = data ^ e stored there, and the feedback register takes c in those bytes and keeps
// `keep` elsewhere (base/rijndael.c:1182,1195: the ciphertext replaces the consumed
// keystream bytes).
template <int W>
__device__ __forceinline__ void cfb_lane_bytes(const uint8_t *p, uint8_t *o, int lo, int hi, const uint32_t (&e)[W],
                                               uint32_t (&iv)[W]) {
#pragma unroll
    for (int w = 0; w < W; w++) {
        const int l = lo - 4 * w, h = hi - 4 * w;
        if (l < 4 && h > 0 && l < h) {
            const uint32_t c = load_word_bytes(p + 4 * w, l, h) ^ e[w];
            store_word_bytes(o + 4 * w, c, l, h);
            const uint32_t m = word_mask(l, h);
            iv[w] = (c & m) | (e[w] & ~m);
        } else {
            iv[w] = e[w];
        }
    }
}

template <int NR, int LAYOUT, int KM, bool STREAM, int NT, int G>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_encrypt_coop(KBatch b) {
    constexpr int W = 4 / G;
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = (int)(threadIdx.x & (G - 1));
    const int wlo = 4 * W * q;  // block bytes [wlo, wlo + 4W) belong to this lane
    constexpr int CH = 8;

    const uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G; t < b.count; t += ngroups) {
        const uint64_t s = b.perm ? b.perm[t] : t;  // longest chains first (ragged batches)
        const Seg g = get_seg<LAYOUT>(b, s);
        const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
        uint32_t rk[NR + 1][W];
#pragma unroll
        for (int r = 0; r <= NR; r++)
#pragma unroll
            for (int w = 0; w < W; w++) rk[r][w] = key->rk[4 * r + W * q + w];

        uint32_t iv[W];  // this lane's words of the 16-byte feedback register
        uint32_t n = 0;
        const uint32_t *ivsrc = STREAM ? reinterpret_cast<const uint32_t *>(b.iv_state + 16 * s)
                                       : reinterpret_cast<const uint32_t *>(key->iv);
#pragma unroll
        for (int w = 0; w < W; w++) iv[w] = ivsrc[W * q + w];
        if (STREAM) n = b.pos_state[s];
        const uint8_t *p = g.in;
        uint8_t *o = g.out;
        uint32_t rem = g.len;
        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
            if (q == 0) store_word_bytes(o, rem, 0, 4);
            o += 4;
        }
        if (STREAM && n != 0 && rem != 0) {  // rest of the partially used keystream block
            const uint32_t take = rem < 16 - n ? rem : 16 - n;
            // bytes [n, n + take) of the block: c = p ^ ivec (ivec already holds the
            // keystream E(C) there), and ivec takes c in those bytes
            uint32_t ks[W];
#pragma unroll
            for (int w = 0; w < W; w++) ks[w] = iv[w];
            cfb_lane_bytes<W>(p - n + wlo, o - n + wlo, (int)n - wlo, (int)(n + take) - wlo, ks, iv);
            p += take;
            o += take;
            rem -= take;
            n = (n + take) & 15u;
        }
        const uint32_t nfull = rem >> 4;
        uint32_t i = 0;
        if (nfull >= CH) {
            uint32_t a[CH][W];
#pragma unroll
            for (int j = 0; j < CH; j++) load_lane<W>(p + 16 * j + wlo, a[j]);
            for (; i + CH <= nfull; i += CH) {
                const bool more = i + 2 * CH <= nfull;
                uint32_t nx[CH][W], c[CH][W];
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    if (more) {
                        load_lane<W>(p + 16 * (CH + j) + wlo, nx[j]);
                    } else {
#pragma unroll
                        for (int w = 0; w < W; w++) nx[j][w] = 0u;
                    }
                }
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    aes_encrypt_group<NR, NT, G>(iv, rk, T);
#pragma unroll
                    for (int w = 0; w < W; w++) {
                        iv[w] ^= a[j][w];  // C_i = P_i ^ E(C_{i-1})
                        c[j][w] = iv[w];
                    }
                }
#pragma unroll
                for (int j = 0; j < CH; j++) store_lane<W>(o + 16 * j + wlo, c[j]);
#pragma unroll
                for (int j = 0; j < CH; j++)
#pragma unroll
                    for (int w = 0; w < W; w++) a[j][w] = nx[j][w];
                p += 16 * CH;
                o += 16 * CH;
            }
        }
        for (; i < nfull; i++) {
            uint32_t pt[W];
            load_lane<W>(p + wlo, pt);
            aes_encrypt_group<NR, NT, G>(iv, rk, T);
#pragma unroll
            for (int w = 0; w < W; w++) iv[w] ^= pt[w];
            store_lane<W>(o + wlo, iv);
            p += 16;
            o += 16;
        }
        rem &= 15u;
        if (rem) {  // partial final block: ivec = E(C) with the first rem bytes replaced
            uint32_t ks[W];
#pragma unroll
            for (int w = 0; w < W; w++) ks[w] = iv[w];
            aes_encrypt_group<NR, NT, G>(ks, rk, T);
            cfb_lane_bytes<W>(p + wlo, o + wlo, -wlo, (int)rem - wlo, ks, iv);
            n = rem;
        }
        if (STREAM) {
            uint32_t *dst = reinterpret_cast<uint32_t *>(b.iv_state + 16 * s);
#pragma unroll
            for (int w = 0; w < W; w++) dst[W * q + w] = iv[w];
            if (q == 0) b.pos_state[s] = n;
        }
    }
}

// ---------------------------------------------------------------------------
// K2q: K2c's group-per-chain cipher with a work queue instead of a grid stride.
// Chains are visited longest first (perm[]); a group that finishes a chain takes the
// next one from a global counter at once, so lanes of a wave never wait for the
// longest chain of their wave (greedy longest-processing-time scheduling).  The loop
// body is one step of up to CH blocks; a block past the chain's end is computed but not
// committed (a select, not a branch).  The wave leaves the loop when no group of it has
// work.  (Two chains per group, round-interleaved, measured 35 % slower on C4: the
// longest chains, which set the end of the launch, then advance at half speed.)  Used
// for ragged batches with more chains than groups (C4), where a static chain-to-lane
// assignment leaves most lanes idle.
template <int NR, int KM, bool STREAM, int NT, int G, bool FIRST_PRIO = true>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_encrypt_queue(KBatch b, uint32_t *next) {
    constexpr int W = 4 / G;
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = (int)(threadIdx.x & (G - 1));
    const int wlo = 4 * W * q;  // block bytes [wlo, wlo + 4W) belong to this lane
    constexpr int CH = 8;
    const uint64_t ngroups = ((uint64_t)gridDim.x * blockDim.x) / G;

    uint32_t rk[NR + 1][W];
    if (KM == KEY_UNIFORM) {
#pragma unroll
        for (int r = 0; r <= NR; r++)
#pragma unroll
            for (int w = 0; w < W; w++) rk[r][w] = b.keys[0].rk[4 * r + W * q + w];
    }
    // chain state
    uint64_t sid = 0;
    const uint8_t *p = nullptr;
    uint8_t *o = nullptr;
    uint32_t nfull = 0, tail = 0, n = 0, iv[W];
#pragma unroll
    for (int w = 0; w < W; w++) iv[w] = 0;
    bool active = false;

    auto begin = [&](uint64_t t) {  // take chain perm[t] (t < count), run its head
        const uint64_t s = b.perm ? b.perm[t] : t;
        sid = s;
        const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
        const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
        if (KM != KEY_UNIFORM) {
#pragma unroll
            for (int r = 0; r <= NR; r++)
#pragma unroll
                for (int w = 0; w < W; w++) rk[r][w] = key->rk[4 * r + W * q + w];
        }
        uint32_t pos = 0;
        const uint32_t *ivsrc = STREAM ? reinterpret_cast<const uint32_t *>(b.iv_state + 16 * s)
                                       : reinterpret_cast<const uint32_t *>(key->iv);
#pragma unroll
        for (int w = 0; w < W; w++) iv[w] = ivsrc[W * q + w];
        if (STREAM) pos = b.pos_state[s];
        const uint8_t *pp = g.in;
        uint8_t *oo = g.out;
        uint32_t rem = g.len;
        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
            if (q == 0) store_word_bytes(oo, rem, 0, 4);
            oo += 4;
        }
        if (STREAM && pos != 0 && rem != 0) {  // rest of the partially used keystream block
            const uint32_t take = rem < 16 - pos ? rem : 16 - pos;
            uint32_t ks[W];
#pragma unroll
            for (int w = 0; w < W; w++) ks[w] = iv[w];
            cfb_lane_bytes<W>(pp - pos + wlo, oo - pos + wlo, (int)pos - wlo, (int)(pos + take) - wlo, ks, iv);
            pp += take;
            oo += take;
            rem -= take;
            pos = (pos + take) & 15u;
        }
        n = pos;
        p = pp;
        o = oo;
        nfull = rem >> 4;
        tail = rem & 15u;
        active = true;
    };
    auto finish = [&]() {  // partial final block and the stream state
        if (tail) {
            uint32_t ks[W];
#pragma unroll
            for (int w = 0; w < W; w++) ks[w] = iv[w];
            aes_encrypt_group<NR, NT, G>(ks, rk, T);
            cfb_lane_bytes<W>(p + wlo, o + wlo, -wlo, (int)tail - wlo, ks, iv);
            n = tail;
        }
        if (STREAM) {
            uint32_t *dst = reinterpret_cast<uint32_t *>(b.iv_state + 16 * sid);
#pragma unroll
            for (int w = 0; w < W; w++) dst[W * q + w] = iv[w];
            if (q == 0) b.pos_state[sid] = n;
        }
    };
    // First chains: the longest (perm[] order) are dealt round-robin over the
    // workgroups -- group j of workgroup w takes chain j * gridDim.x + w -- so the few
    // longest chains, which set the end of the launch, sit on different CUs and in the
    // first wave of each; that wave runs at raised priority so its chain's rounds are
    // not queued behind the 15 other waves' (the critical path of a greedy schedule
    // is its longest job).  Later chains come from the counter (from ngroups on).
    const uint64_t t0 = (uint64_t)(threadIdx.x / G) * gridDim.x + blockIdx.x;
    if (FIRST_PRIO && threadIdx.x < 64) __builtin_amdgcn_s_setprio(2);
    if (t0 < b.count) begin(t0);
    while (true) {
        if (__builtin_amdgcn_ballot_w64(active) == 0) break;
        // a chain with no whole block left: finish it, take the next chain
        if (active && nfull == 0) {
            finish();
            uint32_t tk = 0;
            if (q == 0) tk = atomicAdd(next, 1u);
            // broadcast the group leader's ticket (DPP quad_perm 0,0,0,0 or 0,0,2,2)
            constexpr int kLeader = G == 4 ? 0x00 : 0xa0;
            const uint64_t tt = (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)tk, kLeader, 0xf, 0xf, true) +
                                ngroups;  // 64-bit: no wrap near count = 2^32 - 1
            active = false;
            if (tt < b.count) begin(tt);
        }
        const uint32_t kk = active ? (nfull < CH ? nfull : CH) : 0u;
        uint32_t a[CH][W];
#pragma unroll
        for (int j = 0; j < CH; j++) {
            if (j < (int)kk) {
                load_lane<W>(p + 16 * j + wlo, a[j]);
            } else {
#pragma unroll
                for (int w = 0; w < W; w++) a[j][w] = 0u;
            }
        }
        // (a group with no work still runs the rounds: its results are dropped like
        // those of blocks past a chain's end)
#pragma unroll
        for (int j = 0; j < CH; j++) {
            uint32_t e[W];
#pragma unroll
            for (int w = 0; w < W; w++) e[w] = iv[w];
            aes_encrypt_group<NR, NT, G>(e, rk, T);
#pragma unroll
            for (int w = 0; w < W; w++) {
                const uint32_t c = e[w] ^ a[j][w];  // C_i = P_i ^ E(C_{i-1})
                iv[w] = j < (int)kk ? c : iv[w];
                a[j][w] = c;
            }
        }
#pragma unroll
        for (int j = 0; j < CH; j++)
            if (j < (int)kk) store_lane<W>(o + 16 * j + wlo, a[j]);
        p += 16 * kk;
        o += 16 * kk;
        nfull -= kk;
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

template <int NR, int G>
static void coop_nr(const KBatch &b, Layout layout, KeyMode km, bool stream, int grid, int threads, hipStream_t st) {
#define FPNN_COOP(L, K, S) \
    hipLaunchKernelGGL((k_cfb_encrypt_coop<NR, L, K, S, 4, G>), dim3(grid), dim3(threads), 0, st, b)
    if (layout == LAYOUT_UNIFORM) {
        if (stream) FPNN_COOP(LAYOUT_UNIFORM, KEY_UNIFORM, true); else FPNN_COOP(LAYOUT_UNIFORM, KEY_UNIFORM, false);
    } else if (km == KEY_UNIFORM) {
        if (stream) FPNN_COOP(LAYOUT_GENERAL, KEY_UNIFORM, true); else FPNN_COOP(LAYOUT_GENERAL, KEY_UNIFORM, false);
    } else {
        if (stream) FPNN_COOP(LAYOUT_GENERAL, KEY_LANE, true); else FPNN_COOP(LAYOUT_GENERAL, KEY_LANE, false);
    }
#undef FPNN_COOP
}

template <int NR, int G>
static void queue_nr(const KBatch &b, KeyMode km, bool stream, int grid, int threads, uint32_t *next,
                     hipStream_t st) {
#define FPNN_QUEUE(K, STR) \
    hipLaunchKernelGGL((k_cfb_encrypt_queue<NR, K, STR, 4, G>), dim3(grid), dim3(threads), 0, st, b, next)
    if (km == KEY_UNIFORM) {
        if (stream) FPNN_QUEUE(KEY_UNIFORM, true); else FPNN_QUEUE(KEY_UNIFORM, false);
    } else {
        if (stream) FPNN_QUEUE(KEY_LANE, true); else FPNN_QUEUE(KEY_LANE, false);
    }
#undef FPNN_QUEUE
}

hipError_t launch_encrypt_queue(const KBatch &b, int nrounds, int group, KeyMode km, bool stream, int grid,
                                int threads, uint32_t *next, hipStream_t st) {
    if (group != 2 && group != 4) return hipErrorInvalidValue;
    hipError_t err = hipMemsetAsync(next, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    set_launched("cfb_encrypt_queue");
    switch (nrounds * 8 + group) {
        case 10 * 8 + 4: queue_nr<10, 4>(b, km, stream, grid, threads, next, st); break;
        case 12 * 8 + 4: queue_nr<12, 4>(b, km, stream, grid, threads, next, st); break;
        case 14 * 8 + 4: queue_nr<14, 4>(b, km, stream, grid, threads, next, st); break;
        case 10 * 8 + 2: queue_nr<10, 2>(b, km, stream, grid, threads, next, st); break;
        case 12 * 8 + 2: queue_nr<12, 2>(b, km, stream, grid, threads, next, st); break;
        case 14 * 8 + 2: queue_nr<14, 2>(b, km, stream, grid, threads, next, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_encrypt_coop(const KBatch &b, int nrounds, int group, Layout layout, KeyMode km, bool stream,
                               int grid, int threads, hipStream_t st) {
    set_launched("cfb_encrypt_coop");
    switch (nrounds * 8 + group) {
        case 10 * 8 + 4: coop_nr<10, 4>(b, layout, km, stream, grid, threads, st); break;
        case 12 * 8 + 4: coop_nr<12, 4>(b, layout, km, stream, grid, threads, st); break;
        case 14 * 8 + 4: coop_nr<14, 4>(b, layout, km, stream, grid, threads, st); break;
        case 10 * 8 + 2: coop_nr<10, 2>(b, layout, km, stream, grid, threads, st); break;
        case 12 * 8 + 2: coop_nr<12, 2>(b, layout, km, stream, grid, threads, st); break;
        case 14 * 8 + 2: coop_nr<14, 2>(b, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int blocks_per_cu(const Variant &v, KeyMode km) { return (km == KEY_UNIFORM && v.tables == 2) ? 2 : 1; }

namespace {
thread_local const char *g_launched = "";
}
const char *last_launched() { return g_launched; }
void set_launched(const char *name) { g_launched = name; }

hipError_t launch_encrypt_chains(const KBatch &b, int nrounds, const Variant &v, Layout layout, KeyMode km,
                                 bool stream, int grid, int threads, hipStream_t st) {
    set_launched("cfb_encrypt_chains");
    switch (nrounds) {
        case 10: enc_nr<10>(b, v, layout, km, stream, grid, threads, st); break;
        case 12: enc_nr<12>(b, v, layout, km, stream, grid, threads, st); break;
        case 14: enc_nr<14>(b, v, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
