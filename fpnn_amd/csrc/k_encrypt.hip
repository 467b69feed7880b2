// k_encrypt.hip -- CFB-128 encryption kernels for gfx950 (see segments.hpp for the
// segment semantics and aes_device.hpp for the LDS T-table round function).
//   K2  k_cfb_encrypt_chains : one lane per packet / stream chain.
//        C_i = P_i ^ E(C_{i-1}) is serial inside a chain (base/rijndael.c:1176-1185),
//        so parallelism is across packets (package mode) or streams (stream mode).
//   K2c k_cfb_encrypt_coop   : one lane quad per chain (few / long chains).
//   K2q k_cfb_encrypt_queue  : K2c with a work queue (many ragged chains).
//   All are persistent: workgroups walk the chains with a grid stride or the queue.
#include "coop.hpp"

namespace fpnn_aes {

// ---------------------------------------------------------------------------
// K2: encryption, one lane per chain.

template <int NR, int LAYOUT, int KM, bool STREAM, int NT, int CH, bool FENCE = false>
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
        if (C > 1 && (b.flags & F_ALIGN_CHUNKS)) {
            // a 16-B aligned segment that starts inside a 128-B line (1472-B datagrams:
            // every other one) runs its first blocks singly, so every chunk below reads
            // and writes whole lines (a chunk straddling two lines leaves half of each
            // to a later chunk, by which time L2 has often dropped it: re-read from HBM)
            const uint32_t mis = (uint32_t)(uintptr_t)p & 127u;
            uint32_t h = (mis & 15u) ? 0u : ((128u - mis) & 127u) >> 4;
            h = h < nfull ? h : nfull;
            for (; i < h; i++) {
                iv = aes_encrypt_block<NR, NT>(iv, rk, T) ^ load16(p);
                store16(q, iv);
                p += 16;
                q += 16;
            }
        }
        if (C > 1 && i + C <= nfull) {
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
                    iv = (FENCE ? aes_encrypt_block_fenced<NR, NT>(iv, rk, T) : aes_encrypt_block<NR, NT>(iv, rk, T)) ^ a[j];
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
// K2c: encryption, one lane QUAD per chain.  Lane q of the quad owns state column q:
// per round it does the 4 T-table lookups of its own 4 bytes and the quad sums the
// contributions with DPP quad_perm (VALU only; aes_encrypt_column below).  A chain
// therefore issues 4 LDS reads per lane and round instead of 16 -- 4x the lanes per
// chain and ~4x shorter per-chain critical path -- and holds 15 round-key words per
// lane instead of 60.  Used when chains are few (streams) or long/ragged.

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
// K2q: K2c's quad-per-chain cipher with a work queue instead of a grid stride.
// Chains are visited longest first (perm[]); a quad that finishes a chain takes the
// next one from a global counter at once, so lanes of a wave never wait for the
// longest chain of their wave (greedy longest-processing-time scheduling).  Each quad
// can carry S chains ("slots") whose ciphers run round-interleaved (a K2c round has
// only 4 lookups in flight per lane).  S = 2 measured 35 % slower on C4: the longest
// chains, which set the end of the launch, then advance at half speed.  The launcher
// uses S = 1.  The loop body is one step of up to CH blocks of every slot;
// a block past a slot's chain end is computed but not committed (a select, not a
// branch, so the two ciphers stay in one basic block).  The wave leaves the loop when
// no slot of any quad has work.  Used for ragged batches with more chains than quads
// (C4), where a static chain-to-lane assignment leaves most lanes idle.
template <int NR, int NT, int S>
__device__ __forceinline__ void aes_encrypt_columns(uint32_t (&sq)[S], const uint32_t (&rkq)[S][NR + 1],
                                                    const Tables4<NT> &T) {
    uint32_t st[S];
#pragma unroll
    for (int k = 0; k < S; k++) st[k] = sq[k] ^ rkq[k][0];
#pragma unroll
    for (int r = 1; r < NR; r++) {
#pragma unroll
        for (int k = 0; k < S; k++) {
            const uint32_t t0 = T.template t<0>(st[k]), t1 = T.template t<1>(st[k]), t2 = T.template t<2>(st[k]),
                           t3 = T.template t<3>(st[k]);
            st[k] = xor3(xor_quad_from<1>(t0, t1), xor_quad_from<2>(rkq[k][r], t2), quad_from<3>(t3));
        }
    }
#pragma unroll
    for (int k = 0; k < S; k++) {
        const uint32_t m0 = T.template sraw<0>(st[k]) & 0x000000ffu, m1 = T.template sraw<1>(st[k]) & 0x0000ff00u,
                       m2 = T.template sraw<2>(st[k]) & 0x00ff0000u, m3 = T.template sraw<3>(st[k]) & 0xff000000u;
        sq[k] = xor3(xor_quad_from<1>(m0, m1), xor_quad_from<2>(rkq[k][NR], m2), quad_from<3>(m3));
    }
}

template <int NR, int KM, bool STREAM, int NT, int S, bool FIRST_PRIO = true>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_encrypt_queue(KBatch b, uint32_t *next) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = (int)(threadIdx.x & 3u);
    const int wlo = 4 * q;  // block bytes [wlo, wlo + 4) belong to this lane
    constexpr int CH = 8;
    const uint64_t nquads = ((uint64_t)gridDim.x * blockDim.x) >> 2;

    uint32_t rkq[S][NR + 1];
    if (KM == KEY_UNIFORM) {
#pragma unroll
        for (int r = 0; r <= NR; r++) {
            const uint32_t w = b.keys[0].rk[4 * r + q];
#pragma unroll
            for (int k = 0; k < S; k++) rkq[k][r] = w;
        }
    }
    // per-slot chain state
    uint64_t sid[S];
    const uint8_t *p[S];
    uint8_t *o[S];
    uint32_t nfull[S], tail[S], n[S], iv[S];
    bool active[S];
#pragma unroll
    for (int k = 0; k < S; k++) {
        sid[k] = 0; p[k] = nullptr; o[k] = nullptr;
        nfull[k] = tail[k] = n[k] = iv[k] = 0;
        active[k] = false;
    }

    auto begin = [&](int k, uint64_t t) {  // slot k takes chain perm[t] (t < count), runs its head
        const uint64_t s = b.perm ? b.perm[t] : t;
        sid[k] = s;
        const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
        const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
        if (KM != KEY_UNIFORM) {
#pragma unroll
            for (int r = 0; r <= NR; r++) rkq[k][r] = key->rk[4 * r + q];
        }
        uint32_t v, pos;
        if (STREAM) {
            v = reinterpret_cast<const uint32_t *>(b.iv_state + 16 * s)[q];
            pos = b.pos_state[s];
        } else {
            v = reinterpret_cast<const uint32_t *>(key->iv)[q];
            pos = 0;
        }
        const uint8_t *pp = g.in;
        uint8_t *oo = g.out;
        uint32_t rem = g.len;
        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
            if (q == 0) store_word_bytes(oo, rem, 0, 4);
            oo += 4;
        }
        if (STREAM && pos != 0 && rem != 0) {  // rest of the partially used keystream block
            const uint32_t take = rem < 16 - pos ? rem : 16 - pos;
            const int lo = max((int)pos, wlo) - wlo, hi = min((int)(pos + take), wlo + 4) - wlo;
            if (lo < hi) {
                const uint32_t c = load_word_bytes(pp - pos + wlo, lo, hi) ^ v;
                store_word_bytes(oo - pos + wlo, c, lo, hi);
                const uint32_t m = word_mask(lo, hi);
                v = (c & m) | (v & ~m);
            }
            pp += take;
            oo += take;
            rem -= take;
            pos = (pos + take) & 15u;
        }
        iv[k] = v;
        n[k] = pos;
        p[k] = pp;
        o[k] = oo;
        nfull[k] = rem >> 4;
        tail[k] = rem & 15u;
        active[k] = true;
    };
    auto finish = [&](int k) {  // partial final block and the stream state
        if (tail[k]) {
            const uint32_t ks = aes_encrypt_column<NR, NT>(iv[k], rkq[k], T);
            const int hi = min((int)tail[k], wlo + 4) - wlo;
            if (hi > 0) {
                const uint32_t c = load_word_bytes(p[k] + wlo, 0, hi) ^ ks;
                store_word_bytes(o[k] + wlo, c, 0, hi);
                const uint32_t m = word_mask(0, hi);
                iv[k] = (c & m) | (ks & ~m);
            } else {
                iv[k] = ks;
            }
            n[k] = tail[k];
        }
        if (STREAM) {
            reinterpret_cast<uint32_t *>(b.iv_state + 16 * sid[k])[q] = iv[k];
            if (q == 0) b.pos_state[sid[k]] = n[k];
        }
    };
    // First chains: the longest (perm[] order) are dealt round-robin over the
    // workgroups -- quad j of workgroup w takes chain j * gridDim.x + w -- so the few
    // longest chains, which set the end of the launch, sit on different CUs and in the
    // first wave of each; that wave runs at raised priority so its chain's rounds are
    // not queued behind the 15 other waves' (the critical path of a greedy schedule
    // is its longest job).  Later chains come from the counter (from S * nquads on).
    const uint64_t t0 = (uint64_t)(threadIdx.x >> 2) * gridDim.x + blockIdx.x;
    if (FIRST_PRIO && threadIdx.x < 64) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int k = 0; k < S; k++)
        if (t0 + k * nquads < b.count) begin(k, t0 + k * nquads);
    while (true) {
        bool any = false;
#pragma unroll
        for (int k = 0; k < S; k++) any = any || active[k];
        if (__builtin_amdgcn_ballot_w64(any) == 0) break;
        // slots whose chain has no whole block left: finish it, take the next chain
#pragma unroll
        for (int k = 0; k < S; k++) {
            if (active[k] && nfull[k] == 0) {
                finish(k);
                uint32_t t = 0;
                if (q == 0) t = atomicAdd(next, 1u);
                // broadcast the quad leader's ticket (DPP quad_perm 0,0,0,0)
                const uint64_t tt = (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x00, 0xf, 0xf, true) +
                                    (uint64_t)S * nquads;  // 64-bit: no wrap near count = 2^32 - 1
                active[k] = false;
                if (tt < b.count) begin(k, tt);
            }
        }
        uint32_t kk[S];
        uint32_t a[S][CH];
#pragma unroll
        for (int k = 0; k < S; k++) {
            uint32_t lim = CH;
            if (b.flags & F_ALIGN_CHUNKS) {
                // line-aligned steps (as K2): a chain whose input and output sit at the
                // same 16-B multiple inside a 128-B line takes a short first step to the
                // line boundary, so every later step reads and writes whole lines back to
                // back instead of leaving half of each line to the next step (C4: 64-B
                // packet offsets; write bytes 1.17x -> 1.00x of algorithmic).  Aligning
                // the output alone when the two differ (wire frames: 4-byte prefix)
                // measured 2.4x slower, so those chains keep the unaligned steps.
                const uint32_t xo = (uint32_t)(uintptr_t)o[k] & 127u, xi = (uint32_t)(uintptr_t)p[k] & 127u;
                if (xo == xi && !(xo & 15u)) lim = CH - (xo >> 4);
            }
            kk[k] = active[k] ? (nfull[k] < lim ? nfull[k] : lim) : 0u;
#pragma unroll
            for (int j = 0; j < CH; j++)
                a[k][j] = j < (int)kk[k] ? *reinterpret_cast<const uint32_u *>(p[k] + 16 * j + wlo) : 0u;
        }
        // (a quad with no work in any slot still runs the rounds: its results are
        // dropped like those of blocks past a chain's end)
#pragma unroll
        for (int j = 0; j < CH; j++) {
            uint32_t e[S];
#pragma unroll
            for (int k = 0; k < S; k++) e[k] = iv[k];
            aes_encrypt_columns<NR, NT, S>(e, rkq, T);
#pragma unroll
            for (int k = 0; k < S; k++) {
                const uint32_t c = e[k] ^ a[k][j];  // C_i = P_i ^ E(C_{i-1})
                iv[k] = j < (int)kk[k] ? c : iv[k];
                a[k][j] = c;
            }
        }
#pragma unroll
        for (int k = 0; k < S; k++) {
#pragma unroll
            for (int j = 0; j < CH; j++)
                if (j < (int)kk[k]) *reinterpret_cast<uint32_u *>(o[k] + 16 * j + wlo) = a[k][j];
            p[k] += 16 * kk[k];
            o[k] += 16 * kk[k];
            nfull[k] -= kk[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Launchers (runtime -> template dispatch)

// Variant selection.  Per-packet keys need ~100 VGPRs of round keys, so they always
// use the 4-table layout (one workgroup per CU); uniform-key variants take the
// layout the engine asks for.
template <int NR, int NT, int CH>
static void enc_launch(const KBatch &b, Layout layout, KeyMode km, bool stream, bool fence, int grid, int threads,
                       hipStream_t st) {
#define FPNN_ENC(L, K, S, NTX) \
    hipLaunchKernelGGL((k_cfb_encrypt_chains<NR, L, K, S, NTX, CH>), dim3(grid), dim3(threads), 0, st, b)
    if (layout == LAYOUT_UNIFORM && !stream && fence && NT == 4 && CH == 8) {  // C2 with fenced rounds
        hipLaunchKernelGGL((k_cfb_encrypt_chains<NR, LAYOUT_UNIFORM, KEY_UNIFORM, false, 4, 8, true>), dim3(grid),
                           dim3(threads), 0, st, b);
    } else if (layout == LAYOUT_UNIFORM) {
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
        if (v.enc_chunk == 4) enc_launch<NR, 2, 4>(b, layout, km, stream, v.fence, grid, threads, st);
        else enc_launch<NR, 2, 1>(b, layout, km, stream, v.fence, grid, threads, st);
    } else {
        if (v.enc_chunk == 8) enc_launch<NR, 4, 8>(b, layout, km, stream, v.fence, grid, threads, st);
        else if (v.enc_chunk == 4) enc_launch<NR, 4, 4>(b, layout, km, stream, v.fence, grid, threads, st);
        else enc_launch<NR, 4, 1>(b, layout, km, stream, v.fence, grid, threads, st);
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

template <int NR>
static void queue_nr(const KBatch &b, KeyMode km, bool stream, int grid, int threads, uint32_t *next,
                     hipStream_t st) {
#define FPNN_QUEUE(K, STR) \
    hipLaunchKernelGGL((k_cfb_encrypt_queue<NR, K, STR, 4, 1>), dim3(grid), dim3(threads), 0, st, b, next)
    if (km == KEY_UNIFORM) {
        if (stream) FPNN_QUEUE(KEY_UNIFORM, true); else FPNN_QUEUE(KEY_UNIFORM, false);
    } else {
        if (stream) FPNN_QUEUE(KEY_LANE, true); else FPNN_QUEUE(KEY_LANE, false);
    }
#undef FPNN_QUEUE
}

hipError_t launch_encrypt_queue(const KBatch &b, int nrounds, KeyMode km, bool stream, int grid, int threads,
                                uint32_t *next, hipStream_t st) {
    hipError_t err = hipMemsetAsync(next, 0, sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    set_launched("cfb_encrypt_queue");
    switch (nrounds) {
        case 10: queue_nr<10>(b, km, stream, grid, threads, next, st); break;
        case 12: queue_nr<12>(b, km, stream, grid, threads, next, st); break;
        case 14: queue_nr<14>(b, km, stream, grid, threads, next, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_encrypt_coop(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool stream, int grid,
                               int threads, hipStream_t st) {
    set_launched("cfb_encrypt_coop");
    switch (nrounds) {
        case 10: coop_nr<10>(b, layout, km, stream, grid, threads, st); break;
        case 12: coop_nr<12>(b, layout, km, stream, grid, threads, st); break;
        case 14: coop_nr<14>(b, layout, km, stream, grid, threads, st); break;
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
