// k_encrypt.hip -- CFB-128 encryption kernels for gfx950 (see segments.hpp for the
// segment semantics and aes_device.hpp for the LDS T-table round function).
//   K2  k_cfb_encrypt_chains : one lane per packet / stream chain.
//        C_i = P_i ^ E(C_{i-1}) is serial inside a chain (base/rijndael.c:1176-1185),
//        so parallelism is across packets (package mode) or streams (stream mode).
//   K2c k_cfb_encrypt_coop   : one lane quad per chain (few / long chains).
//   Both are persistent: workgroups walk the chains with a grid stride (ragged batches
//   with more chains than quads go to K2h, k_hybrid.hip).
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
    // Package mode: every chain of a key slot starts from the slot's IV, so its first
    // keystream block E_k(IV) is a per-slot constant (point 3) -- with one
    // key computed once per lane here, with per-lane keys read from the key set's table
    // (b.eiv).  Where a wave's lanes start their chains at the same step (uniform lengths:
    // C2, U1) the wave skips block 0's rounds together.
    constexpr bool kFirst = !STREAM;
    const bool use_eiv = kFirst && (KM == KEY_UNIFORM || b.eiv != nullptr);
    uint4 eiv_u = make_uint4(0, 0, 0, 0);
    if (kFirst && KM == KEY_UNIFORM) eiv_u = aes_encrypt_block<NR, NT>(*reinterpret_cast<const uint4 *>(b.keys->iv), rku, T);

    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    // per-lane keys: kept while the lane's next chain has the same slot (a connection's
    // frames a grid stride apart; Q1's 16 384 connections: every chain of a lane) -- the
    // reload is 240 B per lane from L2 / the Infinity Cache per chain otherwise
    RoundKeys<NR> rk;
    uint32_t rk_slot = ~0u;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < b.count; s += nthreads) {
        const Seg g = get_seg<LAYOUT>(b, s);
        FA_DECL(a_ilo = (uintptr_t)g.in, a_ihi = (uintptr_t)g.in + g.len, a_olo = (uintptr_t)g.out,
                a_ohi = (uintptr_t)g.out + g.len + ((b.flags & F_WIRE_PREFIX) ? 4u : 0u));
        const DevKey *key = FA_AT(b, AB_KEYS, b.keys + (KM == KEY_UNIFORM ? 0u : g.slot), sizeof(DevKey));
        if (KM == KEY_UNIFORM) {
            rk = rku;
        } else if (g.slot != rk_slot) {
            rk = load_round_keys<NR>(key);
            rk_slot = g.slot;
        }
        uint4 eiv = eiv_u;
        if (kFirst && KM != KEY_UNIFORM && use_eiv) eiv = *FA_AT(b, AB_EIV, b.eiv + g.slot, 16);

        uint4 iv;
        uint32_t n = 0;
        if (STREAM) {
            iv = ld_state_iv(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16));
            n = *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4);
        } else {
            iv = *reinterpret_cast<const uint4 *>(key->iv);
        }
        const uint8_t *p = g.in;
        uint8_t *q = g.out;
        uint32_t rem = g.len;

        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {  // htole32(len) ‖ ciphertext (core/Encryptor.cpp:47-48)
            uint8_t *qp = FA_RG(b, AB_OUT, q, 0, 4, a_olo, a_ohi);
            qp[0] = (uint8_t)rem;
            qp[1] = (uint8_t)(rem >> 8);
            qp[2] = (uint8_t)(rem >> 16);
            qp[3] = (uint8_t)(rem >> 24);
            q += 4;
        }

        if (STREAM && n != 0 && rem != 0) {  // finish the partially consumed keystream block
            const uint32_t take = rem < 16 - n ? rem : 16 - n;
            const int lo = (int)n, hi = (int)(n + take);
            const uint4 o = load_bytes(FA_RG(b, AB_IN, p - n, lo, hi, a_ilo, a_ihi), lo, hi) ^ iv;
            store_bytes(FA_RG(b, AB_OUT, q - n, lo, hi, a_olo, a_ohi), o, lo, hi);
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
                iv = (use_eiv && i == 0 ? eiv : aes_encrypt_block<NR, NT>(iv, rk, T)) ^
                     load16(FA_SEG(b, AB_IN, p, 16, a_ilo, a_ihi));
                store16(FA_SEG(b, AB_OUT, q, 16, a_olo, a_ohi), iv);
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
            for (int j = 0; j < C; j++) a[j] = load16(FA_SEG(b, AB_IN, p + 16 * j, 16, a_ilo, a_ihi));
            for (; i + C <= nfull; i += C) {
                // the next chunk's loads, unconditional (the last chunk reads the first
                // DevKey's 128+ bytes, an L2 hit, not its own chunk again: that cost C2 an
                // eighth of its reads in HBM traffic): a load under a branch leaves the
                // waitcnt pass unsure how many are in flight, and it then drains all of them
                // (vmcnt(0)) inside the next chunk
                const bool more = i + 2 * C <= nfull;
                const uint8_t *pn = more ? p + 16 * C : reinterpret_cast<const uint8_t *>(b.keys);
                uint4 nx[C];
#pragma unroll
                for (int j = 0; j < C; j++)
                    nx[j] = load16(more ? FA_SEG(b, AB_IN, pn + 16 * j, 16, a_ilo, a_ihi) : FA_AT(b, AB_KEYS, pn + 16 * j, 16));
#pragma unroll
                for (int j = 0; j < C; j++) {
                    uint4 ks;
                    if (use_eiv && j == 0 && i == 0)  // the chain's first block (wave-uniform)
                        ks = eiv;
                    else
                        ks = FENCE ? aes_encrypt_block_fenced<NR, NT>(iv, rk, T) : aes_encrypt_block<NR, NT>(iv, rk, T);
                    iv = ks ^ a[j];
                    a[j] = iv;
                }
#pragma unroll
                for (int j = 0; j < C; j++) store16(FA_SEG(b, AB_OUT, q + 16 * j, 16, a_olo, a_ohi), a[j]);
#pragma unroll
                for (int j = 0; j < C; j++) a[j] = nx[j];
                p += 16 * C;
                q += 16 * C;
            }
        }
        uint4 pt = i < nfull ? load16(FA_SEG(b, AB_IN, p, 16, a_ilo, a_ihi)) : make_uint4(0, 0, 0, 0);
        for (; i < nfull; i++) {
            const uint4 pn = (i + 1 < nfull) ? load16(FA_SEG(b, AB_IN, p + 16, 16, a_ilo, a_ihi)) : make_uint4(0, 0, 0, 0);  // prefetch
            iv = (use_eiv && i == 0 ? eiv : aes_encrypt_block<NR, NT>(iv, rk, T)) ^ pt;  // C_i = P_i ^ E(C_{i-1})
            store16(FA_SEG(b, AB_OUT, q, 16, a_olo, a_ohi), iv);
            pt = pn;
            p += 16;
            q += 16;
        }
        rem &= 15u;
        if (rem) {  // partial final block: ivec = E(C) with the first rem bytes replaced
            const uint4 ks = use_eiv && nfull == 0 ? eiv : aes_encrypt_block<NR, NT>(iv, rk, T);
            const uint4 o = load_bytes(FA_RG(b, AB_IN, p, 0, rem, a_ilo, a_ihi), 0, (int)rem) ^ ks;
            store_bytes(FA_RG(b, AB_OUT, q, 0, rem, a_olo, a_ohi), o, 0, (int)rem);
            iv = select_bytes(byte_mask(0, (int)rem), o, ks);
            n = rem;
        }
        if (STREAM) {
            *reinterpret_cast<uint4 *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16)) = iv;
            *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4) = n;
        }
    }
}

// ---------------------------------------------------------------------------
// K2s: short frames (FPNN's quests: 145-B frames from many keyed connections, the caller's
// max_len <= kFrameMaxBytes), one lane per chain in grid-stride order like K2, but a
// chain's whole frame is loaded at once, ciphered in registers and stored at once.
// K2 steps through a frame in 4-block chunks; adjacent lanes' frames share their first and
// last 128-byte lines, and with 1024 lanes per CU of ~145-B frames in flight the lines a
// chunk touches left L2 before the chunk that needed their other half came: Q1 moved 2.35x
// its algorithmic HBM bytes (reads 2.52x, writes 2.16x; profiles/r05/Q1s_final, VERDICT r05
// item 3).  Here a wave's 64 frames -- one contiguous span for a collector's flush -- are
// read by back-to-back loads and written by back-to-back stores, so every line is read
// once and written whole while L2 still holds it: 1.01-1.02x.

// A frame past the pipeline's slots (past the caller's bound, or under 16 B) in MAXB-block
// passes: K2s-DB's rare path.
template <int NR, int KM, bool WIRE, int MAXB>
__device__ __forceinline__ void frame_passes(const KBatch &b, const Seg &g, const uint4 &eiv, const RoundKeys<NR> &key,
                                             const Tables4<4> &T, const uint8_t *dummy) {
    constexpr bool kTailSlot = true;
    constexpr int NT = 4;
    FA_DECL(a_ilo = (uintptr_t)g.in, a_ihi = (uintptr_t)g.in + g.len, a_olo = (uintptr_t)g.out,
            a_ohi = (uintptr_t)g.out + g.len + (WIRE ? 4u : 0u));
    uint4 iv = make_uint4(0, 0, 0, 0);
    const uint8_t *p = g.in;
    uint8_t *o = g.out;
    const uint32_t nfull = g.len >> 4, tail = g.len & 15u;
    if (WIRE) {  // htole32(len) || ciphertext (core/Encryptor.cpp:47-48)
        store_bytes(FA_RG(b, AB_OUT, o, 0, 4, a_olo, a_ohi), make_uint4(g.len, 0u, 0u, 0u), 0, 4);
        o += 4;
    }
    // MAXB blocks at a time -- a frame within the caller's bound is ONE pass: its blocks
    // loaded back to back (lanes past their frame's blocks re-read the key table),
    // ciphered in registers, stored back to back.  A partial final block takes the next
    // free slot of its pass as a whole 16-byte block when those 16 bytes lie in one
    // 4 KiB page (the page of its first byte, which the frame's own bytes map): it is
    // then ciphered like the others and costs no round trip of its own (Q1s +17 %,
    // r06h).  The bytes past the frame are read, never used or written.
    uint32_t done = 0;
    bool tail_done = !tail;
    do {
        const uint32_t nb = nfull - done < (uint32_t)MAXB ? nfull - done : (uint32_t)MAXB;
        const uint64_t ta = (uint64_t)(uintptr_t)(p + 16 * nb);
        const bool tin = kTailSlot && !tail_done && done + nb == nfull && nb < (uint32_t)MAXB &&
                         ((ta ^ (ta + 15)) >> 12) == 0;
        uint4 a[MAXB];
        auto load_slot = [&](int j) {
            return load16(j < (int)nb               ? FA_SEG(b, AB_IN, p + 16 * j, 16, a_ilo, a_ihi)
                          : (tin && j == (int)nb) ? FA_SEG(b, AB_IN, p + 16 * j, tail, a_ilo, a_ihi)
                                                  : FA_AT(b, AB_KEYS, dummy + 16 * j, 16));
        };
#pragma unroll
        for (int j = 0; j < MAXB; j++) a[j] = load_slot(j);
        // block 0's keystream is the slot's E_k(IV): every lane of the wave starts its
        // chain here together (point 3)
#pragma unroll
        for (int j = 0; j < MAXB; j++) {
            if (j < (int)nb || (tin && j == (int)nb)) {
                const uint4 ks =
                    j == 0 && done == 0 ? eiv : aes_encrypt_block<NR, NT>(iv, key, T);
                iv = ks ^ a[j];  // C_i = P_i ^ E(C_{i-1})
                a[j] = iv;
            }
        }
        uint4 t = a[0];  // the partial block's slot, picked by selects
#pragma unroll
        for (int j = 1; j < MAXB; j++)
            if (j == (int)nb) t = a[j];
#pragma unroll
        for (int j = 0; j < MAXB; j++)
            if (j < (int)nb) store16(FA_SEG(b, AB_OUT, o + 16 * j, 16, a_olo, a_ohi), a[j]);
        if (tin) store_bytes(FA_RG(b, AB_OUT, o + 16 * nb, 0, tail, a_olo, a_ohi), t, 0, (int)tail);
        p += 16 * nb;
        o += 16 * nb;
        done += nb;
        tail_done |= tin;
    } while (done < nfull);
    if (!tail_done) {  // partial final block after a full pass (or a frame under 16 B):
                       // keystream from the last whole block, or E_k(IV)
        const uint4 ks = nfull == 0 ? eiv : aes_encrypt_block<NR, NT>(iv, key, T);
        const uint4 c = load_bytes(FA_RG(b, AB_IN, p, 0, tail, a_ilo, a_ihi), 0, (int)tail) ^ ks;
        store_bytes(FA_RG(b, AB_OUT, o, 0, tail, a_olo, a_ohi), c, 0, (int)tail);
    }
}

// ---------------------------------------------------------------------------
// K2s-DB: K2s with the next chain's frame in flight while this one is ciphered.  In K2s every
// chain starts with the same two round trips (descriptor, then frame), and the waves of a CU
// start their chains together: at Q1's 10 blocks per chain the CU's LDS idles while 1024
// lanes wait on 160 KiB of loads (0.61 busy, SQ_WAIT_ANY 0.51, profiles/r06/Q1).  Here the
// next chain's descriptor is read at the top of the chain, its frame and E_k(IV) behind this
// chain's block 1, so they land while the rounds run.  Two frames of registers per lane
// (2 x 40 VGPRs) do not fit at 4 waves per SIMD with per-lane round keys: the kernel runs
// OCC waves per SIMD (256 * OCC threads a workgroup, one workgroup per CU).
//
// A frame "fits" when its whole blocks and partial block take at most MAXB slots; its
// partial block is then loaded as the frame's LAST 16 bytes (inside the frame) and shifted
// down.  Frames past the caller's bound and frames under 16 B take frame_passes (encrypt)
// or frame_decrypt_blocks (decrypt).
//
// Measured and not kept (tools/ab_frames.py over tools/probe/build_variant.sh builds, DESIGN
// section 4): K2s at 4 waves per SIMD with no frame in flight (Q1s 903-916, Q1w 754 against
// 960-968 / 891-939); 3 waves per SIMD (spills with AES-256 lane keys); two store bursts
// per frame, the next frame loading into the first half's registers; the next descriptor
// alone loaded ahead; waves of a CU started a chain step apart; a decrypt's passes run 2 or
// 3 at a time, round-interleaved (equal); every global access of the steady state issued
// unconditionally -- buffer stores through an output window, unused slots dropped past it
// -- so that the compiler's waits count them instead of collapsing to vmcnt(0) at each
// join (with fenced rounds: encrypt equal, Q1s decrypt 990 -> 972, profiles/r06/ab_fence).

struct FrameShape {
    uint32_t nfull, tail;
    bool fit;
};

__device__ __forceinline__ FrameShape frame_shape(const Seg &g, int maxb) {
    FrameShape f;
    f.nfull = g.len >> 4;
    f.tail = g.len & 15u;
    f.fit = f.nfull + (f.tail ? 1u : 0u) <= (uint32_t)maxb && (f.nfull > 0 || f.tail == 0);
    return f;
}

template <int MAXB>
__device__ __forceinline__ void frame_issue(const KBatch &b, const Seg &g, const FrameShape &f, uint4 (&x)[MAXB],
                                            const uint8_t *dummy) {
    FA_DECL(a_ilo = (uintptr_t)g.in, a_ihi = (uintptr_t)g.in + g.len);
#pragma unroll
    for (int j = 0; j < MAXB; j++)
        x[j] = load16(j < (int)f.nfull                   ? FA_SEG(b, AB_IN, g.in + 16 * j, 16, a_ilo, a_ihi)
                      : (f.tail && j == (int)f.nfull) ? FA_SEG(b, AB_IN, g.in + g.len - 16, 16, a_ilo, a_ihi)
                                                      : FA_AT(b, AB_KEYS, dummy + 16 * j, 16));
}

// Store a fitted frame's slots in one burst: its whole blocks, then its partial block.
template <int MAXB>
__device__ __forceinline__ void frame_store(const KBatch &b, const uint4 (&A)[MAXB], const FrameShape &f, uint8_t *o,
                                            uint64_t a_olo, uint64_t a_ohi) {
    (void)a_olo;
    (void)a_ohi;
    uint4 t = A[0];  // the partial block's slot, picked by selects
#pragma unroll
    for (int j = 1; j < MAXB; j++)
        if (j == (int)f.nfull) t = A[j];
#pragma unroll
    for (int j = 0; j < MAXB; j++)
        if (j < (int)f.nfull) store16(FA_SEG(b, AB_OUT, o + 16 * j, 16, a_olo, a_ohi), A[j]);
    if (f.tail) store_bytes(FA_RG(b, AB_OUT, o + 16 * f.nfull, 0, f.tail, a_olo, a_ohi), t, 0, (int)f.tail);
}

// One chain of a decrypt past the bound (or under 16 B): block by block.  P_i = C_i ^
// E(C_{i-1}), P_0 = C_0 ^ E_k(IV).
template <int NR>
__device__ __forceinline__ void frame_decrypt_blocks(const KBatch &b, const Seg &g, const uint4 &eiv,
                                                     const RoundKeys<NR> &key, const Tables4<4> &T) {
    FA_DECL(a_ilo = (uintptr_t)g.in, a_ihi = (uintptr_t)g.in + g.len, a_olo = (uintptr_t)g.out,
            a_ohi = (uintptr_t)g.out + g.len);
    const uint32_t nfull = g.len >> 4, tail = g.len & 15u;
    uint4 prev = make_uint4(0, 0, 0, 0);
    for (uint32_t i = 0; i < nfull; i++) {
        const uint4 c = load16(FA_SEG(b, AB_IN, g.in + 16 * i, 16, a_ilo, a_ihi));
        const uint4 ks = i == 0 ? eiv : aes_encrypt_block<NR, 4>(prev, key, T);
        store16(FA_SEG(b, AB_OUT, g.out + 16 * i, 16, a_olo, a_ohi), c ^ ks);
        prev = c;
    }
    if (tail) {
        const uint4 ks = nfull == 0 ? eiv : aes_encrypt_block<NR, 4>(prev, key, T);
        const uint4 c = load_bytes(FA_RG(b, AB_IN, g.in + 16 * nfull, 0, tail, a_ilo, a_ihi), 0, (int)tail);
        store_bytes(FA_RG(b, AB_OUT, g.out + 16 * nfull, 0, tail, a_olo, a_ohi), c ^ ks, 0, (int)tail);
    }
}

// DEC: the same pipeline decrypts (D2s): block j's keystream is E(C_{j-1}), the ciphertext
// just loaded, so a lane's AES passes are independent of each other.
template <int NR, int KM, bool WIRE, int OCC, bool DEC>
__global__ __launch_bounds__(256 * OCC) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void k_cfb_frames_db(
    KBatch b) {
    constexpr int NT = 4, MAXB = kFrameMaxBlocks;
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};

    RoundKeys<NR> rku;
    uint4 eiv_u = make_uint4(0, 0, 0, 0);
    if (KM == KEY_UNIFORM) {
        rku = load_round_keys<NR>(b.keys);
        eiv_u = aes_encrypt_block<NR, NT>(*reinterpret_cast<const uint4 *>(b.keys->iv), rku, T);
    }
    const uint8_t *const dummy = reinterpret_cast<const uint8_t *>(b.keys);  // 272 readable bytes
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    RoundKeys<NR> rk;
    if (KM != KEY_UNIFORM) {
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) rk.k[i] = 0u;
    }
    uint32_t rk_slot = ~0u;
    uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= b.count) return;  // (no barrier below)
    Seg g = get_seg<LAYOUT_GENERAL>(b, s);
    FrameShape fa = frame_shape(g, MAXB);
    uint4 eiv = KM == KEY_UNIFORM ? eiv_u : *FA_AT(b, AB_EIV, b.eiv + g.slot, 16);
    uint4 A[MAXB], B[MAXB];
    if (fa.fit) frame_issue<MAXB>(b, g, fa, A, dummy);
    for (;;) {
        const uint64_t sn = s + nthreads;
        const bool more = sn < b.count;
        const Seg gn = get_seg<LAYOUT_GENERAL>(b, more ? sn : s);  // (read now, used behind block 1)
        if (KM != KEY_UNIFORM && g.slot != rk_slot) {
            rk = load_round_keys<NR>(FA_AT(b, AB_KEYS, b.keys + g.slot, sizeof(DevKey)));
            rk_slot = g.slot;
        }
        FrameShape fb;
        fb.fit = false;
        uint4 eivn = eiv_u;
        if (fa.fit) {
            FA_DECL(a_olo = (uintptr_t)g.out, a_ohi = (uintptr_t)g.out + g.len + (WIRE ? 4u : 0u));
            uint8_t *const o = g.out + (WIRE ? 4 : 0);
            if (WIRE)  // htole32(len) || ciphertext (core/Encryptor.cpp:47-48)
                store_bytes(FA_RG(b, AB_OUT, g.out, 0, 4, a_olo, a_ohi), make_uint4(g.len, 0u, 0u, 0u), 0, 4);
            uint4 iv = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < MAXB; j++) {
                if (j == 2) {  // the next chain's frame and E_k(IV), behind this chain's block 1
                    fb = frame_shape(gn, MAXB);
                    fb.fit = fb.fit && more;
                    if (fb.fit) frame_issue<MAXB>(b, gn, fb, B, dummy);
                    if (KM != KEY_UNIFORM) eivn = *FA_AT(b, AB_EIV, b.eiv + gn.slot, 16);
                }
                if (j < (int)fa.nfull || (fa.tail && j == (int)fa.nfull)) {
                    // fenced rounds (every lookup of a round issued before any fold): Q1 encrypt /
                    // decrypt 784-786 / 782-792 -> 811-813 / 815-823 GiB/s, Q1s 961-963 / 963-966
                    // -> 985-988 / 990-991, Q1w 921 -> 929-931 (profiles/r06/ab_fence)
                    const uint4 ks = j == 0 ? eiv : aes_encrypt_block_fenced<NR, NT>(iv, KM == KEY_UNIFORM ? rku : rk, T);
                    const uint4 x = j == (int)fa.nfull ? shr_bytes(A[j], 16 - (int)fa.tail) : A[j];
                    if (DEC) {  // P_i = C_i ^ E(C_{i-1}); iv carries the ciphertext
                        A[j] = x ^ ks;
                        iv = x;
                    } else {  // C_i = P_i ^ E(C_{i-1})
                        iv = ks ^ x;
                        A[j] = iv;
                    }
                }
            }
            frame_store<MAXB>(b, A, fa, o, FA_ARGS(a_olo, a_ohi));  // (one burst: two measured slower, r06l)
        } else {
            if (DEC) frame_decrypt_blocks<NR>(b, g, eiv, KM == KEY_UNIFORM ? rku : rk, T);
            else frame_passes<NR, KM, WIRE, MAXB>(b, g, eiv, KM == KEY_UNIFORM ? rku : rk, T, dummy);
            fb = frame_shape(gn, MAXB);
            fb.fit = fb.fit && more;
            if (fb.fit) frame_issue<MAXB>(b, gn, fb, B, dummy);
            if (KM != KEY_UNIFORM) eivn = *FA_AT(b, AB_EIV, b.eiv + gn.slot, 16);
        }
        if (!more) break;
        s = sn;
        g = gn;
        fa = fb;
        eiv = eivn;
#pragma unroll
        for (int j = 0; j < MAXB; j++) A[j] = B[j];
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
__global__ __launch_bounds__(kThreads, 4) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_cfb_encrypt_coop(KBatch b) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = (int)(threadIdx.x & 3u);
    constexpr int CH = 8;

    const uint64_t nquads = ((uint64_t)gridDim.x * blockDim.x) >> 2;
    for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; t < b.count; t += nquads) {
        const uint64_t s = b.perm ? min(*FA_AT(b, AB_PERM, b.perm + t, 4), (uint32_t)b.count - 1u) : t;  // longest chains first (ragged batches)
        const Seg g = get_seg<LAYOUT>(b, s);
        FA_DECL(a_ilo = (uintptr_t)g.in, a_ihi = (uintptr_t)g.in + g.len, a_olo = (uintptr_t)g.out,
                a_ohi = (uintptr_t)g.out + g.len + ((b.flags & F_WIRE_PREFIX) ? 4u : 0u));
        const DevKey *key = FA_AT(b, AB_KEYS, b.keys + (KM == KEY_UNIFORM ? 0u : g.slot), sizeof(DevKey));
        uint32_t rkq[NR + 1];
#pragma unroll
        for (int r = 0; r <= NR; r++) rkq[r] = key->rk[4 * r + q];

        uint32_t iv;  // this lane's word of the 16-byte feedback register
        uint32_t n = 0;
        // package mode: block 0's keystream E_k(IV) from the key set's table (the quads of a
        // wave start their chains together on C5-like batches: the wave skips those rounds)
        const bool use_eiv = !STREAM && b.eiv != nullptr;
        uint32_t ew = 0;  // this lane's word of E_k(IV)
        if (STREAM) {
            iv = reinterpret_cast<const uint32_t *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16))[q];
            n = *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4);
        } else {
            iv = reinterpret_cast<const uint32_t *>(key->iv)[q];
            if (use_eiv)
                ew = reinterpret_cast<const uint32_t *>(FA_AT(b, AB_EIV, b.eiv + (KM == KEY_UNIFORM ? 0u : g.slot), 16))[q];
        }
        const uint8_t *p = g.in;
        uint8_t *o = g.out;
        uint32_t rem = g.len;
        if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
            if (q == 0) store_word_bytes(FA_RG(b, AB_OUT, o, 0, 4, a_olo, a_ohi), rem, 0, 4);
            o += 4;
        }
        const int wlo = 4 * q;  // block bytes [wlo, wlo + 4) belong to this lane
        if (STREAM && n != 0 && rem != 0) {  // rest of the partially used keystream block
            const uint32_t take = rem < 16 - n ? rem : 16 - n;
            const int lo = max((int)n, wlo) - wlo, hi = min((int)(n + take), wlo + 4) - wlo;
            if (lo < hi) {
                const uint32_t c = load_word_bytes(FA_RG(b, AB_IN, p - n + wlo, lo, hi, a_ilo, a_ihi), lo, hi) ^ iv;
                store_word_bytes(FA_RG(b, AB_OUT, o - n + wlo, lo, hi, a_olo, a_ohi), c, lo, hi);
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
            for (int j = 0; j < CH; j++) a[j] = *reinterpret_cast<const uint32_u *>(FA_SEG(b, AB_IN, p + 16 * j + wlo, 4, a_ilo, a_ihi));
            // the chain carries C ^ rk[0] (aes_chain_column: its two XORs folded into the keys)
            const uint32_t rkx = rkq[NR] ^ rkq[0];
            uint32_t sw = iv ^ rkq[0];
            for (; i + CH <= nfull; i += CH) {
                // the next step's words, unconditional (the last step reads the first
                // DevKey, an L2 hit): loads under a branch made the waitcnt pass drain them
                // all (vmcnt(0)) at the end of the step's first block -- one memory latency
                // per 8-block step (C5: K2c's SQ_WAIT_ANY 0.40 against SQ_WAIT_INST_LDS 0.09,
                // VERDICT r04 item 5)
                const bool more = i + 2 * CH <= nfull;
                const uint8_t *pn = (more ? p + 16 * CH : reinterpret_cast<const uint8_t *>(b.keys)) + wlo;
                uint32_t nx[CH], c[CH];
#pragma unroll
                for (int j = 0; j < CH; j++)
                    nx[j] = *reinterpret_cast<const uint32_u *>(more ? FA_SEG(b, AB_IN, pn + 16 * j, 4, a_ilo, a_ihi)
                                                                      : FA_AT(b, AB_KEYS, pn + 16 * j, 4));
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    if (j == 0 && use_eiv && i == 0)  // the chain's first block (quad-uniform)
                        sw = ew ^ a[j] ^ rkq[0];
                    else
                        sw = aes_chain_column<NR, NT>(sw, rkq, rkx ^ a[j], T);
                    c[j] = sw ^ rkq[0];
                }
                iv = c[CH - 1];
                // the step's 8 words go out together, each quad's 128-B line in 8 back-to-back
                // stores: stored one per block, a line sat partly written in L2 for a whole
                // step and C5 wrote 1.42x its output bytes to HBM (profiles/r05/C5)
#pragma unroll
                for (int j = 0; j < CH; j++) asm volatile("" : "+v"(c[j]));
#pragma unroll
                for (int j = 0; j < CH; j++) *reinterpret_cast<uint32_u *>(FA_SEG(b, AB_OUT, o + 16 * j + wlo, 4, a_olo, a_ohi)) = c[j];
                // the loaded words are handed on here, after the rounds: without this the
                // register allocator moved each nx[j] into a round's registers as soon as it
                // could, waiting (vmcnt) for loads issued one block earlier
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    asm volatile("" : "+v"(nx[j]));
                    a[j] = nx[j];
                }
                p += 16 * CH;
                o += 16 * CH;
            }
        }
        for (; i < nfull; i++) {
            const uint32_t pt = *reinterpret_cast<const uint32_u *>(FA_SEG(b, AB_IN, p + wlo, 4, a_ilo, a_ihi));
            iv = (use_eiv && i == 0 ? ew : aes_encrypt_column<NR, NT>(iv, rkq, T)) ^ pt;
            *reinterpret_cast<uint32_u *>(FA_SEG(b, AB_OUT, o + wlo, 4, a_olo, a_ohi)) = iv;
            p += 16;
            o += 16;
        }
        rem &= 15u;
        if (rem) {  // partial final block
            const uint32_t ks = use_eiv && nfull == 0 ? ew : aes_encrypt_column<NR, NT>(iv, rkq, T);
            const int lo = 0, hi = min((int)rem, wlo + 4) - wlo;
            if (hi > lo) {
                const uint32_t c = load_word_bytes(FA_RG(b, AB_IN, p + wlo, lo, hi, a_ilo, a_ihi), lo, hi) ^ ks;
                store_word_bytes(FA_RG(b, AB_OUT, o + wlo, lo, hi, a_olo, a_ohi), c, lo, hi);
                const uint32_t m = word_mask(lo, hi);
                iv = (c & m) | (ks & ~m);
            } else {
                iv = ks;
            }
            n = rem;
        }
        if (STREAM) {
            reinterpret_cast<uint32_t *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16))[q] = iv;
            if (q == 0) *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4) = n;
        }
    }
}

// ---------------------------------------------------------------------------
// Launchers (runtime -> template dispatch)

// Which K2 runs (the other sides of these choices were measured slower and removed in
// round 6, their A/B switches with them):
//   * package batches run the fenced round (every lookup of a round issued before any
//     fold): C2 and, on ragged batches, R1's wire send 919-930 -> 966-975 GiB/s, Q1 +1 %
//     (profiles/r05/ab_k2_fence_c4);
//   * per-lane AES-128/192 keys on ragged package batches take 4-block chunks (8-block
//     chunks spilled 14-26 VGPRs): Q1s 559-560 -> 636-638 GiB/s (same profile);
//   * stream batches keep the plain round (more live registers per lane).
template <int NR>
static void enc_nr(const KBatch &b, Layout layout, KeyMode km, bool stream, int grid, int threads, hipStream_t st) {
#define FPNN_ENC(L, K, S, CH, F) \
    hipLaunchKernelGGL((k_cfb_encrypt_chains<NR, L, K, S, 4, CH, F>), dim3(grid), dim3(threads), 0, st, b)
    if (layout == LAYOUT_UNIFORM) {
        if (stream) FPNN_ENC(LAYOUT_UNIFORM, KEY_UNIFORM, true, 8, false);
        else FPNN_ENC(LAYOUT_UNIFORM, KEY_UNIFORM, false, 8, true);
    } else if (stream) {
        if (km == KEY_UNIFORM) FPNN_ENC(LAYOUT_GENERAL, KEY_UNIFORM, true, 8, false);
        else FPNN_ENC(LAYOUT_GENERAL, KEY_LANE, true, 8, false);
    } else if (km == KEY_UNIFORM) {
        FPNN_ENC(LAYOUT_GENERAL, KEY_UNIFORM, false, 8, true);
    } else if (NR != 14) {
        FPNN_ENC(LAYOUT_GENERAL, KEY_LANE, false, 4, true);
    } else {
        FPNN_ENC(LAYOUT_GENERAL, KEY_LANE, false, 8, true);  // (AES-256 per-lane keys chunk by 4 anyway)
    }
#undef FPNN_ENC
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
    set_launched("cfb_encrypt_coop");
    switch (nrounds) {
        case 10: coop_nr<10>(b, layout, km, stream, grid, threads, st); break;
        case 12: coop_nr<12>(b, layout, km, stream, grid, threads, st); break;
        case 14: coop_nr<14>(b, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// K2s-DB's and D2s's waves per SIMD (3 spilled with AES-256 lane keys and measured slower,
// r06k / r06m; probe builds of tools/probe/build_variant.sh may set them)
#ifndef FPNN_AES_K2S_DB_OCC
#define FPNN_AES_K2S_DB_OCC 2
#endif
#ifndef FPNN_AES_D2S_OCC
#define FPNN_AES_D2S_OCC 2
#endif

template <int NR>
static void frames_nr(const KBatch &b, KeyMode km, bool wire, int grid, hipStream_t st) {
#define FPNN_FR(K, W)                                                                                              \
    hipLaunchKernelGGL((k_cfb_frames_db<NR, K, W, FPNN_AES_K2S_DB_OCC, false>), dim3(grid),                 \
                       dim3(256 * FPNN_AES_K2S_DB_OCC), 0, st, b)
    if (km == KEY_UNIFORM) {
        if (wire) FPNN_FR(KEY_UNIFORM, true); else FPNN_FR(KEY_UNIFORM, false);
    } else {
        if (wire) FPNN_FR(KEY_LANE, true); else FPNN_FR(KEY_LANE, false);
    }
#undef FPNN_FR
}

template <int NR>
static void dframes_nr(const KBatch &b, KeyMode km, int grid, hipStream_t st) {
#define FPNN_DF(K)                                                                                                 \
    hipLaunchKernelGGL((k_cfb_frames_db<NR, K, false, FPNN_AES_D2S_OCC, true>), dim3(grid),                 \
                       dim3(256 * FPNN_AES_D2S_OCC), 0, st, b)
    if (km == KEY_UNIFORM) FPNN_DF(KEY_UNIFORM);
    else FPNN_DF(KEY_LANE);
#undef FPNN_DF
}

hipError_t launch_decrypt_frames(const KBatch &b, int nrounds, KeyMode km, int grid, hipStream_t st) {
    set_launched("cfb_decrypt_frames");
    switch (nrounds) {
        case 10: dframes_nr<10>(b, km, grid, st); break;
        case 12: dframes_nr<12>(b, km, grid, st); break;
        case 14: dframes_nr<14>(b, km, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_encrypt_frames(const KBatch &b, int nrounds, KeyMode km, bool wire, int grid, hipStream_t st) {
    set_launched("cfb_encrypt_frames");
    switch (nrounds) {
        case 10: frames_nr<10>(b, km, wire, grid, st); break;
        case 12: frames_nr<12>(b, km, wire, grid, st); break;
        case 14: frames_nr<14>(b, km, wire, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

namespace {
thread_local const char *g_launched = "";
}
const char *last_launched() { return g_launched; }
void set_launched(const char *name) { g_launched = name; }

hipError_t launch_encrypt_chains(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool stream, int grid,
                                 int threads, hipStream_t st) {
    set_launched("cfb_encrypt_chains");
    switch (nrounds) {
        case 10: enc_nr<10>(b, layout, km, stream, grid, threads, st); break;
        case 12: enc_nr<12>(b, layout, km, stream, grid, threads, st); break;
        case 14: enc_nr<14>(b, layout, km, stream, grid, threads, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
