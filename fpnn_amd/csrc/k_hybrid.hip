// k_hybrid.hip -- K2h, CFB-128 encryption of ragged batches that hold more chains than the
// chip has lane quads (C4's Zipf packets, the wire-frame send side of R1).
//
// C_i = P_i ^ E(C_{i-1}) is serial inside a chain (base/rijndael.c:1176-1185), so a chain
// is one unit of work.  Two ways to run one:
//   * lane session (K2's cipher): one lane per chain, 16 independent T-table lookups per
//     lane and round, 1.5 VALU per lookup -- the LDS-efficient form, but a chain advances
//     one block per ~1024 lanes' worth of CU time;
//   * quad session (K2c's cipher): one 4-lane quad per chain, 4 lookups per lane and round
//     summed by DPP -- 4x faster per chain, but with one round in flight per wave the
//     LDS is only ~2/3 busy.
// Chains come longest first (perm[], launch_length_order).  The longest ones -- block
// count at or above the threshold bucket -- form the quad queue: they set the end of the
// launch, so they start at once, on quads, at raised priority, dealt round-robin over the
// CUs.  Everything shorter forms the lane queue.  `quad_waves` waves of every workgroup
// start in the quad session, the rest in the lane session; a wave whose queue runs dry
// joins the other one.
//
// Lane-session steps end on 128-byte line boundaries of the OUTPUT.  Wire frames (the
// htole32(len) prefix of core/Encryptor.cpp:34-51 puts every body 4 bytes off its blocks)
// run on quads alone: each 16-byte output slot is assembled inside the quad from the tails
// and heads of two consecutive cipher blocks (a funnel shift by d = out & 15 bytes).  The
// lane session's own funnel (FPNN_AES_HYB_WIRE_LANES) was slower and was removed in round 6
// together with its knob; it was the variant running when session r05x faulted.
#include "coop.hpp"

namespace fpnn_aes {

// component-wise select (a ternary on uint4 makes the compiler pick a stack slot by address)
__device__ __forceinline__ uint4 sel4(bool c, const uint4 &x, const uint4 &y) {
    return make_uint4(c ? x.x : y.x, c ? x.y : y.y, c ? x.z : y.z, c ? x.w : y.w);
}

// Word q - k (mod 4) of x's quad for a quad-uniform runtime rotation k: the three
// quad_perm rotations, then two levels of selects.
__device__ __forceinline__ uint32_t quad_rot(uint32_t x, uint32_t k) {
    const uint32_t r1 = quad_from<3>(x), r2 = quad_from<2>(x), r3 = quad_from<1>(x);
    const uint32_t l0 = (k & 1u) ? r1 : x, l1 = (k & 1u) ? r3 : r2;
    return (k & 2u) ? l1 : l0;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int NR, int KM, bool STREAM, int NT, int CH, bool SHIFT, bool FENCE, bool LANES = true>
__global__ __launch_bounds__(kThreads, 4) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_cfb_encrypt_hybrid(KBatch b, HybridArgs h) {
    static_assert(!(SHIFT && LANES), "wire frames run on quads alone");
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;

    // perm[0, n_long) = the chains of the long buckets (quad queue); perm[n_long, count) the rest
    uint32_t part = 0;
    if (lane <= h.long_bucket) part += h.buckets[lane];
    if (lane + 64 <= h.long_bucket) part += h.buckets[lane + 64];
    // (at most the batch even when the block's counts are bad, kernels.hpp kFaultLengthOrder)
    const uint64_t n_long = min((uint64_t)__builtin_amdgcn_readfirstlane(wave_sum32(part)), b.count);
    // quad tickets below static_q are dealt at start, the rest come from h.ctr[0]
    const uint64_t static_q = (uint64_t)h.quad_waves * 16u * gridDim.x;
    // wire batches: every body starts on the 4-byte grid (flag set by the length ordering)
    const bool wm = SHIFT && __builtin_amdgcn_readfirstlane(h.buckets[kWireFlagWord]) == 0u;

    RoundKeys<NR> rku;
    if (KM == KEY_UNIFORM) rku = load_round_keys<NR>(b.keys);

    // ---------------- quad session: K2q's cipher over perm[0, n_long) ----------------
    // Steps of 8 blocks; the next step's input words are loaded during this step's rounds.
    // Where input and output share their offset inside a 128-byte line (C4), a short
    // first step aligns the steps to the lines.  SHIFT (wire frames: the output sits 4
    // bytes off the input): steps stay on the INPUT's lines -- aligning them to the output
    // lines instead measured 412 vs 751 GiB/s on R1 -- and every 16-byte output slot is
    // the funnel of two cipher blocks, built inside the quad (quad_rot + alignbyte), so
    // stores are aligned dwords; the slots of a step past the output line boundary at
    // position mq are held back (held[]) and stored with the next step's first mq slots,
    // so each output line is written whole in one burst.  The chain's first slot is stored
    // from byte lo0 on; its last held slots and the d bytes that end its last whole block
    // are stored at the chain's end.
    auto quad_session = [&](bool first) {
        const int q = (int)(lane & 3u);
        const int wlo = 4 * q;  // block bytes [wlo, wlo + 4) belong to this lane
        // (per-lane keys: zero until the quad's first chain -- every lane runs the rounds,
        // and a quad without a chain must not run them on undefined values)
        uint32_t rkq[NR + 1];
#pragma unroll
        for (int r = 0; r <= NR; r++) rkq[r] = KM == KEY_UNIFORM ? b.keys[0].rk[4 * r + q] : 0u;
        uint64_t sid = 0;
        const uint8_t *p = nullptr;
        uint8_t *o = nullptr;
        uint32_t nfull = 0, tail = 0, n = 0, iv = 0;
        FA_DECL(a_ilo = 0, a_ihi = 0, a_olo = 0, a_ohi = 0);  // (audit build: the chain's own bytes)
        // SHIFT state: d = o & 15; the funnel's rotation kl, sources (fl, fh) and
        // byte offset r; pl / ph = the rotated words of the previous raw block, praw its
        // own word; pv / lo0 as in the lane session
        uint32_t d = 0, kl = 0, r = 0, pl = 0, ph = 0, praw = 0, pv = 0, lo0 = 0;
        bool fl = false, fh = false;
        // hold-back: this lane's words j < jt of a step end an output line (jt = 8: no
        // boundary in the step); held[j] (j >= jt) = words of the last step, hk its block
        // count, hdst its base, hv = they are pending
        uint32_t jt = 8, hk = 0, held[8];
        uint8_t *hdst = nullptr;
        bool hv = false;
#pragma unroll
        for (int j = 0; j < 8; j++) held[j] = 0u;
        bool active = false, exhausted = false, fresh = false;
        // package mode: at0 = no block of the chain ciphered yet; ew = this lane's word of the
        // slot's E_k(IV) (kernels.hpp KBatch::eiv), block 0's keystream
        bool at0 = false;
        uint32_t ew = 0;
        uint32_t a[8], nx[8];
#pragma unroll
        for (int j = 0; j < 8; j++) a[j] = nx[j] = 0u;
        const uint8_t *const dummy = reinterpret_cast<const uint8_t *>(b.keys);  // 16 readable bytes
        uint8_t *const sinkw = reinterpret_cast<uint8_t *>(h.sink + 2 * ((uint64_t)blockIdx.x * (kThreads / 64) + wave));
        auto begin = [&](uint64_t t) {
            const uint64_t s = min(*FA_AT(b, AB_PERM, b.perm + t, 4), (uint32_t)b.count - 1u);  // (in range even from a bad block)
            sid = s;
            const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
            FA_SET(a_ilo, (uintptr_t)g.in);
            FA_SET(a_ihi, (uintptr_t)g.in + g.len);
            FA_SET(a_olo, (uintptr_t)g.out);
            FA_SET(a_ohi, (uintptr_t)g.out + g.len + ((b.flags & F_WIRE_PREFIX) ? 4u : 0u));
            const DevKey *key = FA_AT(b, AB_KEYS, b.keys + (KM == KEY_UNIFORM ? 0u : g.slot), sizeof(DevKey));
            if (KM != KEY_UNIFORM) {
#pragma unroll
                for (int r = 0; r <= NR; r++) rkq[r] = key->rk[4 * r + q];
            }
            uint32_t v, pos;
            if (STREAM) {
                v = reinterpret_cast<const uint32_t *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16))[q];
                pos = *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4);
            } else {
                v = reinterpret_cast<const uint32_t *>(key->iv)[q];
                pos = 0;
                at0 = true;
                if (b.eiv)
                    ew = reinterpret_cast<const uint32_t *>(FA_AT(b, AB_EIV, b.eiv + (KM == KEY_UNIFORM ? 0u : g.slot), 16))[q];
            }
            const uint8_t *pp = g.in;
            uint8_t *oo = g.out;
            uint32_t rem = g.len;
            uint32_t pw = 0;  // (SHIFT) this lane's word of the 16 bytes before the body
            pv = 0;
            if (!STREAM && (b.flags & F_WIRE_PREFIX)) {  // htole32(len) ‖ ciphertext (core/Encryptor.cpp:47-48)
                if (q == 0) store_word_bytes(FA_RG(b, AB_OUT, oo, 0, 4, a_olo, a_ohi), rem, 0, 4);
                oo += 4;
                pw = q == 3 ? rem : 0u;
                pv = 4;
            }
            if (STREAM && pos != 0 && rem != 0) {  // rest of the partially used keystream block
                const uint32_t take = rem < 16 - pos ? rem : 16 - pos;
                const int lo = max((int)pos, wlo) - wlo, hi = min((int)(pos + take), wlo + 4) - wlo;
                if (lo < hi) {
                    const uint32_t c = load_word_bytes(FA_RG(b, AB_IN, pp - pos + wlo, lo, hi, a_ilo, a_ihi), lo, hi) ^ v;
                    store_word_bytes(FA_RG(b, AB_OUT, oo - pos + wlo, lo, hi, a_olo, a_ohi), c, lo, hi);
                    const uint32_t m = word_mask(lo, hi);
                    v = (c & m) | (v & ~m);
                }
                pp += take;
                oo += take;
                rem -= take;
                pos = (pos + take) & 15u;
            }
            iv = v;
            n = pos;
            p = pp;
            o = oo;
            nfull = rem >> 4;
            tail = rem & 15u;
            active = true;
            fresh = true;
            if (SHIFT && wm) {  // words stored where they fall (every body 4-byte aligned)
                d = 0;
                lo0 = 0;
                const int bnd = (int)((128u - ((uint32_t)(uintptr_t)oo & 127u)) & 127u) - wlo;  // line end - word
                jt = bnd + wlo == 0 ? 8u : bnd <= 0 ? 0u : (uint32_t)(bnd + 15) >> 4;
                hv = false;
            } else if (SHIFT) {
                d = (uint32_t)(uintptr_t)oo & 15u;
                const uint32_t e = (d + 3u) >> 2;  // slot word q starts in word q - e of its block
                kl = e & 3u;
                fl = (uint32_t)q < e;
                fh = (uint32_t)q + 1u < e;
                r = (0u - d) & 3u;
                pl = quad_rot(pw, kl);
                ph = quad_from<1>(pl);
                praw = pw;
                lo0 = d > pv ? d - pv : 0u;
                const uint32_t m = (8u - (((uint32_t)((uintptr_t)(oo - d) >> 4)) & 7u)) & 7u;
                jt = m == 0 ? 8u : m;
                hv = false;
            }
        };
        auto finish = [&]() {  // the shifted remainder, the partial final block, the stream state
            if (SHIFT) {
                if (hv) {  // the held words of the last step
#pragma unroll
                    for (int j = 0; j < 8; j++)
                        if (j >= (int)jt && j < (int)hk)
                            *FA_SEG(b, AB_OUT, reinterpret_cast<uint32_t *>(hdst + 16 * j), 4, a_olo, a_ohi) = held[j];
                    hv = false;
                }
                // bytes [16 - k, 16) of the last raw block end at o
                const uint32_t k = d < pv ? d : pv;
                const int lo = (int)(16u - k) - wlo;
                if (k && lo < 4)
                    store_word_bytes(FA_RG(b, AB_OUT, o - 16 + wlo, lo > 0 ? lo : 0, 4, a_olo, a_ohi), praw, lo > 0 ? lo : 0, 4);
            }
            if (tail) {
                const uint32_t ks = !STREAM && b.eiv && at0 ? ew : aes_encrypt_column<NR, NT>(iv, rkq, T);
                const int hi = min((int)tail, wlo + 4) - wlo;
                if (hi > 0) {
                    const uint32_t c = load_word_bytes(FA_RG(b, AB_IN, p + wlo, 0, hi, a_ilo, a_ihi), 0, hi) ^ ks;
                    store_word_bytes(FA_RG(b, AB_OUT, o + wlo, 0, hi, a_olo, a_ohi), c, 0, hi);
                    const uint32_t m = word_mask(0, hi);
                    iv = (c & m) | (ks & ~m);
                } else {
                    iv = ks;
                }
                n = tail;
            }
            if (STREAM) {
                reinterpret_cast<uint32_t *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * sid, 16))[q] = iv;
                if (q == 0) *FA_AT(b, AB_POS_STATE, b.pos_state + sid, 4) = n;
            }
        };
        // Tickets: the wave's quads that need a chain take consecutive ones with one atomic,
        // so neighbouring chains (adjacent frames of a send buffer) run side by side in one
        // wave and the output line they share is written in the same step.  The first
        // chains are dealt the same way, 16 per wave: wave w of workgroup g takes chains
        // [16 (w * grid + g), +16) -- the longest 16 * grid (perm[] order) start at once,
        // in the first wave of every workgroup.
        if (first) {
            const uint64_t qi = threadIdx.x >> 2;
            const uint64_t t0 = ((qi >> 4) * gridDim.x + blockIdx.x) * 16u + (qi & 15u);
            if (t0 < n_long) begin(t0);
            else exhausted = true;
        }
        __builtin_amdgcn_s_setprio(2);
        while (true) {
            if (active && nfull == 0) {
                finish();
                active = false;
            }
            const uint64_t need = __builtin_amdgcn_ballot_w64(q == 0 && !active && !exhausted);
            if (need) {
                const uint32_t leader = (uint32_t)__builtin_ctzll(need);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(FA_AT(b, AB_BLOCK, &h.ctr[0], 4), (uint32_t)__builtin_popcountll(need));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
                if (!active && !exhausted) {
                    const uint64_t below = need & ((1ull << (lane & ~3u)) - 1ull);  // needing quads before mine
                    const uint64_t t = (uint64_t)base + (uint64_t)__builtin_popcountll(below) + static_q;
                    if (t < n_long) begin(t);
                    else exhausted = true;
                }
            }
            if (__builtin_amdgcn_ballot_w64(active) == 0) break;
            if (__builtin_amdgcn_ballot_w64(active && nfull != 0) == 0) continue;
            // this step: 8 blocks, or up to the next line boundary where input and output
            // share their line offset; the next step is loaded during this one's rounds
            uint32_t lim = 8u;
            if (!SHIFT) {
                const uint32_t xo = (uint32_t)(uintptr_t)o & 127u, xi = (uint32_t)(uintptr_t)p & 127u;
                if (xo == xi && !(xo & 15u)) lim = 8u - (xo >> 4);
            }
            const uint32_t kk = active ? (nfull < lim ? nfull : lim) : 0u;
            const uint32_t rest = active ? nfull - kk : 0u;
            const uint32_t kk2 = rest < 8u ? rest : 8u;
            // Memory ops of the steady state are unconditional (lanes with nothing to load
            // read the key table, lanes with nothing to store write the wave's sink slot),
            // so the waitcnt pass counts them exactly: the rounds wait only for this step's
            // words (loaded one step earlier), never for the stores or the next prefetch.
            if (__builtin_amdgcn_ballot_w64(fresh) != 0) {  // chains that start: their first words
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (fresh)
                        a[j] = *reinterpret_cast<const uint32_u *>(j < (int)kk ? FA_SEG(b, AB_IN, p + 16 * j + wlo, 4, a_ilo, a_ihi)
                                                                                : FA_AT(b, AB_KEYS, dummy + wlo, 4));
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0), inside the rare branch
            }
#pragma unroll
            for (int j = 0; j < 8; j++)
                nx[j] = *reinterpret_cast<const uint32_u *>(j < (int)kk2 ? FA_SEG(b, AB_IN, p + 16 * (kk + j) + wlo, 4, a_ilo, a_ihi)
                                                                          : FA_AT(b, AB_KEYS, dummy + wlo, 4));
            // the rounds and the stores; FUN: the in-quad funnel (wire bodies off the 4-byte
            // grid somewhere in the batch), else block words are output words
            uint8_t *const dst = o - d + wlo;
            const bool head = SHIFT && lo0 != 0 && kk != 0;  // the chain's first slot: from byte lo0 on
            // every quad that ciphers a block this step is at its chain's block 0: the wave
            // takes that block's keystream from the key set (a quad at block 0 would compute
            // the same value: sw = IV ^ rk[0])
            const bool all0 = !STREAM && b.eiv && __builtin_amdgcn_ballot_w64(kk != 0 && !at0) == 0;
            auto body = [&](auto fun_c) {
                constexpr bool FUN = decltype(fun_c)::value;
                // the chain carries C ^ rk[0] (aes_chain_column: its XORs folded into the keys)
                const uint32_t rkx = rkq[NR] ^ rkq[0];
                uint32_t sw = iv ^ rkq[0];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t nsw =
                        j == 0 && all0 ? ew ^ a[j] ^ rkq[0] : aes_chain_column<NR, NT>(sw, rkq, rkx ^ a[j], T);
                    const uint32_t c = nsw ^ rkq[0];  // C_i = P_i ^ E(C_{i-1})
                    const bool use = j < (int)kk;
                    sw = use ? nsw : sw;
                    if (FUN) {  // slot j = the last d bytes of block j - 1 ‖ the first 16 - d of block j
                        // word q of the slot = bytes of block words q - e and q - e + 1
                        // (cl, ch), from the previous block where those indices wrap (fl, fh)
                        const uint32_t cl = quad_rot(c, kl), ch = quad_from<1>(cl);
                        a[j] = __builtin_amdgcn_alignbyte(fh ? ph : ch, fl ? pl : cl, r);
                        // (after a short step the chain ends: only praw is read again)
                        pl = cl;
                        ph = ch;
                        praw = use ? c : praw;
                    } else {
                        a[j] = c;
                    }
                }
                iv = sw ^ rkq[0];
                if (SHIFT) {
                    // one output line: the last step's held words [jt, 8), then this step's
                    // [0, jt) (4-aligned dwords); then this step's [jt, kk) are held
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const bool now = j < (int)jt;
                        const bool st = now ? j < (int)kk && !(j == 0 && head) : hv && kk != 0;
                        *reinterpret_cast<uint32_t *>(st ? FA_SEG(b, AB_OUT, (now ? dst : hdst) + 16 * j, 4, a_olo, a_ohi)
                                                          : FA_AT(b, AB_SINK, sinkw + wlo, 4)) = now ? a[j] : held[j];
                    }
#pragma unroll
                    for (int j = 0; j < 8; j++) held[j] = j >= (int)jt ? a[j] : held[j];
                    if (kk) {
                        hv = jt < 8u;
                        hk = kk;
                        hdst = dst;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; j++)
                        *reinterpret_cast<uint32_u *>(j < (int)kk ? FA_SEG(b, AB_OUT, dst + 16 * j, 4, a_olo, a_ohi)
                                                                  : FA_AT(b, AB_SINK, sinkw + wlo, 4)) = a[j];
                }
            };
            if (SHIFT && !wm) body(std::true_type{});
            else body(std::false_type{});
            if (SHIFT && __builtin_amdgcn_ballot_w64(head) != 0) {
                const int lo = (int)lo0 - wlo;
                if (head && lo < 4) store_word_bytes(FA_RG(b, AB_OUT, dst, lo > 0 ? lo : 0, 4, a_olo, a_ohi), a[0], lo > 0 ? lo : 0, 4);
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0), inside the rare branch
            }
            if (SHIFT && kk) {
                lo0 = 0;
                pv = 16;
            }
            if (kk) at0 = false;
            p += 16 * kk;
            o += 16 * kk;
            nfull -= kk;
#pragma unroll
            for (int j = 0; j < 8; j++) a[j] = nx[j];
            fresh = false;
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // ---------------- lane session: K2's cipher over perm[n_long, count) ----------------
    // (never for wire frames: their outputs sit 4 bytes off the blocks, and they run on
    // quads alone, whose in-quad funnel stores whole slots -- hybrid_nr)
    auto lane_session = [&]() {
        RoundKeys<NR> rkl;  // (per-lane keys: zero until the lane's first chain, as rkq above)
        if (KM != KEY_UNIFORM) {
#pragma unroll
            for (int i = 0; i < 4 * (NR + 1); i++) rkl.k[i] = 0u;
        }
        uint64_t sid = 0;
        const uint8_t *p = nullptr;
        uint8_t *o = nullptr;
        // nfull/tail: whole blocks / bytes of the partial final block left; n: stream position
        uint32_t nfull = 0, tail = 0, n = 0;
        FA_DECL(a_ilo = 0, a_ihi = 0, a_olo = 0, a_ohi = 0);  // (audit build: the chain's own bytes)
        uint4 iv = make_uint4(0, 0, 0, 0);
        bool valid = false, exhausted = false, fresh = false;
        bool at0 = false;                     // package mode: no block of the chain ciphered yet
        uint4 eivl = make_uint4(0, 0, 0, 0);  // the slot's E_k(IV) (KBatch::eiv)
        uint4 a[CH], nx[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) a[j] = nx[j] = make_uint4(0, 0, 0, 0);
        auto enc = [&](const uint4 &x) {
            if (FENCE)
                return KM == KEY_UNIFORM ? aes_encrypt_block_fenced<NR, NT>(x, rku, T)
                                         : aes_encrypt_block_fenced<NR, NT>(x, rkl, T);
            return KM == KEY_UNIFORM ? aes_encrypt_block<NR, NT>(x, rku, T) : aes_encrypt_block<NR, NT>(x, rkl, T);
        };
        auto begin = [&](uint64_t t) {
            const uint64_t s = min(*FA_AT(b, AB_PERM, b.perm + t, 4), (uint32_t)b.count - 1u);  // (in range even from a bad block)
            sid = s;
            const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
            FA_SET(a_ilo, (uintptr_t)g.in);
            FA_SET(a_ihi, (uintptr_t)g.in + g.len);
            FA_SET(a_olo, (uintptr_t)g.out);
            FA_SET(a_ohi, (uintptr_t)g.out + g.len);
            const DevKey *key = FA_AT(b, AB_KEYS, b.keys + (KM == KEY_UNIFORM ? 0u : g.slot), sizeof(DevKey));
            if (KM != KEY_UNIFORM) rkl = load_round_keys<NR>(key);
            if (STREAM) {
                iv = ld_state_iv(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * s, 16));
                n = *FA_AT(b, AB_POS_STATE, b.pos_state + s, 4);
            } else {
                iv = *reinterpret_cast<const uint4 *>(key->iv);
                n = 0;
                at0 = true;
                if (b.eiv) eivl = *FA_AT(b, AB_EIV, b.eiv + (KM == KEY_UNIFORM ? 0u : g.slot), 16);
            }
            const uint8_t *pp = g.in;
            uint8_t *oo = g.out;
            uint32_t rem = g.len;
            if (STREAM && n != 0 && rem != 0) {  // finish the partially consumed keystream block
                const uint32_t take = rem < 16 - n ? rem : 16 - n;
                const int lo = (int)n, hi = (int)(n + take);
                const uint4 c = load_bytes(FA_RG(b, AB_IN, pp - n, lo, hi, a_ilo, a_ihi), lo, hi) ^ iv;
                store_bytes(FA_RG(b, AB_OUT, oo - n, lo, hi, a_olo, a_ohi), c, lo, hi);
                iv = select_bytes(byte_mask(lo, hi), c, iv);
                pp += take;
                oo += take;
                rem -= take;
                n = (n + take) & 15u;
            }
            p = pp;
            o = oo;
            nfull = rem >> 4;
            tail = rem & 15u;
            valid = true;
            fresh = true;
        };
        for (;;) {
            // chains whose whole blocks are done: the partial final block, the stream state
            const bool fin = valid && nfull == 0;
            if (__builtin_amdgcn_ballot_w64(fin)) {
                uint4 ks = make_uint4(0, 0, 0, 0);
                if (__builtin_amdgcn_ballot_w64(fin && tail != 0)) {
                    // chains of one partial block all at block 0: E_k(IV) from the key set
                    if (!STREAM && b.eiv && __builtin_amdgcn_ballot_w64(fin && tail != 0 && !at0) == 0)
                        ks = eivl;
                    else
                        ks = enc(iv);
                }
                if (fin) {
                    if (tail) {
                        const uint4 c = load_bytes(FA_RG(b, AB_IN, p, 0, tail, a_ilo, a_ihi), 0, (int)tail) ^ ks;
                        store_bytes(FA_RG(b, AB_OUT, o, 0, tail, a_olo, a_ohi), c, 0, (int)tail);
                        iv = select_bytes(byte_mask(0, (int)tail), c, ks);
                        n = tail;
                    }
                    if (STREAM) {
                        *reinterpret_cast<uint4 *>(FA_AT(b, AB_IV_STATE, b.iv_state + 16 * sid, 16)) = iv;
                        *FA_AT(b, AB_POS_STATE, b.pos_state + sid, 4) = n;
                    }
                    valid = false;
                }
            }
            // lanes without a chain take the next ones: one atomic per wave
            const uint64_t need = __builtin_amdgcn_ballot_w64(!valid && !exhausted);
            if (need) {
                const uint32_t leader = (uint32_t)__builtin_ctzll(need);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(FA_AT(b, AB_BLOCK, &h.ctr[1], 4), (uint32_t)__builtin_popcountll(need));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
                if (!valid && !exhausted) {
                    const uint64_t t = n_long + base + lane_rank(need);
                    if (t < b.count) begin(t);
                    else exhausted = true;
                }
            }
            if (__builtin_amdgcn_ballot_w64(valid) == 0) break;
            if (__builtin_amdgcn_ballot_w64(valid && nfull != 0) == 0) continue;  // only sub-block chains

            // one step: up to CH blocks, ending on a CH*16-byte boundary of the output
            const uint32_t slot0 = (uint32_t)((uintptr_t)o >> 4);
            const uint32_t lim = (uint32_t)CH - (slot0 & (uint32_t)(CH - 1));
            const uint32_t kk = valid ? (nfull < lim ? nfull : lim) : 0u;
            const uint32_t rest = valid ? nfull - kk : 0u;
            const uint32_t kk2 = rest < (uint32_t)CH ? rest : (uint32_t)CH;
            // next step's blocks are loaded during this one's rounds (PF), except where the
            // registers are short (per-lane AES-192/256 round keys)
            constexpr bool PF = !(KM == KEY_LANE && NR >= 12);
            if (fresh || !PF) {
#pragma unroll
                for (int j = 0; j < CH; j++) a[j] = j < (int)kk ? load16(FA_SEG(b, AB_IN, p + 16 * j, 16, a_ilo, a_ihi)) : a[j];
            }
            if (PF) {
#pragma unroll
                for (int j = 0; j < CH; j++)
                    if (j < (int)kk2) nx[j] = load16(FA_SEG(b, AB_IN, p + 16 * (kk + j), 16, a_ilo, a_ihi));
            }
            // every lane that ciphers a block this step is at its chain's block 0: the wave
            // takes that block's keystream from the key set (a lane at block 0 would compute
            // the same E_k(IV))
            const bool all0 = !STREAM && b.eiv && __builtin_amdgcn_ballot_w64(kk != 0 && !at0) == 0;
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const uint4 c = (j == 0 && all0 ? eivl : enc(iv)) ^ a[j];  // C_i = P_i ^ E(C_{i-1})
                iv = sel4(j < (int)kk, c, iv);
                a[j] = c;
            }
#pragma unroll
            for (int j = 0; j < CH; j++)
                if (j < (int)kk) store16(FA_SEG(b, AB_OUT, o + 16 * j, 16, a_olo, a_ohi), a[j]);
            if (kk) at0 = false;
            p += 16 * kk;
            o += 16 * kk;
            nfull -= kk;
            if (PF) {
#pragma unroll
                for (int j = 0; j < CH; j++) a[j] = nx[j];
            }
            fresh = false;
        }
    };

    if constexpr (!LANES) {  // every chain on quads (wire frames: the host routes them here)
        quad_session(true);
    } else {
        if (wave < h.quad_waves) quad_session(true);
        lane_session();
        // long chains left (fewer quad waves than the long queue needs): join them
        if (__atomic_load_n(&h.ctr[0], __ATOMIC_RELAXED) + static_q < n_long) quad_session(false);
    }
    length_order_release(h.ctr - kTicketWords);  // the block's last reader: zero it for the next call
}

template <int NR>
static void hybrid_nr(const KBatch &b, const HybridArgs &h, KeyMode km, bool stream, int grid, hipStream_t st) {
#define FPNN_HYB(K, STR, CH, SH, LN) \
    hipLaunchKernelGGL((k_cfb_encrypt_hybrid<NR, K, STR, 4, CH, SH, true, LN>), dim3(grid), dim3(kThreads), 0, st, b, h)
    // wire frames (outputs off the block grid by construction, the 4-byte prefix): every
    // chain on quads, whose funnel stores whole 16-byte slots -- the lane session's funnel
    // measured 653 vs 800 GiB/s on R1 (profiles/r03/ab_r1.json) and was removed in round 6;
    // other ragged outputs are stored as they fall
    const bool shift = !stream && (b.flags & F_WIRE_PREFIX);
    if (km == KEY_UNIFORM) {
        if (stream) FPNN_HYB(KEY_UNIFORM, true, 8, false, true);
        else if (shift) FPNN_HYB(KEY_UNIFORM, false, 8, true, false);
        else FPNN_HYB(KEY_UNIFORM, false, 8, false, true);
    } else {  // per-lane round keys (up to 60 VGPRs): half-line steps
        if (stream) FPNN_HYB(KEY_LANE, true, 4, false, true);
        else if (shift) FPNN_HYB(KEY_LANE, false, 4, true, false);
        else FPNN_HYB(KEY_LANE, false, 4, false, true);
    }
#undef FPNN_HYB
}

hipError_t launch_encrypt_hybrid(const KBatch &b, const HybridArgs &h, int nrounds, KeyMode km, bool stream, int grid,
                                 hipStream_t st) {
    set_launched("cfb_encrypt_hybrid");
    switch (nrounds) {
        case 10: hybrid_nr<10>(b, h, km, stream, grid, st); break;
        case 12: hybrid_nr<12>(b, h, km, stream, grid, st); break;
        case 14: hybrid_nr<14>(b, h, km, stream, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
