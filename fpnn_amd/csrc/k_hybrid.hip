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
// Lane-session output is written in whole 128-byte lines: steps end on line boundaries
// of the OUTPUT, and when the output is not 16-byte aligned with the blocks (the
// htole32(len) prefix of the wire form, core/Encryptor.cpp:34-51, shifts every frame by 4)
// each 16-byte slot is assembled from the tails and heads of two consecutive cipher blocks
// (a funnel shift by d = out & 15 bytes, the d-byte remainder carried to the next step).
// Only a chain's first and last slot are partial stores.
#include "coop.hpp"

namespace fpnn_aes {

// Bytes [16 - d, 32 - d) of the 32-byte sequence prev ‖ cur (d in 1..15): the output slot
// whose first d bytes end the previous block.  c1/c2 = bits 0/1 of the word offset
// (16 - d) >> 2, r = (16 - d) & 3.  20 VALU.
__device__ __forceinline__ uint4 funnel_slot(const uint4 &prev, const uint4 &cur, bool c1, bool c2, uint32_t r) {
    const uint32_t y[8] = {prev.x, prev.y, prev.z, prev.w, cur.x, cur.y, cur.z, cur.w};
    uint32_t z1[7], z2[5];
#pragma unroll
    for (int m = 0; m < 7; m++) z1[m] = c1 ? y[m + 1] : y[m];
#pragma unroll
    for (int m = 0; m < 5; m++) z2[m] = c2 ? z1[m + 2] : z1[m];
    return make_uint4(__builtin_amdgcn_alignbyte(z2[1], z2[0], r), __builtin_amdgcn_alignbyte(z2[2], z2[1], r),
                      __builtin_amdgcn_alignbyte(z2[3], z2[2], r), __builtin_amdgcn_alignbyte(z2[4], z2[3], r));
}

// component-wise select (a ternary on uint4 makes the compiler pick a stack slot by address)
__device__ __forceinline__ uint4 sel4(bool c, const uint4 &x, const uint4 &y) {
    return make_uint4(c ? x.x : y.x, c ? x.y : y.y, c ? x.z : y.z, c ? x.w : y.w);
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int NR, int KM, bool STREAM, int NT, int CH, bool SHIFT, bool FENCE>
__global__ __launch_bounds__(kThreads, 4) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_cfb_encrypt_hybrid(KBatch b, HybridArgs h) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;

    // perm[0, n_long) = the chains of the long buckets (quad queue); perm[n_long, count) the rest
    uint32_t part = 0;
    if (lane <= h.long_bucket) part += h.buckets[lane];
    if (lane + 64 <= h.long_bucket) part += h.buckets[lane + 64];
    const uint64_t n_long = __builtin_amdgcn_readfirstlane(wave_sum32(part));
    // quad tickets below static_q are dealt at start, the rest come from h.ctr[0]
    const uint64_t static_q = (uint64_t)h.quad_waves * 16u * gridDim.x;

    RoundKeys<NR> rku;
    if (KM == KEY_UNIFORM) rku = load_round_keys<NR>(b.keys);

    // ---------------- quad session: K2q's cipher over perm[0, n_long) ----------------
    auto quad_session = [&](bool first) {
        const int q = (int)(lane & 3u);
        const int wlo = 4 * q;  // block bytes [wlo, wlo + 4) belong to this lane
        uint32_t rkq[NR + 1];
        if (KM == KEY_UNIFORM) {
#pragma unroll
            for (int r = 0; r <= NR; r++) rkq[r] = b.keys[0].rk[4 * r + q];
        }
        uint64_t sid = 0;
        const uint8_t *p = nullptr;
        uint8_t *o = nullptr;
        uint32_t nfull = 0, tail = 0, n = 0, iv = 0;
        bool active = false, exhausted = false;
        auto begin = [&](uint64_t t) {
            const uint64_t s = b.perm[t];
            sid = s;
            const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
            const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
            if (KM != KEY_UNIFORM) {
#pragma unroll
                for (int r = 0; r <= NR; r++) rkq[r] = key->rk[4 * r + q];
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
            if (!STREAM && (b.flags & F_WIRE_PREFIX)) {  // htole32(len) ‖ ciphertext (core/Encryptor.cpp:47-48)
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
            iv = v;
            n = pos;
            p = pp;
            o = oo;
            nfull = rem >> 4;
            tail = rem & 15u;
            active = true;
        };
        auto finish = [&]() {  // partial final block and the stream state
            if (tail) {
                const uint32_t ks = aes_encrypt_column<NR, NT>(iv, rkq, T);
                const int hi = min((int)tail, wlo + 4) - wlo;
                if (hi > 0) {
                    const uint32_t c = load_word_bytes(p + wlo, 0, hi) ^ ks;
                    store_word_bytes(o + wlo, c, 0, hi);
                    const uint32_t m = word_mask(0, hi);
                    iv = (c & m) | (ks & ~m);
                } else {
                    iv = ks;
                }
                n = tail;
            }
            if (STREAM) {
                reinterpret_cast<uint32_t *>(b.iv_state + 16 * sid)[q] = iv;
                if (q == 0) b.pos_state[sid] = n;
            }
        };
        auto ticket = [&]() -> uint64_t {  // the quad leader's atomic, broadcast over the quad
            uint32_t t = 0;
            if (q == 0) t = atomicAdd(&h.ctr[0], 1u);
            return (uint64_t)(uint32_t)__builtin_amdgcn_mov_dpp((int)t, 0x00, 0xf, 0xf, true) + static_q;
        };
        if (first) {
            const uint64_t t0 = (uint64_t)(threadIdx.x >> 2) * gridDim.x + blockIdx.x;
            if (t0 < n_long) begin(t0);
            else exhausted = true;
        }
        __builtin_amdgcn_s_setprio(2);
        while (true) {
            if (active && nfull == 0) {
                finish();
                active = false;
            }
            if (!active && !exhausted) {
                const uint64_t t = ticket();
                if (t < n_long) begin(t);
                else exhausted = true;
            }
            if (__builtin_amdgcn_ballot_w64(active) == 0) break;
            if (__builtin_amdgcn_ballot_w64(active && nfull != 0) == 0) continue;
            const uint32_t kk = active ? (nfull < 8u ? nfull : 8u) : 0u;
            uint32_t a[8];
#pragma unroll
            for (int j = 0; j < 8; j++) a[j] = j < (int)kk ? *reinterpret_cast<const uint32_u *>(p + 16 * j + wlo) : 0u;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t c = aes_encrypt_column<NR, NT>(iv, rkq, T) ^ a[j];  // C_i = P_i ^ E(C_{i-1})
                iv = j < (int)kk ? c : iv;
                a[j] = c;
            }
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (j < (int)kk) *reinterpret_cast<uint32_u *>(o + 16 * j + wlo) = a[j];
            p += 16 * kk;
            o += 16 * kk;
            nfull -= kk;
        }
        __builtin_amdgcn_s_setprio(0);
    };

    // ---------------- lane session: K2's cipher over perm[n_long, count) ----------------
    auto lane_session = [&]() {
        RoundKeys<NR> rkl;
        uint64_t sid = 0;
        const uint8_t *p = nullptr;
        uint8_t *o = nullptr;
        // nfull/tail: whole blocks / bytes of the partial final block left; n: stream
        // position; d = o & 15 (output shift against the blocks); pv = trailing bytes of
        // prev that are this chain's own output (rewritable); lo0 = first byte of the
        // chain's first slot that this chain may write
        uint32_t nfull = 0, tail = 0, n = 0, d = 0, pv = 0, lo0 = 0;
        uint4 iv = make_uint4(0, 0, 0, 0), prev = make_uint4(0, 0, 0, 0);
        bool valid = false, exhausted = false, fresh = false;
        uint4 a[CH], nx[CH];
#pragma unroll
        for (int j = 0; j < CH; j++) a[j] = nx[j] = make_uint4(0, 0, 0, 0);
        auto enc = [&](const uint4 &x) {
            if (SHIFT || FENCE)  // (the funnel's live registers make the compiler serialize the lookups)
                return KM == KEY_UNIFORM ? aes_encrypt_block_fenced<NR, NT>(x, rku, T)
                                         : aes_encrypt_block_fenced<NR, NT>(x, rkl, T);
            return KM == KEY_UNIFORM ? aes_encrypt_block<NR, NT>(x, rku, T) : aes_encrypt_block<NR, NT>(x, rkl, T);
        };
        auto begin = [&](uint64_t t) {
            const uint64_t s = b.perm[t];
            sid = s;
            const Seg g = get_seg<LAYOUT_GENERAL>(b, s);
            const DevKey *key = b.keys + (KM == KEY_UNIFORM ? 0u : g.slot);
            if (KM != KEY_UNIFORM) rkl = load_round_keys<NR>(key);
            if (STREAM) {
                iv = ld_state_iv(b.iv_state + 16 * s);
                n = b.pos_state[s];
            } else {
                iv = *reinterpret_cast<const uint4 *>(key->iv);
                n = 0;
            }
            const uint8_t *pp = g.in;
            uint8_t *oo = g.out;
            uint32_t rem = g.len;
            pv = 0;
            if (!STREAM && (b.flags & F_WIRE_PREFIX)) {
                prev = make_uint4(0u, 0u, 0u, rem);  // the prefix = the 4 output bytes before the body
                store_bytes(oo - 12, prev, 12, 16);
                oo += 4;
                pv = 4;
            }
            if (STREAM && n != 0 && rem != 0) {  // finish the partially consumed keystream block
                const uint32_t take = rem < 16 - n ? rem : 16 - n;
                const int lo = (int)n, hi = (int)(n + take);
                const uint4 c = load_bytes(pp - n, lo, hi) ^ iv;
                store_bytes(oo - n, c, lo, hi);
                iv = select_bytes(byte_mask(lo, hi), c, iv);
                pp += take;
                oo += take;
                rem -= take;
                n = (n + take) & 15u;
                prev = c;
                pv = n == 0 ? take : 0u;  // c's last `take` bytes precede oo only if the block is used up
            }
            p = pp;
            o = oo;
            nfull = rem >> 4;
            tail = rem & 15u;
            d = (uint32_t)(uintptr_t)oo & 15u;
            lo0 = d > pv ? d - pv : 0u;
            valid = true;
            fresh = true;
        };
        for (;;) {
            // chains whose whole blocks are done: the shifted remainder, the partial final
            // block, the stream state
            const bool fin = valid && nfull == 0;
            if (__builtin_amdgcn_ballot_w64(fin)) {
                uint4 ks = make_uint4(0, 0, 0, 0);
                if (__builtin_amdgcn_ballot_w64(fin && tail != 0)) ks = enc(iv);
                if (fin) {
                    const uint32_t k = d < pv ? d : pv;
                    if (SHIFT && k) store_bytes(o - 16, prev, (int)(16 - k), 16);
                    if (tail) {
                        const uint4 c = load_bytes(p, 0, (int)tail) ^ ks;
                        store_bytes(o, c, 0, (int)tail);
                        iv = select_bytes(byte_mask(0, (int)tail), c, ks);
                        n = tail;
                    }
                    if (STREAM) {
                        *reinterpret_cast<uint4 *>(b.iv_state + 16 * sid) = iv;
                        b.pos_state[sid] = n;
                    }
                    valid = false;
                }
            }
            // lanes without a chain take the next ones: one atomic per wave
            const uint64_t need = __builtin_amdgcn_ballot_w64(!valid && !exhausted);
            if (need) {
                const uint32_t leader = (uint32_t)__builtin_ctzll(need);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&h.ctr[1], (uint32_t)__builtin_popcountll(need));
                base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
                if (!valid && !exhausted) {
                    const uint64_t t = n_long + base + lane_rank(need);
                    if (t < b.count) begin(t);
                    else exhausted = true;
                }
            }
            if (__builtin_amdgcn_ballot_w64(valid) == 0) break;
            if (__builtin_amdgcn_ballot_w64(valid && nfull != 0) == 0) continue;  // only sub-block chains

            // one step: up to CH blocks, ending on a CH*16-byte boundary of the output slots
            const uint32_t slot0 = (uint32_t)((uintptr_t)(o - d) >> 4);
            const uint32_t lim = (uint32_t)CH - (slot0 & (uint32_t)(CH - 1));
            const uint32_t kk = valid ? (nfull < lim ? nfull : lim) : 0u;
            const uint32_t rest = valid ? nfull - kk : 0u;
            const uint32_t kk2 = rest < (uint32_t)CH ? rest : (uint32_t)CH;
            // next step's blocks are loaded during this one's rounds (PF), except where the
            // registers are short (per-lane AES-192/256 round keys)
            constexpr bool PF = !(KM == KEY_LANE && NR >= 12);
            if (fresh || !PF) {
#pragma unroll
                for (int j = 0; j < CH; j++) a[j] = j < (int)kk ? load16(p + 16 * j) : a[j];
            }
            if (PF) {
#pragma unroll
                for (int j = 0; j < CH; j++)
                    if (j < (int)kk2) nx[j] = load16(p + 16 * (kk + j));
            }
            if (!SHIFT) {
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    const uint4 c = enc(iv) ^ a[j];  // C_i = P_i ^ E(C_{i-1})
                    iv = sel4(j < (int)kk, c, iv);
                    a[j] = c;
                }
#pragma unroll
                for (int j = 0; j < CH; j++)
                    if (j < (int)kk) store16(o + 16 * j, a[j]);
            } else {
                // each block's output slot is assembled as soon as the block is ciphered
                // (only the last raw block, prev, stays live), then the slots go out back
                // to back; lanes with d == 0 store the blocks themselves
                const uint32_t t = 16u - d;
                const bool c1 = (t >> 2) & 1u, c2 = (t >> 3) & 1u;
                const uint32_t r = t & 3u;
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    const uint4 c = enc(iv) ^ a[j];  // C_i = P_i ^ E(C_{i-1})
                    iv = sel4(j < (int)kk, c, iv);
                    a[j] = sel4(d != 0, funnel_slot(prev, c, c1, c2, r), c);
                    prev = sel4(j < (int)kk, c, prev);
                }
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    if (j < (int)kk) {
                        uint8_t *dst = o - d + 16 * j;
                        if (j == 0 && lo0 != 0) store_bytes(dst, a[j], (int)lo0, 16);
                        else store16(dst, a[j]);
                    }
                }
                if (kk) {
                    lo0 = 0;
                    pv = 16;
                }
            }
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

    if (wave < h.quad_waves) quad_session(true);
    lane_session();
    // long chains left (fewer quad waves than the long queue needs): join them
    if (__atomic_load_n(&h.ctr[0], __ATOMIC_RELAXED) + static_q < n_long) quad_session(false);
}

template <int NR, bool F>
static void hybrid_nrf(const KBatch &b, const HybridArgs &h, KeyMode km, bool stream, int grid, hipStream_t st) {
#define FPNN_HYB(K, STR, CH, SH) \
    hipLaunchKernelGGL((k_cfb_encrypt_hybrid<NR, K, STR, 4, CH, SH, F || SH>), dim3(grid), dim3(kThreads), 0, st, b, h)
    // the funnel-shifted whole-slot stores only where outputs sit off the block grid by
    // construction (the wire prefix); other ragged outputs are stored as they fall
    const bool shift = !stream && (b.flags & F_WIRE_PREFIX);
    if (km == KEY_UNIFORM) {
        if (stream) FPNN_HYB(KEY_UNIFORM, true, 8, false);
        else if (shift) FPNN_HYB(KEY_UNIFORM, false, 8, true);
        else FPNN_HYB(KEY_UNIFORM, false, 8, false);
    } else {  // per-lane round keys (up to 60 VGPRs): half-line steps
        if (stream) FPNN_HYB(KEY_LANE, true, 4, false);
        else if (shift) FPNN_HYB(KEY_LANE, false, 4, true);
        else FPNN_HYB(KEY_LANE, false, 4, false);
    }
#undef FPNN_HYB
}

template <int NR>
static void hybrid_nr(const KBatch &b, const HybridArgs &h, KeyMode km, bool stream, bool fence, int grid,
                      hipStream_t st) {
    if (fence) hybrid_nrf<NR, true>(b, h, km, stream, grid, st);
    else hybrid_nrf<NR, false>(b, h, km, stream, grid, st);
}

hipError_t launch_encrypt_hybrid(const KBatch &b, const HybridArgs &h, int nrounds, KeyMode km, bool stream, bool fence,
                                 int grid, hipStream_t st) {
    hipError_t err = hipMemsetAsync(h.ctr, 0, 2 * sizeof(uint32_t), st);
    if (err != hipSuccess) return err;
    set_launched("cfb_encrypt_hybrid");
    switch (nrounds) {
        case 10: hybrid_nr<10>(b, h, km, stream, fence, grid, st); break;
        case 12: hybrid_nr<12>(b, h, km, stream, fence, grid, st); break;
        case 14: hybrid_nr<14>(b, h, km, stream, fence, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
