// k_decrypt.hip -- CFB-128 decryption kernels for gfx950.
//   K1  k_cfb_decrypt_blocks : one lane per 16-byte block (any layout, stream mode).
//        P_i = C_i ^ E(C_{i-1}), C_{-1} = IV (base/rijndael.c:1189-1197).  Every C is
//        known up front, so all blocks of all packets run in parallel; lane l gets
//        C_{i-1} from lane l-1 by DPP wave_shr:1, only lane 0 reloads it.
//   K1d k_cfb_decrypt_dense  : dense whole-block packets (the C2 / C5 shapes).
//   Both keep the T-table image in LDS (aes_device.hpp) and are persistent: one
//   1024-thread workgroup per CU walks the work with a grid stride.
#include "segments.hpp"

namespace fpnn_aes {

// ---------------------------------------------------------------------------
// K1: decryption, one lane per virtual block, 64 consecutive blocks per wave step.

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
template <int NR, bool INPLACE, int NT, bool ALIGNED, int U, int IL, bool PF, bool KEYED, bool FENCE = false>
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
    const uint8_t *inb = b.in;
    uint8_t *outb = b.out;
    // wave-uniform: does the chunk's first block open a packet?
    auto opens = [&](uint64_t c) -> bool { return chunk_bi0<ALIGNED>(c, nb, b.magic) == 0; };

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
        if (!opens(c0))  // wave-uniform; at a packet start the IV is used
            D.f = INPLACE ? b.boundary[c0] : load16(inb + (c0 << 10) - 16);  // any byte alignment
#pragma unroll
        for (int j = 0; j < U; j++) {
            const uint64_t c = st * U + j;
            const uint64_t cl = FULL || c < nchunks ? c : nchunks - 1;  // overhang: recompute the last chunk
            uint32_t lo = lane16;
            if (!FULL && !ALIGNED) {  // partial last chunk: clamp to the last block
                const uint64_t left = total - (cl << 6);
                if (left < 64) lo = min(lane, (uint32_t)left - 1u) * 16u;
            }
            D.x[j] = load16(inb + (cl << 10) + lo);
        }
    };
    auto step = [&](uint64_t st, StepBuf &X, StepBuf &NX, bool pref, auto full_tag) {
        constexpr bool FULL = decltype(full_tag)::value;
        if (KEYED) {
            const uint32_t pkt = fast_div((uint32_t)((st * U) << 6), b.magic);
            set_key(((ConstU32 *)b.key_slot)[pkt]);
        }
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
            aes_encrypt_blocks<NR, NT, IL, FENCE>(grp, rk, T);
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
            store16(outb + (c << 10) + lane16, X.x[j] ^ ks[j]);
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

// K1k: K1d's dense addressing with one key slot per packet and packets that do NOT
// fall on chunk boundaries (UDP datagrams of many connections: 1472-B packets, the U1
// shape).  A chunk then mixes packets, so round keys are per lane (VGPRs, loaded per
// step from the lane's key slot); everything else is K1d: packet / block-in-packet by
// one multiply-high, no segment arrays, the step's ciphertext and key slots prefetched
// one step ahead (ping-pong), lane 0's predecessor loaded with them.
template <int NR, bool INPLACE, int NT>
__global__ __launch_bounds__(kThreads, 4 * Lds<NT>::kBlocksPerCU) void k_cfb_decrypt_lanekey(KBatch b) {
    __shared__ uint4 lds4[Lds<NT>::kBytes / 16];
    lds_fill_tables<NT>(lds4, b.t0le);
    __syncthreads();
    const Tables4<NT> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t total = b.total_blocks;
    const uint64_t nchunks = (total + 63) >> 6;
    const uint32_t nb = b.nb_uniform;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w0 = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);

    struct Buf {
        uint4 x, f;  // this lane's block; lane 0's predecessor (when the chunk opens mid-packet)
        uint32_t slot;
    };
    // lane's global block (clamped into the batch for the partial last chunk)
    auto gblock = [&](uint64_t c) {
        const uint64_t g = (c << 6) + lane;
        return (uint32_t)(g < total ? g : total - 1);
    };
    auto load = [&](uint64_t c, Buf &D) {
        const uint32_t bi0 = chunk_bi0<false>(c, nb, b.magic);
        if (bi0 != 0)  // wave-uniform
            D.f = INPLACE ? b.boundary[c] : *reinterpret_cast<const uint4 *>(b.in + (c << 10) - 16);
        const uint32_t g = gblock(c);
        D.x = load16(b.in + 16ull * g);
        D.slot = b.key_slot[fast_div(g, b.magic)];
    };
    auto step = [&](uint64_t c, Buf &X, Buf &NX, bool pref) {
        const uint32_t g = gblock(c);
        const uint32_t bi = g - nb * fast_div(g, b.magic);
        const RoundKeys<NR> rk = load_round_keys<NR>(b.keys + X.slot);
        const uint4 ivl = *reinterpret_cast<const uint4 *>(b.keys[X.slot].iv);
        // C_{i-1}: lane l-1's block (DPP); lane 0 gets its IV at a packet start, else the
        // block before the chunk; a lane that opens a packet takes its own IV
        uint4 kin = X.x;
        const uint4 fill = bi == 0 ? ivl : X.f;
        kin = make_uint4(wave_shr1(X.x.x, fill.x), wave_shr1(X.x.y, fill.y), wave_shr1(X.x.z, fill.z),
                         wave_shr1(X.x.w, fill.w));
        if (lane != 0 && bi == 0) kin = ivl;
        if (pref) load(c + nwaves, NX);
        // fenced rounds: U1 decrypt 1 147-1 149 -> 1 163-1 173 GiB/s (profiles/r06/ab_k1k_fence)
        const uint4 ks = aes_encrypt_block_fenced<NR, NT>(kin, rk, T);
        if ((c << 6) + lane < total) store16(b.out + 16ull * ((c << 6) + lane), X.x ^ ks);
    };
    uint64_t c = w0;
    if (c >= nchunks) return;
    Buf ba, bb;
    load(c, ba);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the loop header then sees only the back edge
    while (true) {
        step(c, ba, bb, c + nwaves < nchunks);
        c += nwaves;
        if (c >= nchunks) break;
        step(c, bb, ba, c + nwaves < nchunks);
        c += nwaves;
        if (c >= nchunks) break;
    }
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

// 64-block chunks per wave step in K1: 4 where the extra state fits in registers
// (package mode, one key), 1 for stream / per-packet-key variants (they would spill).
constexpr int dec_u(bool stream, int km) { return (!stream && km == KEY_UNIFORM) ? 4 : 1; }

template <int NR, bool INPLACE>
static void dec_launch(const KBatch &b, Layout layout, KeyMode km, bool dense, int grid, hipStream_t st) {
#define FPNN_DEC(L) \
    hipLaunchKernelGGL((k_cfb_decrypt_blocks<NR, L, KEY_UNIFORM, false, INPLACE, 4, 4, 1>), dim3(grid), \
                       dim3(kThreads), 0, st, b)
#define FPNN_DENSE(AL, U, KEYED) \
    hipLaunchKernelGGL((k_cfb_decrypt_dense<NR, INPLACE, 4, AL, U, 1, true, KEYED>), dim3(grid), dim3(kThreads), 0, st, b)
    const bool aligned = b.nb_uniform % 64 == 0;
    set_launched(layout == LAYOUT_FULL && km == KEY_LANE && !aligned ? "cfb_decrypt_lanekey"
                 : layout == LAYOUT_FULL && (km == KEY_LANE || dense) ? "cfb_decrypt_dense"
                                                                       : "cfb_decrypt_blocks");
    if (layout == LAYOUT_FULL && km == KEY_LANE && !aligned) {  // dense, one key per packet, mixed chunks
        hipLaunchKernelGGL((k_cfb_decrypt_lanekey<NR, INPLACE, 4>), dim3(grid), dim3(kThreads), 0, st, b);
    } else if (layout == LAYOUT_FULL && km == KEY_LANE) {  // dense, chunk-aligned, one key per packet
        const uint32_t nbc = b.nb_uniform / 64;
        if (nbc % 4 == 0) FPNN_DENSE(true, 4, true);
        else if (nbc % 2 == 0) FPNN_DENSE(true, 2, true);
        else FPNN_DENSE(true, 1, true);
    } else if (layout == LAYOUT_FULL && dense) {  // K1d with the next step prefetched
        if (aligned)  // the C2 decrypt: fenced rounds
            hipLaunchKernelGGL((k_cfb_decrypt_dense<NR, INPLACE, 4, true, 4, 1, true, false, true>), dim3(grid),
                               dim3(kThreads), 0, st, b);
        else FPNN_DENSE(false, 4, false);
    } else if (layout == LAYOUT_FULL) {
        FPNN_DEC(LAYOUT_FULL);
    } else {  // LAYOUT_UNIFORM package batch with a partial last block per packet
        FPNN_DEC(LAYOUT_UNIFORM);
    }
#undef FPNN_DENSE
#undef FPNN_DEC
}

template <int NR>
static void dec_nr(const KBatch &b, Layout layout, KeyMode km, bool inplace, int grid, hipStream_t st) {
    const bool dense = b.stride == 16ull * b.nb_uniform;
    if (inplace) dec_launch<NR, true>(b, layout, km, dense, grid, st);
    else dec_launch<NR, false>(b, layout, km, dense, grid, st);
}

hipError_t launch_decrypt_blocks(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool inplace, int grid,
                                 hipStream_t st) {
    switch (nrounds) {
        case 10: dec_nr<10>(b, layout, km, inplace, grid, st); break;
        case 12: dec_nr<12>(b, layout, km, inplace, grid, st); break;
        case 14: dec_nr<14>(b, layout, km, inplace, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_boundary_save(const KBatch &b, uint4 *boundary, uint64_t nchunks, hipStream_t st) {
    const int grid = grid_for(nchunks, 256, 4096);
    hipLaunchKernelGGL((k_boundary_save<LAYOUT_UNIFORM, false>), dim3(grid), dim3(256), 0, st, b, boundary, nchunks);
    return hipGetLastError();
}

}  // namespace fpnn_aes
