// k_ragged.hip -- K1r: CFB-128 decryption of a ragged batch with no host round trip.
//
// A ragged batch (offset / length / key-slot arrays, package or stream mode, any byte
// lengths and CFB positions) is decrypted one lane per 16-byte virtual block
// (base/rijndael.c:1189-1197: P_i = C_i ^ E(C_{i-1}), every C known up front), exactly
// as K1, but everything the launch needs is computed on the device:
//   1. the block-map scan (k_support.hip) writes bstart[0..count] (bstart[count] = the
//      total block count, which the host never reads);
//   2. k_ragged_plan gives every wave of the decrypt grid a contiguous range of 64-block
//      chunks, the segment holding its first block and the ciphertext block in front of
//      it (saved before any wave writes, so in-place batches need no other boundary
//      table);
//   3. k_cfb_decrypt_ragged walks its chunk range in order.  A wave keeps a window of
//      64 consecutive bstart[] entries in registers (one per lane); the segment of each
//      lane's block follows from the window by ballots and at most a few readlanes per
//      chunk, so there is no per-chunk scratch (no tile map, no start mask) -- only
//      count- and wave-sized arrays, sized on the host from what it knows.  Lane 0's
//      predecessor is lane 63's block of the previous chunk (registers), or the plan's
//      saved block for the wave's first chunk.  The descriptors of chunk c+2 and the
//      ciphertext of chunk c+1 are in flight while chunk c is enciphered.
// Grid: one 1024-thread workgroup per CU whatever the batch size (waves without chunks
// exit at once), so the launch never depends on the total.
#include "segments.hpp"

namespace fpnn_aes {

__device__ __forceinline__ void wave_chunk_range(uint64_t nchunks, uint64_t nwaves, uint64_t w, uint64_t &c0,
                                                 uint64_t &c1) {
    const uint64_t q = nchunks / nwaves, r = nchunks % nwaves;
    c0 = w * q + (w < r ? w : r);
    c1 = c0 + q + (w < r ? 1 : 0);
}

// Largest s in [0, count) with bstart[s] <= g, for g < bstart[count]: a 64-ary search by
// the whole wave (wave-uniform result; ~log64(count) rounds of one coalesced load).
__device__ __forceinline__ uint64_t wave_find_segment(const uint64_t *__restrict__ bstart, uint64_t count, uint64_t g,
                                                      uint32_t lane) {
    uint64_t lo = 0, n = count;  // answer in [lo, lo + n); bstart[lo] <= g
    while (n > 64) {
        const uint64_t step = (n + 63) >> 6;
        const uint64_t d = (uint64_t)lane * step;
        const bool ok = d < n && bstart[lo + d] <= g;
        const uint64_t m = __builtin_amdgcn_ballot_w64(ok);  // bit 0 always set
        const uint32_t L = 63u - (uint32_t)__builtin_clzll(m);
        lo += (uint64_t)L * step;
        const uint64_t left = n - (uint64_t)L * step;
        n = left < step ? left : step;
    }
    const bool ok = lane < n && bstart[lo + lane] <= g;
    const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
    return lo + (63u - (uint32_t)__builtin_clzll(m));
}

// Block g's predecessor ciphertext block when it is in the same segment (else zero: the
// chunk opens a segment and takes the IV).
template <bool STREAM>
__device__ __forceinline__ uint4 predecessor_block(const KBatch &b, uint64_t s, uint64_t g) {
    const uint64_t bi = g - b.bstart[s];
    if (bi == 0) return make_uint4(0, 0, 0, 0);
    const Seg sg = get_seg<LAYOUT_GENERAL>(b, s);
    const uint32_t n0 = STREAM ? b.pos_snap[s] : 0u;
    const uint4 ivs = STREAM ? b.iv_snap[s] : make_uint4(0, 0, 0, 0);  // package blocks never need it
    return load_cx(sg, n0, (uint32_t)(bi - 1), ivs);
}

// One wave per plan entry: (first segment, predecessor block) of the wave's chunk range.
template <bool STREAM>
__global__ __launch_bounds__(256) void k_ragged_plan(KBatch b, uint64_t nwaves, RaggedPlan *plan) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t w = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    if (w >= nwaves) return;
    const uint64_t total = b.bstart[b.count];
    uint64_t c0, c1;
    wave_chunk_range((total + 63) >> 6, nwaves, w, c0, c1);
    if (c0 >= c1) return;  // this wave has no chunk; its plan entry is never read
    const uint64_t s = wave_find_segment(b.bstart, b.count, c0 << 6, lane);
    if (lane == 0) {
        plan[w].s0 = s;
        plan[w].fill = predecessor_block<STREAM>(b, s, c0 << 6);
    }
}

// Segment descriptors of each lane's block in one chunk (loads issued, not waited for).
struct RDesc {
    uint64_t g;  // the lane's block (clamped into the batch)
    uint64_t bs, io, oo;
    uint32_t s, len, slot, n0;
    bool uni;    // wave-uniform: the whole chunk lies in segment s
};

// The chunk itself: ciphertext block + what its store and CFB fill need.
struct RChunk {
    uint4 x;
    const uint8_t *in;  // segment bases
    uint8_t *out;
    uint32_t s, bi, len, n0, slot;  // count < 2^32 (fpnn_aes_batch.count is 32-bit)
    bool valid;
    bool full;  // the block is 16 whole bytes of the segment (plain 16-B load / store)
};

typedef __attribute__((address_space(4))) const DevKey ConstDevKeyR;
typedef __attribute__((address_space(4))) const uint64_t ConstU64R;
typedef __attribute__((address_space(4))) const uint32_t ConstU32R;

// (the builtins return int: each half goes through uint32_t so the low half is not
// sign-extended into the high one -- offsets past 2 GiB have bit 31 set)
__device__ __forceinline__ uint64_t readfirst64(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
    return ((uint64_t)hi << 32) | lo;
}

// Memory-access discipline of this kernel (what keeps its prefetches in flight): every
// load whose result is needed in the same chunk is consumed inside the (rare) branch
// that issued it; the loads of the pipeline ring (descriptors two chunks ahead,
// ciphertext one to DEPTH-1 chunks ahead) are issued unconditionally in straight-line
// code -- past the wave's last chunk they re-read that chunk -- so the compiler's
// waitcnt pass can count them exactly instead of draining the memory pipe (vmcnt(0)).
// The host guarantees in_off, out_off and len are device arrays (launch_decrypt_ragged).
// Round keys from the key table: the first KS words stay in SGPRs, the rest are copied to
// VGPRs (every lane the same value).  All in SGPRs they push this kernel's scalar state
// past the SGPR file, and the spills cost the cipher its LDS parallelism (the scheduler
// then waits after every one or two lookups); all in VGPRs, AES-256's 60 words push the
// vector state past the 128 VGPRs of 4 waves per SIMD.
template <int NR, int KS = NR == 14 ? 28 : NR == 12 ? 12 : 0>
__device__ __forceinline__ void set_keys(RoundKeys<NR> &rk, ConstDevKeyR *kp) {
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); i++) {
        const uint32_t v = kp->rk[i];
        if (i < KS) rk.k[i] = v;
        else asm volatile("v_mov_b32 %0, %1" : "=v"(rk.k[i]) : "s"(v));
    }
}

// key rows per wave in LDS for chunks spanning several key slots (process()): 8 AES-256
// keys = 1 920 B per wave, 30 KiB per 16-wave workgroup beside the 128 KiB table image
constexpr int kLdsKeys = 8;

template <int NR, bool STREAM, int KM, bool FENCE>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_decrypt_ragged(KBatch b, const RaggedPlan *__restrict__ plan,
                                                                     uint4 *sink) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    // KEY_LANE: each wave's rows for the round keys of up to kLdsKeys slots (process())
    __shared__ uint4 lkeys[KM == KEY_LANE ? (kThreads / 64) * kLdsKeys * (NR + 1) : 1];
    lds_fill_tables<4>(lds4, b.t0le);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u;
    uint4 *const wkeys = lkeys + (KM == KEY_LANE ? (threadIdx.x >> 6) * kLdsKeys * (NR + 1) : 0);
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const uint64_t count = b.count;
    const uint64_t total = ((ConstU64R *)b.bstart)[count];
    uint64_t c0, c1;
    wave_chunk_range((total + 63) >> 6, nwaves, w, c0, c1);
    if (c0 >= c1) return;

    // round keys: the batch's one key; KEY_LANE AES-128 stream batches: the last slot's
    // (VGPRs, reloaded when the slot changes -- a stream's chunks follow each other)
    RoundKeys<NR> rku;
    uint32_t key_slot = ~0u;
    uint4 ivu = make_uint4(0, 0, 0, 0);
    if (KM == KEY_UNIFORM) {
        ConstDevKeyR *kp = (ConstDevKeyR *)b.keys;
        set_keys(rku, kp);
        ConstU32R *ivp = (ConstU32R *)kp->iv;
        ivu = make_uint4(ivp[0], ivp[1], ivp[2], ivp[3]);
    }
    const uint8_t *dummy = reinterpret_cast<const uint8_t *>(b.keys);  // 16 readable bytes
    // 32 writable bytes that nobody reads: this wave's sink entry (not its plan entry,
    // which is read through constant-address loads the compiler may repeat anywhere)
    uint8_t *scratch = reinterpret_cast<uint8_t *>(sink + 2 * w);

    // the wave's first segment and the ciphertext block in front of its first chunk: from
    // the plan launch (in place), or found here when no wave writes what another reads
    uint64_t wb;
    uint4 fill;
    if (plan) {
        wb = ((ConstU64R *)&plan[w].s0)[0];
        ConstU32R *fp = (ConstU32R *)&plan[w].fill;
        fill = make_uint4(fp[0], fp[1], fp[2], fp[3]);
    } else {
        wb = readfirst64(wave_find_segment(b.bstart, count, c0 << 6, lane));
        fill = predecessor_block<STREAM>(b, wb, c0 << 6);
    }
    // window: wv = bstart[wb + lane] (all-ones past bstart[count])
    auto load_window = [&]() -> uint64_t {
        const uint64_t i = wb + lane;
        return i <= count ? b.bstart[i] : ~0ull;
    };
    uint64_t wv = load_window();

    // descriptors of the segment of the last fetched single-segment chunk (SGPRs)
    uint32_t last_s = ~0u, last_len = 0, last_slot = 0, last_n0 = 0;
    uint64_t last_bs = 0, last_io = 0, last_oo = 0;

    // --- segment of every lane's block in chunk c, descriptor loads issued ----------
    auto locate = [&](uint64_t c) -> RDesc {
        RDesc D;
        const uint64_t base = c << 6;
        D.g = base + lane < total ? base + lane : total - 1;  // lanes past the end: clamped, not stored
        const uint32_t gl = (uint32_t)(D.g - base);
        uint32_t r0 = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(lane >= 1 && wv <= base));
        bool slow = false;
        if (readlane64(wv, 63) <= base + 63) {  // rare: segment starts past the window's end
            while (true) {
                if (r0 == 0) {  // 63 starts inside one chunk: search per lane below
                    slow = true;
                    break;
                }
                wb += r0;  // re-window at the segment holding the chunk's first block
                wv = load_window();
                r0 = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(lane >= 1 && wv <= base));
                if (readlane64(wv, 63) > base + 63) break;
            }
        }
        uint32_t s;
        uint64_t m = slow ? ~0ull : __builtin_amdgcn_ballot_w64(lane >= 1 && wv > base && wv <= base + 63);
        D.uni = m == 0;
        if (D.uni && (uint32_t)(wb + r0) == last_s) {
            // the chunk continues the segment of the chunk fetched before it (long
            // segments: almost every chunk): its descriptors are in SGPRs, no loads
            D.s = last_s;
            D.bs = last_bs;
            D.io = last_io;
            D.oo = last_oo;
            D.len = last_len;
            D.slot = last_slot;
            D.n0 = last_n0;
            return D;
        }
        if (!slow) {
            uint32_t r = r0;
            while (m) {  // the segments that open inside this chunk, in order
                const uint32_t k = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const uint32_t pos = __builtin_amdgcn_readlane((uint32_t)wv, k) - (uint32_t)base;
                r += gl >= pos ? 1u : 0u;
            }
            s = (uint32_t)(wb + r);
        } else {
            uint64_t lo = wb, hi = count - 1;  // largest s with bstart[s] <= g
            while (lo < hi) {
                const uint64_t mid = (lo + hi + 1) >> 1;
                if (b.bstart[mid] <= D.g) lo = mid; else hi = mid - 1;
            }
            s = (uint32_t)lo;
        }
        D.s = s;
        D.bs = b.bstart[s];
        D.io = b.in_off[s];
        D.oo = b.out_off[s];
        D.len = b.len[s];
        D.slot = KM == KEY_LANE ? b.key_slot[s] : 0u;
        D.n0 = STREAM ? b.pos_snap[s] : 0u;
        return D;
    };

    // --- ciphertext block of every lane (loads issued) --------------------------------
    auto fetch = [&](const RDesc &D, uint64_t c) -> RChunk {
        RChunk X;
        X.valid = (c << 6) + lane < total;
        X.s = D.s;
        X.bi = (uint32_t)(D.g - D.bs);
        X.len = D.len;
        X.n0 = D.n0;
        X.slot = D.slot;
        X.in = b.in + D.io;
        X.out = b.out + D.oo;
        if (D.uni) {  // remember the segment (uniform values; the loads have arrived by now)
            last_s = D.s;
            last_bs = readfirst64(D.bs);
            last_io = readfirst64(D.io);
            last_oo = readfirst64(D.oo);
            last_len = __builtin_amdgcn_readfirstlane(D.len);
            last_slot = __builtin_amdgcn_readfirstlane(D.slot);
            last_n0 = __builtin_amdgcn_readfirstlane(D.n0);
        }
        const int64_t lo = 16 * (int64_t)X.bi - X.n0;  // the block's first byte in the segment
        X.full = lo >= 0 && lo + 16 <= (int64_t)X.len;
        // Edge blocks of segments of 16+ bytes load the 16 segment bytes nearest to them
        // (the first 16 for a head block, the last 16 for a tail block) and process()
        // shifts them into place; edge blocks of shorter segments are built bytewise there.
        const int64_t at = X.full ? lo : lo < 0 ? 0 : (int64_t)X.len - 16;
        X.x = load16(X.full || X.len >= 16 ? X.in + at : dummy);
        return X;
    };

    // --- decrypt one chunk; returns lane 63's ciphertext block (the next chunk's fill) --
    auto process = [&](RChunk &X, const uint4 &f) -> uint4 {
        // lanes that open their segment take its IV (stream: the carried ivec), loaded here
        // in a branch taken only by chunks where a segment starts (and drained inside it)
        uint4 ivs = ivu;
        if (STREAM || KM == KEY_LANE) {
            if (__builtin_amdgcn_ballot_w64(X.bi == 0) != 0) {
                if (X.bi == 0)
                    ivs = STREAM ? b.iv_snap[X.s] : *reinterpret_cast<const uint4 *>(b.keys[X.slot].iv);
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            }
        }
        if (__builtin_amdgcn_ballot_w64(X.valid && !X.full) != 0) {  // segment edges: byte-exact block
            if (X.valid && !X.full && X.len >= 16) {
                // head block (bi 0 at position n0 > 0): segment bytes [0, 16 - n0) at n0..15,
                // the carried ivec below them; tail block: the last hi bytes at 0..hi-1
                const int hi = (int)((int64_t)X.n0 + X.len - 16 * (int64_t)X.bi);
                if (X.bi == 0 && X.n0 != 0)
                    X.x = select_bytes(byte_mask(0, (int)X.n0), ivs, shl_bytes(X.x, (int)X.n0));
                else
                    X.x = shr_bytes(X.x, 16 - hi);
            }
            if (__builtin_amdgcn_ballot_w64(X.valid && !X.full && X.len < 16) != 0) {
                if (X.valid && !X.full && X.len < 16) X.x = load_cx(Seg{X.in, X.out, X.len, X.slot}, X.n0, X.bi, ivs);
                // drain here, inside the rare branch: the merge below then carries no pending
                // load, and the common path keeps its prefetches in flight
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            }
        }
        uint4 kin = make_uint4(wave_shr1(X.x.x, f.x), wave_shr1(X.x.y, f.y), wave_shr1(X.x.z, f.z),
                               wave_shr1(X.x.w, f.w));
        if (X.bi == 0) kin = ivs;
        uint4 ks;
        if (KM == KEY_UNIFORM) {
            ks = aes_encrypt_block_sel<FENCE, NR, 4>(kin, rku, T);
        } else {
            // The chunk's distinct key slots.  One: a single pass with wave-uniform keys
            // (below).  Two to kLdsKeys (small frames of many connections in one chunk --
            // 145-B quests: about 7): the slots' round keys are staged in this wave's LDS
            // rows and every lane runs ONE pass with its own row (aes_encrypt_block_ldsk);
            // a pass per slot cost that many full AES passes of the wave.  More: one pass
            // per slot as below.
            uint32_t np = 0, kidx = 0, slotv = 0;
            if (NR >= 12 || !STREAM) {
                uint64_t seen = __builtin_amdgcn_read_exec();
                do {
                    const uint32_t first = (uint32_t)__builtin_ctzll(seen);
                    const uint32_t slotk = __builtin_amdgcn_readlane(X.slot, first);
                    const bool mine = X.slot == slotk;
                    seen &= ~__builtin_amdgcn_ballot_w64(mine);
                    if (mine) kidx = np;
                    slotv = lane == np ? slotk : slotv;  // lane k holds the k-th slot
                    np++;
                } while (seen);
            }
            constexpr int kRows = NR + 1;
            if (NR == 10 && !STREAM) {
                // AES-128 package batches (FPNN's receive frames): one slot -- SGPR keys (scalar loads per chunk; the VGPR-cached keys
                // of earlier rounds left no room beside the pipeline state for the LDS-row
                // path); 2..kLdsKeys -- the LDS rows; more -- one pass per slot through row 0.
                const uint32_t slot0 = __builtin_amdgcn_readfirstlane(slotv);
                if (np == 1) {  // one slot: wave-uniform keys from scalar loads (SGPRs), no LDS rows
                    RoundKeys<NR> rk;
                    set_keys<NR, 4 * (NR + 1)>(rk, (ConstDevKeyR *)b.keys + slot0);
                    ks = aes_encrypt_block<NR, 4>(kin, rk, T);
                } else if (np <= (uint32_t)kLdsKeys) {
                    {
                        const uint32_t kk = lane >> 3, r0 = 2 * (lane & 7);
                        const uint32_t sk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * kk), (int)slotv);
                        const uint4 *src = reinterpret_cast<const uint4 *>(b.keys[kk < np ? sk : 0u].rk);
                        uint4 v[2];
#pragma unroll
                        for (int m = 0; m < 2; m++) v[m] = src[(r0 + m) < (uint32_t)kRows ? r0 + m : 0];
#pragma unroll
                        for (int m = 0; m < 2; m++)
                            if (kk < np && r0 + m < (uint32_t)kRows) wkeys[kk * kRows + r0 + m] = v[m];
                    }
                    ks = aes_encrypt_block_ldsk<NR, 4, false>(kin, wkeys + kidx * kRows, T);
                } else {
                    uint64_t todo = __builtin_amdgcn_read_exec();
                    ks = make_uint4(0, 0, 0, 0);
                    do {
                        const uint32_t first = (uint32_t)__builtin_ctzll(todo);
                        const uint32_t slotk = __builtin_amdgcn_readlane(X.slot, first);
                        const bool mine = X.slot == slotk;
                        todo &= ~__builtin_amdgcn_ballot_w64(mine);
                        if (lane < (uint32_t)kRows)
                            wkeys[lane] = reinterpret_cast<const uint4 *>(b.keys[slotk].rk)[lane];
                        const uint4 e = aes_encrypt_block_ldsk<NR, 4, false>(kin, wkeys, T);
                        if (mine) ks = e;
                    } while (todo);
                }
            } else if (np >= 2 && np <= (uint32_t)kLdsKeys) {
                // lane l copies round-key rows [2 (l & 7), +2) of slot (l >> 3)'s key
                const uint32_t kk = lane >> 3, r0 = 2 * (lane & 7);
                const uint32_t sk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * kk), (int)slotv);
                const uint4 *src = reinterpret_cast<const uint4 *>(b.keys[kk < np ? sk : 0u].rk);
                uint4 v[2];
#pragma unroll
                for (int m = 0; m < 2; m++) v[m] = src[(r0 + m) < (uint32_t)kRows ? r0 + m : 0];
#pragma unroll
                for (int m = 0; m < 2; m++)
                    if (kk < np && r0 + m < (uint32_t)kRows) wkeys[kk * kRows + r0 + m] = v[m];
                ks = aes_encrypt_block_ldsk<NR, 4, FENCE && NR != 10>(kin, wkeys + kidx * kRows, T);
            } else {
            // One pass per distinct key slot in the chunk (AES-192/256 with one or more than
            // kLdsKeys slots; AES-128 stream batches, whose VGPR-cached keys leave no room for
            // the LDS rows -- their long segments seldom share a chunk), a lane keeping the
            // pass of its own slot.  Chunks inside one segment (the common case) take one
            // pass.  AES-192/256: SGPR keys from scalar loads per pass (52-60 words fit
            // neither register file for the whole loop beside the pipeline state).
            uint64_t todo = __builtin_amdgcn_read_exec();
            ks = make_uint4(0, 0, 0, 0);
            do {
                const uint32_t first = (uint32_t)__builtin_ctzll(todo);
                const uint32_t slotk = __builtin_amdgcn_readlane(X.slot, first);
                const bool mine = X.slot == slotk;
                todo &= ~__builtin_amdgcn_ballot_w64(mine);
                uint4 e;
                if (NR == 10) {  // (stream batches) VGPR keys, reloaded when the slot changes
                    if (slotk != key_slot) {
                        // fenced rounds hold 16 lookups in flight: 12 key words then stay in SGPRs
                        // (all in VGPRs spill to scratch, more in SGPRs spill SGPRs)
                        set_keys<NR, FENCE ? 12 : 0>(rku, (ConstDevKeyR *)b.keys + slotk);
                        key_slot = slotk;
                    }
                    e = aes_encrypt_block_sel<FENCE, NR, 4>(kin, rku, T);
                } else {
                    RoundKeys<NR> rk;
                    set_keys<NR, 4 * (NR + 1)>(rk, (ConstDevKeyR *)b.keys + slotk);
                    e = aes_encrypt_block_sel<FENCE, NR, 4>(kin, rk, T);
                }
                if (mine) ks = e;
            } while (todo);
            }
        }
        if (STREAM && X.bi == 0 && X.n0 != 0) ks = ivs;  // keystream bytes already in the carried ivec
        // Stores are unconditional (lanes with nothing to store write the wave's scratch
        // slot), so the waitcnt pass always knows how many are in flight; the byte-exact
        // edge stores run in a rare branch that drains before it rejoins.
        const uint4 pt = X.x ^ ks;
        store16(X.valid && X.full ? X.out + (16ull * X.bi - X.n0) : scratch, pt);
        if (__builtin_amdgcn_ballot_w64(X.valid && !X.full) != 0) {
            if (X.valid && !X.full) store_cx(Seg{X.in, X.out, X.len, X.slot}, X.n0, X.bi, pt);
            __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        }
        if (STREAM) {  // the segment's last block exports (ivec, pos) (base/rijndael.c:1171-1201)
            const bool last = X.valid && (uint64_t)X.bi + 1 == seg_blocks(X.len, X.n0);
            if (__builtin_amdgcn_ballot_w64(last) != 0) {  // once per segment: a rare branch
                if (last) {
                    const uint32_t pos = (X.n0 + X.len) & 15u;
                    *reinterpret_cast<uint4 *>(b.iv_state + 16ull * X.s) =
                        pos ? select_bytes(byte_mask(0, (int)pos), X.x, ks) : X.x;
                    b.pos_state[X.s] = pos;
                }
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            }
        }
        return readlane63(X.x);
    };

    // --- interior runs -------------------------------------------------------------
    // A chunk that lies inside one segment (Dx.uni: its descriptors are in last_*) and
    // whose blocks -- and the following chunks' -- are whole interior blocks of it (every
    // block 16 bytes of the segment, none its first block (the IV) or, in stream mode, its
    // last (the state export)) needs none of the general path's per-lane work: addresses
    // are a wave-uniform base + 16 * lane, there are no edges, one key serves them all.
    // run_at(Dx) decides that for chunk c (fetched, not yet deciphered) and sets the run's
    // length and bases; run(x) deciphers chunks [c, c + run_m) in a loop of its own, from
    // chunk c's ciphertext x (already in registers), the next chunk's in flight during each
    // chunk's rounds: the cipher's own VALU cost plus ~14 instructions per chunk against
    // the general path's ~125 (C4: 2.03 VALU per LDS instruction in round 3).  Long
    // segments (C4's Zipf tail, R1's bodies beyond their first chunk) spend most of their
    // chunks there.  FPNN_AES_K1R_RUNS=0 (KBatch::runs) keeps every chunk on the general
    // path, for same-box A/B.
    // Built for one-key AES-256 package batches only: with the run's code the per-key,
    // stream, AES-128 and AES-192 kernels spill the general path's registers to scratch
    // (framed C3, AES-128 per key, measured 881 against 957 GiB/s without it).
    constexpr bool kRuns = KM == KEY_UNIFORM && NR == 14 && !STREAM;
    uint64_t c = c0;  // the chunk the pipeline deciphers next
    // run parameters (wave-uniform), set by run_at; run() re-asserts their uniformity
    // (readfirstlane) so its loop runs on scalar registers
    uint64_t run_m = 0;
    const uint8_t *run_ip = nullptr;
    uint8_t *run_op = nullptr;
    auto run_at = [&](const RDesc &Dx) -> bool {
        if (!kRuns || !b.runs || !Dx.uni) return false;
        const uint32_t n0 = STREAM ? last_n0 : 0u;
        const uint64_t bi_hi = STREAM ? (uint64_t)seg_blocks(last_len, n0) - 1 : (uint64_t)(last_len >> 4);
        uint64_t cend = (last_bs + bi_hi) >> 6;  // chunks below cend end inside the interior
        if (cend > c1) cend = c1;
        if ((c << 6) <= last_bs || cend <= c) return false;
        run_m = cend - c;
        const uint64_t lo = 16 * ((c << 6) - last_bs) - n0;  // the run's first byte in the segment
        run_ip = b.in + last_io + lo;
        run_op = b.out + last_oo + lo;
        return true;
    };
    auto run = [&](uint4 x) {  // x = the run's first chunk, already loaded
        const uint32_t lofs = lane * 16u;
        const uint64_t m = readfirst64(run_m);  // (uniform again after the merge)
        const uint8_t *ip = reinterpret_cast<const uint8_t *>(readfirst64((uint64_t)(uintptr_t)run_ip));
        uint8_t *op = reinterpret_cast<uint8_t *>(readfirst64((uint64_t)(uintptr_t)run_op));
        // C_{i-1}: lane 0 takes lane 63 of the chunk before (wave_ror:1 of it, lane 0 of
        // `prev`), the other lanes their left neighbour (wave_shr:1 over prev)
        uint4 prev = fill;
        for (uint64_t j = 0; j < m; j++) {
            const uint64_t jn = j + 1 < m ? j + 1 : j;
            const uint4 xn = load16(ip + 1024 * jn + lofs);
            const uint4 kin = make_uint4(wave_shr1(x.x, prev.x), wave_shr1(x.y, prev.y), wave_shr1(x.z, prev.z),
                                         wave_shr1(x.w, prev.w));
            const uint4 ks = aes_encrypt_block_sel<FENCE, NR, 4>(kin, rku, T);
            store16(op + 1024 * j + lofs, x ^ ks);
            prev = make_uint4(wave_ror1(x.x), wave_ror1(x.y), wave_ror1(x.z), wave_ror1(x.w));
            x = xn;
        }
        fill = make_uint4(__builtin_amdgcn_readlane(prev.x, 0), __builtin_amdgcn_readlane(prev.y, 0),
                          __builtin_amdgcn_readlane(prev.z, 0), __builtin_amdgcn_readlane(prev.w, 0));
        c += m;
    };

    // Pipeline.  The vector-memory counter retires in issue order, so a wait for a load
    // also waits for everything issued before it.  Each step issues the next chunk's
    // ciphertext load and the descriptor loads of the chunk after it, THEN enciphers the
    // current chunk: the current chunk's ciphertext was issued one cipher earlier, and the
    // back edge follows a cipher, so the loop header (where the compiler rotates its
    // registers and must wait for their loads) only waits for loads issued one cipher ago.
    // Indices past the wave's range are clamped to its last chunk (re-read, never stored).
    const uint64_t clast = c1 - 1;
    auto cl = [&](uint64_t x) { return x < clast ? x : clast; };
    RDesc D1, D0 = locate(c0);
    RChunk X1, X0 = fetch(D0, c0);
    D1 = locate(cl(c0 + 1));
    if constexpr (kRuns) {
        // unrolled by two like the loop below; a run is entered from the first half only
        // (one copy of its loop: a copy per half spills the general path's registers), so
        // it may start one chunk late.  The pipeline restarts after it (the descriptor
        // loads issued for the run's second chunk are dropped).
        while (true) {
            X1 = fetch(D1, cl(c + 1));
            D0 = locate(cl(c + 2));
            fill = process(X0, fill);
            if (++c >= c1) return;
            if (run_at(D1)) {
                run(X1.x);
                if (c >= c1) return;
                D0 = locate(c);
                X0 = fetch(D0, c);
                D1 = locate(cl(c + 1));
                continue;
            }
            X0 = fetch(D0, cl(c + 1));
            D1 = locate(cl(c + 2));
            fill = process(X1, fill);
            if (++c >= c1) return;
        }
    } else {
        // unrolled by two (no register rotation)
        while (true) {
            X1 = fetch(D1, cl(c + 1));
            D0 = locate(cl(c + 2));
            fill = process(X0, fill);
            if (++c >= c1) return;
            X0 = fetch(D0, cl(c + 1));
            D1 = locate(cl(c + 2));
            fill = process(X1, fill);
            if (++c >= c1) return;
        }
    }
}

// For K1r every segment needs in_off / out_off / len arrays: missing ones are written here
// from the stride / uniform length (out_off missing = in_off).
__global__ __launch_bounds__(256) void k_ragged_desc(uint64_t count, uint64_t stride, uint32_t uniform_len,
                                                     uint64_t *in_off, uint32_t *len) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < count;
         s += (uint64_t)gridDim.x * blockDim.x) {
        if (in_off) in_off[s] = s * stride;
        if (len) len[s] = uniform_len;
    }
}

hipError_t launch_ragged_desc(uint64_t count, uint64_t stride, uint32_t uniform_len, uint64_t *in_off, uint32_t *len,
                              hipStream_t st) {
    if (count && (in_off || len))
        hipLaunchKernelGGL(k_ragged_desc, dim3(grid_for(count, 256, 4096)), dim3(256), 0, st, count, stride,
                           uniform_len, in_off, len);
    return hipGetLastError();
}

// Fenced rounds everywhere except the AES-192/256 per-slot passes, which run out of SGPRs
// for their round keys when fenced (spills).  Only the launched variants are instantiated.
template <int NR>
static void ragged_nr(const KBatch &b, KeyMode km, bool stream, const RaggedPlan *plan, uint4 *sink, int grid,
                      hipStream_t st) {
    constexpr bool kLaneFence = NR == 10;
#define FPNN_RAGGED(S, K, F) \
    hipLaunchKernelGGL((k_cfb_decrypt_ragged<NR, S, K, F>), dim3(grid), dim3(kThreads), 0, st, b, plan, sink)
    if (stream) {
        if (km == KEY_LANE) FPNN_RAGGED(true, KEY_LANE, kLaneFence); else FPNN_RAGGED(true, KEY_UNIFORM, true);
    } else {
        if (km == KEY_LANE) FPNN_RAGGED(false, KEY_LANE, kLaneFence); else FPNN_RAGGED(false, KEY_UNIFORM, true);
    }
#undef FPNN_RAGGED
}

hipError_t launch_decrypt_ragged(const KBatch &b, int nrounds, KeyMode km, bool stream, RaggedPlan *plan, uint4 *sink,
                                 bool plan_launch, int grid, hipStream_t st) {
    const uint64_t nwaves = (uint64_t)grid * (kThreads / 64);
    const unsigned pgrid = (unsigned)((nwaves * 64 + 255) / 256);
    if (!plan_launch)
        plan = nullptr;  // out of place: each wave plans itself (k_cfb_decrypt_ragged)
    else if (stream)
        hipLaunchKernelGGL((k_ragged_plan<true>), dim3(pgrid), dim3(256), 0, st, b, nwaves, plan);
    else
        hipLaunchKernelGGL((k_ragged_plan<false>), dim3(pgrid), dim3(256), 0, st, b, nwaves, plan);
    set_launched("cfb_decrypt_ragged");
    switch (nrounds) {
        case 10: ragged_nr<10>(b, km, stream, plan, sink, grid, st); break;
        case 12: ragged_nr<12>(b, km, stream, plan, sink, grid, st); break;
        case 14: ragged_nr<14>(b, km, stream, plan, sink, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
