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
    const uint64_t w = __builtin_amdgcn_readfirstlane(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
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

// Segment of each lane's block in one chunk (descriptor loads issued, not waited for).
struct RDesc {
    uint64_t g, s, bs;
    uint64_t io, oo;
    uint32_t len, slot, n0;
    bool uni;  // wave-uniform: the whole chunk lies in one segment (descriptors by scalar loads)
};

// The chunk itself: ciphertext block + what its store and CFB fill need.
struct RChunk {
    uint4 x, ivs;
    uint8_t *out;
    uint32_t s, bi, len, n0, slot;  // count < 2^32 (fpnn_aes_batch.count is 32-bit)
    bool valid;
    bool simple;  // wave-uniform: one segment and whole 16-byte blocks only (no byte-granular edge)
};

typedef __attribute__((address_space(4))) const DevKey ConstDevKeyR;
typedef __attribute__((address_space(4))) const uint64_t ConstU64R;
typedef __attribute__((address_space(4))) const uint32_t ConstU32R;

template <int NR, bool STREAM, int KM>
__global__ __launch_bounds__(kThreads, 4) void k_cfb_decrypt_ragged(KBatch b, const RaggedPlan *__restrict__ plan) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, b.t0le);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w = __builtin_amdgcn_readfirstlane(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint64_t count = b.count;
    const uint64_t total = ((ConstU64R *)b.bstart)[count];
    uint64_t c0, c1;
    wave_chunk_range((total + 63) >> 6, nwaves, w, c0, c1);
    if (c0 >= c1) return;

    // uniform key (one key slot for the batch): round keys and IV in SGPRs
    RoundKeys<NR> rku;
    uint4 ivu = make_uint4(0, 0, 0, 0);
    if (KM == KEY_UNIFORM) {
        ConstDevKeyR *kp = (ConstDevKeyR *)b.keys;
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) rku.k[i] = kp->rk[i];
        ConstU32R *ivp = (ConstU32R *)kp->iv;
        ivu = make_uint4(ivp[0], ivp[1], ivp[2], ivp[3]);
    }

    // window: wv = bstart[wb + lane] (all-ones past bstart[count])
    uint64_t wb = ((ConstU64R *)&plan[w].s0)[0];
    auto load_window = [&]() -> uint64_t {
        const uint64_t i = wb + lane;
        return i <= count ? b.bstart[i] : ~0ull;
    };
    uint64_t wv = load_window();
    uint4 fill;
    {
        ConstU32R *fp = (ConstU32R *)&plan[w].fill;
        fill = make_uint4(fp[0], fp[1], fp[2], fp[3]);
    }

    // --- segment of every lane's block in chunk c --------------------------------------
    auto locate = [&](uint64_t c) -> RDesc {
        RDesc D;
        const uint64_t base = c << 6;
        D.g = base + lane < total ? base + lane : total - 1;  // lanes past the end: clamped, not stored
        const uint32_t gl = (uint32_t)(D.g - base);
        bool slow = false;
        uint32_t r0;
        while (true) {
            r0 = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(lane >= 1 && wv <= base));
            const uint64_t last = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(wv >> 32), 63) << 32) |
                                  __builtin_amdgcn_readlane((uint32_t)wv, 63);
            if (last > base + 63) break;  // every segment start in the chunk is in the window
            if (r0 == 0) {                // >= 63 starts inside one chunk: search per lane
                slow = true;
                break;
            }
            wb += r0;  // re-window at the segment holding the chunk's first block
            wv = load_window();
        }
        uint64_t m = slow ? ~0ull : __builtin_amdgcn_ballot_w64(lane >= 1 && wv > base && wv <= base + 63);
        D.uni = m == 0;
        if (D.uni) {  // one segment: descriptors are wave-uniform scalar loads
            const uint64_t su = wb + r0;
            D.s = su;
            D.bs = ((ConstU64R *)b.bstart)[su];
            D.io = b.in_off ? ((ConstU64R *)b.in_off)[su] : su * b.stride;
            D.oo = b.out_off ? ((ConstU64R *)b.out_off)[su] : D.io;
            D.len = b.len ? ((ConstU32R *)b.len)[su] : b.uniform_len;
            D.slot = (KM == KEY_LANE && b.key_slot) ? ((ConstU32R *)b.key_slot)[su] : 0u;
            D.n0 = STREAM ? ((ConstU32R *)b.pos_snap)[su] : 0u;
            return D;
        }
        uint64_t s;
        if (!slow) {
            uint32_t r = r0;
            while (m) {  // the segments that open inside this chunk, in order
                const uint32_t k = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const uint32_t pos = __builtin_amdgcn_readlane((uint32_t)wv, k) - (uint32_t)base;
                r += gl >= pos ? 1u : 0u;
            }
            s = wb + r;
        } else {
            uint64_t lo = wb, hi = count - 1;  // largest s with bstart[s] <= g
            while (lo < hi) {
                const uint64_t mid = (lo + hi + 1) >> 1;
                if (b.bstart[mid] <= D.g) lo = mid; else hi = mid - 1;
            }
            s = lo;
        }
        D.s = s;
        D.bs = b.bstart[s];
        D.io = b.in_off ? b.in_off[s] : s * b.stride;
        D.oo = b.out_off ? b.out_off[s] : D.io;
        D.len = b.len ? b.len[s] : b.uniform_len;
        D.slot = (KM == KEY_LANE && b.key_slot) ? b.key_slot[s] : 0u;
        D.n0 = STREAM ? b.pos_snap[s] : 0u;
        return D;
    };

    // --- ciphertext block of every lane (loads issued) --------------------------------
    auto fetch = [&](const RDesc &D, uint64_t c) -> RChunk {
        RChunk X;
        X.valid = (c << 6) + lane < total;
        X.s = (uint32_t)D.s;
        X.bi = (uint32_t)(D.g - D.bs);
        X.len = D.len;
        X.n0 = D.n0;
        X.slot = D.slot;
        const uint8_t *in = b.in + D.io;
        X.out = b.out + D.oo;
        X.ivs = ivu;
        if (X.bi == 0) {  // the lane opens its segment: CFB input = IV (carried IV in stream mode)
            if (STREAM) X.ivs = b.iv_snap[X.s];
            else if (KM == KEY_LANE) X.ivs = *reinterpret_cast<const uint4 *>(b.keys[X.slot].iv);
        }
        // simple chunk: one segment, no partial head block (stream position) and no partial
        // last block inside it -- every lane loads and stores one whole 16-byte block
        X.simple = false;
        if (D.uni) {
            const uint32_t bi0 = __builtin_amdgcn_readfirstlane(X.bi);  // lane 0 is never clamped
            const uint64_t nbs = seg_blocks(X.len, X.n0);
            const bool partial_head = bi0 == 0 && X.n0 != 0;
            const bool partial_tail = ((X.n0 + X.len) & 15u) != 0 && (uint64_t)bi0 + 63 >= nbs - 1;
            X.simple = !partial_head && !partial_tail;
        }
        if (X.simple)
            X.x = load16(in + 16ull * X.bi - X.n0);
        else
            X.x = load_cx(Seg{in, X.out, X.len, X.slot}, X.n0, X.bi, X.ivs);
        return X;
    };

    // --- decrypt one chunk; returns lane 63's ciphertext block (the next chunk's fill) --
    auto process = [&](const RChunk &X, const uint4 &f) -> uint4 {
        uint4 kin = make_uint4(wave_shr1(X.x.x, f.x), wave_shr1(X.x.y, f.y), wave_shr1(X.x.z, f.z),
                               wave_shr1(X.x.w, f.w));
        if (X.bi == 0) kin = X.ivs;
        uint4 ks;
        if (KM == KEY_UNIFORM) {
            ks = aes_encrypt_block<NR, 4>(kin, rku, T);
        } else {
            // one pass per distinct key slot in the chunk, each with wave-uniform (SGPR)
            // round keys; a lane keeps the pass of its own slot.  Chunks inside one segment
            // (the common case) take one pass; no per-lane key registers.
            uint64_t todo = __builtin_amdgcn_read_exec();
            ks = make_uint4(0, 0, 0, 0);
            do {
                const uint32_t first = (uint32_t)__builtin_ctzll(todo);
                const uint32_t slotk = __builtin_amdgcn_readlane(X.slot, first);
                const bool mine = X.slot == slotk;
                todo &= ~__builtin_amdgcn_ballot_w64(mine);
                RoundKeys<NR> rk;
                ConstDevKeyR *kp = (ConstDevKeyR *)b.keys + slotk;
#pragma unroll
                for (int i = 0; i < 4 * (NR + 1); i++) rk.k[i] = kp->rk[i];
                const uint4 e = aes_encrypt_block<NR, 4>(kin, rk, T);
                if (mine) ks = e;
            } while (todo);
        }
        if (STREAM && X.bi == 0 && X.n0 != 0) ks = X.ivs;  // keystream bytes already in the carried ivec
        if (X.valid) {
            if (X.simple)
                store16(X.out + 16ull * X.bi - X.n0, X.x ^ ks);
            else
                store_cx(Seg{nullptr, X.out, X.len, X.slot}, X.n0, X.bi, X.x ^ ks);
            if (STREAM && (uint64_t)X.bi + 1 == seg_blocks(X.len, X.n0)) {  // last block: export (ivec, pos)
                const uint32_t pos = (X.n0 + X.len) & 15u;
                const uint4 nv = pos ? select_bytes(byte_mask(0, (int)pos), X.x, ks) : X.x;
                *reinterpret_cast<uint4 *>(b.iv_state + 16ull * X.s) = nv;
                b.pos_state[X.s] = pos;
            }
        }
        return readlane63(X.x);
    };

    // pipeline: while chunk c is enciphered, the ciphertext of chunks c+1 .. c+DEPTH-1 and
    // the descriptors of the next chunk to fetch are in flight (a ring of DEPTH chunk
    // buffers, one descriptor buffer)
    constexpr int DEPTH = 3;
    RChunk X[DEPTH];
    RDesc D = locate(c0);
    uint64_t next = c0;  // next chunk to fetch; D = its descriptors
#pragma unroll
    for (int j = 0; j < DEPTH; j++) {
        if (next < c1) {
            X[j] = fetch(D, next);
            next++;
            if (next < c1) D = locate(next);
        }
    }
    uint64_t c = c0;
    while (true) {
#pragma unroll
        for (int j = 0; j < DEPTH; j++) {  // X[j] holds chunk c
            fill = process(X[j], fill);
            if (next < c1) {
                X[j] = fetch(D, next);
                next++;
                if (next < c1) D = locate(next);
            }
            if (++c >= c1) return;
        }
    }
}

template <int NR>
static void ragged_nr(const KBatch &b, KeyMode km, bool stream, const RaggedPlan *plan, int grid, hipStream_t st) {
#define FPNN_RAGGED(S, K) \
    hipLaunchKernelGGL((k_cfb_decrypt_ragged<NR, S, K>), dim3(grid), dim3(kThreads), 0, st, b, plan)
    if (stream) {
        if (km == KEY_LANE) FPNN_RAGGED(true, KEY_LANE); else FPNN_RAGGED(true, KEY_UNIFORM);
    } else {
        if (km == KEY_LANE) FPNN_RAGGED(false, KEY_LANE); else FPNN_RAGGED(false, KEY_UNIFORM);
    }
#undef FPNN_RAGGED
}

hipError_t launch_decrypt_ragged(const KBatch &b, int nrounds, KeyMode km, bool stream, RaggedPlan *plan, int grid,
                                 hipStream_t st) {
    const uint64_t nwaves = (uint64_t)grid * (kThreads / 64);
    const unsigned pgrid = (unsigned)((nwaves * 64 + 255) / 256);
    if (stream)
        hipLaunchKernelGGL((k_ragged_plan<true>), dim3(pgrid), dim3(256), 0, st, b, nwaves, plan);
    else
        hipLaunchKernelGGL((k_ragged_plan<false>), dim3(pgrid), dim3(256), 0, st, b, nwaves, plan);
    set_launched("cfb_decrypt_ragged");
    switch (nrounds) {
        case 10: ragged_nr<10>(b, km, stream, plan, grid, st); break;
        case 12: ragged_nr<12>(b, km, stream, plan, grid, st); break;
        case 14: ragged_nr<14>(b, km, stream, plan, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
