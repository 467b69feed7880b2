// k_support.hip -- small gfx950 kernels around the cipher: the ragged decrypt block
// map (scan), the longest-first encrypt ordering, device key expansion and the
// synthetic payload generator.
#include "segments.hpp"

namespace fpnn_aes {

// ---------------------------------------------------------------------------
// General-layout block map: exclusive scan of per-segment block counts.

constexpr int kScanThreads = 256;

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

// Batches of up to kSmallScanMax segments (C3's 4 096 streams, R1's 16 384 connections):
// the whole block map in ONE workgroup -- and, for stream batches, the (iv, pos) snapshot
// the decrypt kernels read -- instead of a look-back launch plus two copies; a framed
// call is launch-bound, so this is most of its fixed cost.  The snapshot is written
// here but the block counts read the live state (nothing has changed it yet).
constexpr int kSmallScanThreads = 1024;
constexpr int kSmallScanItems = 16;
constexpr uint64_t kSmallScanMax = (uint64_t)kSmallScanThreads * kSmallScanItems;

// Round k covers segments [k·1024, k·1024 + 1024), one per thread, so every load and
// store is coalesced.  Segment order is (round, wave, lane): each round's values are
// scanned inside the wave (6 DPP steps), the ≤ 256 wave totals in that same order are
// scanned by wave 0, and two barriers join the halves (the round-1 form held contiguous
// runs per thread and paid 20 barriers of a 1024-wide Hillis-Steele scan: ≈ 10 µs per
// framed call).  Rounds go in groups of four with no per-round branch inside a group (the
// loads past the batch re-read its last segment), so a group's loads share one memory
// round trip and its four scans interleave: the per-round branches of round 3 serialised
// the snapshot's load -> store and the scans, ≈ 7.5 µs per launch at C3's 4 096 streams.
// Inclusive wave64 scan of 64-bit values in DPP moves (no LDS round trips): Hillis-Steele
// inside each 16-lane row (row_shr 1, 2, 4, 8; lanes shifted in from outside the row read
// 0), then row 15's total into rows 1 and 3 (row_bcast:15) and lane 31's into rows 2 and
// 3 (row_bcast:31); disabled rows take `old` = 0.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROWS, 0xf, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xf, true);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x) {
    x += dpp_u64<0x111, 0xf>(x);  // row_shr:1
    x += dpp_u64<0x112, 0xf>(x);  // row_shr:2
    x += dpp_u64<0x114, 0xf>(x);  // row_shr:4
    x += dpp_u64<0x118, 0xf>(x);  // row_shr:8
    x += dpp_u64<0x142, 0xa>(x);  // row_bcast:15 -> rows 1, 3
    x += dpp_u64<0x143, 0xc>(x);  // row_bcast:31 -> rows 2, 3
    return x;
}

constexpr int kScanGroup = 4;
static_assert(kSmallScanItems % kScanGroup == 0 && kScanGroup == 4, "groups of four rounds");

template <bool STREAM>
__global__ __launch_bounds__(kSmallScanThreads) void k_scan_small(KBatch b, const uint4 *__restrict__ iv_src,
                                                                  const uint32_t *__restrict__ pos_src,
                                                                  uint4 *__restrict__ snap_iv,
                                                                  uint32_t *__restrict__ snap_pos,
                                                                  uint64_t *__restrict__ bstart,
                                                                  uint64_t *__restrict__ total_out) {
    constexpr int kWaves = kSmallScanThreads / 64;
    __shared__ uint64_t grp[kSmallScanItems * kWaves + 1];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t count = b.count;  // 1 <= count <= kSmallScanMax (host)
    const uint32_t per = (count + kSmallScanThreads - 1) / kSmallScanThreads;
    const uint32_t *__restrict__ lens = b.len;
    uint32_t len[kSmallScanItems], pos[kSmallScanItems];
#pragma unroll
    for (int k0 = 0; k0 < kSmallScanItems; k0 += kScanGroup) {  // every group's loads first
        if ((uint32_t)k0 < per) {
#pragma unroll
            for (int k = k0; k < k0 + kScanGroup; k++) {
                const uint32_t s = k * kSmallScanThreads + t, sc = s < count ? s : count - 1;
                len[k] = lens ? lens[sc] : b.uniform_len;
                pos[k] = STREAM ? pos_src[sc] : 0u;
            }
        }
    }
    if (STREAM) {  // the (iv, pos) snapshot the decrypt kernels read
#pragma unroll
        for (int k0 = 0; k0 < kSmallScanItems; k0 += kScanGroup) {
            if ((uint32_t)k0 < per) {
                // Lanes past the batch copy its last segment again (the same bytes), so
                // the stores need no predicate and the loads stay in one round trip.
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                const v4u *__restrict__ src = reinterpret_cast<const v4u *>(iv_src);
                v4u *__restrict__ dst = reinterpret_cast<v4u *>(snap_iv);
                v4u iv[kScanGroup];
                uint32_t sc[kScanGroup];
#pragma unroll
                for (int k = 0; k < kScanGroup; k++) {
                    const uint32_t s = (k0 + k) * kSmallScanThreads + t;
                    sc[k] = s < count ? s : count - 1;
                    iv[k] = src[sc[k]];
                }
                asm volatile("" : "+v"(iv[0]), "+v"(iv[1]), "+v"(iv[2]), "+v"(iv[3]));  // one round trip
#pragma unroll
                for (int k = 0; k < kScanGroup; k++) {
                    dst[sc[k]] = iv[k];
                    snap_pos[sc[k]] = pos[k0 + k];
                }
            }
        }
    }
    uint64_t ex[kSmallScanItems];  // exclusive prefix inside the wave, then the segment's bstart
#pragma unroll
    for (int k0 = 0; k0 < kSmallScanItems; k0 += kScanGroup) {
        if ((uint32_t)k0 < per) {
            uint64_t v[kScanGroup], x[kScanGroup];
#pragma unroll
            for (int k = 0; k < kScanGroup; k++) {
                const uint32_t s = (k0 + k) * kSmallScanThreads + t;
                v[k] = s < count ? seg_blocks(len[k0 + k], pos[k0 + k]) : 0;
                x[k] = v[k];
            }
#pragma unroll
            for (int k = 0; k < kScanGroup; k++) x[k] = wave_incl_scan64(x[k]);
#pragma unroll
            for (int k = 0; k < kScanGroup; k++) {
                ex[k0 + k] = x[k] - v[k];
                if (lane == 63) grp[(k0 + k) * kWaves + wv] = x[k];  // rounds >= per are zero
            }
        }
    }
    __syncthreads();
    if (wv == 0) {  // exclusive scan of the wave totals (per rounded up to a group) * 16, 4 per lane
        const uint32_t n = ((per + kScanGroup - 1) / kScanGroup) * kScanGroup * kWaves;
        uint64_t g[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t j = lane * 4 + i;
            g[i] = j < n ? grp[j] : 0;
            sum += g[i];
        }
        const uint64_t x = wave_incl_scan64(sum);
        uint64_t run = x - sum;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t j = lane * 4 + i;
            if (j < n) grp[j] = run;
            run += g[i];
        }
        if (lane == 63) grp[kSmallScanItems * kWaves] = x;  // the block total
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSmallScanItems; k++) {
        const uint32_t s = k * kSmallScanThreads + t;
        if ((uint32_t)k < per && s < count) bstart[s] = grp[k * kWaves + wv] + ex[k];
    }
    if (t == 0) {
        const uint64_t total = grp[kSmallScanItems * kWaves];
        bstart[count] = total;
        *total_out = total;
    }
}

hipError_t launch_block_map_small(const KBatch &b, bool stream, const uint8_t *iv_state, const uint32_t *pos_state,
                                  uint4 *snap_iv, uint32_t *snap_pos, uint64_t *bstart, uint64_t *total,
                                  hipStream_t st) {
    if (stream)
        hipLaunchKernelGGL((k_scan_small<true>), dim3(1), dim3(kSmallScanThreads), 0, st, b,
                           reinterpret_cast<const uint4 *>(iv_state), pos_state, snap_iv, snap_pos, bstart, total);
    else
        hipLaunchKernelGGL((k_scan_small<false>), dim3(1), dim3(kSmallScanThreads), 0, st, b, nullptr, nullptr,
                           nullptr, nullptr, bstart, total);
    return hipGetLastError();
}

uint64_t block_map_small_max() { return kSmallScanMax; }

// ---------------------------------------------------------------------------
// Length ordering for ragged encrypt batches: counting sort into 128 descending
// quarter-octave buckets of the block count (order inside a bucket is arbitrary; it
// only affects speed, never results).

constexpr int kBuckets = 128;

__host__ __device__ inline uint32_t bucket_of_blocks(uint64_t nblocks) {
    const uint64_t nb = nblocks + 1;  // >= 1
    const uint32_t x = nb > 0xffffffffull ? 0xffffffffu : (uint32_t)nb;
    const int lz = 31 - __builtin_clz(x);
    const uint32_t frac = lz >= 2 ? (x >> (lz - 2)) & 3u : (x << (2 - lz)) & 3u;
    return (uint32_t)(kBuckets - 1) - (uint32_t)(4 * lz + frac);  // descending length
}

uint32_t length_bucket_of(uint64_t nblocks) { return bucket_of_blocks(nblocks); }

// A wave whose lanes all fall in one bucket (uniform lengths: R1's frames, C2R) adds to
// it once instead of 64 times: same-address LDS atomics serialise lane by lane.  Returns
// the lane's slot among the wave's additions to bucket k (base = the counter's old value).
__device__ __forceinline__ uint32_t bucket_add(uint32_t *h, uint32_t k, bool live) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t act = __builtin_amdgcn_ballot_w64(live);
    if (!act) return 0;
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)k, (int)__builtin_ctzll(act));
    if (__builtin_amdgcn_ballot_w64(live && k == k0) == act) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(act);
        uint32_t base = 0;
        if (lane == lead) base = atomicAdd(&h[k0], (uint32_t)__builtin_popcountll(act));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)lead);
        return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    }
    return live ? atomicAdd(&h[k], 1u) : 0u;
}

// Both passes take 16 segments per thread with every load issued before the first use:
// unconditional loads (lanes past the batch re-read its last segment), so no load sits
// in a branch of its own with a wait behind it (a loop of load -> atomic per segment
// waited out one memory latency per segment: R1's 1 M frames cost 19 + 14 µs per call).
// The host calls these for ragged batches only (b.len set).
constexpr int kBucketItems = 16;
constexpr uint64_t kBucketTile = 256ull * kBucketItems;

// buckets of segments tile0 + 256 i (kBuckets: past the batch)
template <bool STREAM>
__device__ __forceinline__ void tile_buckets(const KBatch &b, uint64_t tile0, uint32_t (&kb)[kBucketItems]) {
    const uint32_t *__restrict__ lens = b.len;
    uint32_t L[kBucketItems], P[kBucketItems];
#pragma unroll
    for (int i = 0; i < kBucketItems; i++) {
        const uint64_t s = tile0 + 256ull * i, sc = s < b.count ? s : b.count - 1;
        L[i] = *FA_AT(b, AB_LEN, lens + sc, 4);
        P[i] = STREAM ? *FA_AT(b, AB_POS_SNAP, b.pos_snap + sc, 4) : 0u;
    }
#pragma unroll
    for (int i = 0; i < kBucketItems; i++)
        kb[i] = tile0 + 256ull * i < b.count ? bucket_of_blocks(seg_blocks(L[i], P[i])) : (uint32_t)kBuckets;
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_bucket_count(KBatch b, uint32_t *counts) {
    __shared__ uint32_t h[kBuckets];
    __shared__ uint32_t off4;
    if (threadIdx.x < kBuckets) h[threadIdx.x] = 0;
    if (threadIdx.x == 0) off4 = 0;
    __syncthreads();
    const uint64_t tile0 = (uint64_t)blockIdx.x * kBucketTile + threadIdx.x;
    uint32_t kb[kBucketItems], mis = 0;
    if (!STREAM && (b.flags & F_WIRE_PREFIX)) {  // K2h's funnel is needed when an output is off the 4-byte grid
        const uint64_t *__restrict__ op = b.out_off ? b.out_off : b.in_off;
        uint64_t O[kBucketItems];
#pragma unroll
        for (int i = 0; i < kBucketItems; i++) {
            const uint64_t s = tile0 + 256ull * i, sc = s < b.count ? s : b.count - 1;
            O[i] = op ? *FA_AT(b, b.out_off ? AB_OUT_OFF : AB_IN_OFF, op + sc, 8) : sc * b.stride;
        }
#pragma unroll
        for (int i = 0; i < kBucketItems; i++) mis |= (uint32_t)((uintptr_t)b.out + O[i]) & 3u;
    }
    tile_buckets<STREAM>(b, tile0, kb);
#pragma unroll
    for (int i = 0; i < kBucketItems; i++) {
        const bool live = kb[i] < (uint32_t)kBuckets;
        (void)bucket_add(h, live ? kb[i] : 0u, live);
    }
    if (mis) off4 = 1;
    __syncthreads();
    if (threadIdx.x < kBuckets && h[threadIdx.x]) atomicAdd(FA_AT(b, AB_BLOCK, &counts[threadIdx.x], 4), h[threadIdx.x]);
    if (threadIdx.x == 0 && off4) atomicOr(FA_AT(b, AB_BLOCK, &counts[kWireFlagWord], 4), 1u);
}

__global__ __launch_bounds__(kBuckets) void k_bucket_scan(uint32_t *counts, uint32_t *cursor, uint64_t count,
                                                          uint32_t *fault) {
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
    // the counts of a block that was zero on entry add up to the batch
    if (t == kBuckets - 1 && sh[t] != count && fault)
        __hip_atomic_store(fault, kFaultLengthOrder, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_bucket_scatter(KBatch b, uint32_t *cursor, uint32_t *perm, uint32_t *release) {
    __shared__ uint32_t cnt[kBuckets], base[kBuckets];
    if (threadIdx.x < kBuckets) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t tile0 = (uint64_t)blockIdx.x * kBucketTile + threadIdx.x;
    uint32_t kb[kBucketItems];
    tile_buckets<STREAM>(b, tile0, kb);
#pragma unroll
    for (int i = 0; i < kBucketItems; i++) {
        const bool live = kb[i] < (uint32_t)kBuckets;
        (void)bucket_add(cnt, live ? kb[i] : 0u, live);
    }
    __syncthreads();
    if (threadIdx.x < kBuckets) {
        base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(FA_AT(b, AB_BLOCK, &cursor[threadIdx.x], 4), cnt[threadIdx.x]) : 0u;
        cnt[threadIdx.x] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kBucketItems; i++) {
        const bool live = kb[i] < (uint32_t)kBuckets;
        const uint32_t k = live ? kb[i] : 0u;
        const uint32_t slot = bucket_add(cnt, k, live);
        const uint32_t at = base[k] + slot;
        if (live && at < b.count) *FA_AT(b, AB_PERM, perm + at, 4) = (uint32_t)(tile0 + 256ull * i);  // (past it: a bad block, see scan)
    }
    if (release) length_order_release(release);  // K2c follows: nothing reads the block again
}

hipError_t launch_length_order(const KBatch &b, bool stream, uint32_t *perm, uint32_t *block, bool zero_after,
                               uint32_t *fault, hipStream_t st) {
    uint32_t *counts = block, *cursor = block + kBuckets;
    const unsigned grid = (unsigned)((b.count + kBucketTile - 1) / kBucketTile);
    uint32_t *release = zero_after ? block : nullptr;
    if (stream)
        hipLaunchKernelGGL((k_bucket_count<true>), dim3(grid), dim3(256), 0, st, b, counts);
    else
        hipLaunchKernelGGL((k_bucket_count<false>), dim3(grid), dim3(256), 0, st, b, counts);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(kBuckets), 0, st, counts, cursor, b.count, fault);
    if (stream)
        hipLaunchKernelGGL((k_bucket_scatter<true>), dim3(grid), dim3(256), 0, st, b, cursor, perm, release);
    else
        hipLaunchKernelGGL((k_bucket_scatter<false>), dim3(grid), dim3(256), 0, st, b, cursor, perm, release);
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

// Single-pass block map for batches past the one-workgroup map (decoupled look-back): a
// workgroup takes a ticket v (tickets follow the order workgroups start in, so every
// tile it waits for belongs to a running or finished workgroup), scans its 4 096
// segments, publishes the tile's total, sums its predecessors' published totals back to
// the nearest inclusive prefix (one wave, 64 tiles per round trip), publishes its own
// inclusive prefix and writes its bstart entries.  One launch where the three-launch
// scan took ≈ 19 µs per call at R1's 1 M frames.
// lb[0] = ticket, lb[1] = finished workgroups, lb[2] = this launch's epoch (0 = 1), lb[3 + v]
// = tile v's status word: epoch (26 bits, never 0; stale words of earlier launches never
// match) | flag (A = tile total, P = inclusive prefix) | value (36 bits: block totals
// stay below 2^36, 1 TiB of data).  The last workgroup to finish resets the tickets and
// advances the epoch; when the epoch wraps it first clears every status word of the buffer,
// so a word 2^26 launches old cannot match either.  Nothing is passed from the host per
// launch: a captured launch replays correctly (fpnn_aes_engine_reserve, "graph-safe").
constexpr int kOneItems = 16;
constexpr uint64_t kOneTile = (uint64_t)kScanThreads * kOneItems;
static_assert(kOneItems * (kScanThreads / 64) == 64, "one wave scans the tile's group totals");
constexpr uint64_t kLbValue = (1ull << 36) - 1, kLbA = 1ull << 36, kLbP = 2ull << 36, kLbFlags = 3ull << 36;
constexpr uint32_t kLbMaxSpin = 1u << 22;  // a bound, never reached: no wave spins forever

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint64_t kLbEpochMask = (1ull << 26) - 1;

template <bool STREAM>
__global__ __launch_bounds__(kScanThreads) void k_scan_onepass(KBatch b, uint64_t *bstart, uint64_t *lb, uint64_t nwg,
                                                               uint64_t lb_words, uint32_t *fault,
                                                               uint64_t *total_out) {
    __shared__ uint64_t grp[kOneItems * (kScanThreads / 64)];
    __shared__ uint64_t ticket, epoch;
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    if (t == 0) {
        ticket = __hip_atomic_fetch_add(&lb[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t e = lb_load(&lb[2]) & kLbEpochMask;  // written by the previous launch's last workgroup
        epoch = e ? e : 1;
    }
    __syncthreads();
    const uint64_t v = ticket, tile0 = v * kOneTile, tag = epoch << 38;
    uint64_t val[kOneItems], ex[kOneItems];
#pragma unroll
    for (int k = 0; k < kOneItems; k++) val[k] = nblocks_of<STREAM>(b, tile0 + (uint64_t)k * kScanThreads + t);
#pragma unroll
    for (int k = 0; k < kOneItems; k++) {  // segment order (round k, wave, lane), as k_scan_small
        const uint64_t x = wave_incl_scan64(val[k]);
        ex[k] = x - val[k];
        if (lane == 63) grp[k * (kScanThreads / 64) + wv] = x;
    }
    __syncthreads();
    if (wv == 0) {
        uint64_t *const st = lb + 3;
        const uint64_t g = grp[lane];
        const uint64_t x = wave_incl_scan64(g);
        const uint64_t agg = (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63) << 32);
        if (lane == 0) lb_store(&st[v], tag | (v == 0 ? kLbP : kLbA) | agg);
        uint64_t excl = 0;
        for (uint64_t end = v; end > 0;) {  // tiles [end - 64, end), nearest first in lane 0
            const int64_t idx = (int64_t)end - 1 - (int64_t)lane;
            uint64_t w = 0, pm = 0, need = ~0ull;
            for (uint32_t spin = 0;; spin++) {
                w = idx >= 0 ? lb_load(&st[idx]) : (tag | kLbP);  // before tile 0: a prefix of 0
                const bool ok = (w & ~(kLbFlags | kLbValue)) == tag && (w & kLbFlags) != 0;
                pm = __builtin_amdgcn_ballot_w64(ok && (w & kLbP));
                need = pm ? ((pm & (0ull - pm)) << 1) - 1 : ~0ull;  // lanes up to the nearest prefix
                if ((__builtin_amdgcn_ballot_w64(!ok) & need) == 0) break;
                if (spin == kLbMaxSpin) {  // never expected: report it rather than sum stale words silently
                    if (lane == 0) __hip_atomic_store(fault, kFaultLookback, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            const uint64_t part = (need >> lane) & 1ull ? (w & kLbValue) : 0ull;
            const uint64_t sum = wave_incl_scan64(part);
            excl += (uint64_t)__builtin_amdgcn_readlane((int)(uint32_t)sum, 63) |
                    ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sum >> 32), 63) << 32);
            if (pm) break;
            end = end > 64 ? end - 64 : 0;
        }
        if (v > 0 && lane == 0) lb_store(&st[v], tag | kLbP | (excl + agg));
        grp[lane] = excl + x - g;  // the group's first bstart
        if (lane == 0 && v == nwg - 1) {
            bstart[b.count] = excl + agg;
            *total_out = excl + agg;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kOneItems; k++) {
        const uint64_t s = tile0 + (uint64_t)k * kScanThreads + t;
        if (s < b.count) bstart[s] = grp[k * (kScanThreads / 64) + wv] + ex[k];
    }
    if (t == 0 && __hip_atomic_fetch_add(&lb[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
        // every workgroup has its ticket and epoch and is past its look-back
        uint64_t next = (epoch + 1) & kLbEpochMask;
        if (!next) {  // wrapped: no status word of any earlier launch may match epoch 1 again
            for (uint64_t i = 3; i < lb_words; i++) lb_store(&lb[i], 0);
            next = 1;
        }
        lb_store(&lb[2], next);
        lb_store(&lb[0], 0);
        lb_store(&lb[1], 0);
    }
}

uint64_t block_map_onepass_words(uint64_t count) { return 3 + (count + kOneTile - 1) / kOneTile; }

hipError_t launch_block_map_onepass(const KBatch &b, bool stream, uint64_t *bstart, uint64_t *lb, uint64_t lb_words,
                                    uint32_t *fault, uint64_t *total, hipStream_t st) {
    const uint64_t nwg = (b.count + kOneTile - 1) / kOneTile;
    if (!nwg) return hipSuccess;
    if (stream)
        hipLaunchKernelGGL((k_scan_onepass<true>), dim3((unsigned)nwg), dim3(kScanThreads), 0, st, b, bstart, lb, nwg,
                           lb_words, fault, total);
    else
        hipLaunchKernelGGL((k_scan_onepass<false>), dim3((unsigned)nwg), dim3(kScanThreads), 0, st, b, bstart, lb, nwg,
                           lb_words, fault, total);
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

// ---------------------------------------------------------------------------
// Host-mapped frame moves (fpnn_aes_package_host over registered host memory, §8f row 1).
// A MoveJob copies n segments, segment i from address sbase + soff[i] to dbase + doff[i],
// len[i] + extra bytes: the gather of frames from host socket buffers into contiguous HBM
// staging (sbase = 0, soff = device-visible host addresses) or the scatter of results back
// (dbase = 0).  The GPU moves the bytes over PCIe itself: no CPU copy, no pinned bounce
// buffer.  One launch runs TWO jobs -- the gather of chunk t and the scatter of chunk
// t - 2 -- with their segment groups interleaved over the waves, so both link directions
// are busy inside one kernel (separate gather and scatter launches on two streams, many
// per call, overlapped only partially on MI355X: tools/probe/hostmap_bw.hip).
// A wave moves a group of F segments per step in 1 KiB pieces, lane l taking bytes
// [16l, 16l + 16) of a piece (unaligned dwordx4; byte copies for the lane that straddles
// a segment's end); all F pieces' loads go out before their stores.
template <int F>
__device__ __forceinline__ void move_group(const MoveJob &J, uint64_t g, uint32_t lane) {
    const uint8_t *src[F];
    uint8_t *dst[F];
    uint32_t L[F];
    uint32_t maxl = 0;
#pragma unroll
    for (int k = 0; k < F; k++) {
        const uint64_t i = g * F + k;
        L[k] = i < J.n ? J.len[i] + J.extra : 0u;
        src[k] = reinterpret_cast<const uint8_t *>(i < J.n ? J.sbase + J.soff[i] : J.sbase);
        dst[k] = reinterpret_cast<uint8_t *>(i < J.n ? J.dbase + J.doff[i] : J.dbase);
        maxl = L[k] > maxl ? L[k] : maxl;
    }
    for (uint32_t p = 0; p < maxl; p += 1024) {
        const uint32_t b = p + 16 * lane;
        uint4 v[F];
#pragma unroll
        for (int k = 0; k < F; k++) v[k] = b + 16 <= L[k] ? load16(src[k] + b) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < F; k++) {
            if (b + 16 <= L[k]) {
                store16(dst[k] + b, v[k]);
            } else if (b < L[k]) {
                for (uint32_t j = b; j < L[k]; j++) dst[k][j] = src[k][j];
            }
        }
    }
}

template <int F>
__global__ __launch_bounds__(256) void k_move_segments(MoveJob a, MoveJob b) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const uint64_t ga = (a.n + F - 1) / F, gb = (b.n + F - 1) / F;
    const uint64_t both = 2 * (ga < gb ? ga : gb);  // virtual groups [0, both) alternate a, b
    for (uint64_t v = w; v < ga + gb; v += nw) {
        if (v < both) {
            if (v & 1) move_group<F>(b, v >> 1, lane); else move_group<F>(a, v >> 1, lane);
        } else if (ga > gb) {
            move_group<F>(a, v - both / 2, lane);
        } else {
            move_group<F>(b, v - both / 2, lane);
        }
    }
}

hipError_t launch_move_segments(const MoveJob &a, const MoveJob &b, hipStream_t st) {
    const uint64_t groups = (a.n + 3) / 4 + (b.n + 3) / 4;
    if (!groups) return hipSuccess;
    // 256 x 256 threads: 1024 waves x 4 KiB in flight saturate the link (more waves only
    // slow the opposite direction)
    const int grid = grid_for(groups, 4, 256);
    hipLaunchKernelGGL((k_move_segments<4>), dim3(grid), dim3(256), 0, st, a, b);
    return hipGetLastError();
}

}  // namespace fpnn_aes
