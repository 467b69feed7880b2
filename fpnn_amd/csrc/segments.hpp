// segments.hpp -- device-side view of a batch shared by the encrypt and decrypt
// kernels: segment lookup, stream-aligned block loads/stores with the reference's
// exact (ivec, pos) byte semantics, and the uniform/general block locator.
//
//   Segments follow the reference's exact byte semantics (rijndael_cfb_encrypt's
//   (ivec, pos) carry): a stream segment that starts at CFB position n0 != 0 first
//   consumes the keystream bytes ivec[n0..15]; block alignment is relative to the
//   stream, not to memory; partial final blocks leave (ivec, pos) exactly as the
//   reference's byte loop does.  Package mode is the special case n0 = 0,
//   ivec = connection IV, state discarded (core/Encryptor.cpp:10-32).
#pragma once

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
        const uint64_t io = b.in_off ? *FA_AT(b, AB_IN_OFF, b.in_off + s, 8) : s * b.stride;
        const uint64_t oo = b.out_off ? *FA_AT(b, AB_OUT_OFF, b.out_off + s, 8) : io;
        g.in = b.in + io;
        g.out = b.out + oo;
        g.len = b.len ? *FA_AT(b, AB_LEN, b.len + s, 4) : b.uniform_len;
        g.slot = b.key_slot ? *FA_AT(b, AB_SLOT, b.key_slot + s, 4) : 0u;
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
    uint4 d;
    if (g.len >= 16) {
        // An edge block of a segment of 16+ bytes: one 16-byte load that stays inside the
        // segment, shifted into place -- the head block (lo = n0 > 0, hi = 16) holds
        // segment bytes [0, 16 - lo) at positions lo.., the tail block (lo = 0) the
        // segment's last hi bytes at 0..hi-1 -- instead of up to sixteen byte loads.
        d = lo != 0 ? shl_bytes(load16(g.in), lo) : shr_bytes(load16(g.in + g.len - 16), 16 - hi);
    } else {
        d = load_bytes(base, lo, hi);
    }
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

// segment and block-in-segment of virtual block gblk of a uniform layout (clamped into
// the batch for lanes past its end)
template <int LAYOUT>
__device__ __forceinline__ void locate_block(const KBatch &b, uint64_t c, uint64_t gblk, uint64_t total, uint64_t &s,
                                             uint32_t &bi) {
    static_assert(LAYOUT != LAYOUT_GENERAL, "general layouts are located by K1r's window");
    (void)c;
    const uint32_t g32 = (uint32_t)(gblk < total ? gblk : total - 1);
    const uint32_t q = fast_div(g32, b.magic);
    s = q;
    bi = g32 - q * b.nb_uniform;
}

__device__ __forceinline__ uint4 readlane63(const uint4 &v) {
    return make_uint4(__builtin_amdgcn_readlane(v.x, 63), __builtin_amdgcn_readlane(v.y, 63),
                      __builtin_amdgcn_readlane(v.z, 63), __builtin_amdgcn_readlane(v.w, 63));
}

inline int grid_for(uint64_t items, int threads, int cap) {
    uint64_t g = (items + threads - 1) / threads;
    if (g < 1) g = 1;
    return (int)(g > (uint64_t)cap ? cap : g);
}

// The last workgroup of a kernel that reads the length-order block (kernels.hpp) returns it
// to zeros for the next call.  Every workgroup calls this at its very end, all threads.
__device__ __forceinline__ void length_order_release(uint32_t *block) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&block[kDoneWord], 1u) == gridDim.x - 1) {
            for (int i = 0; i < kLengthOrderWords; i++) block[i] = 0u;
            __threadfence();
        }
    }
}

}  // namespace fpnn_aes
