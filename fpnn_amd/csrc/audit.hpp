// audit.hpp -- the address-audit build of the GPU library (`make audit` ->
// fpnn_amd/libfpnn_aes_gpu_audit.so, compiled with -DFPNN_AES_BOUNDS).
//
// Every global load and store of K2h (k_hybrid.hip), K2's ragged path (k_encrypt.hip) and
// the length-order kernels (k_support.hip) names the buffer it indexes through FA_AT /
// FA_SEG / FA_RG.  In the audit build each one checks its byte range against an extent:
//   * the array extents the host supplies per call (AuditTable::lo/hi: descriptor arrays of
//     `count` entries, the key set's slots, perm[] of `count` entries, the wave sinks, the
//     length-order block, the stream state arrays, and the union of the segments' payload);
//   * for payload bytes, the CURRENT SEGMENT's own range as well (in_off[s] .. + len[s], out
//     off[s] .. + len[s] (+ 4 wire prefix bytes)), so a store into a neighbour frame is caught
//     as surely as one past the allocation.
// A violating access is redirected into the table's scratch bytes and the first one is
// recorded (source line, buffer, workgroup, thread, address, extent); the engine reports it
// as FPNN_AES_ERR_DEVICE with the record in fpnn_aes_last_error().  In the product build the
// macros are the bare pointer expressions: the kernels compile exactly as without them.
#pragma once

#include <stdint.h>

namespace fpnn_aes {

enum AuditBuf : uint32_t {
    AB_IN = 0,     // payload read (batch union extent)
    AB_OUT,        // payload written (batch union extent)
    AB_IN_OFF,     // descriptor arrays, `count` entries each
    AB_OUT_OFF,
    AB_LEN,
    AB_SLOT,
    AB_KEYS,       // DevKey table (slots of the key set)
    AB_EIV,        // E_k(IV) per slot
    AB_IV_STATE,   // stream (iv, pos) per segment
    AB_POS_STATE,
    AB_PERM,       // length order, `count` entries
    AB_SINK,       // K2h: 2 x uint4 per wave
    AB_BLOCK,      // the length-order block (kLengthOrderWords)
    AB_POS_SNAP,   // pos snapshot read by the bucket kernels
    AB_SEG_IN,     // payload read outside the current segment
    AB_SEG_OUT,    // payload written outside the current segment (+ wire prefix)
    kAuditBufs
};

struct AuditTable {
    uint64_t lo[kAuditBufs], hi[kAuditBufs];  // [lo, hi) per buffer; hi == 0: not checked
    uint32_t hits;                            // violations seen
    uint32_t site, buf, block, thread, pad;   // the first one
    uint64_t addr, len, elo, ehi;             // its bytes and the extent they left
    alignas(16) uint8_t scratch[64];          // where violating accesses go instead
};

#if defined(FPNN_AES_BOUNDS) && defined(__HIP_DEVICE_COMPILE__)

// Out of line, and as few arguments as the record needs: the checks run at every access of
// kernels that already hold 128 VGPRs, so each extra live value is a spill.  (Recording the
// segment's index and bounds as well, inlined or as extra arguments, doubled the audit
// kernels' scratch and made some of them compute wrong results -- r06c/r06d)
__device__ __noinline__ void audit_record(AuditTable *a, uint32_t buf, uint64_t x, uint64_t n, uint64_t lo, uint64_t hi,
                                          uint32_t site) {
    if (atomicAdd(&a->hits, 1u) == 0u) {
        a->site = site;
        a->buf = buf;
        a->block = blockIdx.x;
        a->thread = threadIdx.x;
        a->addr = x;
        a->len = n;
        a->elo = lo;
        a->ehi = hi;
        __threadfence();
    }
}

// [x, x + n) inside [lo, hi) (no wrap: x near 2^64 must not pass)
__device__ __forceinline__ bool audit_ok(AuditTable *a, uint32_t buf, uint64_t x, uint64_t n, uint64_t lo, uint64_t hi,
                                         uint32_t site) {
    if (!a || n == 0 || hi == 0 || (x >= lo && x < hi && n <= hi - x)) return true;
    audit_record(a, buf, x, n, lo, hi, site);
    return false;
}

// p .. p + n against the buffer's array extent
template <class T>
__device__ __forceinline__ T *audit_at(AuditTable *a, uint32_t buf, T *p, uint64_t n, uint32_t site) {
    if (!a) return p;
    const uint64_t x = (uint64_t)(uintptr_t)p;
    return audit_ok(a, buf, x, n, a->lo[buf], a->hi[buf], site) ? p : reinterpret_cast<T *>(a->scratch);
}

// p .. p + n against the batch union AND the current segment [slo, shi)
template <class T>
__device__ __forceinline__ T *audit_seg(AuditTable *a, uint32_t buf, T *p, uint64_t n, uint64_t slo, uint64_t shi,
                                        uint32_t site) {
    if (!a) return p;
    const uint64_t x = (uint64_t)(uintptr_t)p;
    if (!audit_ok(a, buf, x, n, a->lo[buf], a->hi[buf], site)) return reinterpret_cast<T *>(a->scratch);
    return audit_ok(a, buf == AB_IN ? AB_SEG_IN : AB_SEG_OUT, x, n, slo, shi, site) ? p
                                                                                      : reinterpret_cast<T *>(a->scratch);
}

// the bytes [lo, hi) of base (the helpers store_bytes / load_bytes / *_word_bytes touch
// exactly those) against the batch union and the current segment; a violation returns a
// base whose [lo, hi) lies in the scratch bytes
template <class T>
__device__ __forceinline__ T *audit_rg(AuditTable *a, uint32_t buf, T *base, int lo, int hi, uint64_t slo, uint64_t shi,
                                       uint32_t site) {
    if (!a || lo >= hi) return base;
    const uint64_t x = (uint64_t)(uintptr_t)base + (uint64_t)(int64_t)lo;
    const uint64_t n = (uint64_t)(hi - lo);
    if (audit_ok(a, buf, x, n, a->lo[buf], a->hi[buf], site) &&
        audit_ok(a, buf == AB_IN ? AB_SEG_IN : AB_SEG_OUT, x, n, slo, shi, site))
        return base;
    return reinterpret_cast<T *>(a->scratch + 16 - lo);
}

#define FA_AT(B, BUF, P, N) (::fpnn_aes::audit_at((B).aud, (BUF), (P), (uint64_t)(N), __LINE__))
#define FA_SEG(B, BUF, P, N, SLO, SHI) (::fpnn_aes::audit_seg((B).aud, (BUF), (P), (uint64_t)(N), (SLO), (SHI), __LINE__))
#define FA_RG(B, BUF, BASE, LO, HI, SLO, SHI) \
    (::fpnn_aes::audit_rg((B).aud, (BUF), (BASE), (int)(LO), (int)(HI), (SLO), (SHI), __LINE__))
// per-lane segment extents, declared and set only in the audit build (FA_ARGS passes two of
// them to a helper)
#define FA_DECL(...) uint64_t __VA_ARGS__
#define FA_SET(X, V) ((X) = (uint64_t)(V))
#define FA_ARGS(...) __VA_ARGS__
#define FA_ON 1

#else

#define FA_AT(B, BUF, P, N) (P)
#define FA_SEG(B, BUF, P, N, SLO, SHI) (P)
#define FA_RG(B, BUF, BASE, LO, HI, SLO, SHI) (BASE)
#define FA_DECL(...)
#define FA_SET(X, V) ((void)0)
#define FA_ARGS(...) 0, 0  // (extent arguments of helpers: unused in the product build)
#define FA_ON 0

#endif

}  // namespace fpnn_aes
