// framing.hip -- wire framing of received bytes on the device.
//
// Package mode (core/EncryptedPackageReceiver.cpp:60-118): the bytes received on a
// connection are [htole32(n)][n bytes CFB ciphertext] frames; the length prefix is
// plaintext and n above Config::_max_recv_package_length closes the connection.
// Stream mode (core/EncryptedStreamReceiver.cpp:8-15,72-111 with
// proto/FPMessage.cpp:27-44): the decrypted stream is a sequence of FPNN messages,
// a 12-byte header {magic "FPNN", version, flag, mtype, ss, psize (LE)} followed by
// BodyLen(header) bytes.
//
// Walking a segment (a connection's received bytes) is a chain of dependent header
// reads: latency work, not bandwidth -- the payload bytes are never read here.  Each
// hop loads its whole header with one round of aligned dword loads.  Two kernels:
//   * k_scan_lane: one lane per segment, for batches of many (short) segments;
//   * k_scan_wave: one wavefront per segment, for few long segments.  The wave guesses
//     that the next frames have the length of the last one and reads up to 64 headers
//     at once (lane j at pos + j * guess); the guess holds up to the first lane whose
//     frame differs, and that lane's header is still correctly placed, so every round
//     trip advances at least one frame and a run of equal-length frames costs one
//     round trip per 64.  The number of reading lanes grows eightfold while guesses
//     hold (1, 2, 16, 64: 64 equal frames in 4 round trips, where doubling took 7 --
//     R1's scan 41 µs per call) and drops to 2 when the first guess fails, so ragged
//     streams do not pay 64 loads per frame.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "kernels.hpp"

namespace fpnn_aes {

namespace {

enum : uint32_t { V_ACCEPT = 0xffffffffu };  // otherwise: the walk's final status (SCAN_OK = incomplete)

// bytes h[0, 4W) as W little-endian words; aligned dword loads, none of them of a word
// that holds no byte of the range (so never past the segment, never across a page)
template <int W>
__device__ __forceinline__ void load_words(const uint8_t *h, uint32_t (&w)[W]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(h);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t d[W + 1];
#pragma unroll
    for (int k = 0; k < W; k++) d[k] = q[k];
    d[W] = sh ? q[W] : 0u;
#pragma unroll
    for (int k = 0; k < W; k++) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// package frame at byte pos of a segment of n bytes, reference recvPackage: prefix
// (:62-76), `len > max` (:77-81), body complete
__device__ __forceinline__ uint32_t package_frame(const uint8_t *p, uint64_t pos, uint64_t n, uint32_t max_len,
                                                  uint64_t &flen) {
    if (pos > n || n - pos < 4) return SCAN_OK;
    uint32_t w[1];
    load_words<1>(p + pos, w);
    const uint32_t L = w[0];
    if (L > max_len) return SCAN_TOO_LARGE;
    if (n - pos - 4 < L) return SCAN_OK;
    flen = 4 + (uint64_t)L;
    return V_ACCEPT;
}

// FPNN message at byte pos of a plaintext region of n bytes, reference remainDataLen +
// recvPackage (core/EncryptedStreamReceiver.cpp:8-15, 87-110), FPMessage::isTCP and
// BodyLen (proto/FPMessage.cpp:27-44)
__device__ __forceinline__ uint32_t stream_message(const uint8_t *p, uint64_t pos, uint64_t n, uint32_t max_len,
                                                   uint64_t &flen) {
    if (pos > n || n - pos < 12) return SCAN_OK;  // header not complete
    uint32_t w[3];
    load_words<3>(p + pos, w);
    if (w[0] != 0x4E4E5046u) return SCAN_BAD_MAGIC;  // "FPNN"
    const uint32_t mtype = (w[1] >> 16) & 0xffu, ss = w[1] >> 24, psize = w[2];
    uint32_t body;  // uint32 arithmetic, as BodyLen
    if (mtype == 1)
        body = psize + ss + 4u;  // FP_MT_TWOWAY: + method name + seq
    else if (mtype == 2)
        body = psize + 4u;  // FP_MT_ANSWER: + seq
    else if (mtype == 0)
        body = psize + ss;  // FP_MT_ONEWAY: + method name
    else
        return SCAN_BAD_MTYPE;  // BodyLen throws FPNN_EC_PROTO_METHOD_TYPE
    // remainDataLen(): (int)(sizeof(Header) + BodyLen) - _curr with _curr == 12
    const int64_t length = (int64_t)(int32_t)(uint32_t)(12u + body) - 12;
    if (length <= 0) return SCAN_BAD_LENGTH;  // "Not available FPNN-TCP-Message"
    if (12 + length > (int64_t)max_len) return SCAN_TOO_LARGE;  // _total + length > max
    flen = 12 + (uint64_t)length;
    if (n - pos < flen) return SCAN_OK;  // message not complete
    return V_ACCEPT;
}

struct SegView {
    const uint8_t *p;  // package: segment bytes; stream: region (carry included)
    uint64_t base, n;
    uint32_t slot;
};

template <bool STREAM>
__device__ __forceinline__ SegView seg_view(const KScan &s, uint64_t i) {
    SegView v;
    v.base = s.off ? s.off[i] : i * s.stride;
    const uint64_t len = s.len ? s.len[i] : s.uniform_len;
    if (STREAM) {
        const uint64_t carry = s.carry ? s.carry[i] : 0u;
        v.n = len + carry;
        v.p = s.buf + v.base - carry;
        v.slot = 0;
    } else {
        v.n = len;
        v.p = s.buf + v.base;
        v.slot = s.key_slot ? s.key_slot[i] : 0u;
    }
    return v;
}

template <bool STREAM>
__device__ __forceinline__ uint32_t frame_at(const SegView &g, uint64_t pos, uint32_t max_len, uint64_t &flen) {
    return STREAM ? stream_message(g.p, pos, g.n, max_len, flen) : package_frame(g.p, pos, g.n, max_len, flen);
}

// frame slot k: the frame of flen bytes at pos (package: its body, for the decrypt batch)
template <bool STREAM>
__device__ __forceinline__ void emit(const KScan &s, const SegView &g, uint64_t k, uint64_t pos, uint64_t flen) {
    if (STREAM) {
        s.frame_off[k] = pos;
        s.frame_len[k] = (uint32_t)flen;
    } else {
        s.frame_off[k] = pos + 4;
        s.frame_len[k] = (uint32_t)(flen - 4);
        s.abs_off[k] = g.base + pos + 4;
        if (s.abs_slot) s.abs_slot[k] = g.slot;
    }
}

// unused frame slot k: decrypts nothing
template <bool STREAM>
__device__ __forceinline__ void emit_unused(const KScan &s, const SegView &g, uint64_t k) {
    s.frame_len[k] = 0;
    if (!STREAM) {
        s.abs_off[k] = g.base;
        if (s.abs_slot) s.abs_slot[k] = g.slot;
    }
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_scan_lane(KScan s) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < s.count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const SegView g = seg_view<STREAM>(s, i);
        const uint64_t k0 = i * s.max_frames;
        uint64_t pos = 0;
        uint32_t f = 0, status = SCAN_OK;
        for (;;) {
            uint64_t flen = 0;
            const uint32_t v = frame_at<STREAM>(g, pos, s.max_len, flen);
            if (v != V_ACCEPT) {
                status = v;
                break;
            }
            if (f == s.max_frames) {
                status = SCAN_FULL;
                break;
            }
            emit<STREAM>(s, g, k0 + f, pos, flen);
            f++;
            pos += flen;
        }
        for (uint32_t j = f; j < s.max_frames; j++) emit_unused<STREAM>(s, g, k0 + j);
        s.scan[i] = ScanResult{f, status, pos};
    }
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t l) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
    return ((uint64_t)hi << 32) | lo;
}

template <bool STREAM>
__global__ __launch_bounds__(256) void k_scan_wave(KScan s) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(blockIdx.x * 4u + (threadIdx.x >> 6)));
    for (uint64_t i = w0; i < s.count; i += (uint64_t)gridDim.x * 4) {
        const SegView g = seg_view<STREAM>(s, i);
        const uint64_t mf = s.max_frames, k0 = i * mf;
        uint64_t pos = 0, guess = 0, f = 0;
        uint32_t width = 1, status = SCAN_OK;  // lanes [0, width) read a header this round
        for (;;) {
            const uint64_t pj = pos + lane * guess;
            uint64_t flen = 0;
            uint32_t v = lane < width ? frame_at<STREAM>(g, pj, s.max_len, flen) : SCAN_OK;
            if (v == V_ACCEPT && f + lane >= mf) v = SCAN_FULL;
            const uint64_t brk = __builtin_amdgcn_ballot_w64(!(v == V_ACCEPT && flen == guess));
            const uint32_t jb = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;  // lanes < jb: guessed right
            if (lane < jb || (lane == jb && v == V_ACCEPT)) emit<STREAM>(s, g, k0 + f + lane, pj, flen);
            if (jb >= width) {  // every reading lane guessed right
                f += width;
                pos += width * guess;
                width = width < 8 ? 8 * width : 64;
                continue;
            }
            const uint32_t vb = (uint32_t)__builtin_amdgcn_readlane(v, jb);
            const uint64_t pb = readlane_u64(pj, jb);
            if (vb != V_ACCEPT) {
                f += jb;
                pos = pb;
                status = vb;
                break;
            }
            const uint64_t fb = readlane_u64(flen, jb);
            f += jb + 1;
            pos = pb + fb;
            if (jb == 0) width = 2;  // the guess failed at once: keep one guessing lane
            guess = fb;
        }
        for (uint64_t j = f + lane; j < mf; j += 64) emit_unused<STREAM>(s, g, k0 + j);
        if (lane == 0) s.scan[i] = ScanResult{(uint32_t)f, status, pos};
    }
}

}  // namespace

hipError_t launch_scan_frames(const KScan &s, bool stream, int num_cus, hipStream_t st) {
    if (!s.count) return hipSuccess;
    // FPNN_AES_SCAN=lane|wave forces one walk (tests run the golden cases through both)
    const char *force = getenv("FPNN_AES_SCAN");
    const bool wave = force && force[0] ? force[0] == 'w' : s.count <= (uint64_t)num_cus * 64;
    if (wave) {  // few segments: a wavefront each
        const uint64_t want = (s.count + 3) / 4;
        const int grid = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
        if (stream)
            k_scan_wave<true><<<grid, 256, 0, st>>>(s);
        else
            k_scan_wave<false><<<grid, 256, 0, st>>>(s);
        return hipGetLastError();
    }
    const uint64_t want = (s.count + 255) / 256;
    const int grid = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
    if (stream)
        k_scan_lane<true><<<grid, 256, 0, st>>>(s);
    else
        k_scan_lane<false><<<grid, 256, 0, st>>>(s);
    return hipGetLastError();
}

}  // namespace fpnn_aes
