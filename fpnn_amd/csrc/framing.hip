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
// One lane walks one segment (a connection's received bytes): the walk is a chain of
// dependent header reads, so this is latency work spread over many segments, not a
// bandwidth kernel; the payload bytes themselves are never read here.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace fpnn_aes {

namespace {

__device__ __forceinline__ uint32_t load_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ uint64_t seg_start(const KScan &s, uint64_t i) {
    return s.off ? s.off[i] : i * s.stride;
}

__device__ __forceinline__ uint32_t seg_len(const KScan &s, uint64_t i) {
    return s.len ? s.len[i] : s.uniform_len;
}

// Package wire frames, reference recvPackage: prefix (:62-76), `len > max` check (:77-81), body.
__global__ __launch_bounds__(256) void k_scan_package(KScan s) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < s.count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t base = seg_start(s, i);
        const uint64_t n = seg_len(s, i);
        const uint8_t *p = s.buf + base;
        const uint32_t slot = s.key_slot ? s.key_slot[i] : 0u;
        uint64_t pos = 0;
        uint32_t f = 0, status = SCAN_OK;
        for (;;) {
            if (n - pos < 4) break;  // prefix not complete
            const uint32_t L = load_le32(p + pos);
            if (L > s.max_len) {
                status = SCAN_TOO_LARGE;
                break;
            }
            if (n - pos - 4 < L) break;  // body not complete
            if (f == s.max_frames) {
                status = SCAN_FULL;
                break;
            }
            const uint64_t k = i * s.max_frames + f;
            s.frame_off[k] = pos + 4;
            s.frame_len[k] = L;
            s.abs_off[k] = base + pos + 4;
            if (s.abs_slot) s.abs_slot[k] = slot;
            f++;
            pos += 4 + (uint64_t)L;
        }
        for (uint32_t j = f; j < s.max_frames; j++) {  // unused slots decrypt nothing
            const uint64_t k = i * s.max_frames + j;
            s.frame_len[k] = 0;
            s.abs_off[k] = base;
            if (s.abs_slot) s.abs_slot[k] = slot;
        }
        s.scan[i] = ScanResult{f, status, pos};
    }
}

// FPNN messages in decrypted stream plaintext, reference remainDataLen + recvPackage
// (core/EncryptedStreamReceiver.cpp:8-15, 87-110) and FPMessage::BodyLen
// (proto/FPMessage.cpp:27-44).  The region of segment i starts carry[i] bytes before its
// data: the plaintext of the previous call's incomplete message, kept by the caller.
__global__ __launch_bounds__(256) void k_scan_stream(KScan s) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < s.count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t carry = s.carry ? s.carry[i] : 0u;
        const uint64_t n = seg_len(s, i) + carry;
        const uint8_t *p = s.buf + seg_start(s, i) - carry;
        uint64_t pos = 0;
        uint32_t f = 0, status = SCAN_OK;
        for (;;) {
            if (n - pos < 12) break;  // header not complete
            const uint8_t *h = p + pos;
            if (!(h[0] == 'F' && h[1] == 'P' && h[2] == 'N' && h[3] == 'N')) {  // FPMessage::isTCP
                status = SCAN_BAD_MAGIC;
                break;
            }
            const uint32_t mtype = h[6], ss = h[7], psize = load_le32(h + 8);
            uint32_t body;  // uint32 arithmetic, as BodyLen
            if (mtype == 1)
                body = psize + ss + 4u;  // FP_MT_TWOWAY: + method name + seq
            else if (mtype == 2)
                body = psize + 4u;  // FP_MT_ANSWER: + seq
            else if (mtype == 0)
                body = psize + ss;  // FP_MT_ONEWAY: + method name
            else {
                status = SCAN_BAD_MTYPE;  // BodyLen throws FPNN_EC_PROTO_METHOD_TYPE
                break;
            }
            // remainDataLen(): (int)(sizeof(Header) + BodyLen) - _curr with _curr == 12
            const int64_t length = (int64_t)(int32_t)(uint32_t)(12u + body) - 12;
            if (length <= 0) {
                status = SCAN_BAD_LENGTH;  // "Not available FPNN-TCP-Message"
                break;
            }
            if (12 + length > (int64_t)s.max_len) {  // _total + length > _max_recv_package_length
                status = SCAN_TOO_LARGE;
                break;
            }
            const uint64_t flen = 12 + (uint64_t)length;
            if (n - pos < flen) break;  // message not complete
            if (f == s.max_frames) {
                status = SCAN_FULL;
                break;
            }
            const uint64_t k = i * s.max_frames + f;
            s.frame_off[k] = pos;
            s.frame_len[k] = (uint32_t)flen;
            f++;
            pos += flen;
        }
        for (uint32_t j = f; j < s.max_frames; j++) s.frame_len[i * s.max_frames + j] = 0;
        s.scan[i] = ScanResult{f, status, pos};
    }
}

}  // namespace

hipError_t launch_scan_frames(const KScan &s, bool stream, int num_cus, hipStream_t st) {
    if (!s.count) return hipSuccess;
    const uint64_t want = (s.count + 255) / 256;
    const int grid = (int)(want < (uint64_t)num_cus * 8 ? want : (uint64_t)num_cus * 8);
    if (stream)
        k_scan_stream<<<grid, 256, 0, st>>>(s);
    else
        k_scan_package<<<grid, 256, 0, st>>>(s);
    return hipGetLastError();
}

}  // namespace fpnn_aes
