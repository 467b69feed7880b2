// k_small.hip -- K0, the small single-call CFB kernel behind the synchronous drop-in
// (PackageEncryptor / StreamEncryptor per call, rijndael_cfb_encrypt; core/Encryptor.cpp:10-70,
// base/rijndael.c:1171-1201) for calls of up to kSmallMaxBytes.
//
// One call = one CFB byte stream with the reference's (ivec, *p_num) carry.  The batch
// kernels pay for throughput machinery a single frame never uses: K2c fills the 128 KiB
// replicated LDS image with 64 threads (128 dependent rounds of a global load each), K1r
// launches a block map, a descriptor pass and a 256-workgroup grid for 64 blocks, and the
// call moves its bytes with three DMA copies and waits with the blocking stream sync.  K0
// is one launch of one 256-thread workgroup:
//   * the table image is filled from registers: thread x loads T0[x] once and writes its
//     entry's copies (encrypt: copies 0..3 only, the chain's quad reads nothing else);
//   * the call's bytes are read from and written back to the engine's pinned staging
//     directly over PCIe (one coalesced burst each way through an LDS buffer);
//   * completion is a sequence number the kernel stores to pinned memory after its
//     results (system-scope release); the host spins on it instead of sleeping in
//     hipStreamSynchronize.
// Decrypt: one lane per 16-byte block (block i's keystream is E(C_{i-1})).  Encrypt: the
// serial chain on one quad (K2c's column round, coop.hpp) -- C_i = P_i ^ E(C_{i-1}).
#include "coop.hpp"
#include "kernels.hpp"

namespace fpnn_aes {

namespace {

constexpr int kSmallThreads = 256;

__device__ __forceinline__ void store_seq(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LDS image: copies [0, ncopies) of every (table, x) entry (the layout of aes_device.hpp)
template <int NT>
__device__ __forceinline__ void fill_tables_regs(uint4 *lds4, const uint32_t *__restrict__ t0le, int ncopies) {
    const uint32_t x = threadIdx.x;  // kSmallThreads == 256 entries
    const uint32_t v0 = t0le[x];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t v = rotl32(v0, 8u * k);
        const uint32_t r = k >> 1, h = k & 1;
        uint4 *row = lds4 + ((r * 65536u + x * 256u + h * 128u) >> 4);  // 32 copies = 8 uint4
        for (int c = 0; c < ncopies; c += 4) row[c >> 2] = make_uint4(v, v, v, v);
    }
}

template <int NR, bool ENCRYPT>
__global__ __launch_bounds__(kSmallThreads, 1) void k_cfb_single(SmallArgs a) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    __shared__ uint4 buf[kSmallMaxBytes / 16 + 2];  // head block + body + one spare (prefetch)
    __shared__ uint32_t fhead[4], fout[4];  // feedback register after the head / after the call
    const uint32_t t = threadIdx.x;
    // the call's bytes: the body starts at io + kSmallBodyAt (16-aligned), the head's
    // bytes (pos != 0: the rest of the current keystream block) sit right before it
    const uint32_t rem = a.len - a.head, r = rem & 15u;
    const uint32_t nb = (rem + 15) >> 4;  // body blocks, the last one partial when r != 0
    uint4 *io = reinterpret_cast<uint4 *>(a.io + kSmallBodyAt - 16);
    // first PCIe read in flight before the table fill (both wait on memory, not on each other)
    const uint4 first = t <= nb ? io[t] : make_uint4(0, 0, 0, 0);
    fill_tables_regs<4>(lds4, a.t0le, ENCRYPT ? 4 : 32);
    if (t <= nb) buf[t] = first;  // buf[0]: the head bytes at its end
    for (uint32_t i = t + kSmallThreads; i <= nb; i += kSmallThreads) buf[i] = io[i];
    __syncthreads();
    if (t == 0) {  // head: ivec bytes [pos, pos + head) are keystream already (base/rijndael.c:1180-1195)
        uint8_t *fb = reinterpret_cast<uint8_t *>(fhead);
        *reinterpret_cast<uint4 *>(fhead) = a.iv;
        uint8_t *hb = reinterpret_cast<uint8_t *>(&buf[0]) + 16 - a.head;
        for (uint32_t j = 0; j < a.head; j++) {
            const uint8_t c = hb[j];
            const uint8_t o = c ^ fb[a.pos + j];
            hb[j] = o;
            fb[a.pos + j] = ENCRYPT ? o : c;  // the feedback is always the ciphertext byte
        }
        *reinterpret_cast<uint4 *>(fout) = *reinterpret_cast<const uint4 *>(fhead);  // nb == 0
    }
    __syncthreads();
    const uint4 f0 = *reinterpret_cast<const uint4 *>(fhead);
    if (ENCRYPT) {
        if (t < 4) {  // the chain on one quad: lane q owns column q (coop.hpp)
            const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
            uint32_t rkq[NR + 1];
#pragma unroll
            for (int k = 0; k <= NR; k++) rkq[k] = a.rk[4 * k + t];
            uint32_t fq = word_of(f0, (int)t);
            uint32_t *bw = reinterpret_cast<uint32_t *>(buf + 1);
            uint32_t pw = nb ? bw[t] : 0u;  // P_i, loaded one block ahead of its use
            for (uint32_t i = 0; i < nb; i++) {
                const uint32_t p = pw;
                pw = bw[4 * (i + 1) + t];  // (buf has one spare block past the body)
                const uint32_t k = aes_encrypt_column<NR, 4>(fq, rkq, T);
                const uint32_t c = k ^ p;
                bw[4 * i + t] = c;
                if (i + 1 < nb || r == 0) {
                    fq = c;
                } else {  // partial last block: ivec = C bytes [0, r) + keystream bytes [r, 16)
                    const int lo = (int)r - 4 * (int)t;
                    const uint32_t m = lo >= 4 ? 0xffffffffu : lo <= 0 ? 0u : (0xffffffffu >> (8 * (4 - lo)));
                    fq = (c & m) | (k & ~m);
                }
            }
            if (nb) fout[t] = fq;
        }
        __syncthreads();
        for (uint32_t i = t; i <= nb; i += kSmallThreads) io[i] = buf[i];
    } else {  // one lane per block; plaintext straight back to the staging
        const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
        const RoundKeys<NR> rk = *reinterpret_cast<const RoundKeys<NR> *>(a.rk);
        for (uint32_t i = t; i < nb; i += kSmallThreads) {
            const uint4 k = aes_encrypt_block<NR, 4>(i ? buf[i] : f0, rk, T);  // buf[i] = C_{i-1}
            const uint4 c = buf[i + 1];
            io[i + 1] = c ^ k;
            if (i + 1 == nb)  // ivec after the call: the last C block, or C bytes [0, r) + K
                *reinterpret_cast<uint4 *>(fout) = r ? select_bytes(byte_mask(0, (int)r), c, k) : c;
        }
        __syncthreads();
        if (t == 0) io[0] = buf[0];
    }
    if (t == 0) {
        uint32_t *st = a.state;
        st[0] = fout[0];
        st[1] = fout[1];
        st[2] = fout[2];
        st[3] = fout[3];
        st[4] = nb ? r : (a.pos + a.head) & 15u;
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) store_seq(a.state + 5, a.seq);
}

}  // namespace

hipError_t launch_cfb_single(const SmallArgs &a, int nrounds, bool encrypt, hipStream_t st) {
    set_launched(encrypt ? "cfb_single_encrypt" : "cfb_single_decrypt");
#define FPNN_K0(NR)                                                                                                  \
    do {                                                                                                             \
        if (encrypt) hipLaunchKernelGGL((k_cfb_single<NR, true>), dim3(1), dim3(kSmallThreads), 0, st, a);           \
        else hipLaunchKernelGGL((k_cfb_single<NR, false>), dim3(1), dim3(kSmallThreads), 0, st, a);                  \
    } while (0)
    switch (nrounds) {
        case 10: FPNN_K0(10); break;
        case 12: FPNN_K0(12); break;
        case 14: FPNN_K0(14); break;
        default: return hipErrorInvalidValue;
    }
#undef FPNN_K0
    return hipGetLastError();
}

}  // namespace fpnn_aes
