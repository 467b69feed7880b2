// bs_kernels.hip -- bitsliced CFB kernels (VALU only, no LDS).  They run beside the
// LDS-bound T-table kernels on a second stream, over a share of the batch.
//
//   K1b k_bs_cfb_decrypt: CFB-128 decryption of uniform package batches whose packets
//       are a multiple of 32 blocks.  One lane = 32 consecutive blocks of one packet:
//       keystream inputs X_j = C_{j-1} (X_0 = C_{-1} or the IV), transposed into the
//       bitsliced state, encrypted (bs_aes.hpp), transposed back, P_j = C_j ^ KS_j
//       (base/rijndael.c:1189-1197, core/Encryptor.cpp:10-20).
#include "aes_device.hpp"
#include "bs_aes.hpp"
#include "kernels.hpp"

namespace fpnn_aes {

template <int NR>
__global__ __launch_bounds__(256, 1) void k_bs_cfb_decrypt(KBatch b, uint64_t first_pkt, uint32_t groups_per_pkt,
                                                           uint64_t ngroups) {
    const uint32_t *rk = b.keys->rk;  // uniform: scalar loads
    const uint4 iv = *reinterpret_cast<const uint4 *>(b.keys->iv);
    const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += nthreads) {
        const uint64_t s = first_pkt + g / groups_per_pkt;
        const uint32_t q = (uint32_t)(g % groups_per_pkt);
        const uint8_t *in = b.in + s * b.stride + 512ull * q;
        uint8_t *out = b.out + s * b.stride + 512ull * q;
        uint32_t S[128];
        const uint4 x0 = q == 0 ? iv : load16(in - 16);
        S[0] = x0.x;
        S[32] = x0.y;
        S[64] = x0.z;
        S[96] = x0.w;
#pragma unroll
        for (int j = 1; j < 32; j++) {
            const uint4 c = load16(in + 16 * (j - 1));
            S[j] = c.x;
            S[32 + j] = c.y;
            S[64 + j] = c.z;
            S[96 + j] = c.w;
        }
#pragma unroll
        for (int d = 0; d < 4; d++) bs_transpose32(S + 32 * d);
        bs_aes_encrypt<NR>(S, rk);
#pragma unroll
        for (int d = 0; d < 4; d++) bs_transpose32(S + 32 * d);
#pragma unroll
        for (int j = 0; j < 32; j++) {
            const uint4 c = load16(in + 16 * j);
            store16(out + 16 * j, make_uint4(c.x ^ S[j], c.y ^ S[32 + j], c.z ^ S[64 + j], c.w ^ S[96 + j]));
        }
    }
}

hipError_t launch_bs_decrypt(const KBatch &b, int nrounds, uint64_t first_pkt, uint64_t npkt,
                             uint32_t groups_per_pkt, int grid, hipStream_t st) {
    const uint64_t ngroups = npkt * groups_per_pkt;
    if (!ngroups) return hipSuccess;
    switch (nrounds) {
        case 10:
            hipLaunchKernelGGL(k_bs_cfb_decrypt<10>, dim3(grid), dim3(256), 0, st, b, first_pkt, groups_per_pkt, ngroups);
            break;
        case 12:
            hipLaunchKernelGGL(k_bs_cfb_decrypt<12>, dim3(grid), dim3(256), 0, st, b, first_pkt, groups_per_pkt, ngroups);
            break;
        case 14:
            hipLaunchKernelGGL(k_bs_cfb_decrypt<14>, dim3(grid), dim3(256), 0, st, b, first_pkt, groups_per_pkt, ngroups);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
