// k_modes.hip -- the rest of the rijndael.h surface on the GPU (base/rijndael.h:22-60):
// single-block / ECB encrypt and decrypt (base/rijndael.c:852-1068), CBC encrypt and
// decrypt (:1070-1153) and OFB (:1155-1169).  FPNN's own path only uses CFB; these exist
// so that a program linked against libfpnn_aes.so instead of rijndael.o finds every
// function the reference declares, with the reference's exact results.
//   ECB (both directions) and CBC decrypt are parallel: one lane per 16-byte block,
//   CBC decrypt takes C_{i-1} from the neighbouring lane (DPP) as the CFB decrypt does.
//   CBC encrypt and OFB are one serial chain per call (C_i = E(P_i ^ C_{i-1});
//   O_i = E(O_{i-1})): one lane runs it.
#include "segments.hpp"

namespace fpnn_aes {

template <int NR, int MODE>
__global__ __launch_bounds__(1024) void k_block_modes(ModeArgs a) {
    constexpr bool INV = MODE == MODE_ECB_DEC || MODE == MODE_CBC_DEC;
    __shared__ uint4 lds4[(Lds<4>::kBytes + (INV ? kIsboxBytes : 0)) / 16];
    lds_fill_tables<4>(lds4, INV ? a.td0le : a.t0le);
    if (INV) lds_fill_isbox(reinterpret_cast<uint32_t *>(lds4), a.isbox);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const RoundKeys<NR> rk = load_round_keys<NR>(a.key);
    const uint32_t lane = threadIdx.x & 63u;

    if (MODE == MODE_ECB_ENC || MODE == MODE_ECB_DEC || MODE == MODE_CBC_DEC) {
        const uint4 iv = *reinterpret_cast<const uint4 *>(a.iv);
        const uint64_t nthreads = (uint64_t)gridDim.x * blockDim.x;
        // every lane of a wave runs the loop the same number of times (DPP needs them all)
        for (uint64_t base = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~63ull; base < a.nblocks;
             base += nthreads) {
            const uint64_t i = base + lane;
            const bool valid = i < a.nblocks;
            const uint4 x = valid ? load16(a.in + 16 * i) : make_uint4(0, 0, 0, 0);
            uint4 y = MODE == MODE_ECB_ENC ? aes_encrypt_block<NR, 4>(x, rk, T) : aes_decrypt_block<NR, 4>(x, rk, T);
            if (MODE == MODE_CBC_DEC) {  // P_i = D(C_i) ^ C_{i-1}, C_{-1} = ivec
                uint4 prev = wave_shr1(x);
                if (lane == 0) prev = i == 0 ? iv : load16(a.in + 16 * (i - 1));
                y = y ^ prev;
            }
            if (valid) store16(a.out + 16 * i, y);
        }
        return;
    }
    if (threadIdx.x != 0 || blockIdx.x != 0) return;  // serial chains: one lane
    uint4 v = *reinterpret_cast<const uint4 *>(a.iv);
    if (MODE == MODE_CBC_ENC) {  // the host zero-pads the last partial block (0 ^ iv == iv)
        for (uint64_t i = 0; i < a.nblocks; i++) {
            v = aes_encrypt_block<NR, 4>(load16(a.in + 16 * i) ^ v, rk, T);
            store16(a.out + 16 * i, v);
        }
        *reinterpret_cast<uint4 *>(a.iv) = v;
        return;
    }
    // OFB: keystream block E(ivec) whenever the position wraps to 0; out = in ^ ivec[n]
    uint32_t n = *a.pos;
    uint64_t k = 0, len = a.len;
    if (n != 0) {
        const uint64_t head = len < 16 - n ? len : 16 - n;
        store_bytes(a.out - n, load_bytes(a.in - n, (int)n, (int)(n + head)) ^ v, (int)n, (int)(n + head));
        k = head;
        n = (uint32_t)((n + head) & 15u);
    }
    for (; k + 16 <= len; k += 16) {
        v = aes_encrypt_block<NR, 4>(v, rk, T);
        store16(a.out + k, load16(a.in + k) ^ v);
    }
    if (k < len) {
        v = aes_encrypt_block<NR, 4>(v, rk, T);
        const int rem = (int)(len - k);
        store_bytes(a.out + k, load_bytes(a.in + k, 0, rem) ^ v, 0, rem);
        n = (uint32_t)rem;
    }
    *reinterpret_cast<uint4 *>(a.iv) = v;
    *a.pos = n;
}

template <int NR>
static void modes_nr(const ModeArgs &a, int mode, int grid, hipStream_t st) {
    switch (mode) {
        case MODE_ECB_ENC: hipLaunchKernelGGL((k_block_modes<NR, MODE_ECB_ENC>), dim3(grid), dim3(1024), 0, st, a); break;
        case MODE_ECB_DEC: hipLaunchKernelGGL((k_block_modes<NR, MODE_ECB_DEC>), dim3(grid), dim3(1024), 0, st, a); break;
        case MODE_CBC_DEC: hipLaunchKernelGGL((k_block_modes<NR, MODE_CBC_DEC>), dim3(grid), dim3(1024), 0, st, a); break;
        case MODE_CBC_ENC: hipLaunchKernelGGL((k_block_modes<NR, MODE_CBC_ENC>), dim3(1), dim3(1024), 0, st, a); break;
        default: hipLaunchKernelGGL((k_block_modes<NR, MODE_OFB>), dim3(1), dim3(1024), 0, st, a); break;
    }
}

hipError_t launch_block_modes(const ModeArgs &a, int nrounds, int mode, int num_cus, hipStream_t st) {
    const uint64_t want = (a.nblocks + 1023) / 1024;
    const int grid = (int)(want < (uint64_t)num_cus ? (want ? want : 1) : (uint64_t)num_cus);
    set_launched(mode == MODE_OFB ? "ofb" : mode == MODE_CBC_ENC ? "cbc_encrypt" : mode == MODE_CBC_DEC ? "cbc_decrypt"
                 : mode == MODE_ECB_DEC ? "ecb_decrypt" : "ecb_encrypt");
    switch (nrounds) {
        case 10: modes_nr<10>(a, mode, grid, st); break;
        case 12: modes_nr<12>(a, mode, grid, st); break;
        case 14: modes_nr<14>(a, mode, grid, st); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fpnn_aes
