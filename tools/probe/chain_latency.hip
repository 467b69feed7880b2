// Latency breakdown of one serial CFB chain round on gfx950 (what sets
// C3's whole-stream encrypt, K2c, one quad per chain).  One wave per CU, s_memtime stamps
// around N dependent repetitions; each lane writes cycles/repetition.  Kernels:
//   lds_chase   idx = lds[idx]                    (dependent ds_read_b32 round trip)
//   valu_chain  x = x ^ rotl(x, 7)                (dependent full-rate VALU, 2 instructions)
//   dpp_chain   x = x ^ dpp_quad_rot(x)           (dependent DPP-sourced XOR)
//   k2c_round   s = aes_encrypt_column(s)         (K2c's round: 4 v_perm + 4 ds_read + 4 VALU)
//   k2_round    16-lookup lane-per-chain round     (K2's round, one chain per lane)
//   hipcc -O3 --offload-arch=gfx950 -I fpnn_amd/csrc tools/probe/chain_latency.hip -o tools/probe/chain_latency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "coop.hpp"

using namespace fpnn_aes;

constexpr int kIters = 4096;

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

__global__ __launch_bounds__(64) void k_lds_chase(uint32_t *out, uint32_t seed) {
    __shared__ uint32_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (i * 2654435761u + seed) & 4095u;
    __syncthreads();
    uint32_t idx = threadIdx.x;
    const uint64_t t0 = stamp();
    for (int i = 0; i < kIters; i++) idx = lds[idx];
    const uint64_t t1 = stamp();
    out[threadIdx.x] = (uint32_t)(t1 - t0);
    out[64 + threadIdx.x] = idx;
}

__global__ __launch_bounds__(64) void k_valu_chain(uint32_t *out, uint32_t seed) {
    uint32_t x = seed + threadIdx.x;
    const uint64_t t0 = stamp();
    for (int i = 0; i < kIters; i++) {
        x = x ^ __builtin_rotateleft32(x, 7);
        __builtin_amdgcn_sched_barrier(0);
    }
    const uint64_t t1 = stamp();
    out[threadIdx.x] = (uint32_t)(t1 - t0);
    out[64 + threadIdx.x] = x;
}

__global__ __launch_bounds__(64) void k_dpp_chain(uint32_t *out, uint32_t seed) {
    uint32_t x = seed + threadIdx.x;
    const uint64_t t0 = stamp();
    for (int i = 0; i < kIters; i++) x = x ^ quad_from<1>(x);
    const uint64_t t1 = stamp();
    out[threadIdx.x] = (uint32_t)(t1 - t0);
    out[64 + threadIdx.x] = x;
}

// Issue throughput (8 independent chains per lane) of the ECDH kernel's multiply forms,
// with W waves per SIMD (workgroup of 4*W waves: the CU deals waves to SIMDs round-robin).
__global__ __launch_bounds__(1024) void k_mad64_tput(uint32_t *out, uint32_t seed, int iters) {
    uint64_t acc[8];
    uint32_t a = seed + threadIdx.x, b = seed * 3u + 1u;
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = k;
    const uint64_t t0 = stamp();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = (uint64_t)(a + k) * b + acc[k];  // v_mad_u64_u32
    }
    const uint64_t t1 = stamp();
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) x ^= acc[k];
    if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)(t1 - t0);
    if (x == 42) out[64] = (uint32_t)x;
}

__global__ __launch_bounds__(1024) void k_fma64_tput(uint32_t *out, uint32_t seed, int iters) {
    double acc[8];
    const double a = 1.0 + 1e-9 * (seed + threadIdx.x), b = 0.999999;
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = k;
    const uint64_t t0 = stamp();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = __builtin_fma(acc[k], b, a);  // v_fma_f64
    }
    const uint64_t t1 = stamp();
    double x = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) x += acc[k];
    if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)(t1 - t0);
    if (x == 42.0) out[64] = 1;
}

__global__ __launch_bounds__(1024) void k_add32_tput(uint32_t *out, uint32_t seed, int iters) {
    uint32_t acc[8];
    const uint32_t a = seed + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = k;
    const uint64_t t0 = stamp();
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = (acc[k] ^ a) + k;  // bitop/add pairs
    }
    const uint64_t t1 = stamp();
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) x ^= acc[k];
    if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)(t1 - t0);
    if (x == 42) out[64] = x;
}

template <int NR>
__global__ __launch_bounds__(1024) void k_k2c_round(const uint32_t *t0le, const DevKey *key, uint32_t *out) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, t0le);
    __syncthreads();
    if (threadIdx.x >= 64) return;  // one wave: the chain's latency, nothing competing
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const int q = threadIdx.x & 3;
    uint32_t rkq[NR + 1];
#pragma unroll
    for (int r = 0; r <= NR; r++) rkq[r] = key->rk[4 * r + q];
    uint32_t s = threadIdx.x * 77u;
    const uint64_t t0 = stamp();
    for (int i = 0; i < kIters / NR; i++) s = aes_encrypt_column<NR, 4>(s, rkq, T);
    const uint64_t t1 = stamp();
    out[threadIdx.x] = (uint32_t)(t1 - t0);
    out[64 + threadIdx.x] = s;
}

template <int NR>
__global__ __launch_bounds__(1024) void k_k2_round(const uint32_t *t0le, const DevKey *key, uint32_t *out) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, t0le);
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const RoundKeys<NR> rk = load_round_keys<NR>(key);
    uint4 s = make_uint4(threadIdx.x, 1, 2, 3);
    const uint64_t t0 = stamp();
    for (int i = 0; i < kIters / NR; i++) s = aes_encrypt_block_fenced<NR, 4>(s, rk, T);
    const uint64_t t1 = stamp();
    out[threadIdx.x] = (uint32_t)(t1 - t0);
    out[64 + threadIdx.x] = s.x ^ s.y ^ s.z ^ s.w;
}

int main() {
    uint32_t t0le[256];
    {  // Te0 little-endian from GF(2^8) (same as aes_common.hpp's generator, any table works for timing)
        uint8_t sbox[256];
        uint8_t p = 1, qv = 1;
        do {
            p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1B : 0);
            qv ^= qv << 1;
            qv ^= qv << 2;
            qv ^= qv << 4;
            if (qv & 0x80) qv ^= 0x09;
            const uint8_t x = qv ^ (uint8_t)((qv << 1) | (qv >> 7)) ^ (uint8_t)((qv << 2) | (qv >> 6)) ^
                              (uint8_t)((qv << 3) | (qv >> 5)) ^ (uint8_t)((qv << 4) | (qv >> 4));
            sbox[p] = x ^ 0x63;
        } while (p != 1);
        sbox[0] = 0x63;
        for (int i = 0; i < 256; i++) {
            const uint8_t s = sbox[i], s2 = (uint8_t)((s << 1) ^ (s & 0x80 ? 0x1B : 0)), s3 = s2 ^ s;
            t0le[i] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
        }
    }
    uint32_t *d_t0, *d_out;
    DevKey *d_key;
    DevKey hk{};
    for (int i = 0; i < 60; i++) hk.rk[i] = 0x01020304u * (i + 1);
    (void)hipMalloc(&d_t0, 1024);
    (void)hipMalloc(&d_out, 1024);
    (void)hipMalloc(&d_key, sizeof(DevKey));
    (void)hipMemcpy(d_t0, t0le, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_key, &hk, sizeof hk, hipMemcpyHostToDevice);
    std::vector<uint32_t> h(128);
    auto run = [&](const char *name, double reps, auto launch) {
        double best = 1e30;
        for (int k = 0; k < 5; k++) {
            launch();
            (void)hipMemcpy(h.data(), d_out, 512, hipMemcpyDeviceToHost);
            best = std::min(best, h[0] / reps);
        }
        printf("%s\"%s\": %.1f", name[0] == 'l' && name[1] == 'd' ? "" : ", ", name, best);
    };
    printf("{\"unit\": \"cycles per repetition (s_memtime), one wave\", ");
    run("lds_chase", kIters, [&] { hipLaunchKernelGGL(k_lds_chase, dim3(1), dim3(64), 0, 0, d_out, 7u); });
    run("valu_chain_2instr", kIters, [&] { hipLaunchKernelGGL(k_valu_chain, dim3(1), dim3(64), 0, 0, d_out, 7u); });
    run("dpp_xor_chain", kIters, [&] { hipLaunchKernelGGL(k_dpp_chain, dim3(1), dim3(64), 0, 0, d_out, 7u); });
    run("k2c_round_aes128", (kIters / 10) * 10, [&] {
        hipLaunchKernelGGL((k_k2c_round<10>), dim3(1), dim3(1024), 0, 0, d_t0, d_key, d_out);
    });
    run("k2c_round_aes256", (kIters / 14) * 14, [&] {
        hipLaunchKernelGGL((k_k2c_round<14>), dim3(1), dim3(1024), 0, 0, d_t0, d_key, d_out);
    });
    run("k2_round_aes128", (kIters / 10) * 10, [&] {
        hipLaunchKernelGGL((k_k2_round<10>), dim3(1), dim3(1024), 0, 0, d_t0, d_key, d_out);
    });
    // multiply-form throughput: cycles per instruction per wave, 1 / 2 / 4 waves per SIMD
    for (int w : {1, 2, 4}) {
        const int iters = 2048;
        auto tput = [&](const char *name, double instr_per_iter, auto kern) {
            double best = 1e30;
            for (int k = 0; k < 5; k++) {
                hipLaunchKernelGGL(kern, dim3(1), dim3(256 * w), 0, 0, d_out, 7u, iters);
                (void)hipMemcpy(h.data(), d_out, 4, hipMemcpyDeviceToHost);
                best = std::min(best, h[0] / (iters * instr_per_iter));
            }
            printf(", \"%s_w%d\": %.2f", name, w, best);
        };
        tput("mad_u64_u32_cyc", 8, k_mad64_tput);
        tput("fma_f64_cyc", 8, k_fma64_tput);
        tput("xor_add_u32_cyc", 16, k_add32_tput);
    }
    printf("}\n");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
