// Compute-only ceiling of the T-table AES round function on one MI355X: the same LDS
// image and round code as K1/K2 (aes_device.hpp), no HBM traffic.  Every lane runs
// IL independent AES-256 chains for ITERS blocks each (output fed back as input), so
// the measured blocks/s is what the LDS + VALU can do with nothing else in the way.
// Also a pure lookup loop (perm + ds_read + xor, no AES structure) for the LDS rate.
//   hipcc -O3 --offload-arch=gfx950 -I fpnn_amd/csrc tools/probe/lds_ceiling.hip -o tools/probe/lds_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "aes_device.hpp"

using namespace fpnn_aes;

template <int IL>
__global__ __launch_bounds__(1024, 1) void k_aes_only(const uint32_t *t0le, const DevKey *key, uint4 *out, int iters) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, t0le);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const RoundKeys<14> rk = load_round_keys<14>(key);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 st[IL];
#pragma unroll
    for (int m = 0; m < IL; m++) st[m] = make_uint4(g, m, g * 7u, m * 13u);
    for (int i = 0; i < iters; i++) aes_encrypt_blocks<14, 4, IL>(st, rk, T);
    uint4 acc = st[0];
#pragma unroll
    for (int m = 1; m < IL; m++) acc = acc ^ st[m];
    out[g] = acc;
}

// The 2-table image (T0, T2: 64 KiB) lets two 1024-thread workgroups share a CU
// (8 waves per SIMD) at the price of rotations for T1 / T3.
template <int IL>
__global__ __launch_bounds__(1024, 2) void k_aes_only_nt2(const uint32_t *t0le, const DevKey *key, uint4 *out, int iters) {
    __shared__ uint4 lds4[Lds<2>::kBytes / 16];
    lds_fill_tables<2>(lds4, t0le);
    __syncthreads();
    const Tables4<2> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const RoundKeys<14> rk = load_round_keys<14>(key);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 st[IL];
#pragma unroll
    for (int m = 0; m < IL; m++) st[m] = make_uint4(g, m, g * 7u, m * 13u);
    for (int i = 0; i < iters; i++) aes_encrypt_blocks<14, 2, IL>(st, rk, T);
    uint4 acc = st[0];
#pragma unroll
    for (int m = 1; m < IL; m++) acc = acc ^ st[m];
    out[g] = acc;
}

// 16 lookups + 8 xor3 per "round", 4 independent words per lane (like one block).
__global__ __launch_bounds__(1024, 1) void k_lookup_only(const uint32_t *t0le, uint32_t *out, int iters) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, t0le);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    uint32_t s0 = threadIdx.x, s1 = s0 * 3u, s2 = s0 * 5u, s3 = s0 * 9u;
    for (int i = 0; i < iters; i++) {
        const uint32_t t0 = xor3(xor3(T.t<0>(s0), T.t<1>(s1), T.t<2>(s2)), T.t<3>(s3), 1u);
        const uint32_t t1 = xor3(xor3(T.t<0>(s1), T.t<1>(s2), T.t<2>(s3)), T.t<3>(s0), 2u);
        const uint32_t t2 = xor3(xor3(T.t<0>(s2), T.t<1>(s3), T.t<2>(s0)), T.t<3>(s1), 3u);
        const uint32_t t3 = xor3(xor3(T.t<0>(s3), T.t<1>(s0), T.t<2>(s1)), T.t<3>(s2), 4u);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
}


// ---- ds_read_b64 (MI355X_MICROARCH.md "LDS": ds_read_b64 takes the
// same 2 LDS-array cycles per wave-instruction as ds_read_b32, 2 x 32 lane groups, banks
// (a/4) mod 64, and one wave per SIMD reaches 95-99 % of its rate issuing continuously).
// Image of 8-byte entries: region r (64 KiB) holds [T_2r[x] | T_2r+1[x]] for x = 0..255,
// entry stride 256 B, copy c (= lane & 31) at +8c, so a 32-lane group covers all 64 banks
// once: conflict-free, 128 KiB like the 4-table image.  Each lookup reads the pair and uses
// one half (the read is volatile so the compiler keeps it 8 bytes wide).
__device__ __forceinline__ void lds_fill_pairs(uint2 *lds2, const uint32_t *__restrict__ t0le) {
    for (uint32_t i = threadIdx.x; i < 131072u / 8; i += blockDim.x) {
        const uint32_t r = i >> 13, x = (i >> 5) & 255;  // i = r * 8192 + x * 32 + c
        const uint32_t v = __ldg(t0le + x);
        lds2[i] = make_uint2(rotl32(v, 16u * r), rotl32(v, 16u * r + 8u));
    }
}

typedef const volatile uint64_t __attribute__((address_space(3))) *lds_u64p;
typedef const volatile uint32_t __attribute__((address_space(3))) *lds_u32p;

struct Tables8 {
    const char *lds;
    uint32_t lb0, lb1;
    __device__ __forceinline__ Tables8(const char *l) : lds(l) {
        lb0 = (threadIdx.x & 31u) << 3;
        lb1 = lb0 | 0x10000u;
    }
    template <int J>
    __device__ __forceinline__ uint32_t t(uint32_t w) const {
        const uint32_t a = __builtin_amdgcn_perm(J < 2 ? lb0 : lb1, w, sel(J));
        const uint64_t v = *(lds_u64p)(lds + a);
        return (J & 1) ? (uint32_t)(v >> 32) : (uint32_t)v;
    }
    template <int J>
    __device__ __forceinline__ uint32_t sraw(uint32_t w) const {  // S at byte J: T0 bytes 1,2 / T2 bytes 0,3
        constexpr bool from_t2 = (J == 0 || J == 3);
        const uint32_t a = __builtin_amdgcn_perm(from_t2 ? lb1 : lb0, w, sel(J));
        return (uint32_t)*(lds_u64p)(lds + a);
    }
};

template <int IL>
__global__ __launch_bounds__(1024, 1) void k_aes_only_b64(const uint32_t *t0le, const DevKey *key, uint4 *out, int iters) {
    __shared__ uint2 lds2[131072 / 8];
    lds_fill_pairs(lds2, t0le);
    __syncthreads();
    const Tables8 T(reinterpret_cast<const char *>(lds2));
    const RoundKeys<14> rk = load_round_keys<14>(key);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s[IL][4];
#pragma unroll
    for (int m = 0; m < IL; m++) { s[m][0] = g; s[m][1] = m; s[m][2] = g * 7u; s[m][3] = m * 13u; }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int m = 0; m < IL; m++) {
            uint32_t s0 = s[m][0] ^ rk.k[0], s1 = s[m][1] ^ rk.k[1], s2 = s[m][2] ^ rk.k[2], s3 = s[m][3] ^ rk.k[3];
#pragma unroll
            for (int r = 1; r < 14; r++) {
                const uint32_t t0 = xor3(xor3(T.t<0>(s0), T.t<1>(s1), T.t<2>(s2)), T.t<3>(s3), rk.k[4 * r + 0]);
                const uint32_t t1 = xor3(xor3(T.t<0>(s1), T.t<1>(s2), T.t<2>(s3)), T.t<3>(s0), rk.k[4 * r + 1]);
                const uint32_t t2 = xor3(xor3(T.t<0>(s2), T.t<1>(s3), T.t<2>(s0)), T.t<3>(s1), rk.k[4 * r + 2]);
                const uint32_t t3 = xor3(xor3(T.t<0>(s3), T.t<1>(s0), T.t<2>(s1)), T.t<3>(s2), rk.k[4 * r + 3]);
                s0 = t0; s1 = t1; s2 = t2; s3 = t3;
            }
            auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
                const uint32_t lo = __builtin_amdgcn_perm(T.sraw<1>(b), T.sraw<0>(a), 0x0c0c0500u);
                const uint32_t hi = __builtin_amdgcn_perm(T.sraw<3>(d), T.sraw<2>(c), 0x07020c0cu);
                return xor3(lo, hi, k);
            };
            s[m][0] = last(s0, s1, s2, s3, rk.k[56]);
            s[m][1] = last(s1, s2, s3, s0, rk.k[57]);
            s[m][2] = last(s2, s3, s0, s1, rk.k[58]);
            s[m][3] = last(s3, s0, s1, s2, rk.k[59]);
        }
    }
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < IL; m++) acc = acc ^ make_uint4(s[m][0], s[m][1], s[m][2], s[m][3]);
    out[g] = acc;
}

// bare b64 lookup loop: 16 lookups + 8 xor3 per "round", like k_lookup_only
__global__ __launch_bounds__(1024, 1) void k_lookup_only_b64(const uint32_t *t0le, uint32_t *out, int iters) {
    __shared__ uint2 lds2[131072 / 8];
    lds_fill_pairs(lds2, t0le);
    __syncthreads();
    const Tables8 T(reinterpret_cast<const char *>(lds2));
    uint32_t s0 = threadIdx.x, s1 = s0 * 3u, s2 = s0 * 5u, s3 = s0 * 9u;
    for (int i = 0; i < iters; i++) {
        const uint32_t t0 = xor3(xor3(T.t<0>(s0), T.t<1>(s1), T.t<2>(s2)), T.t<3>(s3), 1u);
        const uint32_t t1 = xor3(xor3(T.t<0>(s1), T.t<1>(s2), T.t<2>(s3)), T.t<3>(s0), 2u);
        const uint32_t t2 = xor3(xor3(T.t<0>(s2), T.t<1>(s3), T.t<2>(s0)), T.t<3>(s1), 3u);
        const uint32_t t3 = xor3(xor3(T.t<0>(s3), T.t<1>(s0), T.t<2>(s1)), T.t<3>(s2), 4u);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3;
}

// pure issue-rate loops: NL independent lookups per iteration, results summed (no AES
// dependency chain), b32 vs b64, to see the array's own ceiling for each width
template <bool B64, int NL>
__global__ __launch_bounds__(1024, 1) void k_lds_rate(const uint32_t *t0le, uint32_t *out, int iters) {
    __shared__ uint2 lds2[131072 / 8];
    lds_fill_pairs(lds2, t0le);
    __syncthreads();
    const char *lds = reinterpret_cast<const char *>(lds2);
    const uint32_t base = B64 ? (threadIdx.x & 31u) << 3 : (threadIdx.x & 31u) << 2;
    uint32_t st[NL], acc[NL];
#pragma unroll
    for (int k = 0; k < NL; k++) { st[k] = threadIdx.x * (2 * k + 1); acc[k] = 0; }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < NL; k++) {
            const uint32_t a = __builtin_amdgcn_perm(base, st[k], sel(k & 3));
            uint32_t v;
            if (B64) {
                const uint64_t w = *(lds_u64p)(lds + a);
                v = (uint32_t)w ^ (uint32_t)(w >> 32);
            } else {
                v = *(lds_u32p)(lds + a);
            }
            acc[k] ^= v;
            st[k] = st[k] * 0x01000193u + v;  // next index depends on the last value (a chain per k)
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < NL; k++) r ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// ---- LDS + vector-L1 (TCP) hybrid: R of the 16 lookups of a round go to a 4 KiB
// global copy of T0..T3 through buffer_load (offset = byte << 2, table = imm offset).
template <int J>
__device__ __forceinline__ uint32_t tcp_t(__amdgpu_buffer_rsrc_t r, uint32_t w) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, ((w >> (8 * J)) & 0xffu) << 2, 0, 0) ;
}

template <int R, int J, int C>
__device__ __forceinline__ uint32_t hyb(const Tables4<4> &T, __amdgpu_buffer_rsrc_t r, uint32_t w) {
    // lookup slot k = J*4 + C taken by the TCP for k >= 16 - R (T3 first, then T2 ...)
    constexpr int k = (3 - J) * 4 + C;
    if (k < R) {
        if (J == 0) return tcp_t<0>(r, w);
        if (J == 1) return __builtin_amdgcn_raw_buffer_load_b32(r, ((w >> 8) & 0xffu) << 2, 1024, 0);
        if (J == 2) return __builtin_amdgcn_raw_buffer_load_b32(r, ((w >> 16) & 0xffu) << 2, 2048, 0);
        return __builtin_amdgcn_raw_buffer_load_b32(r, (w >> 24) << 2, 3072, 0);
    }
    return T.template t<J>(w);
}

template <int R, int IL>
__global__ __launch_bounds__(1024, 1) void k_hybrid(const uint32_t *t0le, const uint32_t *gt, uint4 *out, int iters) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    lds_fill_tables<4>(lds4, t0le);
    __syncthreads();
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gt, 0, 4096, 0x00020000);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t s[IL][4];
#pragma unroll
    for (int m = 0; m < IL; m++) { s[m][0] = g; s[m][1] = g * 3u + m; s[m][2] = g * 5u; s[m][3] = g * 9u + m; }
    for (int i = 0; i < iters; i++) {
        uint32_t t[IL][4];
#pragma unroll
        for (int m = 0; m < IL; m++) {
            t[m][0] = xor3(xor3(hyb<R, 0, 0>(T, rs, s[m][0]), hyb<R, 1, 0>(T, rs, s[m][1]), hyb<R, 2, 0>(T, rs, s[m][2])), hyb<R, 3, 0>(T, rs, s[m][3]), 1u);
            t[m][1] = xor3(xor3(hyb<R, 0, 1>(T, rs, s[m][1]), hyb<R, 1, 1>(T, rs, s[m][2]), hyb<R, 2, 1>(T, rs, s[m][3])), hyb<R, 3, 1>(T, rs, s[m][0]), 2u);
            t[m][2] = xor3(xor3(hyb<R, 0, 2>(T, rs, s[m][2]), hyb<R, 1, 2>(T, rs, s[m][3]), hyb<R, 2, 2>(T, rs, s[m][0])), hyb<R, 3, 2>(T, rs, s[m][1]), 3u);
            t[m][3] = xor3(xor3(hyb<R, 0, 3>(T, rs, s[m][3]), hyb<R, 1, 3>(T, rs, s[m][0]), hyb<R, 2, 3>(T, rs, s[m][1])), hyb<R, 3, 3>(T, rs, s[m][2]), 4u);
        }
#pragma unroll
        for (int m = 0; m < IL; m++)
#pragma unroll
            for (int c = 0; c < 4; c++) s[m][c] = t[m][c];
    }
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int m = 0; m < IL; m++) acc = acc ^ make_uint4(s[m][0], s[m][1], s[m][2], s[m][3]);
    out[g] = acc;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint32_t *d_t0;
    DevKey *d_key;
    uint4 *d_out;
    CK(hipMalloc(&d_t0, 1024));
    CK(hipMemcpy(d_t0, kTables.t0le, 1024, hipMemcpyHostToDevice));
    DevKey hk{};
    for (int i = 0; i < 60; i++) hk.rk[i] = 0x01020304u * (i + 1);
    CK(hipMalloc(&d_key, sizeof(DevKey)));
    CK(hipMemcpy(d_key, &hk, sizeof(DevKey), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, (size_t)cus * 1024 * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int iters = 2048;
    auto run = [&](const char *name, auto launch, double blocks, double lookups) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        // lookups/clk/CU at the nominal 2.4 GHz and implied clock if LDS ran at 32/clk
        const double lps = lookups / (best * 1e-3);
        printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"payload_GBs\": %.1f, \"lookups_per_ns_per_cu\": %.2f, "
               "\"lds_bound_clock_GHz_at_32_per_clk\": %.3f}\n",
               name, best, blocks * 16 / (best * 1e-3) / 1e9, lps / 1e9 / cus, lps / cus / 32 / 1e9);
    };
    const double lanes = (double)cus * 1024;
    run("aes_only_il1", [&] { hipLaunchKernelGGL(k_aes_only<1>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters); },
        lanes * iters, lanes * iters * 224);
    run("aes_only_il2", [&] { hipLaunchKernelGGL(k_aes_only<2>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters / 2); },
        lanes * iters, lanes * iters * 224);
    run("aes_only_il4", [&] { hipLaunchKernelGGL(k_aes_only<4>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters / 4); },
        lanes * iters, lanes * iters * 224);
    CK(hipFree(d_out));
    CK(hipMalloc(&d_out, (size_t)2 * cus * 1024 * 16));
    run("aes_only_nt2_2wg", [&] { hipLaunchKernelGGL(k_aes_only_nt2<1>, dim3(2 * cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters / 2); },
        lanes * iters, lanes * iters * 224);
    run("aes_only_nt2_1wg", [&] { hipLaunchKernelGGL(k_aes_only_nt2<1>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters); },
        lanes * iters, lanes * iters * 224);
    run("lookup_only", [&] { hipLaunchKernelGGL(k_lookup_only, dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 14); },
        lanes * iters, lanes * iters * 224);

    // ds_read_b64 rows, beside the b32 rows above
    run("aes_only_b64_il1", [&] { hipLaunchKernelGGL(k_aes_only_b64<1>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters); },
        lanes * iters, lanes * iters * 224);
    run("aes_only_b64_il2", [&] { hipLaunchKernelGGL(k_aes_only_b64<2>, dim3(cus), dim3(1024), 0, 0, d_t0, d_key, d_out, iters / 2); },
        lanes * iters, lanes * iters * 224);
    run("lookup_only_b64", [&] { hipLaunchKernelGGL(k_lookup_only_b64, dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 14); },
        lanes * iters, lanes * iters * 224);
    // (a "block" here = 224 lookups, so lookups_per_ns_per_cu is the comparable column)
    run("rate_b32_nl8", [&] { hipLaunchKernelGGL((k_lds_rate<false, 8>), dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 28); },
        lanes * iters, lanes * iters * 224);
    run("rate_b64_nl8", [&] { hipLaunchKernelGGL((k_lds_rate<true, 8>), dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 28); },
        lanes * iters, lanes * iters * 224);
    run("rate_b32_nl16", [&] { hipLaunchKernelGGL((k_lds_rate<false, 16>), dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 14); },
        lanes * iters, lanes * iters * 224);
    run("rate_b64_nl16", [&] { hipLaunchKernelGGL((k_lds_rate<true, 16>), dim3(cus), dim3(1024), 0, 0, d_t0, (uint32_t *)d_out, iters * 14); },
        lanes * iters, lanes * iters * 224);

    uint32_t *d_gt;
    CK(hipMalloc(&d_gt, 4096));
    {
        uint32_t h[1024];
        for (int k = 0; k < 4; k++)
            for (int x = 0; x < 256; x++) h[256 * k + x] = (kTables.t0le[x] << (8 * k)) | (k ? kTables.t0le[x] >> (32 - 8 * k) : 0);
        CK(hipMemcpy(d_gt, h, 4096, hipMemcpyHostToDevice));
    }
#define HYB(R, IL) run("hybrid_r" #R "_il" #IL, [&] { hipLaunchKernelGGL((k_hybrid<R, IL>), dim3(cus), dim3(1024), 0, 0, d_t0, d_gt, d_out, iters * 14 / IL); }, lanes * iters, lanes * iters * 224)
    HYB(0, 2); HYB(1, 2); HYB(2, 2); HYB(3, 2); HYB(4, 2); HYB(6, 2); HYB(8, 2); HYB(16, 2);
    HYB(2, 4); HYB(4, 4);
    CK(hipGetLastError());
    return 0;
}
