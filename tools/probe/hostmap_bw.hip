// PROBE (not part of the product): how fast can gfx950 kernels gather frames from, and
// scatter frames to, registered (GPU-mapped) host memory over PCIe, compared with
// hipMemcpyAsync DMA from pinned staging?  Frames are 1 KiB at shuffled host addresses
// (the host-frame path's shape: 1M frames).  One wave moves F frames per step
// (lane = 16 B of a frame, loads of all F frames issued before the stores).
//   hipcc -O3 --offload-arch=gfx950 hostmap_bw.hip -o hostmap_bw && ./hostmap_bw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int F = 4;

// dst[i*L ..] = src + off[i]  (gather: src host, dst device)
__global__ __launch_bounds__(256) void k_gather(const uint8_t *src, const uint64_t *off, uint8_t *dst, uint32_t n,
                                                uint32_t L) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * blockDim.x / 64;
    for (uint64_t f0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64 * F; f0 < n; f0 += nw * F) {
        uint4 v[F];
#pragma unroll
        for (int k = 0; k < F; k++)
            if (f0 + k < n) v[k] = *(const uint4 *)(src + off[f0 + k] + 16 * lane);
#pragma unroll
        for (int k = 0; k < F; k++)
            if (f0 + k < n) *(uint4 *)(dst + (f0 + k) * L + 16 * lane) = v[k];
    }
}

// dst + off[i] = src[i*L ..]  (scatter: src device, dst host)
__global__ __launch_bounds__(256) void k_scatter(const uint8_t *src, const uint64_t *off, uint8_t *dst, uint32_t n,
                                                 uint32_t L) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * blockDim.x / 64;
    for (uint64_t f0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64 * F; f0 < n; f0 += nw * F) {
        uint4 v[F];
#pragma unroll
        for (int k = 0; k < F; k++)
            if (f0 + k < n) v[k] = *(const uint4 *)(src + (f0 + k) * L + 16 * lane);
#pragma unroll
        for (int k = 0; k < F; k++)
            if (f0 + k < n) *(uint4 *)(dst + off[f0 + k] + 16 * lane) = v[k];
    }
}

// the product's k_move_segments (k_support.hip) restated: descriptor arrays per segment
typedef uint4 __attribute__((aligned(1))) uint4_u;
__global__ __launch_bounds__(256) void k_move(uint64_t sbase, const uint64_t *__restrict__ soff, uint64_t dbase,
                                              const uint64_t *__restrict__ doff, const uint32_t *__restrict__ len,
                                              uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t w = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    for (uint64_t g = w * F; g < n; g += nw * F) {
        const uint8_t *src[F];
        uint8_t *dst[F];
        uint32_t L[F];
        uint32_t maxl = 0;
#pragma unroll
        for (int k = 0; k < F; k++) {
            const uint64_t i = g + k;
            L[k] = i < n ? len[i] : 0u;
            src[k] = reinterpret_cast<const uint8_t *>(i < n ? sbase + soff[i] : sbase);
            dst[k] = reinterpret_cast<uint8_t *>(i < n ? dbase + doff[i] : dbase);
            maxl = L[k] > maxl ? L[k] : maxl;
        }
        for (uint32_t p = 0; p < maxl; p += 1024) {
            const uint32_t b = p + 16 * lane;
            uint4 v[F];
#pragma unroll
            for (int k = 0; k < F; k++) v[k] = b + 16 <= L[k] ? *(const uint4_u *)(src[k] + b) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < F; k++) {
                if (b + 16 <= L[k]) {
                    *(uint4_u *)(dst[k] + b) = v[k];
                } else if (b < L[k]) {
                    for (uint32_t j = b; j < L[k]; j++) dst[k][j] = src[k][j];
                }
            }
        }
    }
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const uint32_t L = 1024, n = 1u << 20;
    const size_t bytes = (size_t)n * L;
    int grid = argc > 1 ? atoi(argv[1]) : 1024;
    const unsigned rflags = argc > 2 ? (unsigned)atoi(argv[2]) : hipHostRegisterDefault;
    // host arena: frames at shuffled positions
    std::vector<uint64_t> off(n);
    for (uint32_t i = 0; i < n; i++) off[i] = (uint64_t)i * L;
    std::shuffle(off.begin(), off.end(), std::mt19937_64(7));
    uint8_t *ha = (uint8_t *)aligned_alloc(4096, bytes), *hb = (uint8_t *)aligned_alloc(4096, bytes);
    memset(ha, 1, bytes);
    memset(hb, 2, bytes);
    double t0 = now();
    CK(hipHostRegister(ha, bytes, rflags));
    CK(hipHostRegister(hb, bytes, rflags));
    printf("{\"register_flags\": %u}\n", rflags);
    double treg = (now() - t0) / 2;
    uint8_t *da, *db;
    CK(hipHostGetDevicePointer((void **)&da, ha, 0));
    CK(hipHostGetDevicePointer((void **)&db, hb, 0));
    uint8_t *d0, *d1;
    uint64_t *doff;
    CK(hipMalloc(&d0, bytes));
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&doff, n * 8));
    CK(hipMemcpy(doff, off.data(), n * 8, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CK(hipStreamCreate(&s1));
    CK(hipStreamCreate(&s2));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn, double gb) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            double t = now();
            fn();
            CK(hipDeviceSynchronize());
            best = std::min<float>(best, (float)(now() - t));
        }
        printf("{\"probe\": \"%s\", \"grid\": %d, \"ms\": %.3f, \"GBs\": %.1f}\n", name, grid, best * 1e3, gb / best / 1e9);
    };
    printf("{\"hipHostRegister_1GiB_ms\": %.1f}\n", treg * 1e3);
    timeit("gather host->dev (kernel, shuffled 1 KiB frames)", [&] {
        hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, s1, da, doff, d0, n, L);
    }, (double)bytes);
    timeit("scatter dev->host (kernel, shuffled 1 KiB frames)", [&] {
        hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(256), 0, s1, d0, doff, db, n, L);
    }, (double)bytes);
    timeit("gather + scatter concurrently (two streams)", [&] {
        hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, s1, da, doff, d0, n, L);
        hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(256), 0, s2, d1, doff, db, n, L);
    }, (double)bytes);  // GB/s per direction
    timeit("DMA H2D (registered, contiguous)", [&] { CK(hipMemcpyAsync(d0, ha, bytes, hipMemcpyHostToDevice, s1)); },
           (double)bytes);
    timeit("DMA D2H (registered, contiguous)", [&] { CK(hipMemcpyAsync(hb, d0, bytes, hipMemcpyDeviceToHost, s1)); },
           (double)bytes);
    timeit("DMA H2D + D2H concurrently", [&] {
        CK(hipMemcpyAsync(d0, ha, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(hb, d1, bytes, hipMemcpyDeviceToHost, s2));
    }, (double)bytes);
    // the product kernel: absolute host addresses + dense device offsets
    {
        std::vector<uint64_t> habs(n), dofs(n);
        std::vector<uint32_t> lens(n, L);
        for (uint32_t i = 0; i < n; i++) { habs[i] = (uint64_t)(uintptr_t)da + off[i]; dofs[i] = (uint64_t)i * L; }
        std::vector<uint64_t> habs_b(n);
        for (uint32_t i = 0; i < n; i++) habs_b[i] = (uint64_t)(uintptr_t)db + off[i];
        uint64_t *d_habs, *d_dofs, *d_habs_b; uint32_t *d_len;
        CK(hipMalloc(&d_habs, n * 8)); CK(hipMalloc(&d_dofs, n * 8)); CK(hipMalloc(&d_habs_b, n * 8)); CK(hipMalloc(&d_len, n * 4));
        CK(hipMemcpy(d_habs, habs.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_habs_b, habs_b.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_dofs, dofs.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_len, lens.data(), n * 4, hipMemcpyHostToDevice));
        for (uint32_t chunk : {n, 65536u}) {
            char name[128];
            auto gat = [&](hipStream_t s) { for (uint32_t c = 0; c < n; c += chunk) hipLaunchKernelGGL(k_move, dim3(grid), dim3(256), 0, s, 0, d_habs + c, (uint64_t)(uintptr_t)d0, d_dofs + c, d_len + c, std::min(chunk, n - c)); };
            auto sca = [&](hipStream_t s) { for (uint32_t c = 0; c < n; c += chunk) hipLaunchKernelGGL(k_move, dim3(grid), dim3(256), 0, s, (uint64_t)(uintptr_t)d1, d_dofs + c, 0, d_habs_b + c, d_len + c, std::min(chunk, n - c)); };
            snprintf(name, sizeof name, "k_move gather, %u frames per launch", chunk);
            timeit(name, [&] { gat(s1); }, (double)bytes);
            snprintf(name, sizeof name, "k_move scatter, %u frames per launch", chunk);
            timeit(name, [&] { sca(s1); }, (double)bytes);
            snprintf(name, sizeof name, "k_move gather + scatter concurrently, %u frames per launch", chunk);
            timeit(name, [&] { gat(s1); sca(s2); }, (double)bytes);
        }
    }
    // verify the gather once
    hipLaunchKernelGGL(k_gather, dim3(grid), dim3(256), 0, s1, da, doff, d0, n, L);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> chk(L);
    bool ok = true;
    for (uint32_t i = 0; i < n && ok; i += 4099) {
        CK(hipMemcpy(chk.data(), d0 + (size_t)i * L, L, hipMemcpyDeviceToHost));
        ok = memcmp(chk.data(), ha + off[i], L) == 0;
    }
    printf("{\"gather_ok\": %s}\n", ok ? "true" : "false");
    CK(hipHostUnregister(ha));
    CK(hipHostUnregister(hb));
    return 0;
}
