// Probe: does gfx950 need wait states between a VALU carry-out write and the next VALU's
// carry-in read?  hipcc's hazard recognizer pads `v_add_co` -> `v_addc` (vcc or an SGPR pair)
// with 2 wait states (s_nop), which costs issue slots in the ECDH field arithmetic.  This
// runs the same 8-limb carry chains inside inline asm with NO padding (the pattern the
// ECDH kernel's mad -> addc macs have always used) and with the padding, on inputs that
// make every limb carry, and counts lanes whose result differs from plain C.
//   hipcc --offload-arch=gfx950 -O3 carry_hazard.hip -o carry_hazard && ./carry_hazard
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__device__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// 8-limb a + b, carry chain in vcc, back to back (no wait states)
__device__ void add8_nopad(const uint32_t *a, const uint32_t *b, uint32_t *r) {
    uint32_t r0, r1, r2, r3, r4, r5, r6, r7;
    asm volatile(
        "v_add_co_u32 %0, vcc, %8, %16\n\t"
        "v_addc_co_u32 %1, vcc, %9, %17, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %10, %18, vcc\n\t"
        "v_addc_co_u32 %3, vcc, %11, %19, vcc\n\t"
        "v_addc_co_u32 %4, vcc, %12, %20, vcc\n\t"
        "v_addc_co_u32 %5, vcc, %13, %21, vcc\n\t"
        "v_addc_co_u32 %6, vcc, %14, %22, vcc\n\t"
        "v_addc_co_u32 %7, vcc, %15, %23, vcc"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(b[0]),
          "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
        : "vcc");
    r[0] = r0, r[1] = r1, r[2] = r2, r[3] = r3, r[4] = r4, r[5] = r5, r[6] = r6, r[7] = r7;
}

// the same chain with the carry in an SGPR pair
__device__ void add8_nopad_s(const uint32_t *a, const uint32_t *b, uint32_t *r) {
    uint32_t r0, r1, r2, r3, r4, r5, r6, r7;
    uint64_t cy;
    asm volatile(
        "v_add_co_u32 %0, %8, %9, %17\n\t"
        "v_addc_co_u32 %1, %8, %10, %18, %8\n\t"
        "v_addc_co_u32 %2, %8, %11, %19, %8\n\t"
        "v_addc_co_u32 %3, %8, %12, %20, %8\n\t"
        "v_addc_co_u32 %4, %8, %13, %21, %8\n\t"
        "v_addc_co_u32 %5, %8, %14, %22, %8\n\t"
        "v_addc_co_u32 %6, %8, %15, %23, %8\n\t"
        "v_addc_co_u32 %7, %8, %16, %24, %8"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7), "=&s"(cy)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(b[0]),
          "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    r[0] = r0, r[1] = r1, r[2] = r2, r[3] = r3, r[4] = r4, r[5] = r5, r[6] = r6, r[7] = r7;
}

// mad -> addc (the ECDH mac): 8 partial products into one 96-bit accumulator
__device__ void mac8_nopad(const uint32_t *a, const uint32_t *b, uint32_t *r) {
    uint64_t lo = 0;
    uint32_t hi = 0;
    for (int j = 0; j < 8; j++)
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                     : "+v"(lo), "+v"(hi)
                     : "v"(a[j]), "v"(b[j])
                     : "vcc");
    r[0] = (uint32_t)lo, r[1] = (uint32_t)(lo >> 32), r[2] = hi;
}

__global__ void k_probe(uint32_t seed, int mode, unsigned long long *bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a[8], b[8], r[8], e[8];
    for (int j = 0; j < 8; j++) {
        const uint32_t x = mix(seed + 16u * i + j), y = mix(~seed + 16u * i + j);
        // mostly all-ones limbs: every limb carries; sometimes random
        a[j] = (x & 3u) ? 0xffffffffu - (x >> 28) : x;
        b[j] = (y & 3u) ? 1u + (y >> 29) : y;
    }
    uint32_t c = 0;
    for (int j = 0; j < 8; j++) {
        const uint64_t s = (uint64_t)a[j] + b[j] + c;
        e[j] = (uint32_t)s;
        c = (uint32_t)(s >> 32);
    }
    int n = 8;
    if (mode == 0) add8_nopad(a, b, r);
    else if (mode == 1) add8_nopad_s(a, b, r);
    else {
        mac8_nopad(a, b, r);
        unsigned __int128 acc = 0;
        for (int j = 0; j < 8; j++) acc += (unsigned __int128)((uint64_t)a[j] * b[j]);
        e[0] = (uint32_t)acc, e[1] = (uint32_t)(acc >> 32), e[2] = (uint32_t)(acc >> 64);
        n = 3;
    }
    bool ok = true;
    for (int j = 0; j < n; j++) ok &= r[j] == e[j];
    if (!ok) atomicAdd(bad, 1ull);
}

int main() {
    unsigned long long *d;
    CHECK(hipMalloc(&d, 8));
    const char *names[3] = {"add_co/addc chain, vcc, no pad", "add_co/addc chain, SGPR pair, no pad",
                            "mad_u64_u32 -> addc (ECDH mac), vcc, no pad"};
    const int blocks = 4096, threads = 256, reps = 8;
    for (int mode = 0; mode < 3; mode++) {
        unsigned long long total = 0;
        for (int rep = 0; rep < reps; rep++) {
            CHECK(hipMemset(d, 0, 8));
            hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(threads), 0, 0, 0x9e3779b9u * (rep + 1), mode, d);
            CHECK(hipDeviceSynchronize());
            unsigned long long h;
            CHECK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
            total += h;
        }
        printf("{\"probe\": \"%s\", \"lanes\": %llu, \"wrong\": %llu}\n", names[mode],
               (unsigned long long)blocks * threads * reps, total);
    }
    CHECK(hipFree(d));
    return 0;
}
