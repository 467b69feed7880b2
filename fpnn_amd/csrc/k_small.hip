// k_small.hip -- the small single-call CFB kernels behind the synchronous drop-in
// (PackageEncryptor / StreamEncryptor per call, rijndael_cfb_encrypt; core/Encryptor.cpp:10-70,
// base/rijndael.c:1171-1201) for calls of up to kSmallMaxBytes.
//
// One call = one CFB byte stream with the reference's (ivec, *p_num) carry.  The batch
// kernels pay for throughput machinery a single frame never uses: K2c fills the 128 KiB
// replicated LDS image with 64 threads (128 dependent rounds of a global load each), K1r
// launches a block map, a descriptor pass and a 256-workgroup grid for 64 blocks, and the
// call moved its bytes with three DMA copies and waited in the blocking stream sync.
//   K0  k_cfb_single : one launch of one 256-thread workgroup per call.  The table image is
//       filled from registers (thread x loads T0[x] once); the bytes are read from and
//       written back to the engine's pinned staging directly over PCIe; completion is a
//       sequence number the kernel stores to pinned memory after its results
//       (system-scope release), on which the host spins.
//   K0s k_cfb_server : the same call body in a workgroup that stays resident while calls
//       keep coming: it polls a mailbox in pinned host memory, serves each request and
//       publishes its sequence number; between requests it checks an idle interval, a
//       lifetime bound, a stop flag and the device's batch-activity word (bumped by the
//       host before it queues batch kernels), and leaves on any of them.  No launch, no table
//       fill and no kernel-argument fetch per call; the host relaunches it once it has left.
// Decrypt: one lane per 16-byte block (block i's keystream is E(C_{i-1})).  Encrypt: the
// serial chain on one quad (K2c's column round, coop.hpp) -- C_i = P_i ^ E(C_{i-1}).
#include "coop.hpp"
#include "kernels.hpp"

namespace fpnn_aes {

namespace {

constexpr int kSmallThreads = 256;

__device__ __forceinline__ void store_release(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t load_acquire(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The first 16 bytes of the request (seq, op, len, head) in ONE system-coherent vector
// load (sc0 sc1: past both GPU caches to host memory), so a poll that sees a new sequence
// number has the call's header in the same PCIe round trip.  The host writes op, len and
// head before it release-stores seq, all in this one 16-byte block of one cache line
// (x86 stores become visible in program order, and the line is read whole), so a new seq
// comes with its own header.  The acquire fence that follows orders the body's loads.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
// with the batch-activity word read beside it (both in flight together: one PCIe round
// trip per poll)
__device__ __forceinline__ u32x4_t load_sys16_and(const void *p, const uint32_t *q, uint32_t &y) {
    u32x4_t v;
    asm volatile("global_load_dwordx4 %0, %2, off sc0 sc1\n\tglobal_load_dword %1, %3, off sc0 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(v), "=&v"(y) : "v"(p), "v"(q) : "memory");
    return v;
}

// LDS image: copies [0, ncopies) of every (table, x) entry (the layout of aes_device.hpp)
__device__ __forceinline__ void fill_tables_regs(uint4 *lds4, uint32_t v0, int ncopies) {
    const uint32_t x = threadIdx.x;  // kSmallThreads == 256 entries
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t v = rotl32(v0, 8u * k);
        const uint32_t r = k >> 1, h = k & 1;
        uint4 *row = lds4 + ((r * 65536u + x * 256u + h * 128u) >> 4);  // 32 copies = 8 uint4
        for (int c = 0; c < ncopies; c += 4) row[c >> 2] = make_uint4(v, v, v, v);
    }
}

struct SmallShared {
    uint4 buf[kSmallMaxBytes / 16 + 2];  // head block + body + one spare (prefetch)
    uint32_t fhead[4], fout[4];          // feedback register after the head / after the call
};

// One call (after buf[0..nb] holds the staging's blocks): head, body, write-back, and the
// (ivec, pos) result into state[0..4].  Every thread of the workgroup calls it.
template <int NR, bool ENCRYPT>
__device__ __forceinline__ void small_body(uint32_t len, uint32_t head, uint32_t pos, uint4 iv, const uint32_t *rkp,
                                           uint4 *io, uint32_t *state, const uint4 *lds4, SmallShared &S) {
    const uint32_t t = threadIdx.x;
    const uint32_t rem = len - head, r = rem & 15u;
    const uint32_t nb = (rem + 15) >> 4;  // body blocks, the last one partial when r != 0
    uint4 *buf = S.buf;
    if (t == 0) {  // head: ivec bytes [pos, pos + head) are keystream already (base/rijndael.c:1180-1195)
        uint8_t *fb = reinterpret_cast<uint8_t *>(S.fhead);
        *reinterpret_cast<uint4 *>(S.fhead) = iv;
        uint8_t *hb = reinterpret_cast<uint8_t *>(&buf[0]) + 16 - head;
        for (uint32_t j = 0; j < head; j++) {
            const uint8_t c = hb[j];
            const uint8_t o = c ^ fb[pos + j];
            hb[j] = o;
            fb[pos + j] = ENCRYPT ? o : c;  // the feedback is always the ciphertext byte
        }
        *reinterpret_cast<uint4 *>(S.fout) = *reinterpret_cast<const uint4 *>(S.fhead);  // nb == 0
    }
    __syncthreads();
    const uint4 f0 = *reinterpret_cast<const uint4 *>(S.fhead);
    if (ENCRYPT) {
        if (t < 4) {  // the chain on one quad: lane q owns column q (coop.hpp)
            const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
            uint32_t rkq[NR + 1];
#pragma unroll
            for (int k = 0; k <= NR; k++) rkq[k] = rkp[4 * k + t];
            uint32_t fq = word_of(f0, (int)t);
            const uint32_t *bw = reinterpret_cast<const uint32_t *>(buf + 1);
            uint32_t *ow = reinterpret_cast<uint32_t *>(io + 1);  // the body's words in the staging
            uint32_t pw = nb ? bw[t] : 0u;  // P_i, loaded one block ahead of its use
            // the chain carries C ^ rk[0] (aes_chain_column: both XORs folded into the keys)
            uint32_t sw = fq ^ rkq[0];
            const uint32_t rkx = rkq[NR] ^ rkq[0];
            for (uint32_t i = 0; i < nb; i++) {
                const uint32_t p = pw;
                pw = bw[4 * (i + 1) + t];  // (buf has one spare block past the body)
                const uint32_t nsw = aes_chain_column<NR, 4>(sw, rkq, rkx ^ p, T);
                const uint32_t c = nsw ^ rkq[0];
                ow[4 * i + t] = c;  // straight out (posted writes during the chain)
                sw = nsw;
                if (i + 1 < nb || r == 0) {
                    fq = c;
                } else {  // partial last block: ivec = C bytes [0, r) + keystream bytes [r, 16)
                    const uint32_t k = c ^ p;
                    const int lo = (int)r - 4 * (int)t;
                    const uint32_t m = lo >= 4 ? 0xffffffffu : lo <= 0 ? 0u : (0xffffffffu >> (8 * (4 - lo)));
                    fq = (c & m) | (k & ~m);
                }
            }
            if (nb) S.fout[t] = fq;
        }
        __syncthreads();
        if (t == 0) io[0] = buf[0];  // the head's block
    } else {  // one lane per block; plaintext straight back to the staging
        const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
        const RoundKeys<NR> rk = *reinterpret_cast<const RoundKeys<NR> *>(rkp);
        for (uint32_t i = t; i < nb; i += kSmallThreads) {
            const uint4 k = aes_encrypt_block<NR, 4>(i ? buf[i] : f0, rk, T);  // buf[i] = C_{i-1}
            const uint4 c = buf[i + 1];
            io[i + 1] = c ^ k;
            if (i + 1 == nb)  // ivec after the call: the last C block, or C bytes [0, r) + K
                *reinterpret_cast<uint4 *>(S.fout) = r ? select_bytes(byte_mask(0, (int)r), c, k) : c;
        }
        __syncthreads();
        if (t == 0) io[0] = buf[0];
    }
    if (t == 0) {
        state[0] = S.fout[0];
        state[1] = S.fout[1];
        state[2] = S.fout[2];
        state[3] = S.fout[3];
        state[4] = nb ? r : (pos + head) & 15u;
    }
}

template <int NR, bool ENCRYPT>
__global__ __launch_bounds__(kSmallThreads, 1) void k_cfb_single(SmallArgs a) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    __shared__ SmallShared S;
    const uint32_t t = threadIdx.x;
    // the call's bytes: the body starts at io + kSmallBodyAt (16-aligned), the head's
    // bytes (pos != 0: the rest of the current keystream block) sit right before it
    const uint32_t nb = (a.len - a.head + 15) >> 4;
    uint4 *io = reinterpret_cast<uint4 *>(a.io + kSmallBodyAt - 16);
    // first PCIe read in flight before the table fill (both wait on memory, not on each other)
    const uint4 first = t <= nb ? io[t] : make_uint4(0, 0, 0, 0);
    fill_tables_regs(lds4, a.t0le[t], ENCRYPT ? 4 : 32);  // encrypt: the chain's quad reads copies 0..3
    if (t <= nb) S.buf[t] = first;  // buf[0]: the head bytes at its end
    for (uint32_t i = t + kSmallThreads; i <= nb; i += kSmallThreads) S.buf[i] = io[i];
    __syncthreads();
    small_body<NR, ENCRYPT>(a.len, a.head, a.pos, a.iv, a.rk, io, a.state, lds4, S);
    __threadfence_system();
    __syncthreads();
    if (t == 0) store_release(a.state + 5, a.seq);
}

// K0s.  Mailbox (pinned host memory, kernels.hpp SmallMailbox): the host writes a request
// (fields, then its sequence number with a release store), the server serves every new
// sequence number in order and stores it into resp.done after the results.
__global__ __launch_bounds__(kSmallThreads, 1) void k_cfb_server(SmallMailbox *mb, const uint32_t *t0le,
                                                                 uint32_t epoch, uint64_t idle_ticks,
                                                                 uint64_t life_ticks, const uint32_t *yield,
                                                                 uint32_t y0) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    __shared__ SmallShared S;
    __shared__ SmallReq rq;
    __shared__ uint32_t ctl[2][4];  // [iteration parity][action, sequence number, body blocks]
    const uint32_t t = threadIdx.x;
    fill_tables_regs(lds4, t0le[t], 32);
    uint32_t done = 0;
    uint64_t t_start = 0, t_idle = 0;
    if (t == 0) {
        done = load_acquire(&mb->resp.done);
        t_start = t_idle = wall_clock64();
    }
    __syncthreads();
    uint4 *io = reinterpret_cast<uint4 *>(mb->io + kSmallBodyAt - 16);
    for (uint32_t it = 0;; it++) {
        // Thread 0 polls until there is a request or a reason to leave; the other waves wait
        // at the barrier meanwhile (no barrier per poll).  An idle poll is one PCIe round trip:
        // the stop flag is a second read, made every 32nd poll only (engine teardown waits
        // for the idle exit anyway).
        if (t == 0) {  // 1 = serve, 2 = leave
            uint32_t action = 0, s = done, nb = 0;
            for (uint32_t np = 0; action == 0; np++) {
                uint32_t y;
                const u32x4_t h = load_sys16_and(&mb->req, yield, y);  // seq, op, len, head; batch word
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                s = h.x;
                const uint64_t now = wall_clock64();
                if (s != done) {
                    action = 1;
                    nb = (h.z - h.w + 15) >> 4;
                    nb = nb < kSmallMaxBytes / 16 ? nb : kSmallMaxBytes / 16;  // the host never asks for more
                } else if (y != y0 || now - t_idle > idle_ticks || now - t_start > life_ticks ||
                           ((np & 31u) == 31u &&
                            __hip_atomic_load(&mb->req.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) {
                    action = 2;
                } else {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            ctl[it & 1][0] = action;
            ctl[it & 1][1] = s;
            ctl[it & 1][2] = nb;
        }
        __syncthreads();
        const uint32_t action = ctl[it & 1][0], s = ctl[it & 1][1], nb = ctl[it & 1][2];
        if (action == 2) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // this wave sees the host's request
        // request header and the call's bytes into LDS
        if (t < sizeof(SmallReq) / 16)
            reinterpret_cast<uint4 *>(&rq)[t] = reinterpret_cast<const uint4 *>(&mb->req)[t];
        for (uint32_t i = t; i <= nb; i += kSmallThreads) S.buf[i] = io[i];
        __syncthreads();
        const uint4 iv = make_uint4(rq.iv[0], rq.iv[1], rq.iv[2], rq.iv[3]);
        uint32_t *st = mb->resp.state;
        const bool enc = rq.op & 1u;
        switch (rq.nrounds) {
            case 10:
                if (enc) small_body<10, true>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                else small_body<10, false>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                break;
            case 12:
                if (enc) small_body<12, true>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                else small_body<12, false>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                break;
            default:
                if (enc) small_body<14, true>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                else small_body<14, false>(rq.len, rq.head, rq.pos, iv, rq.rk, io, st, lds4, S);
                break;
        }
        __threadfence_system();
        __syncthreads();
        if (t == 0) {
            store_release(&mb->resp.done, s);
            done = s;
            t_idle = wall_clock64();
        }
    }
    if (t == 0) store_release(&mb->resp.exited, epoch);
}

// E_k(IV) of key slots: the keystream block every package-mode chain of a slot starts
// with (the IV is the same for every frame, core/Encryptor.cpp:12-19; SURVEY section 0,
// point 3).  The batch encrypt kernels use it for block 0 and skip its rounds where a whole
// wave starts its chains together.  One thread per slot, after every key-set write.
template <int NR>
__global__ __launch_bounds__(kSmallThreads, 1) void k_slot_eiv(const DevKey *keys, uint32_t first, uint32_t count,
                                                               const uint32_t *t0le, uint4 *eiv) {
    __shared__ uint4 lds4[Lds<4>::kBytes / 16];
    fill_tables_regs(lds4, t0le[threadIdx.x], 32);
    __syncthreads();
    const uint32_t i = blockIdx.x * kSmallThreads + threadIdx.x;
    if (i >= count) return;
    const Tables4<4> T{reinterpret_cast<const char *>(lds4), LaneBase()};
    const DevKey *k = keys + first + i;
    const RoundKeys<NR> rk = load_round_keys<NR>(k);
    eiv[first + i] = aes_encrypt_block<NR, 4>(*reinterpret_cast<const uint4 *>(k->iv), rk, T);
}

}  // namespace

hipError_t launch_slot_eiv(const DevKey *keys, uint32_t first, uint32_t count, int nrounds, const uint32_t *t0le,
                           uint4 *eiv, hipStream_t st) {
    if (count == 0) return hipSuccess;
    const dim3 grid((count + kSmallThreads - 1) / kSmallThreads);
    switch (nrounds) {
        case 10: hipLaunchKernelGGL(k_slot_eiv<10>, grid, dim3(kSmallThreads), 0, st, keys, first, count, t0le, eiv); break;
        case 12: hipLaunchKernelGGL(k_slot_eiv<12>, grid, dim3(kSmallThreads), 0, st, keys, first, count, t0le, eiv); break;
        case 14: hipLaunchKernelGGL(k_slot_eiv<14>, grid, dim3(kSmallThreads), 0, st, keys, first, count, t0le, eiv); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

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

hipError_t launch_cfb_server(SmallMailbox *mb, const uint32_t *t0le, uint32_t epoch, uint64_t idle_ticks,
                             uint64_t life_ticks, const uint32_t *yield, uint32_t y0, hipStream_t st) {
    set_launched("cfb_server");
    hipLaunchKernelGGL(k_cfb_server, dim3(1), dim3(kSmallThreads), 0, st, mb, t0le, epoch, idle_ticks, life_ticks,
                       yield, y0);
    return hipGetLastError();
}

}  // namespace fpnn_aes
