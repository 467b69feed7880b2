// engine.hip -- implementation of the C-ABI declared in include/fpnn_aes.h.
//
// Host-side responsibilities only: argument checking, key-set management, scratch
// sizing, choosing the kernel variant (uniform vs general layout, uniform vs
// per-packet keys, package vs stream, in-place) and queuing it on the engine's
// HIP stream.  There is no CPU cipher in this library: every byte of payload is
// transformed by the HIP kernels in k_encrypt.hip / k_decrypt.hip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdint>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/fpnn_aes.h"
#include "../../include/fpnn_ecdh.h"
#include "ecc.hpp"
#include "hostcopy.hpp"
#include "numa_place.hpp"
#include "aes_common.hpp"
#include "kernels.hpp"

using namespace fpnn_aes;

namespace {

thread_local std::string g_last_error;

// FPNN_AES_DEBUG_FAIL_CALL=N (tests only): the N-th host-data call of the process (cfb_host,
// package_host, stream_host, stream_recv -- the calls the C++ classes make) returns
// FPNN_AES_ERR_DEVICE as a failed device would, so the drop-in's failure contract can be
// driven through FPNN's own IO code (fail_policy.hpp, tests/test_gpu_dropin.py).
int debug_fail_point() {
    static const long long at = [] {
        const char *v = getenv("FPNN_AES_DEBUG_FAIL_CALL");
        return v ? atoll(v) : 0ll;
    }();
    if (at <= 0) return 0;
    static std::atomic<long long> calls{0};
    if (calls.fetch_add(1, std::memory_order_relaxed) + 1 != at) return 0;
    g_last_error = "injected device error (FPNN_AES_DEBUG_FAIL_CALL)";
    return FPNN_AES_ERR_DEVICE;
}

int hip_fail(hipError_t err, const char *what) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(err), (int)err);
    g_last_error = buf;
    return FPNN_AES_ERR_HIP;
}

#define HIP_TRY(expr)                                          \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return hip_fail(_e, #expr);      \
    } while (0)

struct EventPair {
    hipEvent_t beg, end;
};

// memcpy job of the host-frame gather/scatter
struct CopyJob {
    uint8_t *dst;
    const uint8_t *src;
    uint64_t n;
};

// Pinned host memory on `node` (the engine's NUMA placement; < 0: the runtime's default).
// hipHostMallocNumaUser makes the allocation follow the calling thread's memory policy,
// which NumaPreferScope points at the node for the call.
hipError_t pinned_host_alloc(int node, void **p, size_t n) {
    fpnn_aes::NumaPreferScope prefer(node);
    return hipHostMalloc(p, n, prefer.active() ? hipHostMallocNumaUser : 0u);
}

// One slot of the host-frame pipeline (fpnn_aes_package_host / fpnn_aes_stream_host):
// pinned + device staging and its own stream, so the copies of one chunk overlap the
// kernel of the other.
struct HostSlot {
    uint8_t *h = nullptr, *d = nullptr;
    uint64_t cap = 0;
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;    // chunk's D2H finished
    hipEvent_t staged = nullptr;  // chunk's H2D finished (the engine stream may cipher it)
    hipEvent_t kdone = nullptr;   // chunk's kernel finished (the slot stream may copy it back)
    bool busy = false;
    std::vector<CopyJob> scatter;  // staged output -> callers' buffers, run after `done`
    uint64_t scatter_bytes = 0;
    // package chunks scatter whole frames [first, first + count) straight from the staged
    // out_off array instead (no per-frame job list)
    const fpnn_aes_host_frame *frames = nullptr;
    uint32_t first = 0, count = 0;
    uint64_t pre = 0, out_at = 0;
    const uint64_t *out_off = nullptr;  // pinned, inside h
};

// One slot of the host-mapped frame pipeline (frames in memory registered with
// fpnn_aes_host_register): device staging for one chunk (input | output | descriptors),
// the pinned descriptor block the host fills, and the events that hand the chunk from
// the move stream to the engine stream and back.
struct MapSlot {
    uint8_t *d = nullptr;  // device: in | out | desc
    uint64_t dcap = 0;
    uint8_t *h = nullptr;  // pinned: desc
    uint64_t hcap = 0;
    hipEvent_t gathered = nullptr;  // chunk staged in HBM (the engine stream may cipher it)
    hipEvent_t ciphered = nullptr;  // cipher done (the move stream may scatter)
    hipEvent_t done = nullptr;      // the slot's descriptors went H2D (its pinned block is free)
    bool busy = false;
};

// Persistent host workers for the host-frame path.  Gathering 1M separate 1 KiB frames
// into pinned staging (and scattering the results back) is the host-memory-bound part
// of fpnn_aes_package_host; threads are kept across calls so a chunk does not pay
// thread start-up.  run(k, fn) calls fn(0..k-1) across the caller and k-1 workers.
class HostPool {
public:
    // workers run on the engine's NUMA placement (numa_place.hpp: the GPU's node's CPUs)
    HostPool(unsigned workers, const fpnn_aes::NumaPlacement &pl) : pl_(pl) {
        for (unsigned t = 0; t < workers; t++) th_.emplace_back([this, t] { loop(t + 1); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    // parts a host-frame call splits its copies into: this pool's threads + the caller,
    // shared fairly among the engines whose host-frame calls run at the same moment (every
    // engine has a pool of min(16, cores) threads: several IO threads flushing at once would
    // otherwise oversubscribe the box's CPU share many times over)
    // (per device: the GPU box grants each GPU its own CPU share)
    unsigned parts() const {
        const unsigned all = max_parts();
        const unsigned active = std::max(1u, g_host_active[device_ & 63].load(std::memory_order_relaxed));
        return std::max(1u, all / active);
    }
    unsigned max_parts() const { return (unsigned)th_.size() + 1; }
    void set_device(int d) { device_ = d; }
    static std::atomic<unsigned> g_host_active[64];

    template <class F>
    void run(unsigned want, const F &fn) {
        want = std::max(1u, std::min(want, max_parts()));
        if (want == 1) {
            fn(0u);
            return;
        }
        const std::function<void(unsigned)> f(fn);
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &f;
            active_ = want;
            pending_ = want - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

    // memcpy jobs split into contiguous, byte-balanced ranges
    void copy(const std::vector<CopyJob> &jobs, uint64_t total, unsigned want) {
        want = std::max(1u, std::min<unsigned>(want, (unsigned)std::min<size_t>(jobs.size(), max_parts())));
        std::vector<size_t> cut(want + 1, jobs.size());
        cut[0] = 0;
        uint64_t acc = 0;
        unsigned p = 1;
        for (size_t i = 0; i < jobs.size() && p < want; i++) {
            acc += jobs[i].n;
            while (p < want && acc >= total * p / want) cut[p++] = i + 1;
        }
        run(want, [&](unsigned q) {
            for (size_t i = cut[q]; i < cut[q + 1]; i++) copy_streaming(jobs[i].dst, jobs[i].src, jobs[i].n);
            copy_fence();
        });
    }

private:
    void loop(unsigned me) {
        (void)fpnn_aes::numa_pin_thread(pl_);
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (me >= active_) continue;
            const std::function<void(unsigned)> *f = fn_;
            lk.unlock();
            (*f)(me);
            lk.lock();
            if (--pending_ == 0) done_cv_.notify_one();
        }
    }

    const fpnn_aes::NumaPlacement pl_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)> *fn_ = nullptr;
    unsigned active_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
    int device_ = 0;
};

std::atomic<unsigned> HostPool::g_host_active[64];

// a host-frame call in progress on a device (HostPool::parts shares the copy threads
// among the calls of that device)
struct HostActive {
    int d;
    explicit HostActive(int device) : d(device & 63) { HostPool::g_host_active[d].fetch_add(1, std::memory_order_relaxed); }
    ~HostActive() { HostPool::g_host_active[d].fetch_sub(1, std::memory_order_relaxed); }
};


}  // namespace

struct fpnn_aes_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int num_cus = 256;
    Variant variant;
    uint8_t *d_tables = nullptr;  // t0le[256] (1 KiB), sbox[256], td0le[256] (1 KiB), isbox[256]
    // general-layout scratch
    uint64_t *d_bstart = nullptr;
    uint64_t cap_bstart = 0;
    uint4 *d_boundary = nullptr;
    uint64_t cap_boundary = 0;
    uint4 *d_snap_iv = nullptr;  // stream-decrypt state snapshot
    uint64_t cap_snap_iv = 0;
    uint32_t *d_snap_pos = nullptr;
    uint64_t cap_snap_pos = 0;
    uint32_t *d_perm = nullptr;  // ragged encrypt: longest-first order
    uint64_t cap_perm = 0;
    uint32_t *d_buckets = nullptr;  // the length-order block (kLengthOrderWords; zeroed when grown, then
    uint64_t cap_buckets = 0;       // zeroed again by its last reader, kernels.hpp)
    uint64_t *d_fr_off = nullptr;  // package receive: absolute body offset per frame slot
    uint64_t cap_fr_off = 0;
    uint32_t *d_fr_slot = nullptr;  // package receive: key slot per frame slot
    uint64_t cap_fr_slot = 0;
    RaggedPlan *d_plan = nullptr;  // K1r: one entry per wave of the decrypt grid
    uint64_t cap_plan = 0;
    uint4 *d_sink = nullptr;  // K1r: 2 x uint4 per wave, stores of lanes with nothing to store
    uint64_t cap_sink = 0;
    uint64_t *d_desc_off = nullptr;  // K1r: materialized in_off / len of stride / uniform batches
    uint64_t cap_desc_off = 0;
    uint32_t *d_desc_len = nullptr;
    uint64_t cap_desc_len = 0;
    uint64_t *d_total = nullptr;  // ragged block total (bstart[count]), device only
    uint64_t *d_lookback = nullptr;  // one-pass block map: tickets, epoch, tile status (zeroed when grown)
    uint64_t cap_lookback = 0;
    // device-side consistency checks (kFault*): a pinned word kernels may set, read when the
    // stream is idle (fpnn_aes_engine_sync, synchronous calls) and reported as FPNN_AES_ERR_DEVICE
    uint32_t *h_fault = nullptr;
    uint32_t *d_fault = nullptr;
    uint8_t *d_ecdh = nullptr;  // ECDH host forms / keyset: peers | keys | ivs | ok (grown, kept)
    uint64_t cap_ecdh = 0;
    uint8_t *d_sstate = nullptr;  // stream host frames: (iv, pos) of the call's streams (grown, kept)
    uint64_t cap_sstate = 0;
    uint8_t *h_sstate = nullptr;  // its pinned twin
    uint64_t cap_hsstate = 0;
    bool pools = false;            // stream-ordered allocation from `pool` for grow()
    hipMemPool_t mpool = nullptr;  // the engine's own memory pool (keeps freed scratch for reuse)
    std::vector<void *> deferred;  // grown-out scratch awaiting an idle stream (no pools)
    // K0 (k_small.hip): pinned staging of the small synchronous calls, its device view,
    // and the sequence number the kernel stores when a call is done
    uint8_t *h_small = nullptr;
    uint8_t *d_small = nullptr;
    uint32_t small_seq = 0;
    // K0s: the resident small-call server's mailbox (pinned), its device view, the last
    // request number and the epoch of the last server launched (0: none yet)
    SmallMailbox *h_mb = nullptr;
    SmallMailbox *d_mb = nullptr;
    uint32_t mb_seq = 0;
    uint32_t srv_epoch = 0;
    // the last batch work this engine queued while small-call servers exist on the device
    // (a server relaunch on another engine waits for it: batch_fence)
    hipEvent_t batch_ev = nullptr;
    std::atomic<bool> batch_pending{false};  // batch kernels about to be queued (batch_signal)
    std::atomic<bool> batch_ev_live{false};  // batch_ev marks the end of queued batch work
    uint64_t srv_idle_ticks = 0, srv_life_ticks = 0;
    // host staging for fpnn_aes_cfb_host
    uint8_t *h_stage = nullptr;
    uint8_t *d_stage = nullptr;
    uint64_t cap_stage = 0;
    // host-frame pipeline
    HostSlot hs[3];  // chunk i on slot i % 3: gather(i) runs beside scatter(i - 2)
    MapSlot ms[4];   // host-mapped chunks: gather(t) + scatter(t - 2) || cipher(t - 1), upload(t + 1)
    hipStream_t map_stream = nullptr;  // host-mapped moves (both PCIe directions in one launch)
    const char *host_path = "";  // "host_staged" / "host_mapped": the last host-frame call's path
    std::unique_ptr<HostPool> pool;  // created on first use
    fpnn_aes::NumaPlacement numa;    // where the pinned arenas and the pool's threads live
    // the address-audit build (audit.hpp): the extent table kernels check against
    AuditTable *d_aud = nullptr;
    // instrumentation
    bool timing = false;
    const char *last_kernel[2] = {"", ""};  // base name of the last main kernel per direction
    std::vector<EventPair> ev[2];
    size_t ev_used[2] = {0, 0};
};

struct fpnn_aes_keyset {
    fpnn_aes_engine *e = nullptr;  // creating engine (may be destroyed before the key set)
    int device = 0;
    DevKey *d_keys = nullptr;
    uint4 *d_eiv = nullptr;  // E_k(IV) per slot (launch_slot_eiv after every write)
    uint32_t count = 0;
    int nrounds = 0;
    uint32_t keylen = 0;
    // updatable tables (fpnn_aes_keyset_reserve / _set)
    uint32_t capacity = 0;
    DevKey *h_up = nullptr;    // pinned upload staging
    uint32_t cap_up = 0;       // DevKeys
    hipEvent_t up_done = nullptr;  // last upload out of h_up
    bool up_pending = false;
};

namespace {

// device table block: t0le (1 KiB) | sbox (256) | td0le (1 KiB) | isbox (256)
const uint32_t *t0le_of(const fpnn_aes_engine *e) { return reinterpret_cast<const uint32_t *>(e->d_tables); }
const uint8_t *sbox_of(const fpnn_aes_engine *e) { return e->d_tables + 1024; }
const uint32_t *td0le_of(const fpnn_aes_engine *e) { return reinterpret_cast<const uint32_t *>(e->d_tables + 1280); }
const uint8_t *isbox_of(const fpnn_aes_engine *e) { return e->d_tables + 2304; }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Scratch growth on the call path never frees synchronously: hipFree waits for the whole
// device, so one thread's first large call would stall every other engine's queued work.
// With stream-ordered pools the old buffer is released by hipFreeAsync behind the work
// already queued on this engine's stream; without them it is kept until the stream is
// next idle (engine_sync, the end of a synchronous host call, engine_destroy).
template <class T>
int grow(fpnn_aes_engine *e, T *&ptr, uint64_t &cap, uint64_t need) {
    if (need <= cap) return FPNN_AES_OK;
    uint64_t n = cap ? cap : 1024;
    while (n < need) n *= 2;
    T *np = nullptr;
    if (e->pools)
        HIP_TRY(hipMallocFromPoolAsync(reinterpret_cast<void **>(&np), n * sizeof(T), e->mpool, e->stream));
    else
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&np), n * sizeof(T)));
    if (ptr) {
        if (e->pools) HIP_TRY(hipFreeAsync(ptr, e->stream));
        else e->deferred.push_back(ptr);
    }
    ptr = np;
    cap = n;
    return FPNN_AES_OK;
}

// a grow()-managed buffer at engine teardown (the stream is idle)
void release_scratch(fpnn_aes_engine *e, void *p) {
    if (!p) return;
    if (e->pools) (void)hipFreeAsync(p, e->stream);
    else (void)hipFree(p);
}

void free_deferred(fpnn_aes_engine *e) {  // the engine's stream is idle
    for (void *p : e->deferred) (void)hipFree(p);
    e->deferred.clear();
}

// The engine's stream is idle: release grown-out scratch, and report (once) a consistency
// check a kernel failed since the last look (kernels.hpp, kFault*).
int stream_idle(fpnn_aes_engine *e) {
    free_deferred(e);
    const uint32_t f = e->h_fault ? __atomic_exchange_n(e->h_fault, 0u, __ATOMIC_ACQ_REL) : 0u;
    if (!f) return FPNN_AES_OK;
    if ((f & kFaultLengthOrder) && e->d_buckets)  // start the next ragged call from a zero block
        (void)hipMemsetAsync(e->d_buckets, 0, e->cap_buckets * sizeof(uint32_t), e->stream);
    g_last_error = (f & kFaultLookback)      ? "block map: a look-back gave up waiting for a tile (results of that call invalid)"
                   : (f & kFaultLengthOrder) ? "length order: bucket counts did not add up to the batch (results of that call invalid)"
                                             : "device-side check failed";
    return FPNN_AES_ERR_DEVICE;
}

// (below, with the small-call server)
void batch_signal(fpnn_aes_engine *e);
void batch_queued(fpnn_aes_engine *e);
void register_engine(fpnn_aes_engine *e);
void unregister_engine(fpnn_aes_engine *e);

// batch_signal for the lifetime of a call: the pending flag that batch_signal sets (and
// batch_queued clears once the kernels are queued) is cleared on EVERY exit, so a call
// that returns an error between the two never leaves other engines' server relaunches
// spinning out their batch_fence bound
struct BatchScope {
    fpnn_aes_engine *e;
    explicit BatchScope(fpnn_aes_engine *eng) : e(eng) { batch_signal(e); }
    ~BatchScope();
    BatchScope(const BatchScope &) = delete;
    BatchScope &operator=(const BatchScope &) = delete;
};

int timing_begin(fpnn_aes_engine *e, int which, EventPair **pair) {
    *pair = nullptr;
    if (!e->timing) return FPNN_AES_OK;
    auto &v = e->ev[which];
    if (e->ev_used[which] == v.size()) {
        EventPair p;
        HIP_TRY(hipEventCreate(&p.beg));
        HIP_TRY(hipEventCreate(&p.end));
        v.push_back(p);
    }
    *pair = &v[e->ev_used[which]++];
    HIP_TRY(hipEventRecord((*pair)->beg, e->stream));
    return FPNN_AES_OK;
}

// after the main kernel of a call: close its timing pair, remember what was launched
int timing_end(fpnn_aes_engine *e, EventPair *pair, int which) {
    e->last_kernel[which] = last_launched();
    batch_queued(e);
    if (pair) HIP_TRY(hipEventRecord(pair->end, e->stream));
    return FPNN_AES_OK;
}

// ceil(2^64 / d) for 1 <= d < 2^32
uint64_t magic_for(uint32_t d) {
    if (d == 1) return 0;  // unused: fast path divides by 1 via umulhi(g, 0) -> wrong, handled below
    const unsigned __int128 one = (unsigned __int128)1 << 64;
    return (uint64_t)((one + d - 1) / d);
}

int check_batch(const fpnn_aes_engine *e, const fpnn_aes_batch *b) {
    if (!e || !b || !b->keys) return FPNN_AES_ERR_ARG;
    if (b->count && (!b->in || !b->out)) return FPNN_AES_ERR_ARG;
    if (b->keys->device != e->device) return FPNN_AES_ERR_ARG;
    if (b->keys->count == 0) return FPNN_AES_ERR_ARG;
    return FPNN_AES_OK;
}

KBatch make_kbatch(const fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state) {
    KBatch k;
    memset(&k, 0, sizeof k);
    k.in = b->in;
    k.out = b->out;
    k.count = b->count;
    k.stride = b->stride;
    k.uniform_len = b->uniform_len;
    k.flags = b->flags;
    k.in_off = b->in_off;
    k.out_off = b->out_off;
    k.len = b->len;
    k.key_slot = b->key_slot;
    k.keys = b->keys->d_keys;
    k.iv_state = iv_state;
    k.pos_state = pos_state;
    k.t0le = t0le_of(e);
    k.eiv = b->keys->d_eiv;
    return k;
}

bool is_uniform_layout(const fpnn_aes_batch *b) {
    return !b->in_off && !b->out_off && !b->len && !b->key_slot;
}


#ifdef FPNN_AES_BOUNDS
// ---- the address-audit build (audit.hpp, `make audit`) ----------------------------------
// Before an encrypt call: the extents of every buffer the call's kernels may touch, in the
// engine's table (synchronous; the audit build is a checker, not a product).  The scratch
// the call grows is grown here first so that its extent is known.
int audit_begin(fpnn_aes_engine *e, const fpnn_aes_batch *b, const uint8_t *iv_state, const uint32_t *pos_state,
                KBatch &k) {
    int rc;
    if (!e->d_aud) HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_aud), sizeof(AuditTable)));
    if ((rc = grow(e, e->d_perm, e->cap_perm, b->count))) return rc;
    if ((rc = grow(e, e->d_sink, e->cap_sink, 2ull * e->num_cus * (kThreads / 64)))) return rc;
    if (kLengthOrderWords > e->cap_buckets) {
        if ((rc = grow(e, e->d_buckets, e->cap_buckets, kLengthOrderWords))) return rc;
        HIP_TRY(hipMemsetAsync(e->d_buckets, 0, e->cap_buckets * sizeof(uint32_t), e->stream));
    }
    HIP_TRY(hipStreamSynchronize(e->stream));
    AuditTable t;
    memset(&t, 0, sizeof t);
    const uint64_t n = b->count;
    auto set = [&](AuditBuf i, const void *p, uint64_t bytes) {
        if (!p) return;
        t.lo[i] = (uint64_t)(uintptr_t)p;
        t.hi[i] = t.lo[i] + bytes;
    };
    set(AB_IN_OFF, b->in_off, 8 * n);
    set(AB_OUT_OFF, b->out_off, 8 * n);
    set(AB_LEN, b->len, 4 * n);
    set(AB_SLOT, b->key_slot, 4 * n);
    const uint64_t slots = std::max<uint64_t>(b->keys->count, b->keys->capacity);
    set(AB_KEYS, b->keys->d_keys, sizeof(DevKey) * slots);
    set(AB_EIV, b->keys->d_eiv, 16 * slots);
    set(AB_IV_STATE, iv_state, 16 * n);
    set(AB_POS_STATE, pos_state, 4 * n);
    set(AB_POS_SNAP, pos_state, 4 * n);
    set(AB_PERM, e->d_perm, 4 * n);
    set(AB_SINK, e->d_sink, 16 * e->cap_sink);
    set(AB_BLOCK, e->d_buckets, 4 * (uint64_t)kLengthOrderWords);
    // the payload: the union of the segments' byte ranges (the kernels also check each
    // access against its own segment)
    std::vector<uint64_t> io(n), oo(n);
    std::vector<uint32_t> ln(n);
    if (b->in_off) HIP_TRY(hipMemcpy(io.data(), b->in_off, 8 * n, hipMemcpyDeviceToHost));
    else for (uint64_t i = 0; i < n; i++) io[i] = i * b->stride;
    if (b->out_off) HIP_TRY(hipMemcpy(oo.data(), b->out_off, 8 * n, hipMemcpyDeviceToHost));
    else oo = io;
    if (b->len) HIP_TRY(hipMemcpy(ln.data(), b->len, 4 * n, hipMemcpyDeviceToHost));
    else std::fill(ln.begin(), ln.end(), b->uniform_len);
    const uint64_t wire = (b->flags & FPNN_AES_F_WIRE_PREFIX) ? 4 : 0;
    uint64_t ilo = UINT64_MAX, ihi = 0, olo = UINT64_MAX, ohi = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (ln[i]) {
            ilo = std::min(ilo, io[i]);
            ihi = std::max(ihi, io[i] + ln[i]);
        }
        if (ln[i] + wire) {
            olo = std::min(olo, oo[i]);
            ohi = std::max(ohi, oo[i] + ln[i] + wire);
        }
    }
    if (ihi) set(AB_IN, b->in + ilo, ihi - ilo);
    else set(AB_IN, b->in, 1);  // (nothing may be read)
    if (ohi) set(AB_OUT, b->out + olo, ohi - olo);
    else set(AB_OUT, b->out, 1);
    // (the audit's own test: an `out` extent this many bytes short must be reported)
    if (const char *v = getenv("FPNN_AES_AUDIT_SHRINK_OUT"))
        if (t.hi[AB_OUT] > t.lo[AB_OUT] + (uint64_t)atoll(v)) t.hi[AB_OUT] -= (uint64_t)atoll(v);
    HIP_TRY(hipMemcpy(e->d_aud, &t, sizeof t, hipMemcpyHostToDevice));
    k.aud = e->d_aud;
    return FPNN_AES_OK;
}

const char *audit_buf_name(uint32_t i) {
    static const char *const names[kAuditBufs] = {"in", "out", "in_off", "out_off", "len", "key_slot", "keys", "eiv",
                                                  "iv_state", "pos_state", "perm", "sink", "length-order block",
                                                  "pos_snap", "in (outside its segment)", "out (outside its segment)"};
    return i < kAuditBufs ? names[i] : "?";
}

// After the call's kernels: wait, and report the first access outside its extent.
int audit_end(fpnn_aes_engine *e, int rc) {
    if (rc != FPNN_AES_OK || !e->d_aud) return rc;
    HIP_TRY(hipStreamSynchronize(e->stream));
    AuditTable t;
    HIP_TRY(hipMemcpy(&t, e->d_aud, sizeof t, hipMemcpyDeviceToHost));
    if (!t.hits) return FPNN_AES_OK;
    char buf[640];
    snprintf(buf, sizeof buf,
             "address audit: %u access(es) outside their extent; first: %s (%s) line %u, workgroup %u thread %u, "
             "bytes [0x%llx, +%llu) against [0x%llx, 0x%llx)",
             t.hits, last_launched(), audit_buf_name(t.buf), t.site, t.block, t.thread, (unsigned long long)t.addr,
             (unsigned long long)t.len, (unsigned long long)t.elo, (unsigned long long)t.ehi);
    g_last_error = buf;
    fprintf(stderr, "[fpnn_aes audit] %s\n", buf);
    return FPNN_AES_ERR_DEVICE;
}
#endif

int run_encrypt_calls(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state, bool stream);

int run_encrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state, bool stream) {
#ifdef FPNN_AES_BOUNDS
    return audit_end(e, run_encrypt_calls(e, b, iv_state, pos_state, stream));
#else
    return run_encrypt_calls(e, b, iv_state, pos_state, stream);
#endif
}

int run_encrypt_calls(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state, bool stream) {
    int rc = check_batch(e, b);
    if (rc) return rc;
    if (stream && b->count && (!iv_state || !pos_state || ((uintptr_t)iv_state & 15))) return FPNN_AES_ERR_ARG;
    if (!stream && (b->flags & FPNN_AES_F_WIRE_PREFIX) && (b->out_off == nullptr && b->in == b->out))
        return FPNN_AES_ERR_ARG;  // the 4-byte prefix needs a distinct output layout
    if (!b->count) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    const BatchScope batch_scope(e);  // (an early return clears the pending flag)
    KBatch k = make_kbatch(e, b, iv_state, pos_state);
#ifdef FPNN_AES_BOUNDS
    if ((rc = audit_begin(e, b, iv_state, pos_state, k))) return rc;
#endif
    const Layout layout = is_uniform_layout(b) ? LAYOUT_UNIFORM : LAYOUT_GENERAL;
    const KeyMode km = (b->key_slot && b->keys->count > 1) ? KEY_LANE : KEY_UNIFORM;
    // Few chains (fewer than the lanes of a full chip) or ragged lengths: one quad per
    // chain (K2c); otherwise one lane per chain with 8-block chunks (K2).
    const uint64_t full_chip = (uint64_t)e->num_cus * kThreads;

    // Ragged package batches of many short frames (the caller's max_len bound): one lane
    // per chain in grid-stride order (K2) -- Q1, 2 M x 145-B quests of 16 384 keyed
    // connections: 705 against K2h's 343 GiB/s (its work-queue atomics and length-order
    // indirection per chain; profiles/r05/ab_k2_short, ab_k2_align), from one chain per
    // GPU lane on (Q1h, 2 per lane: K2 767-770 against K2h 182-184 GiB/s,
    // profiles/r05/ab_k2_short_min).  Without a bound K2h, which also balances
    // Zipf-like lengths (C4 on K2: 88 GiB/s).
    const bool k2_ragged = b->len && !stream && b->max_len && b->max_len <= 2048 && b->count >= full_chip;
    if ((b->count < full_chip || b->len != nullptr) && !k2_ragged) {
        const uint64_t lanes = 4 * b->count;
        int threads = 64;
        while (threads < kThreads && (uint64_t)threads * e->num_cus < lanes) threads *= 2;
        const uint64_t want = (lanes + threads - 1) / threads;
        const int grid = (int)(want < (uint64_t)e->num_cus ? (want ? want : 1) : (uint64_t)e->num_cus);
        // ragged with more chains than quads: K2h (short chains one per lane, the longest
        // on quads, both from work queues); with fewer every quad holds at most one chain
        // and K2c's grid stride is cheaper
        const bool hybrid = b->len && b->count > 1 && (lanes > full_chip || e->variant.hyb_force);
        uint32_t *block = nullptr;  // the length-order block (ragged batches)
        // (everything that can fail is done before the length order is queued: its block is
        // left dirty until its last reader runs)
        if (hybrid && (rc = grow(e, e->d_sink, e->cap_sink, 2ull * e->num_cus * (kThreads / 64)))) return rc;
        if (b->len && b->count > 1) {  // ragged: visit the longest chains first, similar lengths per wave
            if ((rc = grow(e, e->d_perm, e->cap_perm, b->count))) return rc;
            if (kLengthOrderWords > e->cap_buckets) {  // starts zeroed; afterwards its last reader zeroes it
                if ((rc = grow(e, e->d_buckets, e->cap_buckets, kLengthOrderWords))) return rc;
                HIP_TRY(hipMemsetAsync(e->d_buckets, 0, e->cap_buckets * sizeof(uint32_t), e->stream));
            }
            if (stream) {  // bucket sizes read pos_state (the encrypt kernel reads it later)
                k.pos_snap = pos_state;
            }
            block = e->d_buckets;
            if (e->variant.poison_order > 0) {  // (tests) bucket counts left over as if by a lost call
                e->variant.poison_order--;
                HIP_TRY(hipMemsetAsync(block, 0x01, kWireFlagWord / 2 * sizeof(uint32_t), e->stream));
            }
            HIP_TRY(launch_length_order(k, stream, e->d_perm, block, !hybrid, e->d_fault, e->stream));
            k.perm = e->d_perm;
        }
        EventPair *ev;
        if ((rc = timing_begin(e, FPNN_AES_K_ENCRYPT, &ev))) {
            if (block) (void)hipMemsetAsync(block, 0, kLengthOrderWords * sizeof(uint32_t), e->stream);
            return rc;
        }
        if (hybrid) {  // K2h: one lane per chain, quads for the longest; one workgroup per CU
            k.flags |= F_ALIGN_CHUNKS;
            HybridArgs h;
            h.ctr = block + kTicketWords;
            h.buckets = block;
            h.long_bucket = length_bucket_of((uint64_t)e->variant.hyb_long);
            h.quad_waves = (uint32_t)e->variant.hyb_quad_waves;
            h.sink = e->d_sink;
            if (b->flags & FPNN_AES_F_WIRE_PREFIX) {
                // wire frames (htole32(len) || C): every chain on quads (k_hybrid.hip's
                // launcher takes the quads-only kernel for them)
                h.long_bucket = 127;
                h.quad_waves = 16;
            }
            HIP_TRY(launch_encrypt_hybrid(k, h, b->keys->nrounds, km, stream, e->num_cus, e->stream));
        } else {
            HIP_TRY(launch_encrypt_coop(k, b->keys->nrounds, layout, km, stream, grid, threads, e->stream));
        }
        return timing_end(e, ev, FPNN_AES_K_ENCRYPT);
    }
    // One lane per chain.  Workgroup size: the smallest power of two (>= one wave) that
    // still spreads the chains over every CU -- with few chains (C3: 4096 streams) a
    // 1024-thread workgroup would pack them onto a handful of CUs whose LDS they then
    // saturate, while the rest of the chip idles.
    const uint64_t slots = (uint64_t)e->num_cus;
    int threads = 64;
    while (threads < kThreads && (uint64_t)threads * slots < b->count) threads *= 2;
    const uint64_t want = (b->count + threads - 1) / threads;
    const int grid = (int)(want < slots ? (want ? want : 1) : slots);
    // (not for ragged batches by default, Variant::k2_align_ragged: a few 16-B aligned
    // frames per wave made the whole wave run their singles)
    if (!b->len) k.flags |= F_ALIGN_CHUNKS;
    EventPair *ev;
    if ((rc = timing_begin(e, FPNN_AES_K_ENCRYPT, &ev))) return rc;
    if (k2_ragged && b->max_len <= kFrameMaxBytes)  // FPNN's quests: whole frames at once (K2s-DB)
        HIP_TRY(launch_encrypt_frames(k, b->keys->nrounds, km, (b->flags & FPNN_AES_F_WIRE_PREFIX) != 0,
                                      e->num_cus, e->stream));
    else
        HIP_TRY(launch_encrypt_chains(k, b->keys->nrounds, layout, km, stream, grid, threads, e->stream));
    return timing_end(e, ev, FPNN_AES_K_ENCRYPT);
}

int run_decrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state, bool stream) {
    int rc = check_batch(e, b);
    if (rc) return rc;
    if (stream && b->count && (!iv_state || !pos_state || ((uintptr_t)iv_state & 15))) return FPNN_AES_ERR_ARG;
    if (b->flags & FPNN_AES_F_WIRE_PREFIX) return FPNN_AES_ERR_ARG;
    if (!b->count) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    const BatchScope batch_scope(e);  // (an early return clears the pending flag)
    KBatch k = make_kbatch(e, b, iv_state, pos_state);
    // small ragged batches: block map (+ stream snapshot) in one single-workgroup kernel
    const bool small_map = b->count <= block_map_small_max();
    if (stream) {  // snapshot the incoming (iv, pos) state, see KBatch::iv_snap
        if ((rc = grow(e, e->d_snap_iv, e->cap_snap_iv, b->count))) return rc;
        if ((rc = grow(e, e->d_snap_pos, e->cap_snap_pos, b->count))) return rc;
        if (!small_map) {  // (stream batches always take the general layout below)
            HIP_TRY(hipMemcpyAsync(e->d_snap_iv, iv_state, 16ull * b->count, hipMemcpyDeviceToDevice, e->stream));
            HIP_TRY(hipMemcpyAsync(e->d_snap_pos, pos_state, 4ull * b->count, hipMemcpyDeviceToDevice, e->stream));
        }
        k.iv_snap = e->d_snap_iv;
        k.pos_snap = e->d_snap_pos;
    }
    // In place whenever the buffers coincide (K1 / K1d: a wave may overwrite the
    // ciphertext block another wave's lane 0 still needs, so chunk boundaries are saved
    // first; K1r saves its waves' boundaries in its plan in any case).
    const bool inplace = b->in == b->out;
    const KeyMode km = (b->key_slot && b->keys->count > 1) ? KEY_LANE : KEY_UNIFORM;
    // Uniform layout: every segment has the same block count, known on the host.
    // (Stream mode only when there is a single segment, whose position the caller
    // supplies through the host path; otherwise positions differ per stream.)
    Layout layout = LAYOUT_GENERAL;
    if (is_uniform_layout(b) && !stream) {
        const uint64_t nb = ((uint64_t)b->uniform_len + 15) >> 4;
        const uint64_t total = nb * b->count;
        if (nb > 0 && total < (1ull << 32) && nb > 1) {
            layout = (b->uniform_len & 15) == 0 ? LAYOUT_FULL : LAYOUT_UNIFORM;
            k.total_blocks = total;
            k.nb_uniform = (uint32_t)nb;
            k.magic = magic_for((uint32_t)nb);
        }
    } else if (!stream && km == KEY_LANE && !b->in_off && !b->out_off && !b->len &&
               b->uniform_len >= 32 && b->uniform_len % 16 == 0 && b->stride == b->uniform_len) {
        // dense whole-block packets, one key slot each: K1d with a wave-uniform key per
        // step when packets are whole 64-block chunks (C5), K1k with per-lane keys
        // otherwise (U1)
        const uint64_t nb = b->uniform_len >> 4;
        const uint64_t total = nb * b->count;
        if (total < (1ull << 32)) {
            layout = LAYOUT_FULL;
            k.total_blocks = total;
            k.nb_uniform = (uint32_t)nb;
            k.magic = magic_for((uint32_t)nb);
        }
    }
    // Ragged package batches of FPNN's quests (the caller's max_len bound, at least one frame
    // per GPU lane): one lane per frame, its blocks decrypted as independent AES passes from
    // registers (D2s).  K1r's 64-block chunks span ~7 frames and key slots there.
    if (layout == LAYOUT_GENERAL && !stream && b->len && b->max_len && b->max_len <= kFrameMaxBytes &&
        b->count >= (uint64_t)e->num_cus * kThreads) {
        EventPair *ev = nullptr;
        if ((rc = timing_begin(e, FPNN_AES_K_DECRYPT, &ev))) return rc;
        HIP_TRY(launch_decrypt_frames(k, b->keys->nrounds, km, e->num_cus, e->stream));
        return timing_end(e, ev, FPNN_AES_K_DECRYPT);
    }
    if (layout == LAYOUT_GENERAL) {
        // K1r: block-map scan, per-wave plan and decrypt all on the device; the host
        // never learns the block total, so nothing here waits for the GPU
        if ((rc = grow(e, e->d_bstart, e->cap_bstart, b->count + 1))) return rc;
        const int grid = e->num_cus;
        if ((rc = grow(e, e->d_plan, e->cap_plan, (uint64_t)grid * (kThreads / 64)))) return rc;
        if ((rc = grow(e, e->d_sink, e->cap_sink, 2ull * grid * (kThreads / 64)))) return rc;
        if (small_map)
            HIP_TRY(launch_block_map_small(k, stream, iv_state, pos_state, e->d_snap_iv, e->d_snap_pos, e->d_bstart,
                                           e->d_total, e->stream));
        else {
            const uint64_t words = block_map_onepass_words(b->count);
            if (words > e->cap_lookback) {  // the kernel expects zeros on first use
                if ((rc = grow(e, e->d_lookback, e->cap_lookback, words))) return rc;
                HIP_TRY(hipMemsetAsync(e->d_lookback, 0, e->cap_lookback * sizeof(uint64_t), e->stream));
            }
            HIP_TRY(launch_block_map_onepass(k, stream, e->d_bstart, e->d_lookback, e->cap_lookback, e->d_fault,
                                             e->d_total, e->stream));
        }
        k.bstart = e->d_bstart;
        if (!k.in_off || !k.len) {  // K1r reads descriptor arrays: materialize the missing ones
            if (!k.in_off && (rc = grow(e, e->d_desc_off, e->cap_desc_off, b->count))) return rc;
            if (!k.len && (rc = grow(e, e->d_desc_len, e->cap_desc_len, b->count))) return rc;
            HIP_TRY(launch_ragged_desc(b->count, b->stride, b->uniform_len, k.in_off ? nullptr : e->d_desc_off,
                                       k.len ? nullptr : e->d_desc_len, e->stream));
            if (!k.in_off) k.in_off = e->d_desc_off;
            if (!k.len) k.len = e->d_desc_len;
        }
        if (!k.out_off) k.out_off = k.in_off;
        k.runs = (uint32_t)e->variant.k1r_runs;
        EventPair *ev = nullptr;
        if ((rc = timing_begin(e, FPNN_AES_K_DECRYPT, &ev))) return rc;
        // in place (in == out, identical offsets: fpnn_aes.h) the predecessor blocks of the
        // waves' first chunks are saved by a plan launch before any wave writes; otherwise
        // every wave finds its own at the start of the decrypt kernel (one launch fewer)
        HIP_TRY(launch_decrypt_ragged(k, b->keys->nrounds, km, stream, e->d_plan, e->d_sink, inplace, grid,
                                      e->stream));
        return timing_end(e, ev, FPNN_AES_K_DECRYPT);
    }
    EventPair *ev = nullptr;
    const uint64_t nchunks = (k.total_blocks + 63) >> 6;
    if (inplace) {
        if ((rc = grow(e, e->d_boundary, e->cap_boundary, nchunks))) return rc;
        HIP_TRY(launch_boundary_save(k, e->d_boundary, nchunks, e->stream));
        k.boundary = e->d_boundary;
    }
    const uint64_t want = (nchunks + 63) / 64;  // 16 waves per workgroup x up to 4 chunks per wave step
    const uint64_t cap = (uint64_t)e->num_cus;
    const int grid = (int)(want < cap ? (want ? want : 1) : cap);
    if ((rc = timing_begin(e, FPNN_AES_K_DECRYPT, &ev))) return rc;
    HIP_TRY(launch_decrypt_blocks(k, b->keys->nrounds, layout, km, inplace, grid, e->stream));
    return timing_end(e, ev, FPNN_AES_K_DECRYPT);
}

}  // namespace

// ===========================================================================
// C-ABI

extern "C" {

// (fpnn_aes_strerror lives in the front library, front.cpp: it must work without this one)

const char *fpnn_aes_last_error(void) { return g_last_error.c_str(); }

const char *fpnn_aes_version(void) {
    return "fpnn_aes 0.4 (gfx950; T-tables 32-way replicated in LDS; v_perm addressing; "
           "decrypt: K1d dense/keyed, K1k lane keys, K1r ragged (no host sync; interior runs), K1 uniform, "
           "one lane per block; encrypt: K2 lane per chain, K2c quad per chain, K2h lanes + quads for ragged "
           "batches; single calls <= 16 KiB: K0s resident server (K0 per launch); "
           "ECDH: one lane per derivation, special-prime folds as carry chains)";
}

int fpnn_aes_setup_encrypt(fpnn_aes_schedule *ctx, const uint8_t *key, size_t keylen) {
    if (!ctx || !key) return FPNN_AES_ERR_ARG;
    const int nr = expand_key_be(ctx->rk, key, keylen);
    ctx->nrounds = nr;
    return nr ? FPNN_AES_OK : FPNN_AES_ERR_KEYLEN;
}

int fpnn_aes_setup_decrypt(fpnn_aes_schedule *ctx, const uint8_t *key, size_t keylen) {
    if (!ctx || !key) return FPNN_AES_ERR_ARG;
    const int nr = expand_key_dec_be(ctx->rk, key, keylen);
    ctx->nrounds = nr;
    return nr ? FPNN_AES_OK : FPNN_AES_ERR_KEYLEN;
}

int fpnn_aes_device_count(int *count) {
    if (!count) return FPNN_AES_ERR_ARG;
    int n = 0;
    hipError_t err = hipGetDeviceCount(&n);
    if (err != hipSuccess) {
        *count = 0;
        hip_fail(err, "hipGetDeviceCount");
        return FPNN_AES_ERR_NODEV;
    }
    *count = n;
    return FPNN_AES_OK;
}

int fpnn_aes_engine_create(int device, void *hip_stream, fpnn_aes_engine **out) {
    if (!out) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        g_last_error = "no HIP device with that index";
        return FPNN_AES_ERR_NODEV;
    }
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        g_last_error = std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950";
        return FPNN_AES_ERR_NODEV;
    }
    DeviceGuard g(device);
    fpnn_aes_engine *e = new fpnn_aes_engine();
    e->device = device;
    e->num_cus = prop.multiProcessorCount;
    {  // the GPU's NUMA node: pinned arenas and copy threads go there (numa_place.hpp)
        char bdf[64] = {0};
        e->numa = fpnn_aes::numa_placement(hipDeviceGetPCIBusId(bdf, sizeof bdf, device) == hipSuccess ? bdf : nullptr);
    }
    // K2h split (tests set these so that small batches exercise each session)
    if (const char *v = getenv("FPNN_AES_HYB_LONG")) e->variant.hyb_long = std::max(1, atoi(v));
    if (const char *v = getenv("FPNN_AES_HYB_QW")) e->variant.hyb_quad_waves = std::min(16, std::max(0, atoi(v)));
    if (const char *v = getenv("FPNN_AES_HYB_FORCE")) e->variant.hyb_force = atoi(v) != 0;
    if (const char *v = getenv("FPNN_AES_DEBUG_POISON_ORDER")) e->variant.poison_order = std::max(0, atoi(v));
    if (const char *v = getenv("FPNN_AES_K1R_RUNS")) e->variant.k1r_runs = atoi(v) != 0;
    {  // stream-ordered scratch allocation from a pool of the engine's own: it keeps freed
       // memory for reuse (release threshold: never) without changing the device's
       // default pool, which other code in the process allocates from
        int pools = 0;
        const char *v = getenv("FPNN_AES_POOLS");
        if ((!v || atoi(v) != 0) &&
            hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, device) == hipSuccess && pools) {
            hipMemPoolProps props;
            memset(&props, 0, sizeof props);
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = device;
            if (hipMemPoolCreate(&e->mpool, &props) == hipSuccess) {
                uint64_t keep = UINT64_MAX;
                (void)hipMemPoolSetAttribute(e->mpool, hipMemPoolAttrReleaseThreshold, &keep);
                e->pools = true;
            } else {
                (void)hipGetLastError();
                e->mpool = nullptr;
            }
        }
    }
    int rc = FPNN_AES_OK;
    do {
        if (hip_stream != FPNN_AES_OWN_STREAM) {
            e->stream = (hipStream_t)hip_stream;  // NULL: the null stream
        } else {
            hipError_t err = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
            if (err != hipSuccess) { rc = hip_fail(err, "hipStreamCreate"); break; }
            e->own_stream = true;
        }
        hipError_t err = hipMalloc(reinterpret_cast<void **>(&e->d_tables), 2 * (1024 + 256));
        if (err != hipSuccess) { rc = hip_fail(err, "hipMalloc(tables)"); break; }
        err = hipMemcpy(e->d_tables, kTables.t0le, 1024, hipMemcpyHostToDevice);
        if (err == hipSuccess) err = hipMemcpy(e->d_tables + 1024, kTables.sbox, 256, hipMemcpyHostToDevice);
        if (err == hipSuccess) err = hipMemcpy(e->d_tables + 1280, kTables.td0le, 1024, hipMemcpyHostToDevice);
        if (err == hipSuccess) err = hipMemcpy(e->d_tables + 2304, kTables.isbox, 256, hipMemcpyHostToDevice);
        if (err != hipSuccess) { rc = hip_fail(err, "hipMemcpy(tables)"); break; }
        err = hipMalloc(reinterpret_cast<void **>(&e->d_total), sizeof(uint64_t));
        if (err != hipSuccess) { rc = hip_fail(err, "hipMalloc(total)"); break; }
        err = hipHostMalloc(reinterpret_cast<void **>(&e->h_fault), 64, hipHostMallocCoherent);
        if (err == hipSuccess) {
            *e->h_fault = 0;
            err = hipHostGetDevicePointer(reinterpret_cast<void **>(&e->d_fault), e->h_fault, 0);
        }
        if (err != hipSuccess) { rc = hip_fail(err, "hipHostMalloc(fault)"); break; }
    } while (0);
    if (rc) {
        fpnn_aes_engine_destroy(e);
        return rc;
    }
    register_engine(e);
    *out = e;
    return FPNN_AES_OK;
}

int fpnn_aes_engine_destroy(fpnn_aes_engine *e) {
    if (!e) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->d_tables);
    for (void *p : {(void *)e->d_bstart, (void *)e->d_boundary, (void *)e->d_snap_iv,
                    (void *)e->d_snap_pos, (void *)e->d_perm, (void *)e->d_buckets,
                    (void *)e->d_fr_off, (void *)e->d_fr_slot, (void *)e->d_plan, (void *)e->d_sink,
                    (void *)e->d_desc_off, (void *)e->d_desc_len, (void *)e->d_ecdh, (void *)e->d_sstate,
                    (void *)e->d_lookback})
        release_scratch(e, p);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    free_deferred(e);
    if (e->mpool) {  // (its blocks were freed above, behind the stream)
        (void)hipStreamSynchronize(e->stream);
        (void)hipMemPoolDestroy(e->mpool);
    }
    (void)hipFree(e->d_total);
    if (e->d_aud) (void)hipFree(e->d_aud);
    if (e->h_fault) (void)hipHostFree(e->h_fault);
    (void)hipFree(e->d_stage);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->h_small) (void)hipHostFree(e->h_small);
    if (e->h_mb) {  // the server left already (idle) or leaves now; the stream sync above waited
        __atomic_store_n(&e->h_mb->req.stop, 1u, __ATOMIC_RELEASE);
        if (e->stream) (void)hipStreamSynchronize(e->stream);
        (void)hipHostFree(e->h_mb);
    }
    if (e->h_sstate) (void)hipHostFree(e->h_sstate);
    for (auto &v : e->ev)
        for (auto &p : v) {
            (void)hipEventDestroy(p.beg);
            (void)hipEventDestroy(p.end);
        }
    for (auto &h : e->hs) {
        if (h.h) (void)hipHostFree(h.h);
        if (h.d) (void)hipFree(h.d);
        if (h.done) (void)hipEventDestroy(h.done);
        if (h.staged) (void)hipEventDestroy(h.staged);
        if (h.kdone) (void)hipEventDestroy(h.kdone);
        if (h.st) (void)hipStreamDestroy(h.st);
    }
    if (e->map_stream) (void)hipStreamSynchronize(e->map_stream);
    for (auto &m : e->ms) {
        if (m.h) (void)hipHostFree(m.h);
        if (m.d) (void)hipFree(m.d);
        if (m.gathered) (void)hipEventDestroy(m.gathered);
        if (m.ciphered) (void)hipEventDestroy(m.ciphered);
        if (m.done) (void)hipEventDestroy(m.done);
    }
    if (e->map_stream) (void)hipStreamDestroy(e->map_stream);
    unregister_engine(e);  // (no-op for an engine whose creation failed)
    if (e->batch_ev) (void)hipEventDestroy(e->batch_ev);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return FPNN_AES_OK;
}

int fpnn_aes_engine_sync(fpnn_aes_engine *e) {
    if (!e) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    HIP_TRY(hipStreamSynchronize(e->stream));
    return stream_idle(e);
}

void *fpnn_aes_engine_stream(fpnn_aes_engine *e) { return e ? (void *)e->stream : nullptr; }

// Devices the C++ classes' engine pool uses, in round-robin order (thread_engine.hpp).
static int pool_devices(int ndev, int *d, int cap) {
    int n = 0;
    if (const char *v = getenv("FPNN_AES_DEVICES")) {
        for (const char *p = v; *p && n < cap;) {
            char *end = nullptr;
            const long x = strtol(p, &end, 10);
            if (end == p) {
                p++;
                continue;
            }
            if (x >= 0 && x < ndev) d[n++] = (int)x;
            p = end;
        }
    } else if (const char *one = getenv("FPNN_AES_DEVICE")) {
        const int x = atoi(one);
        if (x >= 0 && x < ndev) d[n++] = x;
    } else {
        for (int i = 0; i < ndev && n < cap; i++) d[n++] = i;
    }
    return n;
}

int fpnn_aes_thread_engine_device(uint32_t k, int ndev) {
    int d[256];
    const int n = pool_devices(ndev, d, 256);
    return n ? d[k % (uint32_t)n] : -1;
}

int fpnn_aes_max_thread_engines(int ndev) {
    if (const char *v = getenv("FPNN_AES_MAX_ENGINES")) return std::max(1, atoi(v));
    int d[256];
    return std::max(1, 16 * pool_devices(ndev, d, 256));
}

int fpnn_aes_engine_reserve(fpnn_aes_engine *e, uint64_t max_segments, uint64_t max_blocks) {
    if (!e) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    int rc;
    if ((rc = grow(e, e->d_bstart, e->cap_bstart, max_segments + 1))) return rc;
    if (block_map_onepass_words(max_segments) > e->cap_lookback) {
        if ((rc = grow(e, e->d_lookback, e->cap_lookback, block_map_onepass_words(max_segments)))) return rc;
        HIP_TRY(hipMemsetAsync(e->d_lookback, 0, e->cap_lookback * sizeof(uint64_t), e->stream));
    }
    const uint64_t nchunks = (max_blocks + 63) / 64;
    if ((rc = grow(e, e->d_boundary, e->cap_boundary, nchunks + 1))) return rc;
    const uint64_t nwaves = (uint64_t)e->num_cus * (kThreads / 64);
    if ((rc = grow(e, e->d_plan, e->cap_plan, nwaves))) return rc;
    if ((rc = grow(e, e->d_sink, e->cap_sink, 2 * nwaves))) return rc;
    // ragged encrypt ordering, stream-decrypt snapshot, materialised descriptors
    if ((rc = grow(e, e->d_perm, e->cap_perm, max_segments))) return rc;
    if (kLengthOrderWords > e->cap_buckets) {
        if ((rc = grow(e, e->d_buckets, e->cap_buckets, kLengthOrderWords))) return rc;
        HIP_TRY(hipMemsetAsync(e->d_buckets, 0, e->cap_buckets * sizeof(uint32_t), e->stream));
    }
    if ((rc = grow(e, e->d_snap_iv, e->cap_snap_iv, max_segments))) return rc;
    if ((rc = grow(e, e->d_snap_pos, e->cap_snap_pos, max_segments))) return rc;
    if ((rc = grow(e, e->d_desc_off, e->cap_desc_off, max_segments))) return rc;
    if ((rc = grow(e, e->d_desc_len, e->cap_desc_len, max_segments))) return rc;
    return FPNN_AES_OK;
}

// ---- key sets ---------------------------------------------------------------

int fpnn_aes_keyset_create(fpnn_aes_engine *e, uint32_t count, size_t keylen, const uint8_t *keys,
                           const uint8_t *ivs, int keys_on_host, fpnn_aes_keyset **out) {
    if (!e || !out || !keys || count == 0) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    if (keylen != 16 && keylen != 24 && keylen != 32) return FPNN_AES_ERR_KEYLEN;
    DeviceGuard g(e->device);
    fpnn_aes_keyset *ks = new fpnn_aes_keyset();
    ks->e = e;
    ks->device = e->device;
    ks->count = count;
    ks->keylen = (uint32_t)keylen;
    ks->nrounds = (int)keylen / 4 + 6;
    uint8_t *d_raw = nullptr;
    int rc = FPNN_AES_OK;
    do {
        hipError_t err = hipMalloc(reinterpret_cast<void **>(&ks->d_keys), sizeof(DevKey) * (size_t)count);
        if (err != hipSuccess) { rc = hip_fail(err, "hipMalloc(keys)"); break; }
        const uint8_t *k_dev = keys, *iv_dev = ivs;
        if (keys_on_host) {
            const size_t kb = (size_t)count * keylen, ib = ivs ? (size_t)count * 16 : 0;
            err = hipMalloc(reinterpret_cast<void **>(&d_raw), kb + ib);
            if (err == hipSuccess) err = hipMemcpy(d_raw, keys, kb, hipMemcpyHostToDevice);
            if (err == hipSuccess && ivs) err = hipMemcpy(d_raw + kb, ivs, ib, hipMemcpyHostToDevice);
            if (err != hipSuccess) { rc = hip_fail(err, "upload(keys)"); break; }
            k_dev = d_raw;
            iv_dev = ivs ? d_raw + kb : nullptr;
        }
        err = launch_expand_keys(k_dev, (uint32_t)keylen, iv_dev, count, sbox_of(e), ks->d_keys, e->stream);
        if (err == hipSuccess) err = hipMalloc(reinterpret_cast<void **>(&ks->d_eiv), sizeof(uint4) * (size_t)count);
        if (err == hipSuccess)
            err = launch_slot_eiv(ks->d_keys, 0, count, ks->nrounds, t0le_of(e), ks->d_eiv, e->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "expand_keys"); break; }
    } while (0);
    if (d_raw) (void)hipFree(d_raw);
    if (rc) {
        fpnn_aes_keyset_destroy(ks);
        return rc;
    }
    *out = ks;
    return FPNN_AES_OK;
}

int fpnn_aes_keyset_from_schedules(fpnn_aes_engine *e, uint32_t count, const fpnn_aes_schedule *ctx,
                                   const uint8_t *ivs, fpnn_aes_keyset **out) {
    if (!e || !out || !ctx || count == 0) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    const int nr = ctx[0].nrounds;
    if (nr != 10 && nr != 12 && nr != 14) return FPNN_AES_ERR_KEYLEN;
    std::vector<DevKey> host(count);
    for (uint32_t i = 0; i < count; i++) {
        if (ctx[i].nrounds != nr) return FPNN_AES_ERR_ARG;
        DevKey &d = host[i];
        memset(&d, 0, sizeof d);
        for (int k = 0; k < 4 * (nr + 1); k++) d.rk[k] = bswap32(ctx[i].rk[k]);
        d.nrounds = (uint32_t)nr;
        d.keylen = (uint32_t)(nr - 6) * 4;
        if (ivs) memcpy(d.iv, ivs + 16 * (size_t)i, 16);
    }
    DeviceGuard g(e->device);
    fpnn_aes_keyset *ks = new fpnn_aes_keyset();
    ks->e = e;
    ks->device = e->device;
    ks->count = count;
    ks->nrounds = nr;
    ks->keylen = (uint32_t)(nr - 6) * 4;
    hipError_t err = hipMalloc(reinterpret_cast<void **>(&ks->d_keys), sizeof(DevKey) * (size_t)count);
    if (err == hipSuccess) err = hipMemcpy(ks->d_keys, host.data(), sizeof(DevKey) * (size_t)count, hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipMalloc(reinterpret_cast<void **>(&ks->d_eiv), sizeof(uint4) * (size_t)count);
    if (err == hipSuccess) err = launch_slot_eiv(ks->d_keys, 0, count, nr, t0le_of(e), ks->d_eiv, e->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) {
        int rc = hip_fail(err, "upload(schedules)");
        fpnn_aes_keyset_destroy(ks);
        return rc;
    }
    *out = ks;
    return FPNN_AES_OK;
}

int fpnn_aes_keyset_destroy(fpnn_aes_keyset *ks) {
    if (!ks) return FPNN_AES_OK;
    DeviceGuard g(ks->device);
    if (ks->up_done) {
        if (ks->up_pending) (void)hipEventSynchronize(ks->up_done);
        (void)hipEventDestroy(ks->up_done);
    }
    if (ks->h_up) (void)hipHostFree(ks->h_up);
    if (ks->d_keys) (void)hipFree(ks->d_keys);  // hipFree waits for outstanding work on the device
    if (ks->d_eiv) (void)hipFree(ks->d_eiv);
    delete ks;
    return FPNN_AES_OK;
}

int fpnn_aes_keyset_reserve(fpnn_aes_engine *e, uint32_t capacity, int nrounds, fpnn_aes_keyset **out) {
    if (!e || !out) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    if (nrounds != 10 && nrounds != 12 && nrounds != 14) return FPNN_AES_ERR_KEYLEN;
    capacity = std::max<uint32_t>(capacity, 1);
    DeviceGuard g(e->device);
    fpnn_aes_keyset *ks = new fpnn_aes_keyset();
    ks->e = e;
    ks->device = e->device;
    ks->nrounds = nrounds;
    ks->keylen = (uint32_t)(nrounds - 6) * 4;
    ks->capacity = capacity;
    hipError_t err = hipMalloc(reinterpret_cast<void **>(&ks->d_keys), sizeof(DevKey) * (size_t)capacity);
    if (err == hipSuccess) err = hipMemsetAsync(ks->d_keys, 0, sizeof(DevKey) * (size_t)capacity, e->stream);
    if (err == hipSuccess) err = hipMalloc(reinterpret_cast<void **>(&ks->d_eiv), sizeof(uint4) * (size_t)capacity);
    if (err == hipSuccess)  // (unset slots too: a batch naming one sees what the rounds would give)
        err = launch_slot_eiv(ks->d_keys, 0, capacity, nrounds, t0le_of(e), ks->d_eiv, e->stream);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&ks->up_done, hipEventDisableTiming);
    if (err != hipSuccess) {
        const int rc = hip_fail(err, "keyset_reserve");
        fpnn_aes_keyset_destroy(ks);
        return rc;
    }
    *out = ks;
    return FPNN_AES_OK;
}

int fpnn_aes_keyset_set(fpnn_aes_keyset *ks, uint32_t first, uint32_t count, const fpnn_aes_schedule *ctx,
                        const uint8_t *ivs) {
    if (!ks || !ks->e || (count && !ctx) || !ks->up_done) return FPNN_AES_ERR_ARG;
    if (count == 0) return FPNN_AES_OK;
    if ((uint64_t)first + count > 0xffffffffull) return FPNN_AES_ERR_RANGE;
    for (uint32_t i = 0; i < count; i++)
        if (ctx[i].nrounds != ks->nrounds) return FPNN_AES_ERR_KEYLEN;
    fpnn_aes_engine *e = ks->e;
    DeviceGuard g(ks->device);
    const uint32_t need = first + count;
    if (need > ks->capacity) {  // grow, keeping the table (queued after everything before it)
        uint32_t cap = ks->capacity;
        while (cap < need) cap = cap > 0x7fffffffu ? need : 2 * cap;
        DevKey *nk = nullptr;
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&nk), sizeof(DevKey) * (size_t)cap));
        HIP_TRY(hipMemsetAsync(nk + ks->capacity, 0, sizeof(DevKey) * (size_t)(cap - ks->capacity), e->stream));
        HIP_TRY(hipMemcpyAsync(nk, ks->d_keys, sizeof(DevKey) * (size_t)ks->capacity, hipMemcpyDeviceToDevice,
                               e->stream));
        uint4 *ne = nullptr;
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&ne), sizeof(uint4) * (size_t)cap));
        HIP_TRY(hipMemcpyAsync(ne, ks->d_eiv, sizeof(uint4) * (size_t)ks->capacity, hipMemcpyDeviceToDevice,
                               e->stream));
        HIP_TRY(launch_slot_eiv(nk, ks->capacity, cap - ks->capacity, ks->nrounds, t0le_of(e), ne, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));  // the old table may still be read by queued kernels
        (void)hipFree(ks->d_keys);
        (void)hipFree(ks->d_eiv);
        ks->d_keys = nk;
        ks->d_eiv = ne;
        ks->capacity = cap;
    }
    if (ks->up_pending) {  // the staging still feeds the previous upload
        HIP_TRY(hipEventSynchronize(ks->up_done));
        ks->up_pending = false;
    }
    if (count > ks->cap_up) {
        if (ks->h_up) (void)hipHostFree(ks->h_up);
        ks->h_up = nullptr;
        ks->cap_up = 0;
        const uint32_t c = std::max<uint32_t>(count, 256);
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&ks->h_up), sizeof(DevKey) * (size_t)c, 0));
        ks->cap_up = c;
    }
    for (uint32_t i = 0; i < count; i++) {
        DevKey &d = ks->h_up[i];
        memset(&d, 0, sizeof d);
        for (int k = 0; k < 4 * (ks->nrounds + 1); k++) d.rk[k] = bswap32(ctx[i].rk[k]);
        d.nrounds = (uint32_t)ks->nrounds;
        d.keylen = ks->keylen;
        if (ivs) memcpy(d.iv, ivs + 16 * (size_t)i, 16);
    }
    HIP_TRY(hipMemcpyAsync(ks->d_keys + first, ks->h_up, sizeof(DevKey) * (size_t)count, hipMemcpyHostToDevice,
                           e->stream));
    HIP_TRY(hipEventRecord(ks->up_done, e->stream));
    HIP_TRY(launch_slot_eiv(ks->d_keys, first, count, ks->nrounds, t0le_of(e), ks->d_eiv, e->stream));
    ks->up_pending = true;
    ks->count = std::max(ks->count, need);
    return FPNN_AES_OK;
}

uint32_t fpnn_aes_keyset_count(const fpnn_aes_keyset *ks) { return ks ? ks->count : 0; }

int fpnn_aes_keyset_nrounds(const fpnn_aes_keyset *ks) { return ks ? ks->nrounds : 0; }

int fpnn_aes_keyset_get_schedule(fpnn_aes_keyset *ks, uint32_t slot, fpnn_aes_schedule *out) {
    if (!ks || !out || slot >= ks->count) return FPNN_AES_ERR_ARG;
    DeviceGuard g(ks->device);
    DevKey d;
    HIP_TRY(hipMemcpy(&d, ks->d_keys + slot, sizeof d, hipMemcpyDeviceToHost));
    memset(out, 0, sizeof *out);
    out->nrounds = (int)d.nrounds;
    for (int k = 0; k < 4 * ((int)d.nrounds + 1); k++) out->rk[k] = bswap32(d.rk[k]);
    return FPNN_AES_OK;
}

// ---- batches ---------------------------------------------------------------------

int fpnn_aes_package_encrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b) {
    return run_encrypt(e, b, nullptr, nullptr, false);
}

int fpnn_aes_package_decrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b) {
    return run_decrypt(e, b, nullptr, nullptr, false);
}

int fpnn_aes_stream_encrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state) {
    if (b && (b->flags & FPNN_AES_F_WIRE_PREFIX)) return FPNN_AES_ERR_ARG;
    return run_encrypt(e, b, iv_state, pos_state, true);
}

int fpnn_aes_stream_decrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state) {
    return run_decrypt(e, b, iv_state, pos_state, true);
}

// ---- receive side: wire framing on the device ------------------------------------

int fpnn_aes_package_recv(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint32_t max_len, uint32_t max_frames,
                          uint64_t *frame_off, uint32_t *frame_len, fpnn_aes_frame_scan *scan) {
    int rc = check_batch(e, b);
    if (rc) return rc;
    if ((rc = debug_fail_point())) return rc;
    if (b->out_off || b->flags) return FPNN_AES_ERR_ARG;
    if (!b->count) return FPNN_AES_OK;
    if (!frame_off || !frame_len || !scan || !max_frames) return FPNN_AES_ERR_ARG;
    const uint64_t slots = (uint64_t)b->count * max_frames;
    if (slots > 0xffffffffull) return FPNN_AES_ERR_RANGE;
    DeviceGuard g(e->device);
    const bool per_key = b->key_slot && b->keys->count > 1;
    if ((rc = grow(e, e->d_fr_off, e->cap_fr_off, slots))) return rc;
    if (per_key && (rc = grow(e, e->d_fr_slot, e->cap_fr_slot, slots))) return rc;
    KScan s;
    memset(&s, 0, sizeof s);
    s.buf = b->in;
    s.count = b->count;
    s.off = b->in_off;
    s.stride = b->stride;
    s.len = b->len;
    s.uniform_len = b->uniform_len;
    s.max_len = max_len;
    s.key_slot = per_key ? b->key_slot : nullptr;
    s.max_frames = max_frames;
    s.frame_off = frame_off;
    s.frame_len = frame_len;
    s.scan = reinterpret_cast<ScanResult *>(scan);
    s.abs_off = e->d_fr_off;
    s.abs_slot = per_key ? e->d_fr_slot : nullptr;
    static_assert(sizeof(ScanResult) == sizeof(fpnn_aes_frame_scan), "scan layout");
    const BatchScope batch_scope(e);  // (an early return clears the pending flag)
    HIP_TRY(launch_scan_frames(s, false, e->num_cus, e->stream));
    batch_queued(e);
    // every frame slot is one package segment (unused ones have length 0)
    fpnn_aes_batch fb;
    memset(&fb, 0, sizeof fb);
    fb.in = b->in;
    fb.out = b->out;
    fb.count = (uint32_t)slots;
    fb.in_off = e->d_fr_off;
    fb.len = frame_len;
    fb.key_slot = per_key ? e->d_fr_slot : nullptr;
    fb.keys = b->keys;
    fb.max_len = max_len;  // (every frame the scan accepts is within it: D2s for FPNN's quests)
    return run_decrypt(e, &fb, nullptr, nullptr, false);
}

int fpnn_aes_stream_recv(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state,
                         const uint32_t *carry, uint32_t max_len, uint32_t max_frames, uint64_t *frame_off,
                         uint32_t *frame_len, fpnn_aes_frame_scan *scan) {
    int rc = check_batch(e, b);
    if (rc) return rc;
    if ((rc = debug_fail_point())) return rc;
    if (!b->count) return FPNN_AES_OK;
    if (!frame_off || !frame_len || !scan || !max_frames) return FPNN_AES_ERR_ARG;
    if ((uint64_t)b->count * max_frames > 0xffffffffull) return FPNN_AES_ERR_RANGE;
    if ((rc = run_decrypt(e, b, iv_state, pos_state, true))) return rc;
    DeviceGuard g(e->device);
    KScan s;
    memset(&s, 0, sizeof s);
    s.buf = b->out;
    s.count = b->count;
    s.off = b->out_off ? b->out_off : b->in_off;
    s.stride = b->stride;
    s.len = b->len;
    s.uniform_len = b->uniform_len;
    s.max_len = max_len;
    s.carry = carry;
    s.max_frames = max_frames;
    s.frame_off = frame_off;
    s.frame_len = frame_len;
    s.scan = reinterpret_cast<ScanResult *>(scan);
    const BatchScope batch_scope(e);  // (an early return clears the pending flag)
    HIP_TRY(launch_scan_frames(s, true, e->num_cus, e->stream));
    batch_queued(e);
    return FPNN_AES_OK;
}

// ---- single call from host memory ------------------------------------------------

}  // extern "C"

namespace {

// pinned + device staging of the synchronous single-call paths, grown on demand
int stage_reserve(fpnn_aes_engine *e, uint64_t need) {
    if (need <= e->cap_stage) return FPNN_AES_OK;
    uint64_t n = e->cap_stage ? e->cap_stage : 65536;
    while (n < need) n *= 2;
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    if (e->d_stage) (void)hipFree(e->d_stage);
    e->h_stage = nullptr;
    e->d_stage = nullptr;
    e->cap_stage = 0;
    HIP_TRY(pinned_host_alloc(e->numa.node, reinterpret_cast<void **>(&e->h_stage), n));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&e->d_stage), n));
    e->cap_stage = n;
    return FPNN_AES_OK;
}

// DevKey of a host schedule (rijndael_context layout, big-endian rk words)
void devkey_from_schedule(DevKey *hk, const fpnn_aes_schedule *ctx) {
    memset(hk, 0, sizeof *hk);
    for (int k = 0; k < 4 * (ctx->nrounds + 1); k++) hk->rk[k] = bswap32(ctx->rk[k]);
    hk->nrounds = (uint32_t)ctx->nrounds;
}

bool valid_rounds(int nr) { return nr == 10 || nr == 12 || nr == 14; }

// K0 for calls of up to kSmallMaxBytes (FPNN_AES_SMALL=0 routes them through the batch
// kernels, the A/B baseline).
bool small_enabled() {
    static const bool on = [] {
        const char *v = getenv("FPNN_AES_SMALL");
        return !v || atoi(v) != 0;
    }();
    return on;
}

// One small synchronous CFB call through K0 (k_small.hip): the bytes go into pinned
// staging, one launch ciphers them in place there, and the kernel's sequence-number store
// says the results are in.  The wait spins on that word; after 20 ms it falls back to the
// stream sync, which also reports a kernel that failed.
constexpr uint64_t kSmallStage = kSmallBodyAt + kSmallMaxBytes + 64;
int cfb_small_launch(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, bool encrypt, const uint8_t *in, uint8_t *out,
                     size_t len, uint8_t ivec[16], size_t *p_num) {
    if (!e->h_small) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_small), kSmallStage, hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&e->d_small), e->h_small, 0));
    }
    const uint32_t pos = (uint32_t)*p_num;
    const uint32_t head = pos ? (uint32_t)std::min<size_t>(len, 16 - pos) : 0u;
    memcpy(e->h_small + kSmallBodyAt - head, in, len);
    SmallArgs a;
    a.io = e->d_small;
    a.len = (uint32_t)len;
    a.head = head;
    a.pos = pos;
    a.seq = ++e->small_seq;
    memcpy(&a.iv, ivec, 16);
    for (int k = 0; k < 4 * (ctx->nrounds + 1); k++) a.rk[k] = bswap32(ctx->rk[k]);
    a.t0le = t0le_of(e);
    a.state = reinterpret_cast<uint32_t *>(e->d_small + kSmallStage - 32);
    volatile uint32_t *hstate = reinterpret_cast<volatile uint32_t *>(e->h_small + kSmallStage - 32);
    const int which = encrypt ? FPNN_AES_K_ENCRYPT : FPNN_AES_K_DECRYPT;
    EventPair *ev;
    if (int rc = timing_begin(e, which, &ev)) return rc;
    HIP_TRY(launch_cfb_single(a, ctx->nrounds, encrypt, e->stream));
    if (int rc = timing_end(e, ev, which)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0; __atomic_load_n(&hstate[5], __ATOMIC_ACQUIRE) != a.seq; spins++) {
        __builtin_ia32_pause();
        if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {
            HIP_TRY(hipStreamSynchronize(e->stream));
            if (__atomic_load_n(&hstate[5], __ATOMIC_ACQUIRE) != a.seq) {
                g_last_error = "small-call kernel finished without publishing its result";
                return FPNN_AES_ERR_HIP;
            }
            break;
        }
    }
    memcpy(out, e->h_small + kSmallBodyAt - head, len);
    for (int i = 0; i < 4; i++) {
        const uint32_t w = hstate[i];
        memcpy(ivec + 4 * i, &w, 4);
    }
    *p_num = hstate[4];
    return FPNN_AES_OK;
}

// K0s, the resident server (FPNN_AES_SMALL_SERVER=0: a K0 launch per call instead).  The
// request goes into the mailbox, its number last (release); if no server of this engine is
// alive one is launched on the engine stream (it starts after whatever is queued there);
// the host spins until the server stores the number into resp.done.  A server that left
// (idle, lifetime) before seeing the request is relaunched; after 20 ms of spinning the
// stream sync -- which returns once the server has left, and reports a failed kernel --
// settles it.
// Batch-activity words, one per device (64-byte apart) in pinned host memory, created with
// the first server: the host bumps its device's word before it queues batch kernels, and
// every server of that device leaves after its current request (kernels.hpp,
// launch_cfb_server).  An idle server would otherwise hold a CU -- and its hardware queue,
// which the box shares among streams (GPU_MAX_HW_QUEUES = 4) -- for up to its 2 ms
// lifetime while a persistent batch grid waits for it.
std::atomic<uint32_t *> g_yield{nullptr};
std::mutex g_yield_mu;

uint32_t *yield_words() {
    uint32_t *y = g_yield.load(std::memory_order_acquire);
    if (y) return y;
    std::lock_guard<std::mutex> lk(g_yield_mu);
    y = g_yield.load(std::memory_order_relaxed);
    if (!y) {
        void *p = nullptr;
        if (hipHostMalloc(&p, 64 * 64, hipHostMallocCoherent | hipHostMallocPortable | hipHostMallocMapped) != hipSuccess)
            return nullptr;
        memset(p, 0, 64 * 64);
        y = static_cast<uint32_t *>(p);
        g_yield.store(y, std::memory_order_release);
    }
    return y;
}

// before batch kernels are queued on a device (no-op until a server ever ran): servers
// leave, and no server is relaunched until the work is done (batch_fence)
void batch_signal(fpnn_aes_engine *e) {
    if (uint32_t *y = g_yield.load(std::memory_order_acquire)) {
        e->batch_pending.store(true, std::memory_order_release);
        __atomic_fetch_add(y + 16 * (e->device & 63), 1u, __ATOMIC_RELEASE);
    }
}

BatchScope::~BatchScope() { e->batch_pending.store(false, std::memory_order_release); }

// Engines per device, for batch_fence.
struct DeviceEngines {
    std::mutex mu;
    std::vector<fpnn_aes_engine *> list;
};
DeviceEngines g_dev_engines[64];

void register_engine(fpnn_aes_engine *e) {
    DeviceEngines &d = g_dev_engines[e->device & 63];
    std::lock_guard<std::mutex> lk(d.mu);
    d.list.push_back(e);
}

void unregister_engine(fpnn_aes_engine *e) {
    DeviceEngines &d = g_dev_engines[e->device & 63];
    std::lock_guard<std::mutex> lk(d.mu);
    d.list.erase(std::remove(d.list.begin(), d.list.end(), e), d.list.end());
}

// after an engine queued batch kernels (once servers exist): remember where they end
void batch_queued(fpnn_aes_engine *e) {
    if (!g_yield.load(std::memory_order_acquire)) return;  // no server ever ran: nothing waits
    if (e->batch_ev || hipEventCreateWithFlags(&e->batch_ev, hipEventDisableTiming) == hipSuccess)
        if (hipEventRecord(e->batch_ev, e->stream) == hipSuccess) e->batch_ev_live.store(true, std::memory_order_release);
    e->batch_pending.store(false, std::memory_order_release);
}

// Before (re)launching a small-call server: wait until the batch work other engines queued
// on this device has finished.  A server launched meanwhile would take a CU from a
// persistent batch grid (every workgroup holds a static share of the work, so the whole
// call waits for that CU) -- servers leave when batch work is queued (batch_signal), and
// do not come back until it is done.  The per-call request waits for the batch instead,
// which it would do anyway: the batch grid holds every CU.
// The wait is bounded (kBatchFenceMs): an engine that queues batch after batch would
// otherwise starve the per-call path; past the bound the server is launched and waits for
// a CU like any kernel.
void batch_fence(fpnn_aes_engine *e) {
    constexpr int kBatchFenceMs = 5;
    DeviceEngines &d = g_dev_engines[e->device & 63];
    std::lock_guard<std::mutex> lk(d.mu);
    const auto t0 = std::chrono::steady_clock::now();
    auto late = [&]() { return std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(kBatchFenceMs); };
    for (fpnn_aes_engine *o : d.list) {
        if (o == e) continue;
        for (uint32_t spins = 0;; spins++) {
            if (o->batch_pending.load(std::memory_order_acquire)) {  // its kernels are being queued
                __builtin_ia32_pause();
            } else if (o->batch_ev_live.load(std::memory_order_acquire)) {
                const hipError_t q = hipEventQuery(o->batch_ev);
                if (q != hipErrorNotReady) {
                    if (q == hipSuccess) o->batch_ev_live.store(false, std::memory_order_release);
                    break;
                }
                __builtin_ia32_pause();
            } else {
                break;
            }
            if ((spins & 255) == 255 && late()) return;
        }
    }
}

bool server_enabled() {
    static const bool on = [] {
        const char *v = getenv("FPNN_AES_SMALL_SERVER");
        return !v || atoi(v) != 0;
    }();
    return on;
}

// Relaunch order: read the device's batch-activity value y0 FIRST, then wait out batch
// work (batch_fence), then launch the server with y0.  A batch that signals after the read
// makes the server leave at its first poll; one that signalled before it set its pending
// flag first (batch_signal), so the fence waits for it.  (Reading y0 after the fence let a
// batch slip in between: its server then never saw a change and held a CU through it.)
int launch_server(fpnn_aes_engine *e) {
    if (!e->srv_idle_ticks) {
        int khz = 0;  // device wall clock (wall_clock64), kHz
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, e->device) != hipSuccess || khz <= 0)
            khz = 100000;
        e->srv_idle_ticks = (uint64_t)khz / 20;   // 50 us without a request
        e->srv_life_ticks = (uint64_t)khz * 2;    // 2 ms in any case
    }
    uint32_t *yh = yield_words();
    if (!yh) return hip_fail(hipErrorOutOfMemory, "hipHostMalloc(yield)");
    uint32_t *yd = nullptr;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&yd), yh + 16 * (e->device & 63), 0));
    const uint32_t y0 = __atomic_load_n(yh + 16 * (e->device & 63), __ATOMIC_ACQUIRE);
    batch_fence(e);
    const uint32_t epoch = ++e->srv_epoch;
    HIP_TRY(launch_cfb_server(e->d_mb, t0le_of(e), epoch, e->srv_idle_ticks, e->srv_life_ticks, yd, y0, e->stream));
    return FPNN_AES_OK;
}

int cfb_small_server(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, bool encrypt, const uint8_t *in, uint8_t *out,
                     size_t len, uint8_t ivec[16], size_t *p_num) {
    if (!e->h_mb) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_mb), sizeof(SmallMailbox), hipHostMallocCoherent));
        memset(e->h_mb, 0, sizeof(SmallMailbox));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void **>(&e->d_mb), e->h_mb, 0));
    }
    SmallMailbox *mb = e->h_mb;
    const uint32_t pos = (uint32_t)*p_num;
    const uint32_t head = pos ? (uint32_t)std::min<size_t>(len, 16 - pos) : 0u;
    memcpy(mb->io + kSmallBodyAt - head, in, len);
    mb->req.op = encrypt ? 1u : 0u;
    mb->req.len = (uint32_t)len;
    mb->req.head = head;
    mb->req.pos = pos;
    mb->req.nrounds = (uint32_t)ctx->nrounds;
    memcpy(mb->req.iv, ivec, 16);
    for (int k = 0; k < 4 * (ctx->nrounds + 1); k++) mb->req.rk[k] = bswap32(ctx->rk[k]);
    const uint32_t seq = ++e->mb_seq;
    __atomic_store_n(&mb->req.seq, seq, __ATOMIC_RELEASE);
    const int which = encrypt ? FPNN_AES_K_ENCRYPT : FPNN_AES_K_DECRYPT;
    e->last_kernel[which] = "cfb_server";
    // a server is alive unless none was launched or the last one has stored its epoch
    if (e->srv_epoch == 0 || __atomic_load_n(&mb->resp.exited, __ATOMIC_ACQUIRE) == e->srv_epoch) {
        if (int rc = launch_server(e)) return rc;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0; __atomic_load_n(&mb->resp.done, __ATOMIC_ACQUIRE) != seq; spins++) {
        __builtin_ia32_pause();
        if (__atomic_load_n(&mb->resp.exited, __ATOMIC_ACQUIRE) == e->srv_epoch &&
            __atomic_load_n(&mb->resp.done, __ATOMIC_ACQUIRE) != seq) {
            if (int rc = launch_server(e)) return rc;  // it left before seeing this request
            continue;
        }
        if ((spins & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) {
            HIP_TRY(hipStreamSynchronize(e->stream));
            if (__atomic_load_n(&mb->resp.done, __ATOMIC_ACQUIRE) != seq) {
                g_last_error = "small-call server left without serving the request";
                return FPNN_AES_ERR_HIP;
            }
            break;
        }
    }
    memcpy(out, mb->io + kSmallBodyAt - head, len);
    memcpy(ivec, mb->resp.state, 16);
    *p_num = mb->resp.state[4];
    return FPNN_AES_OK;
}

int cfb_small(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, bool encrypt, const uint8_t *in, uint8_t *out,
              size_t len, uint8_t ivec[16], size_t *p_num) {
    DeviceGuard g(e->device);
    return server_enabled() ? cfb_small_server(e, ctx, encrypt, in, out, len, ivec, p_num)
                            : cfb_small_launch(e, ctx, encrypt, in, out, len, ivec, p_num);
}

// One synchronous rijndael.h call in the non-CFB modes (k_modes.hip).  Staging:
// [DevKey 272][iv 16][pos 4 | pad 12][in: in_bytes, 16-padded][out: out_bytes]
int modes_call(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int mode, const uint8_t *in, uint64_t in_copy,
               uint64_t in_bytes, uint8_t *out, uint64_t out_copy, uint64_t nblocks, uint64_t len, uint8_t *ivec,
               size_t *p_num) {
    const uint64_t hdr = sizeof(DevKey) + 32;
    const uint64_t ipad = (in_bytes + 15) & ~15ull, opad = (std::max(out_copy, nblocks * 16) + 15) & ~15ull;
    DeviceGuard g(e->device);
    if (int rc = stage_reserve(e, hdr + ipad + opad)) return rc;
    devkey_from_schedule(reinterpret_cast<DevKey *>(e->h_stage), ctx);
    uint8_t *h_iv = e->h_stage + sizeof(DevKey);
    uint32_t *h_pos = reinterpret_cast<uint32_t *>(h_iv + 16);
    if (ivec) memcpy(h_iv, ivec, 16); else memset(h_iv, 0, 16);
    *h_pos = p_num ? (uint32_t)*p_num : 0u;
    if (in_copy) memcpy(e->h_stage + hdr, in, in_copy);
    if (ipad > in_copy) memset(e->h_stage + hdr + in_copy, 0, ipad - in_copy);  // CBC: zero padding
    HIP_TRY(hipMemcpyAsync(e->d_stage, e->h_stage, hdr + ipad, hipMemcpyHostToDevice, e->stream));
    ModeArgs a;
    a.in = e->d_stage + hdr;
    a.out = e->d_stage + hdr + ipad;
    a.nblocks = nblocks;
    a.len = len;
    a.key = reinterpret_cast<const DevKey *>(e->d_stage);
    a.iv = e->d_stage + sizeof(DevKey);
    a.pos = reinterpret_cast<uint32_t *>(a.iv + 16);
    a.t0le = t0le_of(e);
    a.td0le = td0le_of(e);
    a.isbox = isbox_of(e);
    HIP_TRY(launch_block_modes(a, ctx->nrounds, mode, e->num_cus, e->stream));
    e->last_kernel[FPNN_AES_K_ENCRYPT] = last_launched();
    HIP_TRY(hipMemcpyAsync(h_iv, a.iv, 32, hipMemcpyDeviceToHost, e->stream));
    if (out_copy) HIP_TRY(hipMemcpyAsync(e->h_stage + hdr + ipad, a.out, out_copy, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (int rf = stream_idle(e)) return rf;
    if (out_copy) memcpy(out, e->h_stage + hdr + ipad, out_copy);
    if (ivec && mode != MODE_CBC_DEC) memcpy(ivec, h_iv, 16);
    if (p_num) *p_num = *h_pos;
    return FPNN_AES_OK;
}

}  // namespace

extern "C" {

int fpnn_aes_ecb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt, const uint8_t *in, uint8_t *out,
                      size_t nblocks) {
    if (!e || !ctx || (nblocks && (!in || !out))) return FPNN_AES_ERR_ARG;
    if (!valid_rounds(ctx->nrounds)) return FPNN_AES_ERR_KEYLEN;
    if (!nblocks) return FPNN_AES_OK;
    return modes_call(e, ctx, encrypt ? MODE_ECB_ENC : MODE_ECB_DEC, in, 16ull * nblocks, 16ull * nblocks, out,
                      16ull * nblocks, nblocks, 0, nullptr, nullptr);
}

int fpnn_aes_cbc_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt, const uint8_t *in, uint8_t *out,
                      size_t len, uint8_t ivec[16]) {
    if (!e || !ctx || !ivec || (len && (!in || !out))) return FPNN_AES_ERR_ARG;
    if (!valid_rounds(ctx->nrounds)) return FPNN_AES_ERR_KEYLEN;
    if (!len) return FPNN_AES_OK;
    const uint64_t nb = (len + 15) / 16, whole = 16 * nb;
    if (encrypt)  // reads len bytes (the last block zero-padded), writes whole blocks
        return modes_call(e, ctx, MODE_CBC_ENC, in, len, whole, out, whole, nb, len, ivec, nullptr);
    // decrypt reads whole blocks, writes len bytes; ivec := the last ciphertext block
    uint8_t last[16];
    memcpy(last, in + whole - 16, 16);  // before an in-place call overwrites it
    const int rc = modes_call(e, ctx, MODE_CBC_DEC, in, whole, whole, out, len, nb, len, ivec, nullptr);
    if (rc == FPNN_AES_OK) memcpy(ivec, last, 16);
    return rc;
}

int fpnn_aes_ofb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, const uint8_t *in, uint8_t *out, size_t len,
                      uint8_t ivec[16], size_t *p_num) {
    if (!e || !ctx || !ivec || !p_num || (len && (!in || !out))) return FPNN_AES_ERR_ARG;
    if (!valid_rounds(ctx->nrounds)) return FPNN_AES_ERR_KEYLEN;
    if (*p_num > 15) return FPNN_AES_ERR_ARG;
    if (!len) return FPNN_AES_OK;
    return modes_call(e, ctx, MODE_OFB, in, len, len, out, len, 0, len, ivec, p_num);
}

int fpnn_aes_cfb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt, const uint8_t *in,
                      uint8_t *out, size_t len, uint8_t ivec[16], size_t *p_num) {
    if (!e || !ctx || !ivec || !p_num || (len && (!in || !out))) return FPNN_AES_ERR_ARG;
    if (int rc = debug_fail_point()) return rc;
    const int nr = ctx->nrounds;
    if (nr != 10 && nr != 12 && nr != 14) return FPNN_AES_ERR_KEYLEN;
    if (*p_num > 15) return FPNN_AES_ERR_ARG;
    if (len == 0) return FPNN_AES_OK;
    if (len > 0xffffffffull) return FPNN_AES_ERR_RANGE;
    if (len <= kSmallMaxBytes && small_enabled()) return cfb_small(e, ctx, encrypt != 0, in, out, len, ivec, p_num);
    DeviceGuard g(e->device);
    // staging layout: [DevKey 272][iv 16][pos 4 | pad 12][payload len] ... [out len]
    const uint64_t hdr = sizeof(DevKey) + 32;
    const uint64_t pay = (len + 15) & ~15ull;
    if (int rc = stage_reserve(e, hdr + 2 * pay)) return rc;
    devkey_from_schedule(reinterpret_cast<DevKey *>(e->h_stage), ctx);
    uint8_t *h_iv = e->h_stage + sizeof(DevKey);
    uint32_t *h_pos = reinterpret_cast<uint32_t *>(h_iv + 16);
    memcpy(h_iv, ivec, 16);
    *h_pos = (uint32_t)*p_num;
    memcpy(e->h_stage + hdr, in, len);
    // (Letting the kernels read and write the pinned staging block directly instead of the
    // three copies measured the same per-call time, 71 / 32 us: the launches and the sync
    // are the cost, not the copies.)
    HIP_TRY(hipMemcpyAsync(e->d_stage, e->h_stage, hdr + len, hipMemcpyHostToDevice, e->stream));

    fpnn_aes_keyset ks;
    ks.e = e;
    ks.device = e->device;
    ks.d_keys = reinterpret_cast<DevKey *>(e->d_stage);
    ks.count = 1;
    ks.nrounds = nr;
    ks.keylen = (uint32_t)(nr - 6) * 4;
    uint8_t *d_iv = e->d_stage + sizeof(DevKey);
    uint32_t *d_pos = reinterpret_cast<uint32_t *>(d_iv + 16);
    fpnn_aes_batch b;
    memset(&b, 0, sizeof b);
    b.in = e->d_stage + hdr;
    b.out = e->d_stage + hdr + pay;
    b.count = 1;
    b.uniform_len = (uint32_t)len;
    b.stride = 0;
    b.keys = &ks;
    int rc = encrypt ? run_encrypt(e, &b, d_iv, d_pos, true) : run_decrypt(e, &b, d_iv, d_pos, true);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h_iv, d_iv, 32, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipMemcpyAsync(e->h_stage + hdr + pay, e->d_stage + hdr + pay, len, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (int rf = stream_idle(e)) return rf;
    memcpy(out, e->h_stage + hdr + pay, len);
    memcpy(ivec, h_iv, 16);
    *p_num = *h_pos;
    return FPNN_AES_OK;
}

// ---- many frames from host memory -----------------------------------------------------

namespace {

// Host threads for gathering/scattering frames: FPNN_AES_HOST_THREADS, default
// min(16, hardware threads) -- the GPU box grants a 16-CPU share per GPU.
unsigned host_threads() {
    unsigned hw = std::thread::hardware_concurrency();
    unsigned n = std::min(16u, hw ? hw : 1u);
    if (const char *v = getenv("FPNN_AES_HOST_THREADS")) n = (unsigned)std::max(1, atoi(v));
    return std::min(n, 64u);  // package chunks keep per-part sums in a 64-entry array
}

HostPool *pool_of(fpnn_aes_engine *e) {
    if (!e->pool) {
        e->pool.reset(new HostPool(host_threads() - 1, e->numa));
        e->pool->set_device(e->device);
    }
    return e->pool.get();
}

// parts for `bytes` of copying: about 1 MiB per thread at least
unsigned copy_parts(fpnn_aes_engine *e, uint64_t bytes) {
    // 1 MiB per copy thread (256 KiB / 64 KiB grains measured within run-to-run spread on
    // the IO-plumbing echo, profiles/r05/io_multi/r05cg_*; the A/B switch was removed in round 6)
    constexpr int grain = 20;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(pool_of(e)->parts(), bytes >> grain));
}

void parallel_copy(fpnn_aes_engine *e, const std::vector<CopyJob> &jobs, uint64_t total) {
    pool_of(e)->copy(jobs, total, copy_parts(e, total));
}

int slot_reserve(HostSlot &s, int node, uint64_t need) {
    if (!s.st) {
        HIP_TRY(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s.staged, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&s.kdone, hipEventDisableTiming));
    }
    if (need <= s.cap) return FPNN_AES_OK;
    uint64_t n = s.cap ? s.cap : (8u << 20);
    while (n < need) n *= 2;
    if (s.h) (void)hipHostFree(s.h);
    if (s.d) (void)hipFree(s.d);
    s.h = nullptr;
    s.d = nullptr;
    s.cap = 0;
    HIP_TRY(pinned_host_alloc(node, reinterpret_cast<void **>(&s.h), n));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&s.d), n));
    s.cap = n;
    return FPNN_AES_OK;
}

// FPNN_AES_HOST_STATS=1: per-call breakdown of the host-frame pipeline on stderr
struct HostStats {
    bool on = getenv("FPNN_AES_HOST_STATS") != nullptr;
    double gather = 0, scatter = 0, wait = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};

// part p of `parts` of a package chunk's scatter (whole frames, straight from the staged
// out_off array)
void scatter_frames_part(const HostSlot &s, unsigned p, unsigned parts) {
    const uint32_t a = (uint32_t)((uint64_t)s.count * p / parts), b = (uint32_t)((uint64_t)s.count * (p + 1) / parts);
    for (uint32_t t = a; t < b; t++) {
        const fpnn_aes_host_frame &f = s.frames[s.first + t];
        copy_streaming(f.dst, s.h + s.out_at + s.out_off[t], f.len + s.pre);
    }
    copy_fence();
}

// wait for a slot's chunk and scatter its outputs to the callers' buffers
int slot_drain(fpnn_aes_engine *e, HostSlot &s, HostStats &st) {
    if (!s.busy) return FPNN_AES_OK;
    s.busy = false;
    const double t0 = st.on ? HostStats::now() : 0;
    HIP_TRY(hipEventSynchronize(s.done));
    const double t1 = st.on ? HostStats::now() : 0;
    if (s.frames) {
        const unsigned parts = copy_parts(e, s.scatter_bytes);
        pool_of(e)->run(parts, [&](unsigned p) { scatter_frames_part(s, p, parts); });
        s.frames = nullptr;
    } else {
        parallel_copy(e, s.scatter, s.scatter_bytes);
    }
    if (st.on) {
        st.wait += t1 - t0;
        st.scatter += HostStats::now() - t1;
    }
    return FPNN_AES_OK;
}

}  // namespace

// ---- utilities --------------------------------------------------------------------------

namespace {

// A contiguous part of one frame's bytes, in staging order.
struct Piece {
    uint32_t frame, off, len;
};

// stream-state scratch of the host-frame calls: device (grow(): no free on the call path)
// and its pinned twin (grown only between calls' uses: the engine stream is drained)
int sstate_reserve(fpnn_aes_engine *e, uint64_t bytes) {
    if (int rc = grow(e, e->d_sstate, e->cap_sstate, bytes)) return rc;
    if (bytes > e->cap_hsstate) {
        uint64_t c = e->cap_hsstate ? e->cap_hsstate : 4096;
        while (c < bytes) c *= 2;
        HIP_TRY(hipStreamSynchronize(e->stream));  // a previous call's state copies are done
        if (e->h_sstate) (void)hipHostFree(e->h_sstate);
        e->h_sstate = nullptr;
        e->cap_hsstate = 0;
        HIP_TRY(pinned_host_alloc(e->numa.node, reinterpret_cast<void **>(&e->h_sstate), c));
        e->cap_hsstate = c;
    }
    return FPNN_AES_OK;
}

// Stream-mode host frames grouped by stream: order[] lists the frame indices by key slot,
// each stream's frames in array order (a stable sort), and segs the streams that carry
// bytes, in slot order ({slot, first, nframes, bytes}: frames order[first .. +nframes)).
// A serial counting sort whose first pass also sums each slot's bytes, so the segments
// come from the histogram, not from a walk of frames[order[i]] (one cache miss per frame
// in arrival order).  A parallel form on the host pool (per-part histograms, prefix over
// slot ranges, per-part placement) measured 5-8 ms per 1M frames on the GPU box against
// this form's 3 (S1, gpurun_out r04k / r04l): four pool passes over a 16-CPU share cost
// more than they split.  Sparse slot ranges take std::stable_sort.
struct StreamSeg {
    uint32_t slot, first, nframes;
    uint64_t bytes;
};

void group_streams(const fpnn_aes_host_frame *frames, uint32_t n, uint32_t nkeys, std::vector<uint32_t> &order,
                   std::vector<StreamSeg> &segs) {
    order.resize(n);
    segs.clear();
    if ((uint64_t)nkeys > 4ull * n + 1024) {  // sparse
        for (uint32_t i = 0; i < n; i++) order[i] = i;
        std::stable_sort(order.begin(), order.end(),
                         [frames](uint32_t x, uint32_t y) { return frames[x].key_slot < frames[y].key_slot; });
        for (uint32_t i = 0; i < n;) {
            const uint32_t slot = frames[order[i]].key_slot;
            uint32_t j = i;
            uint64_t bytes = 0;
            while (j < n && frames[order[j]].key_slot == slot) bytes += frames[order[j++]].len;
            if (bytes) segs.push_back({slot, i, j - i, bytes});  // empty streams keep their state
            i = j;
        }
        return;
    }
    std::vector<uint32_t> cnt((size_t)nkeys + 1, 0);
    std::vector<uint64_t> byt(nkeys, 0);
    for (uint32_t i = 0; i < n; i++) {
        cnt[frames[i].key_slot + 1]++;
        byt[frames[i].key_slot] += frames[i].len;
    }
    for (uint32_t k = 0; k < nkeys; k++) {
        if (byt[k]) segs.push_back({k, cnt[k], cnt[k + 1], byt[k]});
        cnt[k + 1] += cnt[k];
    }
    for (uint32_t i = 0; i < n; i++) order[cnt[frames[i].key_slot]++] = i;
}

// Host-frame pipeline shared by the package and stream entry points.
//   package: one segment per frame (key slot frames[i].key_slot, fresh chain).
//   stream : one segment per distinct stream slot = the concatenation of that
//            stream's frames in array order (CFB over a concatenation equals the
//            successive calls, base/rijndael.c:1171-1201 carries ivec/num), whose
//            state lives in iv_state/pos_state[slot] on the host.
// Chunks of <= kChunk input bytes are gathered into pinned staging by the copy pool,
// then H2D and D2H run on the slot's stream and the kernel on the engine stream (events
// hand the chunk over) while the host gathers the next chunk.  Kernels of successive
// chunks are therefore ordered: they share the engine's scratch, and in stream mode a
// stream split across chunks continues from the state the previous chunk left.
int host_pipeline(fpnn_aes_engine *e, bool encrypt, bool stream, const fpnn_aes_host_frame *frames, uint32_t n,
                  const fpnn_aes_keyset *keys, uint32_t flags, uint8_t *iv_state, uint32_t *pos_state) {
    const HostActive active_call(e->device);
    const uint64_t pre = (!stream && (flags & FPNN_AES_F_WIRE_PREFIX)) ? 4 : 0;
    // input bytes per pipeline chunk.  (Quarter-call chunks for small calls, so one IO
    // cycle's 8 MiB flush would overlap its steps, measured slower: 1.37 against 0.83 ms
    // per flush, each chunk's copies getting fewer threads, gpurun_out r05d.)
    const uint64_t kChunk = 32ull << 20;
    // ---- segments in staging order -------------------------------------------------
    std::vector<uint32_t> order;  // frame indices
    std::vector<StreamSeg> segs;  // stream mode only (package chunks walk `frames` directly)
    if (stream) group_streams(frames, n, keys->count, order, segs);
    if (stream && segs.empty()) return FPNN_AES_OK;
    e->host_path = "host_staged";
    const uint64_t nseg = stream ? segs.size() : n;
    HostStats hst;
    const double t_call = hst.on ? HostStats::now() : 0;
    uint64_t nchunks = 0;
    DeviceGuard g(e->device);
    hipStream_t main_stream = e->stream;
    // order the slot streams after work already queued on the engine stream
    for (auto &sl : e->hs)
        if (int rc = slot_reserve(sl, e->numa.node, 0)) return rc;
    HIP_TRY(hipEventRecord(e->hs[0].kdone, main_stream));
    for (auto &sl : e->hs) HIP_TRY(hipStreamWaitEvent(sl.st, e->hs[0].kdone, 0));
    // ---- stream state: compact (iv, pos) of the touched streams on the device ----------
    uint8_t *d_state = nullptr, *h_state = nullptr;
    // stream round-robin cursors: bytes left, frame cursor, host model of pos (for the
    // decrypt block count) per segment
    struct {
        std::vector<uint64_t> rem;
        std::vector<uint32_t> fi, fo, pos;
        uint64_t left = 0, next = 0, chunk = 0, quota = 0;
    } sr;
    if (stream) {
        const uint64_t bytes = nseg * 20;
        if (int rc = sstate_reserve(e, bytes)) return rc;
        h_state = e->h_sstate;
        d_state = e->d_sstate;
        // (a fresh d_state is stream-ordered on the engine stream: the upload below waits for it)
        HIP_TRY(hipEventRecord(e->hs[0].kdone, main_stream));
        HIP_TRY(hipStreamWaitEvent(e->hs[0].st, e->hs[0].kdone, 0));
        sr.rem.resize(nseg);
        sr.fi.assign(nseg, 0);
        sr.fo.assign(nseg, 0);
        sr.pos.resize(nseg);
        uint32_t *hp = reinterpret_cast<uint32_t *>(h_state + 16 * nseg);
        for (uint64_t t = 0; t < nseg; t++) {
            memcpy(h_state + 16 * t, iv_state + 16ull * segs[t].slot, 16);
            hp[t] = sr.pos[t] = pos_state[segs[t].slot] & 15u;
            sr.rem[t] = segs[t].bytes;
            sr.left += segs[t].bytes;
        }
        // bigger chunks for few long streams (more chain steps per launch), quota per
        // stream so one chunk spans as many streams as it can
        sr.chunk = std::min<uint64_t>(256ull << 20, std::max<uint64_t>(kChunk, sr.left / 4));
        sr.quota = std::max<uint64_t>(16u << 10, (sr.chunk / nseg + 15) & ~15ull);
        (void)hipMemcpyAsync(d_state, h_state, bytes, hipMemcpyHostToDevice, e->hs[0].st);
    }
    int rc = FPNN_AES_OK;
    uint64_t si = 0;  // package: next segment; stream: nseg once every byte is queued
    int k = 0;
    HostSlot *prev = nullptr;
    std::vector<Piece> pieces;
    std::vector<CopyJob> gather;
    const int kSlots = (int)(sizeof(e->hs) / sizeof(e->hs[0]));
    while (si < nseg && rc == FPNN_AES_OK) {
        HostSlot &s = e->hs[k];
        if ((rc = slot_drain(e, s, hst))) break;  // package: already scattered beside a gather
        // package: the chunk two back is scattered by half the copy threads while the other
        // half gathers this one (host memory, not one thread group, is the limit)
        HostSlot *sc = nullptr;
        if (!stream) {
            HostSlot &o = e->hs[(k + 1) % kSlots];
            if (o.busy && o.frames) {
                const double tw = hst.on ? HostStats::now() : 0;
                HIP_TRY(hipEventSynchronize(o.done));
                if (hst.on) hst.wait += HostStats::now() - tw;
                o.busy = false;
                sc = &o;
            }
        }
        // ---- choose this chunk's segments / pieces ----
        pieces.clear();
        struct CSeg {
            uint32_t slot;
            uint64_t at, len;
            uint32_t pos;
        };
        std::vector<CSeg> cs;
        uint64_t state0 = si;  // stream: state index of the chunk's first segment
        uint64_t in_b = 0;
        uint32_t cnt = 0, uni_len = 0;  // uni_len: stream chunk whose segments all take this many bytes
        uint64_t out_b = 0, in_pad = 0, out_pad = 0, arr = 0, out_at = 0;
        if (!stream) {
            // whole frames [si, j) with <= kChunk input bytes (at least one frame)
            uint64_t j = si;
            while (j < n && (j == si || in_b + frames[j].len <= kChunk)) in_b += frames[j++].len;
            cnt = (uint32_t)(j - si);
            out_b = in_b + pre * cnt;
            in_pad = (in_b + 15) & ~15ull;
            out_pad = (out_b + 15) & ~15ull;
            arr = (uint64_t)cnt * (8 + 8 + 4 + 4);
            out_at = in_pad + ((arr + 15) & ~15ull);
            if ((rc = slot_reserve(s, e->numa.node, in_pad + out_pad + arr + 64))) break;
            uint64_t *in_off = reinterpret_cast<uint64_t *>(s.h + in_pad);
            uint64_t *out_off = in_off + cnt;
            uint32_t *lens = reinterpret_cast<uint32_t *>(out_off + cnt);
            uint32_t *slots = lens + cnt;
            // frame-parallel: per-part byte sums, then offsets + arrays + gather per part
            const unsigned all = pool_of(e)->parts();
            const unsigned sparts = sc ? std::max(1u, all / 2) : 0;
            const unsigned parts = sc ? std::max(1u, all - sparts) : copy_parts(e, in_b);
            uint64_t psum[64 + 1] = {0};
            const fpnn_aes_host_frame *fr = frames + si;
            auto range = [&](unsigned p, uint32_t &a, uint32_t &b) {
                a = (uint32_t)((uint64_t)cnt * p / parts);
                b = (uint32_t)((uint64_t)cnt * (p + 1) / parts);
            };
            const double tg = hst.on ? HostStats::now() : 0;
            pool_of(e)->run(parts, [&](unsigned p) {
                uint32_t a, b;
                range(p, a, b);
                uint64_t sum = 0;
                for (uint32_t t = a; t < b; t++) sum += fr[t].len;
                psum[p + 1] = sum;
            });
            for (unsigned p = 0; p < parts; p++) psum[p + 1] += psum[p];
            uint8_t *h_in = s.h;
            pool_of(e)->run(parts + sparts, [&](unsigned p) {
                if (p >= parts) {
                    scatter_frames_part(*sc, p - parts, sparts);
                    return;
                }
                uint32_t a, b;
                range(p, a, b);
                uint64_t io = psum[p], oo = psum[p] + pre * a;
                for (uint32_t t = a; t < b; t++) {
                    const fpnn_aes_host_frame &f = fr[t];
                    in_off[t] = io;
                    out_off[t] = oo;
                    lens[t] = f.len;
                    slots[t] = f.key_slot;
                    copy_streaming(h_in + io, f.src, f.len);
                    io += f.len;
                    oo += f.len + pre;
                }
                copy_fence();
            });
            if (hst.on) hst.gather += HostStats::now() - tg;
            if (sc) sc->frames = nullptr;
            s.frames = frames;
            s.first = (uint32_t)si;
            s.count = cnt;
            s.pre = pre;
            s.out_at = out_at;
            s.out_off = out_off;
            s.scatter_bytes = out_b;
            si = j;
        } else {
            // Round robin: each chunk takes up to `quota` bytes from each of a run of
            // consecutive streams, so every kernel advances many CFB chains at once (the
            // encrypt chain is serial: parallelism = streams per kernel).
            uint64_t t = sr.next < nseg ? sr.next : 0;
            while (sr.rem[t] == 0) t = t + 1 < nseg ? t + 1 : 0;  // left_total > 0: terminates
            state0 = t;
            for (; t < nseg && in_b < sr.chunk; t++) {
                const StreamSeg &sg = segs[t];
                const uint64_t take = std::min(sr.rem[t], sr.quota);
                uint64_t took = 0;
                while (took < take) {
                    const fpnn_aes_host_frame &f = frames[order[sg.first + sr.fi[t]]];
                    const uint32_t part = (uint32_t)std::min<uint64_t>(f.len - sr.fo[t], take - took);
                    if (part) pieces.push_back({order[sg.first + sr.fi[t]], sr.fo[t], part});
                    took += part;
                    sr.fo[t] += part;
                    if (sr.fo[t] == f.len) {
                        sr.fi[t]++;
                        sr.fo[t] = 0;
                    }
                }
                cs.push_back({sg.slot, in_b, take, sr.pos[t]});
                sr.pos[t] = (uint32_t)((sr.pos[t] + take) & 15u);
                sr.rem[t] -= take;
                sr.left -= take;
                in_b += take;
            }
            sr.next = t;
            if (sr.left == 0) si = nseg;
            // stream chunk: arrays and gather/scatter jobs from the pieces
            cnt = (uint32_t)cs.size();
            out_b = in_b;
            in_pad = (in_b + 15) & ~15ull;
            out_pad = in_pad;
            arr = (uint64_t)cnt * (8 + 8 + 4 + 4);
            out_at = in_pad + ((arr + 15) & ~15ull);
            if ((rc = slot_reserve(s, e->numa.node, in_pad + out_pad + arr + 64))) break;
            uint64_t *in_off = reinterpret_cast<uint64_t *>(s.h + in_pad);
            uint64_t *out_off = in_off + cnt;
            uint32_t *lens = reinterpret_cast<uint32_t *>(out_off + cnt);
            uint32_t *slots = lens + cnt;
            uni_len = cnt ? (uint32_t)cs[0].len : 0u;
            for (uint32_t t = 0; t < cnt; t++) {
                in_off[t] = out_off[t] = cs[t].at;
                lens[t] = (uint32_t)cs[t].len;
                slots[t] = cs[t].slot;
                if (lens[t] != uni_len) uni_len = 0;
            }
            gather.clear();
            s.scatter.clear();
            s.scatter_bytes = in_b;
            uint64_t at = 0;
            for (const Piece &pc : pieces) {
                const fpnn_aes_host_frame &f = frames[pc.frame];
                gather.push_back({s.h + at, f.src + pc.off, pc.len});
                s.scatter.push_back({f.dst + pc.off, s.h + out_at + at, pc.len});
                at += pc.len;
            }
            const double tg = hst.on ? HostStats::now() : 0;
            parallel_copy(e, gather, in_b);
            if (hst.on) hst.gather += HostStats::now() - tg;
        }
        nchunks++;
        HIP_TRY(hipMemcpyAsync(s.d, s.h, in_pad + arr, hipMemcpyHostToDevice, s.st));
        // The cipher runs on the engine stream: chunks share the engine's scratch (block
        // map, plan, length order, queue counter), so their kernels must not overlap --
        // and stream chunks continue from the state the previous chunk left.  The copies
        // of the slots still overlap each other and the kernels.
        HIP_TRY(hipEventRecord(s.staged, s.st));
        HIP_TRY(hipStreamWaitEvent(main_stream, s.staged, 0));
        fpnn_aes_batch b;
        memset(&b, 0, sizeof b);
        b.in = s.d;
        b.out = s.d + out_at;
        b.count = cnt;
        b.in_off = reinterpret_cast<const uint64_t *>(s.d + in_pad);
        b.out_off = pre ? b.in_off + cnt : nullptr;
        b.len = reinterpret_cast<const uint32_t *>(s.d + in_pad + 16ull * cnt);
        b.key_slot = keys->count > 1 ? b.len + cnt : nullptr;
        if (stream && encrypt && uni_len) {
            // every stream takes the same quota (segments back to back): a uniform batch,
            // so the encrypt skips the ragged length ordering (mapped_stream_pipeline)
            b.in_off = nullptr;
            b.len = nullptr;
            b.stride = uni_len;
            b.uniform_len = uni_len;
        }
        b.keys = keys;
        b.flags = pre ? FPNN_AES_F_WIRE_PREFIX : 0;
        uint8_t *ivp = stream ? d_state + 16 * state0 : nullptr;
        uint32_t *posp = stream ? reinterpret_cast<uint32_t *>(d_state + 16 * nseg) + state0 : nullptr;
        rc = encrypt ? run_encrypt(e, &b, ivp, posp, stream) : run_decrypt(e, &b, ivp, posp, stream);
        if (rc) break;
        HIP_TRY(hipEventRecord(s.kdone, main_stream));
        HIP_TRY(hipStreamWaitEvent(s.st, s.kdone, 0));
        HIP_TRY(hipMemcpyAsync(s.h + out_at, s.d + out_at, out_pad, hipMemcpyDeviceToHost, s.st));
        HIP_TRY(hipEventRecord(s.done, s.st));
        s.busy = true;
        prev = &s;
        k = (k + 1) % kSlots;
    }
    for (auto &sl : e->hs) {
        const int r2 = slot_drain(e, sl, hst);
        if (!rc) rc = r2;
    }
    if (stream) {
        if (!rc && prev) {
            const hipError_t err = hipMemcpy(h_state, d_state, nseg * 20, hipMemcpyDeviceToHost);
            if (err != hipSuccess) rc = hip_fail(err, "hipMemcpy(stream state)");
        }
        if (!rc) {
            const uint32_t *hp = reinterpret_cast<const uint32_t *>(h_state + 16 * nseg);
            for (uint64_t t = 0; t < nseg; t++) {
                memcpy(iv_state + 16ull * segs[t].slot, h_state + 16 * t, 16);
                pos_state[segs[t].slot] = hp[t];
            }
        }
    }
    if (hst.on)
        fprintf(stderr, "[fpnn_aes host] %s %s: %u frames, %llu segments, %llu chunks, %.2f ms total, gather %.2f, "
                "scatter %.2f, wait %.2f ms, %u copy threads\n", stream ? "stream" : "package",
                encrypt ? "encrypt" : "decrypt", n, (unsigned long long)nseg, (unsigned long long)nchunks,
                1e3 * (HostStats::now() - t_call), 1e3 * hst.gather, 1e3 * hst.scatter, 1e3 * hst.wait,
                e->pool ? e->pool->parts() : 1u);
    return rc;
}

int check_host_frames(const fpnn_aes_engine *e, const fpnn_aes_host_frame *frames, uint32_t n,
                      const fpnn_aes_keyset *keys) {
    if (!e || !keys || (n && !frames)) return FPNN_AES_ERR_ARG;
    if (keys->device != e->device) return FPNN_AES_ERR_ARG;
    for (uint32_t i = 0; i < n; i++)
        if ((frames[i].len && (!frames[i].src || !frames[i].dst)) || frames[i].key_slot >= keys->count)
            return FPNN_AES_ERR_ARG;
    return FPNN_AES_OK;
}

// ---- host-mapped frames ------------------------------------------------------------------
// Host ranges registered with fpnn_aes_host_register (process-wide, portable: every GPU may
// access them).  A range's device-visible address is looked up per device on first use.
constexpr int kMapDevices = 64;
struct MappedRange {
    uintptr_t lo, hi;
    intptr_t delta[kMapDevices];  // device address - host address per device (INTPTR_MIN: not looked up)
};
std::mutex g_map_mu;
std::vector<MappedRange> g_mapped;  // sorted by lo, disjoint

// One call's view of the registry: the ranges and this device's address deltas.
struct MapView {
    std::vector<uintptr_t> lo, hi;
    std::vector<intptr_t> delta;
    // the range holding [p, p + n), or -1
    long find(const void *ptr, uint64_t n) const {
        const uintptr_t p = (uintptr_t)ptr;
        auto it = std::upper_bound(lo.begin(), lo.end(), p);
        if (it == lo.begin()) return -1;
        const size_t i = (size_t)(it - lo.begin()) - 1;
        return p + n <= hi[i] && p + n >= p ? (long)i : -1;
    }
};

int map_view(int device, MapView &v) {
    std::lock_guard<std::mutex> lk(g_map_mu);
    v.lo.clear();
    v.hi.clear();
    v.delta.clear();
    if (device < 0 || device >= kMapDevices) return FPNN_AES_OK;  // (no mapped path there)
    for (auto &r : g_mapped) {
        if (r.delta[device] == INTPTR_MIN) {
            DeviceGuard g(device);
            void *dp = nullptr;
            HIP_TRY(hipHostGetDevicePointer(&dp, reinterpret_cast<void *>(r.lo), 0));
            r.delta[device] = (intptr_t)dp - (intptr_t)r.lo;
        }
        v.lo.push_back(r.lo);
        v.hi.push_back(r.hi);
        v.delta.push_back(r.delta[device]);
    }
    return FPNN_AES_OK;
}

int mslot_reserve(MapSlot &m, int node, uint64_t dneed, uint64_t hneed) {
    if (!m.gathered) {
        HIP_TRY(hipEventCreateWithFlags(&m.gathered, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&m.ciphered, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&m.done, hipEventDisableTiming));
    }
    if (dneed > m.dcap) {
        uint64_t c = m.dcap ? m.dcap : (16u << 20);
        while (c < dneed) c *= 2;
        if (m.d) (void)hipFree(m.d);
        m.d = nullptr;
        m.dcap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&m.d), c));
        m.dcap = c;
    }
    if (hneed > m.hcap) {
        uint64_t c = m.hcap ? m.hcap : (1u << 20);
        while (c < hneed) c *= 2;
        if (m.h) (void)hipHostFree(m.h);
        m.h = nullptr;
        m.hcap = 0;
        HIP_TRY(pinned_host_alloc(node, reinterpret_cast<void **>(&m.h), c));
        m.hcap = c;
    }
    return FPNN_AES_OK;
}

// Package-mode host frames that all lie in registered memory.  The call is cut into
// chunks of whole frames; chunk t lives in slot t % 4 (HBM staging in | out | descriptors,
// pinned descriptor block).  Step t: on the move stream ONE launch gathers chunk t from
// host memory into its staging AND scatters chunk t - 2's results to the frames'
// destinations (k_move_segments: both PCIe directions busy in one kernel); meanwhile the
// engine stream ciphers chunk t - 1 as an ordinary device batch (uniform lengths keep the
// dense K2 / K1d paths) and then uploads chunk t + 1's descriptors (40 B per frame,
// written by the host threads during step t), so the move stream never waits for a copy.
// Events hand each chunk between the two streams.  The host threads only write
// descriptors.
int mapped_pipeline(fpnn_aes_engine *e, bool encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                    const fpnn_aes_keyset *keys, uint32_t flags, const MapView &v, uint32_t *done) {
    const HostActive active_call(e->device);
    const uint64_t pre = (flags & FPNN_AES_F_WIRE_PREFIX) ? 4 : 0;
    static const uint64_t kChunk = [] {     // input bytes per full chunk (FPNN_AES_MAP_CHUNK_MB)
        const char *x = getenv("FPNN_AES_MAP_CHUNK_MB");
        return (x && atoi(x) > 0 ? (uint64_t)atoi(x) : 32ull) << 20;
    }();
    const uint32_t kMaxFrames = 1u << 20;   // frames per chunk (descriptor block <= 40 MiB)
    constexpr int kSlots = (int)(sizeof(e->ms) / sizeof(e->ms[0]));
    static_assert(kSlots >= 4, "a chunk's staging is live for three steps, plus the upload ahead");
    HostStats hst;
    const double t_call = hst.on ? HostStats::now() : 0;
    DeviceGuard g(e->device);
    for (auto &m : e->ms)
        if (int rc = mslot_reserve(m, e->numa.node, 0, 0)) return rc;
    if (!e->map_stream) HIP_TRY(hipStreamCreateWithFlags(&e->map_stream, hipStreamNonBlocking));
    hipStream_t ms = e->map_stream;
    // the move stream starts after work already queued on the engine stream
    HIP_TRY(hipEventRecord(e->ms[0].ciphered, e->stream));
    HIP_TRY(hipStreamWaitEvent(ms, e->ms[0].ciphered, 0));
    struct Chunk {
        uint32_t first = 0, cnt = 0;  // cnt = 0: no chunk in the slot
        bool uniform = false;
        uint64_t out_at = 0, desc_at = 0, desc_b = 0;
    } ch[kSlots];
    auto jobs_of = [&](int slot, MoveJob &gather, MoveJob &scatter) {
        const Chunk &c = ch[slot];
        MapSlot &m = e->ms[slot];
        const uint64_t *d_src = reinterpret_cast<const uint64_t *>(m.d + c.desc_at);
        const uint64_t *d_so = d_src + c.cnt, *d_dst = d_so + c.cnt, *d_oo = d_dst + c.cnt;
        const uint32_t *d_len = reinterpret_cast<const uint32_t *>(d_oo + c.cnt);
        gather = MoveJob{0, d_src, (uint64_t)(uintptr_t)m.d, d_so, d_len, 0, c.cnt};
        scatter = MoveJob{(uint64_t)(uintptr_t)(m.d + c.out_at), d_oo, 0, d_dst, d_len, (uint32_t)pre, c.cnt};
    };
    uint32_t si = 0;
    bool stop = false;  // a frame outside registered memory ended the mapped chunks
    // host: the descriptors of chunk t into its slot's pinned block (false: no chunk t)
    auto prepare = [&](uint64_t t, int &rc) -> bool {
        const int k = (int)(t % kSlots);
        Chunk &c = ch[k];
        c.cnt = 0;
        if (si >= n || stop) return false;
        MapSlot &m = e->ms[k];
        if (m.busy) {  // the slot's previous pinned block went H2D
            const double tw = hst.on ? HostStats::now() : 0;
            if (hipError_t err = hipEventSynchronize(m.done)) {
                rc = hip_fail(err, "hipEventSynchronize");
                return false;
            }
            if (hst.on) hst.wait += HostStats::now() - tw;
            m.busy = false;
        }
        const double tf = hst.on ? HostStats::now() : 0;
        uint64_t in_b = 0;
        uint32_t j = si;
        while (j < n && (j == si || (in_b + frames[j].len <= kChunk && j - si < kMaxFrames))) in_b += frames[j++].len;
        uint32_t cnt = j - si;
        const fpnn_aes_host_frame *fr = frames + si;
        // every frame of the chunk inside registered memory?  The chunk ends before the
        // first one that is not (the caller takes the rest through the staged path).
        {
            const unsigned parts = cnt >= 16384 ? pool_of(e)->parts() : 1u;
            std::atomic<uint32_t> bad{cnt};
            pool_of(e)->run(parts, [&](unsigned p) {
                const uint32_t a0 = (uint32_t)((uint64_t)cnt * p / parts), b0 = (uint32_t)((uint64_t)cnt * (p + 1) / parts);
                long rs = -1, rd = -1;
                for (uint32_t q = a0; q < b0; q++) {
                    const fpnn_aes_host_frame &f = fr[q];
                    const uintptr_t xs = (uintptr_t)f.src, xd = (uintptr_t)f.dst;
                    bool ok = true;
                    if (f.len && (rs < 0 || xs < v.lo[rs] || xs + f.len > v.hi[rs])) ok = (rs = v.find(f.src, f.len)) >= 0;
                    if (ok && f.len + pre && (rd < 0 || xd < v.lo[rd] || xd + f.len + pre > v.hi[rd]))
                        ok = (rd = v.find(f.dst, f.len + pre)) >= 0;
                    if (!ok) {
                        uint32_t cur = bad.load();
                        while (q < cur && !bad.compare_exchange_weak(cur, q)) {
                        }
                        return;
                    }
                }
            });
            if (bad.load() < cnt) {
                cnt = bad.load();
                j = si + cnt;
                in_b = 0;
                for (uint32_t q = 0; q < cnt; q++) in_b += fr[q].len;
                stop = true;  // no chunk after this one
                if (!cnt) return false;
            }
        }
        const uint64_t out_b = in_b + pre * cnt;
        const uint64_t in_pad = (in_b + 255) & ~255ull, out_pad = (out_b + 255) & ~255ull;
        c.first = si;
        c.out_at = in_pad;
        c.desc_at = in_pad + out_pad;
        c.desc_b = (uint64_t)cnt * 40;
        if (c.desc_at + c.desc_b + 64 > m.dcap || c.desc_b + 64 > m.hcap) {
            // growing frees the slot's buffers: let every queued use of them finish
            hipError_t err = hipStreamSynchronize(ms);
            if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
            if (err != hipSuccess) {
                rc = hip_fail(err, "hipStreamSynchronize");
                return false;
            }
            if ((rc = mslot_reserve(m, e->numa.node, c.desc_at + c.desc_b + 64, c.desc_b + 64))) return false;
        }
        // descriptor block (same layout in h and at d + desc_at):
        //   src u64 | so u64 | dst u64 | oo u64 | len u32 | slot u32   (cnt entries each)
        uint64_t *h_src = reinterpret_cast<uint64_t *>(m.h);
        uint64_t *h_so = h_src + cnt, *h_dst = h_so + cnt, *h_oo = h_dst + cnt;
        uint32_t *h_len = reinterpret_cast<uint32_t *>(h_oo + cnt), *h_slot = h_len + cnt;
        const unsigned parts = cnt >= 16384 ? pool_of(e)->parts() : 1u;
        uint64_t psum[64 + 1] = {0};
        uint8_t same[64];
        auto range = [&](unsigned p, uint32_t &a0, uint32_t &b0) {
            a0 = (uint32_t)((uint64_t)cnt * p / parts);
            b0 = (uint32_t)((uint64_t)cnt * (p + 1) / parts);
        };
        pool_of(e)->run(parts, [&](unsigned p) {
            uint32_t a0, b0;
            range(p, a0, b0);
            uint64_t sum = 0;
            bool eq = true;
            for (uint32_t q = a0; q < b0; q++) {
                sum += fr[q].len;
                eq = eq && fr[q].len == fr[0].len;
            }
            psum[p + 1] = sum;
            same[p] = eq;
        });
        c.uniform = true;
        for (unsigned p = 0; p < parts; p++) {
            psum[p + 1] += psum[p];
            c.uniform = c.uniform && same[p];
        }
        pool_of(e)->run(parts, [&](unsigned p) {
            uint32_t a0, b0;
            range(p, a0, b0);
            uint64_t io = psum[p], oo = psum[p] + pre * a0;
            long rs = -1, rd = -1;  // last range hit (frames of one arena: one search each)
            for (uint32_t q = a0; q < b0; q++) {
                const fpnn_aes_host_frame &f = fr[q];
                uint64_t sa = 0, da = 0;
                if (f.len) {
                    const uintptr_t x = (uintptr_t)f.src;
                    if (rs < 0 || x < v.lo[rs] || x + f.len > v.hi[rs]) rs = v.find(f.src, f.len);
                    sa = (uint64_t)((intptr_t)x + v.delta[rs]);
                }
                if (f.len + pre) {
                    const uintptr_t x = (uintptr_t)f.dst;
                    if (rd < 0 || x < v.lo[rd] || x + f.len + pre > v.hi[rd]) rd = v.find(f.dst, f.len + pre);
                    da = (uint64_t)((intptr_t)x + v.delta[rd]);
                }
                h_src[q] = sa;
                h_so[q] = io;
                h_dst[q] = da;
                h_oo[q] = oo;
                h_len[q] = f.len;
                h_slot[q] = f.key_slot;
                io += f.len;
                oo += f.len + pre;
            }
        });
        c.cnt = cnt;
        si = j;
        if (hst.on) hst.gather += HostStats::now() - tf;  // (descriptor fill)
        return true;
    };
    // engine stream: chunk t's descriptors H2D; `done` doubles as "descriptors on the device"
    auto upload = [&](uint64_t t) -> int {
        const int k = (int)(t % kSlots);
        MapSlot &m = e->ms[k];
        HIP_TRY(hipMemcpyAsync(m.d + ch[k].desc_at, m.h, ch[k].desc_b, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipEventRecord(m.done, e->stream));
        m.busy = true;
        return FPNN_AES_OK;
    };
    int rc = FPNN_AES_OK;
    if (prepare(0, rc)) rc = upload(0);
    const MoveJob none{0, nullptr, 0, nullptr, nullptr, 0, 0};
    for (uint64_t t = 0; rc == FPNN_AES_OK; t++) {
        const int kt = (int)(t % kSlots), k1 = (int)((t + kSlots - 1) % kSlots), k2 = (int)((t + kSlots - 2) % kSlots);
        const bool gather_t = ch[kt].cnt != 0;
        const bool cipher_t1 = t >= 1 && ch[k1].cnt != 0;
        const bool scatter_t2 = t >= 2 && ch[k2].cnt != 0;
        if (!gather_t && !cipher_t1 && !scatter_t2) break;
        // move stream: gather t || scatter t - 2
        MoveJob gj = none, sj = none, tmp;
        if (gather_t) {
            HIP_TRY(hipStreamWaitEvent(ms, e->ms[kt].done, 0));
            jobs_of(kt, gj, tmp);
        }
        if (scatter_t2) {
            HIP_TRY(hipStreamWaitEvent(ms, e->ms[k2].ciphered, 0));
            jobs_of(k2, tmp, sj);
        }
        HIP_TRY(launch_move_segments(gj, sj, ms));
        if (gather_t) HIP_TRY(hipEventRecord(e->ms[kt].gathered, ms));
        // engine stream: cipher t - 1, then upload chunk t + 1 (its slot's previous chunk,
        // t - 3, was scattered by step t - 1's launch, which the cipher waited for); the
        // cipher is queued before the host prepares chunk t + 1's descriptors
        bool next = false, prepared = false;
        if (cipher_t1) {
            const Chunk &c = ch[k1];
            MapSlot &m = e->ms[k1];
            HIP_TRY(hipStreamWaitEvent(e->stream, m.gathered, 0));
            MoveJob gq, sq;
            jobs_of(k1, gq, sq);
            fpnn_aes_batch bt;
            memset(&bt, 0, sizeof bt);
            bt.in = m.d;
            bt.out = m.d + c.out_at;
            bt.count = c.cnt;
            bt.keys = keys;
            bt.flags = pre ? FPNN_AES_F_WIRE_PREFIX : 0u;
            if (c.uniform && !pre) {  // dense uniform staging: the K2 / K1d fast paths
                bt.stride = frames[c.first].len;
                bt.uniform_len = frames[c.first].len;
            } else {
                bt.in_off = gq.doff;
                bt.out_off = sq.soff;
                bt.len = gq.len;
            }
            if (keys->count > 1) bt.key_slot = gq.len + c.cnt;
            rc = encrypt ? run_encrypt(e, &bt, nullptr, nullptr, false) : run_decrypt(e, &bt, nullptr, nullptr, false);
            if (rc) break;
            HIP_TRY(hipEventRecord(m.ciphered, e->stream));
        }
        // host: chunk t + 1's descriptors while the GPU moves and ciphers
        if (!prepared) next = prepare(t + 1, rc);
        if (rc) break;
        // (chunk t + 1 exists only if chunk t - 1 does, for t >= 1: the upload always
        // follows a cipher; at t = 0 the slot is unused)
        if (next && (rc = upload(t + 1))) break;
        if (scatter_t2) ch[k2].cnt = 0;  // (its slot's next chunk is prepared at step t + 1)
    }
    const double td = hst.on ? HostStats::now() : 0;
    HIP_TRY(hipStreamSynchronize(ms));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (int rf = stream_idle(e)) rc = rc ? rc : rf;
    for (auto &m : e->ms) m.busy = false;
    for (auto &c : ch) c.cnt = 0;
    *done = si;
    e->host_path = "host_mapped";
    if (hst.on)
        fprintf(stderr, "[fpnn_aes host] mapped %s: %u frames, %.2f ms total, descriptors %.2f, slot waits %.2f, "
                "final drain %.2f ms, chunk %llu MiB\n", encrypt ? "encrypt" : "decrypt", n,
                1e3 * (HostStats::now() - t_call), 1e3 * hst.gather, 1e3 * hst.wait, 1e3 * (HostStats::now() - td),
                (unsigned long long)(kChunk >> 20));
    return rc;
}

// Stream-mode host frames that all lie in registered memory: the chunking of host_pipeline
// (one segment per stream = its frames in array order, round-robin quotas so a chunk
// advances many chains) with mapped_pipeline's moves: on the move stream one launch per
// step gathers chunk t's pieces from host memory and scatters chunk t - 2's results to
// the frames' destinations; the engine stream ciphers chunk t - 1 with the streams'
// carried (iv, pos) -- chunks in order, so a stream split across chunks continues from
// the state the previous chunk left -- then uploads chunk t + 1's descriptors.
// Descriptor block of a chunk: per piece src u64 | so u64 | dst u64 | oo u64 | len u32,
// then per stream segment off u64 | len u32 | slot u32.
int mapped_stream_pipeline(fpnn_aes_engine *e, bool encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                           const fpnn_aes_keyset *keys, const MapView &v, uint8_t *iv_state, uint32_t *pos_state) {
    const HostActive active_call(e->device);
    static const uint64_t kChunk = [] {
        const char *x = getenv("FPNN_AES_MAP_CHUNK_MB");
        return (x && atoi(x) > 0 ? (uint64_t)atoi(x) : 32ull) << 20;
    }();
    constexpr int kSlots = (int)(sizeof(e->ms) / sizeof(e->ms[0]));
    // ---- streams in array order (group_streams) ----
    HostStats hst;
    const double t_call = hst.on ? HostStats::now() : 0;
    std::vector<uint32_t> order;
    std::vector<StreamSeg> segs;
    group_streams(frames, n, keys->count, order, segs);
    if (segs.empty()) return FPNN_AES_OK;
    const uint64_t nseg = segs.size();
    const double t_sorted = hst.on ? HostStats::now() : 0;
    DeviceGuard g(e->device);
    for (auto &m : e->ms)
        if (int rc = mslot_reserve(m, e->numa.node, 0, 0)) return rc;
    if (!e->map_stream) HIP_TRY(hipStreamCreateWithFlags(&e->map_stream, hipStreamNonBlocking));
    hipStream_t ms = e->map_stream;
    // ---- the streams' (iv, pos), compact, on the device (engine stream) ----
    if (int rc = sstate_reserve(e, nseg * 20)) return rc;
    uint8_t *h_state = e->h_sstate, *d_state = e->d_sstate;
    std::vector<uint64_t> rem(nseg);
    std::vector<uint32_t> fi(nseg, 0), fo(nseg, 0);
    uint64_t left = 0;
    {
        uint32_t *hp = reinterpret_cast<uint32_t *>(h_state + 16 * nseg);
        for (uint64_t t = 0; t < nseg; t++) {
            memcpy(h_state + 16 * t, iv_state + 16ull * segs[t].slot, 16);
            hp[t] = pos_state[segs[t].slot] & 15u;
            rem[t] = segs[t].bytes;
            left += segs[t].bytes;
        }
    }
    HIP_TRY(hipMemcpyAsync(d_state, h_state, nseg * 20, hipMemcpyHostToDevice, e->stream));
    // Chunks of kChunk bytes (as the package path: the moves of chunk t overlap the cipher
    // of chunk t - 1, so more, smaller chunks pipeline better than a few large ones), each
    // taking a quota from as many streams as fit: the encrypt of a chunk is one serial CFB
    // chain per stream, so its parallelism is the number of streams it spans.
    const uint64_t chunk = kChunk;
    const uint64_t quota = std::max<uint64_t>(1024, (chunk / nseg + 15) & ~15ull);
    // the move stream starts after work already queued on the engine stream
    HIP_TRY(hipEventRecord(e->ms[0].ciphered, e->stream));
    HIP_TRY(hipStreamWaitEvent(ms, e->ms[0].ciphered, 0));
    struct Chunk {
        uint32_t np = 0, ns = 0;  // pieces, stream segments (np = 0: no chunk in the slot)
        uint32_t uni = 0;         // every segment this many bytes (0: ragged)
        uint64_t state0 = 0, out_at = 0, desc_at = 0, desc_b = 0;
    } ch[kSlots];
    uint64_t next = 0;  // round-robin cursor over segs
    auto jobs_of = [&](int slot, MoveJob &gather, MoveJob &scatter) {
        const Chunk &c = ch[slot];
        MapSlot &m = e->ms[slot];
        const uint64_t *d_src = reinterpret_cast<const uint64_t *>(m.d + c.desc_at);
        const uint64_t *d_so = d_src + c.np, *d_dst = d_so + c.np, *d_oo = d_dst + c.np;
        const uint32_t *d_len = reinterpret_cast<const uint32_t *>(d_oo + c.np);
        gather = MoveJob{0, d_src, (uint64_t)(uintptr_t)m.d, d_so, d_len, 0, c.np};
        scatter = MoveJob{(uint64_t)(uintptr_t)(m.d + c.out_at), d_oo, 0, d_dst, d_len, 0, c.np};
    };
    auto seg_arrays = [&](int slot, const uint64_t *&off, const uint32_t *&len, const uint32_t *&sl) {
        const Chunk &c = ch[slot];
        const uint8_t *base = e->ms[slot].d + c.desc_at + (uint64_t)c.np * 36;
        const uint64_t a = ((uint64_t)(uintptr_t)base + 7) & ~7ull;
        off = reinterpret_cast<const uint64_t *>(a);
        len = reinterpret_cast<const uint32_t *>(off + c.ns);
        sl = len + c.ns;
    };
    // host: chunk t's pieces and descriptors into its slot's pinned block
    auto prepare = [&](uint64_t t, int &rc) -> bool {
        const int k = (int)(t % kSlots);
        Chunk &c = ch[k];
        c.np = c.ns = 0;
        if (left == 0) return false;
        MapSlot &m = e->ms[k];
        if (m.busy) {
            const double tw = hst.on ? HostStats::now() : 0;
            if (hipError_t err = hipEventSynchronize(m.done)) {
                rc = hip_fail(err, "hipEventSynchronize");
                return false;
            }
            if (hst.on) hst.wait += HostStats::now() - tw;
            m.busy = false;
        }
        const double tf = hst.on ? HostStats::now() : 0;
        std::vector<Piece> pieces;
        struct CS {
            uint32_t slot;
            uint64_t at, len;
        };
        std::vector<CS> cs;
        uint64_t s = next < nseg ? next : 0;
        while (rem[s] == 0) s = s + 1 < nseg ? s + 1 : 0;  // left > 0: terminates
        c.state0 = s;
        uint64_t in_b = 0;
        for (; s < nseg && in_b < chunk; s++) {
            const StreamSeg &sg = segs[s];
            const uint64_t take = std::min(rem[s], quota);
            uint64_t took = 0;
            while (took < take) {
                const uint32_t fidx = order[sg.first + fi[s]];
                const fpnn_aes_host_frame &f = frames[fidx];
                const uint32_t part = (uint32_t)std::min<uint64_t>(f.len - fo[s], take - took);
                if (part) pieces.push_back({fidx, fo[s], part});
                took += part;
                fo[s] += part;
                if (fo[s] == f.len) {
                    fi[s]++;
                    fo[s] = 0;
                }
            }
            cs.push_back({sg.slot, in_b, take});
            rem[s] -= take;
            left -= take;
            in_b += take;
        }
        next = s;
        const uint32_t np = (uint32_t)pieces.size(), ns = (uint32_t)cs.size();
        const uint64_t in_pad = (in_b + 255) & ~255ull;
        c.out_at = in_pad;
        c.desc_at = 2 * in_pad;
        c.desc_b = (uint64_t)np * 36 + 8 + (uint64_t)ns * 16;
        if (c.desc_at + c.desc_b + 64 > m.dcap || c.desc_b + 64 > m.hcap) {
            hipError_t err = hipStreamSynchronize(ms);  // growing frees the slot's buffers
            if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
            if (err != hipSuccess) {
                rc = hip_fail(err, "hipStreamSynchronize");
                return false;
            }
            if ((rc = mslot_reserve(m, e->numa.node, c.desc_at + c.desc_b + 64, c.desc_b + 64))) return false;
        }
        uint64_t *h_src = reinterpret_cast<uint64_t *>(m.h);
        uint64_t *h_so = h_src + np, *h_dst = h_so + np, *h_oo = h_dst + np;
        uint32_t *h_len = reinterpret_cast<uint32_t *>(h_oo + np);
        const unsigned parts = np >= 16384 ? pool_of(e)->parts() : 1u;
        std::vector<uint64_t> at(np);
        {
            uint64_t a = 0;
            for (uint32_t q = 0; q < np; q++) {
                at[q] = a;
                a += pieces[q].len;
            }
        }
        pool_of(e)->run(parts, [&](unsigned p) {
            const uint32_t a0 = (uint32_t)((uint64_t)np * p / parts), b0 = (uint32_t)((uint64_t)np * (p + 1) / parts);
            long rs = -1, rd = -1;
            for (uint32_t q = a0; q < b0; q++) {
                const Piece &pc = pieces[q];
                const fpnn_aes_host_frame &f = frames[pc.frame];
                const uintptr_t xs = (uintptr_t)f.src + pc.off, xd = (uintptr_t)f.dst + pc.off;
                if (rs < 0 || xs < v.lo[rs] || xs + pc.len > v.hi[rs]) rs = v.find((const void *)xs, pc.len);
                if (rd < 0 || xd < v.lo[rd] || xd + pc.len > v.hi[rd]) rd = v.find((const void *)xd, pc.len);
                h_src[q] = (uint64_t)((intptr_t)xs + v.delta[rs]);
                h_so[q] = at[q];
                h_dst[q] = (uint64_t)((intptr_t)xd + v.delta[rd]);
                h_oo[q] = at[q];
                h_len[q] = pc.len;
            }
        });
        const uint64_t sa = (((uint64_t)(uintptr_t)(m.h + (uint64_t)np * 36)) + 7) & ~7ull;
        uint64_t *h_off = reinterpret_cast<uint64_t *>(sa);
        uint32_t *h_slen = reinterpret_cast<uint32_t *>(h_off + ns), *h_sslot = h_slen + ns;
        for (uint32_t q = 0; q < ns; q++) {
            h_off[q] = cs[q].at;
            h_slen[q] = (uint32_t)cs[q].len;
            h_sslot[q] = cs[q].slot;
        }
        c.np = np;
        c.ns = ns;
        c.uni = (uint32_t)cs[0].len;  // (segments lie back to back: equal lengths = a stride)
        for (uint32_t q = 1; q < ns && c.uni; q++)
            if (cs[q].len != c.uni) c.uni = 0;
        if (hst.on) hst.gather += HostStats::now() - tf;
        return true;
    };
    auto upload = [&](uint64_t t) -> int {
        const int k = (int)(t % kSlots);
        MapSlot &m = e->ms[k];
        HIP_TRY(hipMemcpyAsync(m.d + ch[k].desc_at, m.h, ch[k].desc_b, hipMemcpyHostToDevice, e->stream));
        HIP_TRY(hipEventRecord(m.done, e->stream));
        m.busy = true;
        return FPNN_AES_OK;
    };
    int rc = FPNN_AES_OK;
    if (prepare(0, rc)) rc = upload(0);
    const MoveJob none{0, nullptr, 0, nullptr, nullptr, 0, 0};
    for (uint64_t t = 0; rc == FPNN_AES_OK; t++) {
        const int kt = (int)(t % kSlots), k1 = (int)((t + kSlots - 1) % kSlots), k2 = (int)((t + kSlots - 2) % kSlots);
        const bool gather_t = ch[kt].np != 0;
        const bool cipher_t1 = t >= 1 && ch[k1].np != 0;
        const bool scatter_t2 = t >= 2 && ch[k2].np != 0;
        if (!gather_t && !cipher_t1 && !scatter_t2) break;
        MoveJob gj = none, sj = none, tmp;
        if (gather_t) {
            HIP_TRY(hipStreamWaitEvent(ms, e->ms[kt].done, 0));
            jobs_of(kt, gj, tmp);
        }
        if (scatter_t2) {
            HIP_TRY(hipStreamWaitEvent(ms, e->ms[k2].ciphered, 0));
            jobs_of(k2, tmp, sj);
        }
        HIP_TRY(launch_move_segments(gj, sj, ms));
        if (gather_t) HIP_TRY(hipEventRecord(e->ms[kt].gathered, ms));
        // the cipher of chunk t - 1 is queued before the host prepares chunk t + 1 (the
        // engine stream is not left empty while the host works)
        bool more = false, prepared = false;
        if (cipher_t1) {
            const Chunk &c = ch[k1];
            MapSlot &m = e->ms[k1];
            HIP_TRY(hipStreamWaitEvent(e->stream, m.gathered, 0));
            const uint64_t *off;
            const uint32_t *len, *sl;
            seg_arrays(k1, off, len, sl);
            fpnn_aes_batch bt;
            memset(&bt, 0, sizeof bt);
            bt.in = m.d;
            bt.out = m.d + c.out_at;
            bt.count = c.ns;
            if (encrypt && c.uni) {
                // every stream takes the same quota (S1's middle chunks): a uniform batch,
                // so the encrypt skips the ragged length ordering (its bucket counters see
                // one length: 16 384 atomics on one word, ~1 ms per chunk in the r04q trace)
                bt.stride = c.uni;
                bt.uniform_len = c.uni;
            } else {
                bt.in_off = off;
                bt.len = len;
            }
            bt.key_slot = keys->count > 1 ? sl : nullptr;
            bt.keys = keys;
            uint8_t *ivp = d_state + 16 * c.state0;
            uint32_t *posp = reinterpret_cast<uint32_t *>(d_state + 16 * nseg) + c.state0;
            rc = encrypt ? run_encrypt(e, &bt, ivp, posp, true) : run_decrypt(e, &bt, ivp, posp, true);
            if (rc) break;
            HIP_TRY(hipEventRecord(m.ciphered, e->stream));
        }
        if (!prepared) more = prepare(t + 1, rc);
        if (rc) break;
        if (more && (rc = upload(t + 1))) break;
        if (scatter_t2) ch[k2].np = 0;
    }
    const double td = hst.on ? HostStats::now() : 0;
    HIP_TRY(hipStreamSynchronize(ms));
    HIP_TRY(hipStreamSynchronize(e->stream));
    if (int rf = stream_idle(e)) rc = rc ? rc : rf;
    for (auto &m : e->ms) m.busy = false;
    for (auto &c : ch) c.np = 0;
    if (!rc) {
        HIP_TRY(hipMemcpy(h_state, d_state, nseg * 20, hipMemcpyDeviceToHost));
        const uint32_t *hp = reinterpret_cast<const uint32_t *>(h_state + 16 * nseg);
        for (uint64_t t = 0; t < nseg; t++) {
            memcpy(iv_state + 16ull * segs[t].slot, h_state + 16 * t, 16);
            pos_state[segs[t].slot] = hp[t];
        }
    }
    e->host_path = "host_mapped";
    if (hst.on)
        fprintf(stderr, "[fpnn_aes host] mapped stream %s: %u frames, %llu streams, %.2f ms total, sort %.2f, "
                "descriptors %.2f, slot waits %.2f, final drain %.2f ms\n", encrypt ? "encrypt" : "decrypt", n,
                (unsigned long long)nseg, 1e3 * (HostStats::now() - t_call), 1e3 * (t_sorted - t_call),
                1e3 * hst.gather, 1e3 * hst.wait, 1e3 * (HostStats::now() - td));
    return rc;
}

// every frame of the call (source and destination) inside registered memory
bool all_mapped(const fpnn_aes_engine *e, const fpnn_aes_host_frame *frames, uint32_t n, const MapView &v) {
    std::atomic<bool> ok{true};
    const unsigned parts = n >= 16384 ? pool_of(const_cast<fpnn_aes_engine *>(e))->parts() : 1u;
    pool_of(const_cast<fpnn_aes_engine *>(e))->run(parts, [&](unsigned p) {
        const uint32_t a0 = (uint32_t)((uint64_t)n * p / parts), b0 = (uint32_t)((uint64_t)n * (p + 1) / parts);
        long rs = -1, rd = -1;
        for (uint32_t q = a0; q < b0 && ok.load(std::memory_order_relaxed); q++) {
            const fpnn_aes_host_frame &f = frames[q];
            if (!f.len) continue;
            const uintptr_t xs = (uintptr_t)f.src, xd = (uintptr_t)f.dst;
            if ((rs < 0 || xs < v.lo[rs] || xs + f.len > v.hi[rs]) && (rs = v.find(f.src, f.len)) < 0) ok = false;
            if ((rd < 0 || xd < v.lo[rd] || xd + f.len > v.hi[rd]) && (rd = v.find(f.dst, f.len)) < 0) ok = false;
        }
    });
    return ok.load();
}

bool mapped_enabled() {
    const char *v = getenv("FPNN_AES_HOST_MAPPED");
    return !v || atoi(v) != 0;
}

}  // namespace

int fpnn_aes_package_host(fpnn_aes_engine *e, int encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                          const fpnn_aes_keyset *keys, uint32_t flags) {
    if (int rc = check_host_frames(e, frames, n, keys)) return rc;
    if (int rc = debug_fail_point()) return rc;
    if (!encrypt && (flags & FPNN_AES_F_WIRE_PREFIX)) return FPNN_AES_ERR_ARG;
    if (flags & FPNN_AES_F_WIRE_PREFIX)
        for (uint32_t i = 0; i < n; i++)
            if (!frames[i].dst) return FPNN_AES_ERR_ARG;
    if (!n) return FPNN_AES_OK;
    if (mapped_enabled()) {  // every frame in registered host memory: the GPU moves the bytes
        MapView v;
        if (int rc = map_view(e->device, v)) return rc;
        const uint64_t pre = (flags & FPNN_AES_F_WIRE_PREFIX) ? 4 : 0;
        if (!v.lo.empty() && (!frames[0].len || v.find(frames[0].src, frames[0].len) >= 0) &&
            (!(frames[0].len + pre) || v.find(frames[0].dst, frames[0].len + pre) >= 0)) {
            // frames in registered memory from the first on: mapped until the first frame
            // that is not, the rest (if any) staged -- package frames are independent
            uint32_t done = 0;
            if (int rc = mapped_pipeline(e, encrypt != 0, frames, n, keys, flags, v, &done)) return rc;
            if (done == n) return FPNN_AES_OK;
            frames += done;
            n -= done;
            const int rc = host_pipeline(e, encrypt != 0, false, frames, n, keys, flags, nullptr, nullptr);
            if (done) e->host_path = "host_mapped+staged";
            return rc;
        }
    }
    return host_pipeline(e, encrypt != 0, false, frames, n, keys, flags, nullptr, nullptr);
}

int fpnn_aes_host_register(void *ptr, size_t len) {
    if (!ptr || !len) return FPNN_AES_ERR_ARG;
    const uintptr_t lo = (uintptr_t)ptr, hi = lo + len;
    if (hi < lo) return FPNN_AES_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_map_mu);
    auto it = std::lower_bound(g_mapped.begin(), g_mapped.end(), lo,
                               [](const MappedRange &r, uintptr_t x) { return r.lo < x; });
    if ((it != g_mapped.end() && it->lo < hi) || (it != g_mapped.begin() && std::prev(it)->hi > lo)) {
        g_last_error = "fpnn_aes_host_register: range overlaps a registered range";
        return FPNN_AES_ERR_ARG;
    }
    HIP_TRY(hipHostRegister(ptr, len, hipHostRegisterPortable | hipHostRegisterMapped));
    MappedRange r;
    r.lo = lo;
    r.hi = hi;
    for (auto &d : r.delta) d = INTPTR_MIN;
    g_mapped.insert(it, r);
    return FPNN_AES_OK;
}

int fpnn_aes_host_unregister(void *ptr) {
    std::lock_guard<std::mutex> lk(g_map_mu);
    auto it = std::find_if(g_mapped.begin(), g_mapped.end(), [ptr](const MappedRange &r) { return r.lo == (uintptr_t)ptr; });
    if (it == g_mapped.end()) return FPNN_AES_ERR_ARG;
    g_mapped.erase(it);
    HIP_TRY(hipHostUnregister(ptr));
    return FPNN_AES_OK;
}

int fpnn_aes_host_is_mapped(const void *ptr, size_t len) {
    std::lock_guard<std::mutex> lk(g_map_mu);
    const uintptr_t p = (uintptr_t)ptr;
    for (const auto &r : g_mapped)
        if (p >= r.lo && p + len <= r.hi && p + len >= p) return 1;
    return 0;
}

int fpnn_aes_stream_host(fpnn_aes_engine *e, int encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                         const fpnn_aes_keyset *keys, uint8_t *iv_state, uint32_t *pos_state) {
    if (int rc = check_host_frames(e, frames, n, keys)) return rc;
    if (int rc = debug_fail_point()) return rc;
    if (n && (!iv_state || !pos_state)) return FPNN_AES_ERR_ARG;
    if (!n) return FPNN_AES_OK;
    if (mapped_enabled()) {  // every frame in registered host memory: the GPU moves the bytes
        MapView v;
        if (int rc = map_view(e->device, v)) return rc;
        if (!v.lo.empty() && all_mapped(e, frames, n, v))
            return mapped_stream_pipeline(e, encrypt != 0, frames, n, keys, v, iv_state, pos_state);
    }
    return host_pipeline(e, encrypt != 0, true, frames, n, keys, 0, iv_state, pos_state);
}

// ---- one host batch over several engines (GPUs) ------------------------------------------
// Each engine runs its share through its own host_pipeline in its own thread (engine 0's in
// the caller's), on that engine's NUMA node; errors are collected and the first one (by
// engine index) is returned, with its message.
static int run_multi(fpnn_aes_engine *const *engines, int n_engines, const std::function<int(int)> &fn) {
    std::vector<int> rc(n_engines, FPNN_AES_OK);
    std::vector<std::string> msg(n_engines);
    std::vector<std::thread> th;
    for (int k = 1; k < n_engines; k++)
        th.emplace_back([&, k] {
            (void)fpnn_aes::numa_pin_thread(engines[k]->numa);
            rc[k] = fn(k);
            if (rc[k]) msg[k] = g_last_error;
        });
    rc[0] = fn(0);
    if (rc[0]) msg[0] = g_last_error;
    for (auto &t : th) t.join();
    for (int k = 0; k < n_engines; k++)
        if (rc[k]) {
            g_last_error = "engine " + std::to_string(k) + ": " + msg[k];
            return rc[k];
        }
    return FPNN_AES_OK;
}

int fpnn_aes_package_host_multi(fpnn_aes_engine *const *engines, const fpnn_aes_keyset *const *keys, int n_engines,
                                int encrypt, const fpnn_aes_host_frame *frames, uint32_t n, uint32_t flags) {
    if (!engines || !keys || n_engines < 1 || (n && !frames)) return FPNN_AES_ERR_ARG;
    for (int k = 0; k < n_engines; k++)
        if (!engines[k] || !keys[k] || keys[k]->count != keys[0]->count || keys[k]->nrounds != keys[0]->nrounds)
            return FPNN_AES_ERR_ARG;
    if (n_engines == 1 || n < 2) return fpnn_aes_package_host(engines[0], encrypt, frames, n, keys[0], flags);
    // byte-balanced contiguous ranges of frames
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += frames[i].len;
    std::vector<uint32_t> cut(n_engines + 1, n);
    cut[0] = 0;
    uint64_t acc = 0;
    int p = 1;
    for (uint32_t i = 0; i < n && p < n_engines; i++) {
        acc += frames[i].len;
        while (p < n_engines && acc * n_engines >= total * p) cut[p++] = i + 1;
    }
    return run_multi(engines, n_engines, [&](int k) {
        return fpnn_aes_package_host(engines[k], encrypt, frames + cut[k], cut[k + 1] - cut[k], keys[k], flags);
    });
}

int fpnn_aes_stream_host_multi(fpnn_aes_engine *const *engines, const fpnn_aes_keyset *const *keys, int n_engines,
                               int encrypt, const fpnn_aes_host_frame *frames, uint32_t n, uint8_t *iv_state,
                               uint32_t *pos_state) {
    if (!engines || !keys || n_engines < 1 || (n && (!frames || !iv_state || !pos_state))) return FPNN_AES_ERR_ARG;
    for (int k = 0; k < n_engines; k++)
        if (!engines[k] || !keys[k] || keys[k]->count != keys[0]->count || keys[k]->nrounds != keys[0]->nrounds)
            return FPNN_AES_ERR_ARG;
    if (n_engines == 1 || n < 2)
        return fpnn_aes_stream_host(engines[0], encrypt, frames, n, keys[0], iv_state, pos_state);
    // whole streams to engines, longest first onto the least-loaded engine (a stream's frames
    // stay in order on one engine: its CFB state chains through them)
    std::unordered_map<uint32_t, uint64_t> bytes;
    for (uint32_t i = 0; i < n; i++) bytes[frames[i].key_slot] += frames[i].len;
    std::vector<std::pair<uint64_t, uint32_t>> order;
    order.reserve(bytes.size());
    for (const auto &kv : bytes) order.push_back({kv.second, kv.first});
    std::sort(order.begin(), order.end(), [](const std::pair<uint64_t, uint32_t> &a,
                                             const std::pair<uint64_t, uint32_t> &b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    std::vector<uint64_t> load(n_engines, 0);
    std::unordered_map<uint32_t, int> owner;
    for (const auto &o : order) {
        const int k = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        owner[o.second] = k;
        load[k] += o.first;
    }
    std::vector<std::vector<fpnn_aes_host_frame>> part(n_engines);
    for (uint32_t i = 0; i < n; i++) part[owner[frames[i].key_slot]].push_back(frames[i]);
    return run_multi(engines, n_engines, [&](int k) {
        return fpnn_aes_stream_host(engines[k], encrypt, part[k].data(), (uint32_t)part[k].size(), keys[k], iv_state,
                                    pos_state);
    });
}

int fpnn_aes_device_alloc(fpnn_aes_engine *e, size_t bytes, void **out) {
    if (!e || !out) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    DeviceGuard g(e->device);
    HIP_TRY(hipMalloc(out, bytes ? bytes : 1));
    return FPNN_AES_OK;
}

int fpnn_aes_device_free(fpnn_aes_engine *e, void *p) {
    if (!e) return FPNN_AES_ERR_ARG;
    if (!p) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    HIP_TRY(hipFree(p));
    return FPNN_AES_OK;
}

int fpnn_aes_pinned_alloc(fpnn_aes_engine *e, size_t bytes, void **out) {
    if (!e || !out) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    DeviceGuard g(e->device);
    HIP_TRY(pinned_host_alloc(e->numa.node, out, bytes ? bytes : 1));
    return FPNN_AES_OK;
}

int fpnn_aes_engine_numa(fpnn_aes_engine *e, int *node, int *device_node, int *ncpus) {
    if (!e) return FPNN_AES_ERR_ARG;
    if (node) *node = e->numa.node;
    if (device_node) *device_node = e->numa.device_node;
    if (ncpus) *ncpus = e->numa.ncpus;
    g_last_error = e->numa.why;
    return FPNN_AES_OK;
}

int fpnn_aes_pinned_free(fpnn_aes_engine *e, void *p) {
    if (!e) return FPNN_AES_ERR_ARG;
    if (!p) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    HIP_TRY(hipHostFree(p));
    return FPNN_AES_OK;
}

int fpnn_aes_copy_async(fpnn_aes_engine *e, void *dst, const void *src, size_t bytes) {
    if (!e || (bytes && (!dst || !src))) return FPNN_AES_ERR_ARG;
    if (!bytes) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, e->stream));
    return FPNN_AES_OK;
}

int fpnn_aes_fill_synthetic(fpnn_aes_engine *e, uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset) {
    if (!e || (nbytes && !dst)) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    HIP_TRY(launch_fill_synthetic(dst, nbytes, seed, byte_offset, e->num_cus * 8, e->stream));
    return FPNN_AES_OK;
}

int fpnn_aes_engine_set_timing(fpnn_aes_engine *e, int enable) {
    if (!e) return FPNN_AES_ERR_ARG;
    e->timing = enable != 0;
    return FPNN_AES_OK;
}

int fpnn_aes_engine_kernel_stats(fpnn_aes_engine *e, int which, uint64_t *launches, double *total_ms) {
    if (!e || which < 0 || which > 1 || !launches || !total_ms) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    HIP_TRY(hipStreamSynchronize(e->stream));
    double sum = 0;
    for (size_t i = 0; i < e->ev_used[which]; i++) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, e->ev[which][i].beg, e->ev[which][i].end));
        sum += ms;
    }
    *launches = e->ev_used[which];
    *total_ms = sum;
    return FPNN_AES_OK;
}

const char *fpnn_aes_engine_last_kernel(fpnn_aes_engine *e, int which) {
    if (!e || which < 0 || which > 2) return "";
    if (which == FPNN_AES_K_HOST) return e->host_path;
    return e->last_kernel[which];
}

int fpnn_aes_engine_reset_stats(fpnn_aes_engine *e) {
    if (!e) return FPNN_AES_ERR_ARG;
    e->ev_used[0] = e->ev_used[1] = 0;
    return FPNN_AES_OK;
}

}  // extern "C"

// ---- ECDH key derivation (include/fpnn_ecdh.h, k_ecdh.hip) -------------------------------
namespace {

int ecdh_const(int curve, EccConst &c) {
    if (!ecc_fill_const(curve, c)) {
        g_last_error = "unknown ECDH curve";
        return FPNN_AES_ERR_ARG;
    }
    return FPNN_AES_OK;
}

bool aligned4(const void *p) { return ((uintptr_t)p & 3u) == 0; }

int ecdh_launch(fpnn_aes_engine *e, int curve, const EccConst &c, const EcdhJob &j) {
    if (j.count == 0) return FPNN_AES_OK;
    if (!aligned4(j.priv) || !aligned4(j.pub) || !aligned4(j.key_out) || !aligned4(j.iv_out) ||
        !aligned4(j.pub_out)) {
        g_last_error = "ECDH device buffers must be 4-byte aligned";
        return FPNN_AES_ERR_ARG;
    }
    DeviceGuard g(e->device);
    const BatchScope batch_scope(e);  // (an early return clears the pending flag)
    HIP_TRY(launch_ecdh(c, j, curve, e->stream));
    batch_queued(e);
    return FPNN_AES_OK;
}

}  // namespace

extern "C" {

int fpnn_ecdh_curve(const char *name) {
    if (!name) return -1;
    for (int i = 0; i < ECC_NCURVES; i++)
        if (strcmp(name, ecc_curve_info(i).name) == 0) return i;
    return -1;
}

int fpnn_ecdh_secret_len(int curve) {
    return curve >= 0 && curve < ECC_NCURVES ? ecc_curve_info(curve).num_bytes : -1;
}

int fpnn_ecdh_private_len(int curve) {
    return curve >= 0 && curve < ECC_NCURVES ? (ecc_curve_info(curve).num_n_bits + 7) / 8 : -1;
}

const char *fpnn_ecdh_curve_name(int curve) {
    return curve >= 0 && curve < ECC_NCURVES ? ecc_curve_info(curve).name : nullptr;
}

int fpnn_ecdh_random_private(int curve, uint8_t *out) {
    EccConst c;
    if (!out || !ecc_fill_const(curve, c)) return 0;
    const int nw = c.nw, bits = c.num_n_bits;
    for (int tries = 0; tries < 64; tries++) {
        uint32_t k[8] = {0};
        size_t got = 0;
        while (got < sizeof(uint32_t) * nw) {
            const ssize_t r = getrandom(reinterpret_cast<uint8_t *>(k) + got, sizeof(uint32_t) * nw - got, 0);
            if (r < 0) {
                if (errno == EINTR) continue;
                return 0;
            }
            got += (size_t)r;
        }
        if (bits < 32 * nw) k[nw - 1] &= 0xFFFFFFFFu >> (32 * nw - bits);
        bool zero = true, below = false, decided = false;
        for (int w = nw - 1; w >= 0; w--) {
            zero = zero && k[w] == 0;
            if (!decided && k[w] != c.n[w]) {
                below = k[w] < c.n[w];
                decided = true;
            }
        }
        if (zero || !below) continue;
        const int pb = c.private_bytes;
        for (int i = 0; i < pb; i++) out[i] = (uint8_t)(k[(pb - 1 - i) / 4] >> (8 * ((pb - 1 - i) % 4)));
        return 1;
    }
    return 0;
}

int fpnn_ecdh_calc_keys(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                        uint32_t count, int keylen, uint8_t *keys, uint8_t *ivs, uint8_t *ok) {
    if (!e || !private_key || (count && (!peer_public || !keys || !ivs || !ok))) return FPNN_AES_ERR_ARG;
    if (keylen != 16 && keylen != 32) return FPNN_AES_ERR_KEYLEN;
    EccConst c;
    int rc = ecdh_const(curve, c);
    if (rc) return rc;
    ecc_set_uniform_scalar(c, private_key);
    EcdhJob j{};
    j.pub = peer_public;
    j.count = count;
    j.mode = ECDH_KEYS;
    j.keylen = keylen;
    j.key_out = keys;
    j.iv_out = ivs;
    j.ok_out = ok;
    return ecdh_launch(e, curve, c, j);
}

int fpnn_ecdh_calc_keys_client(fpnn_aes_engine *e, int curve, const uint8_t *private_keys,
                               const uint8_t *server_public, uint32_t count, int keylen, uint8_t *keys,
                               uint8_t *ivs, uint8_t *ok) {
    if (!e || !server_public || (count && (!private_keys || !keys || !ivs || !ok))) return FPNN_AES_ERR_ARG;
    if (keylen != 16 && keylen != 32) return FPNN_AES_ERR_KEYLEN;
    EccConst c;
    int rc = ecdh_const(curve, c);
    if (rc) return rc;
    ecc_set_uniform_point(c, server_public);
    EcdhJob j{};
    j.priv = private_keys;
    j.count = count;
    j.mode = ECDH_KEYS;
    j.keylen = keylen;
    j.key_out = keys;
    j.iv_out = ivs;
    j.ok_out = ok;
    return ecdh_launch(e, curve, c, j);
}

int fpnn_ecdh_public_keys(fpnn_aes_engine *e, int curve, const uint8_t *private_keys, uint32_t count,
                          uint8_t *public_keys, uint8_t *ok) {
    if (!e || (count && (!private_keys || !public_keys || !ok))) return FPNN_AES_ERR_ARG;
    EccConst c;
    int rc = ecdh_const(curve, c);  // px, py = G
    if (rc) return rc;
    EcdhJob j{};
    j.priv = private_keys;
    j.count = count;
    j.mode = ECDH_PUBLIC;
    j.pub_out = public_keys;
    j.ok_out = ok;
    return ecdh_launch(e, curve, c, j);
}

int fpnn_ecdh_keyset(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                     uint32_t count, int keylen, uint8_t *ok, fpnn_aes_keyset **out) {
    if (!e || !out || count == 0) return FPNN_AES_ERR_ARG;
    *out = nullptr;
    if (keylen != 16 && keylen != 32) return FPNN_AES_ERR_KEYLEN;
    DeviceGuard g(e->device);
    const size_t kb = (size_t)count * keylen, ib = (size_t)count * 16;
    int rc = grow(e, e->d_ecdh, e->cap_ecdh, kb + ib + count);  // keys | ivs | ok, engine scratch
    if (rc) return rc;
    uint8_t *tmp = e->d_ecdh;
    rc = fpnn_ecdh_calc_keys(e, curve, private_key, peer_public, count, keylen, tmp, tmp + kb, ok ? ok : tmp + kb + ib);
    if (!rc) rc = fpnn_aes_keyset_create(e, count, (size_t)keylen, tmp, tmp + kb, 0, out);  // synchronizes
    return rc;
}

int fpnn_ecdh_calc_keys_host(fpnn_aes_engine *e, int curve, const uint8_t *private_key, const uint8_t *peer_public,
                             uint32_t count, int keylen, uint8_t *keys, uint8_t *ivs, uint8_t *ok) {
    if (!e || !private_key || (count && (!peer_public || !keys || !ivs || !ok))) return FPNN_AES_ERR_ARG;
    if (keylen != 16 && keylen != 32) return FPNN_AES_ERR_KEYLEN;
    const int sl = fpnn_ecdh_secret_len(curve);
    if (sl < 0) return FPNN_AES_ERR_ARG;
    if (count == 0) return FPNN_AES_OK;
    DeviceGuard g(e->device);
    const size_t pb = (size_t)count * 2 * sl, kb = (size_t)count * keylen, ib = (size_t)count * 16;
    int rc = grow(e, e->d_ecdh, e->cap_ecdh, pb + kb + ib + count);  // peers | keys | ivs | ok
    if (rc) return rc;
    uint8_t *d = e->d_ecdh;
    do {
        hipError_t err = hipMemcpyAsync(d, peer_public, pb, hipMemcpyHostToDevice, e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh upload"); break; }
        if ((rc = fpnn_ecdh_calc_keys(e, curve, private_key, d, count, keylen, d + pb, d + pb + kb,
                                      d + pb + kb + ib)))
            break;
        err = hipMemcpyAsync(keys, d + pb, kb, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipMemcpyAsync(ivs, d + pb + kb, ib, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipMemcpyAsync(ok, d + pb + kb + ib, count, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh download"); break; }
    } while (0);
    return rc;
}

int fpnn_ecdh_calc_key_host(fpnn_aes_engine *e, const char *curve, const uint8_t *private_key, size_t private_len,
                            const uint8_t *peer_public, size_t peer_len, int keylen, uint8_t *key, uint8_t *iv) {
    if (!e) return FPNN_AES_ERR_ARG;
    // ECCKeyExchange::init + calcKey's own checks, in the reference's order
    const int cv = fpnn_ecdh_curve(curve);
    if (cv < 0 || (int)private_len != fpnn_ecdh_private_len(cv) || !private_key) return 0;
    if ((int)peer_len != 2 * fpnn_ecdh_secret_len(cv) || !peer_public) return 0;
    if (keylen != 16 && keylen != 32) return 0;
    if (!key || !iv) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    int rc = grow(e, e->d_ecdh, e->cap_ecdh, 64 + 32 + 16 + 16);  // peer (<= 64) | key (32) | iv (16) | ok
    if (rc) return rc;
    uint8_t *d = e->d_ecdh;
    uint8_t res[32 + 16 + 1];
    do {
        hipError_t err = hipMemcpyAsync(d, peer_public, peer_len, hipMemcpyHostToDevice, e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh upload"); break; }
        if ((rc = fpnn_ecdh_calc_keys(e, cv, private_key, d, 1, keylen, d + 64, d + 96, d + 112))) break;
        err = hipMemcpyAsync(res, d + 64, sizeof res, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh download"); break; }
    } while (0);
    if (rc) return rc;
    if (!res[48]) return 0;
    memcpy(key, res, (size_t)keylen);
    memcpy(iv, res + 32, 16);
    return 1;
}

int fpnn_ecdh_public_key_host(fpnn_aes_engine *e, int curve, const uint8_t *private_key, uint8_t *public_key) {
    if (!e || !private_key || !public_key) return FPNN_AES_ERR_ARG;
    const int pl = fpnn_ecdh_private_len(curve), sl = fpnn_ecdh_secret_len(curve);
    if (pl < 0) return FPNN_AES_ERR_ARG;
    DeviceGuard g(e->device);
    int rc = grow(e, e->d_ecdh, e->cap_ecdh, 32 + 64 + 16);  // private (<= 32) | public (<= 64) | ok
    if (rc) return rc;
    uint8_t *d = e->d_ecdh;
    uint8_t res[64 + 1];
    do {
        hipError_t err = hipMemcpyAsync(d, private_key, (size_t)pl, hipMemcpyHostToDevice, e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh upload"); break; }
        if ((rc = fpnn_ecdh_public_keys(e, curve, d, 1, d + 32, d + 96))) break;
        err = hipMemcpyAsync(res, d + 32, 64, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipMemcpyAsync(res + 64, d + 96, 1, hipMemcpyDeviceToHost, e->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
        if (err != hipSuccess) { rc = hip_fail(err, "ecdh download"); break; }
    } while (0);
    if (rc) return rc;
    memcpy(public_key, res, (size_t)(2 * sl));
    return res[64] ? 1 : 0;
}

}  // extern "C"
