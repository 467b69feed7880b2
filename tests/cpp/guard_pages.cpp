// guard_pages.cpp -- ragged encrypt batches over buffers that end (or start) exactly at an
// unmapped page (the r05x illegal-address fault).
//
// Every array a call reads or writes -- payload in / out, in_off, out_off, len, key_slot,
// the stream (iv, pos) state -- gets a virtual-memory mapping of its own
// (hipMemAddressReserve / hipMemCreate / hipMemMap) with an unmapped granule on each side,
// and is placed so that its LAST byte is the mapping's last byte ("end") or its FIRST byte
// the mapping's first ("start").  A kernel that touches one byte past either end of any
// array then faults at once and every time, instead of only when a torch allocation happens
// to end at a mapping boundary.  Outputs are compared with the oracle (oracle/aes_oracle.c,
// test infrastructure), the gap bytes between frames included.
//
// The shapes are tests/test_gpu_hybrid.py's wire-frame and ragged cases (the r05x test was
// test_wire_frames_every_offset[1-16-1-hybrid_lane_engine]: 2 500 wire frames, AES-128), the
// stream segments, and FPNN's short quests through K2 (max_len), each on the engine settings
// the tests use.  With FPNN_AES_GPU_LIB pointing at libfpnn_aes_gpu_audit.so the same run
// also checks every access of K2h / K2 / the length order against its extent (audit.hpp).
//
//   guard_pages [--direct-copy] [--malloc] [--keep-going] [--reuse-va] [filter]
//                one line per (case, engine, placement); exit 0 when all pass
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/fpnn_aes.h"
#include "../../oracle/aes_oracle.h"

namespace {

#define HIPCHK(x)                                                                               \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(3);                                                                            \
        }                                                                                       \
    } while (0)

size_t g_gran = 0;
bool g_direct_copy = false;  // --direct-copy: hipMemcpy of the array's bytes only (else whole mapped pages)
bool g_malloc = false;       // --malloc: plain hipMalloc allocations of the exact size (no guard pages)
bool g_keep_going = false;   // --keep-going: run every case after a failure
// --reuse-va: unmap and release each case's mappings when it ends (their virtual addresses
// come back for the next case's arrays); by default they stay mapped until the process
// exits, so no device virtual address is ever mapped twice in one run
bool g_reuse_va = false;

// one array in a mapping of its own, an unmapped granule before and after it
struct Guarded {
    void *va = nullptr;  // the reservation (guard | mapping | guard)
    size_t va_size = 0, map_size = 0;
    hipMemGenericAllocationHandle_t h{};
    uint8_t *ptr = nullptr;  // the array
    size_t n = 0;
    Guarded(size_t bytes, bool at_end) : n(bytes) {
        if (g_malloc) {
            HIPCHK(hipMalloc(reinterpret_cast<void **>(&ptr), bytes ? bytes : 1));
            return;
        }
        map_size = (bytes + g_gran - 1) / g_gran * g_gran;
        if (map_size == 0) map_size = g_gran;
        va_size = map_size + 2 * g_gran;
        HIPCHK(hipMemAddressReserve(&va, va_size, g_gran, nullptr, 0));
        hipMemAllocationProp prop;
        memset(&prop, 0, sizeof prop);
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = 0;
        HIPCHK(hipMemCreate(&h, map_size, &prop, 0));
        uint8_t *mid = static_cast<uint8_t *>(va) + g_gran;
        HIPCHK(hipMemMap(mid, map_size, 0, h, 0));
        hipMemAccessDesc acc;
        memset(&acc, 0, sizeof acc);
        acc.location.type = hipMemLocationTypeDevice;
        acc.location.id = 0;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        HIPCHK(hipMemSetAccess(mid, map_size, &acc, 1));
        ptr = at_end ? mid + map_size - bytes : mid;
    }
    ~Guarded() {
        if (g_malloc) {
            (void)hipFree(ptr);
            return;
        }
        if (!g_reuse_va) return;  // (left mapped: the process exit releases it)
        uint8_t *mid = static_cast<uint8_t *>(va) + g_gran;
        (void)hipMemUnmap(mid, map_size);
        (void)hipMemRelease(h);
        (void)hipMemAddressFree(va, va_size);
    }
    // Copies move whole mapped pages from / to a host image (page-aligned, whole-page copies),
    // and every upload is read back and compared, so a copy path that mishandles a
    // destination at an odd address inside a mapping cannot pass for a kernel error.
    uint8_t *mid() const { return static_cast<uint8_t *>(va) + g_gran; }
    bool put(const void *src) {
        if (g_malloc || g_direct_copy) {
            HIPCHK(hipMemcpy(ptr, src, n, hipMemcpyHostToDevice));
        } else {
            std::vector<uint8_t> img(map_size, 0);
            memcpy(&img[ptr - mid()], src, n);
            HIPCHK(hipMemcpy(mid(), img.data(), map_size, hipMemcpyHostToDevice));
        }
        std::vector<uint8_t> back(n);
        get(back.data());
        return memcmp(back.data(), src, n) == 0;
    }
    void get(void *dst) const {
        if (g_malloc || g_direct_copy) {
            HIPCHK(hipMemcpy(dst, ptr, n, hipMemcpyDeviceToHost));
            return;
        }
        std::vector<uint8_t> img(map_size);
        HIPCHK(hipMemcpy(img.data(), mid(), map_size, hipMemcpyDeviceToHost));
        memcpy(dst, &img[ptr - mid()], n);
    }
    Guarded(const Guarded &) = delete;
    Guarded &operator=(const Guarded &) = delete;
};

struct Rng {  // splitmix64
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
    void bytes(std::vector<uint8_t> &v) {
        for (auto &b : v) b = (uint8_t)next();
    }
};

struct Case {
    const char *name;
    int kind;  // 0 wire frames, 1 ragged package, 2 stream segments, 3 short quests (K2, max_len)
    uint32_t n, keylen, nkeys, grid, maxlen;
};

struct EngineKind {
    const char *name;
    const char *env[4][2];
};

// tests/conftest.py's HYBRID_ENGINES (+ the default engine); variables an engine does not
// know are ignored by it
const EngineKind kEngines[] = {
    {"engine", {{nullptr, nullptr}}},
    {"hybrid_engine", {{"FPNN_AES_HYB_FORCE", "1"}, {"FPNN_AES_HYB_LONG", "64"}, {"FPNN_AES_HYB_QW", "3"}, {nullptr, nullptr}}},
    {"hybrid_lane_engine",
     {{"FPNN_AES_HYB_FORCE", "1"}, {"FPNN_AES_HYB_LONG", "1000000000"}, {"FPNN_AES_HYB_QW", "2"}, {nullptr, nullptr}}},
    {"hybrid_quad_engine", {{"FPNN_AES_HYB_FORCE", "1"}, {"FPNN_AES_HYB_LONG", "1"}, {"FPNN_AES_HYB_QW", "0"}, {nullptr, nullptr}}},
};

const Case kCases[] = {
    {"wire_g1_aes128", 0, 2500, 16, 1, 1, 0},   // the r05x shape
    {"wire_g4_aes128", 0, 2500, 16, 1, 4, 0},
    {"wire_g1_aes192_5k", 0, 2500, 24, 5, 1, 0},
    {"wire_g1_aes256_200k", 0, 2500, 32, 200, 1, 0},
    {"ragged_aes256", 1, 3000, 32, 1, 1, 0},
    {"ragged_aes128_7k", 1, 3000, 16, 7, 1, 0},
    {"stream_aes128", 2, 3000, 16, 3000, 1, 0},
    {"stream_aes256", 2, 3000, 32, 3000, 1, 0},
    {"quests_aes256", 3, 300000, 32, 4096, 1, 145},  // > one chain per GPU lane: K2 under max_len
    {"quests_wire_aes128", 3, 300000, 16, 4096, 1, 145},
};

int run_case(const Case &c, fpnn_aes_engine *e, bool at_end, uint64_t seed, std::string &why) {
    Rng r(seed);
    const uint32_t n = c.n;
    std::vector<uint32_t> len(n), slot(n);
    std::vector<uint64_t> in_off(n), out_off(n);
    static const uint32_t special[] = {0, 1, 4, 11, 12, 15, 16, 17, 28, 32, 124, 127, 128, 129, 1024, 1025};
    const bool wire = c.kind == 0 || (c.kind == 3 && c.keylen == 16);
    uint64_t ip = 3, op = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t L;
        if (c.kind == 3) L = 100 + r.below(c.maxlen - 99);  // FPNN quests: 100..145 B
        else if (c.kind == 1) L = 64 * (1 + (r.below(1000) < 30 ? r.below(1024) : r.below(16))) + (r.below(4) ? 0 : r.below(16));
        else L = r.below(10) < 3 ? special[r.below(16)] : r.below(3001);
        len[i] = L;
        in_off[i] = ip;
        ip += L + (c.kind == 3 ? 0 : 5);
        const uint32_t gap = c.kind == 3 ? 0 : r.below(18);
        out_off[i] = op;
        uint64_t span = (uint64_t)L + (wire ? 4 : 0) + gap;
        span = (span + c.grid - 1) / c.grid * c.grid;
        op += span;
        slot[i] = c.nkeys > 1 ? r.below(c.nkeys) : 0;
    }
    (void)op;
    uint64_t in_bytes = 1, out_bytes = 1;  // no slack: the arrays end where the last frame ends
    for (uint32_t i = 0; i < n; i++) {
        in_bytes = std::max<uint64_t>(in_bytes, in_off[i] + len[i]);
        out_bytes = std::max<uint64_t>(out_bytes, out_off[i] + len[i] + (wire ? 4 : 0));
    }
    std::vector<uint8_t> plain(in_bytes), dst0(out_bytes), keys(c.nkeys * c.keylen), ivs(16 * c.nkeys);
    r.bytes(plain);
    r.bytes(dst0);
    r.bytes(keys);
    r.bytes(ivs);
    std::vector<uint8_t> exp = dst0;
    std::vector<uint8_t> iv_state, iv_exp;
    std::vector<uint32_t> pos_state, pos_exp;
    if (c.kind == 2) {
        iv_state.resize(16 * (size_t)n);
        pos_state.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            memcpy(&iv_state[16 * (size_t)i], &ivs[16 * (size_t)slot[i] % ivs.size()], 16);
            pos_state[i] = r.below(16);
            slot[i] = i % c.nkeys;
        }
        iv_exp = iv_state;
        pos_exp = pos_state;
        ao_stream_batch(1, plain.data(), exp.data(), n, in_off.data(), out_off.data(), len.data(), slot.data(),
                        keys.data(), c.keylen, iv_exp.data(), pos_exp.data(), 8);
    } else if (wire) {
        std::vector<uint64_t> body(n);
        for (uint32_t i = 0; i < n; i++) body[i] = out_off[i] + 4;
        ao_package_batch(1, plain.data(), exp.data(), n, 0, 0, in_off.data(), body.data(), len.data(),
                         c.nkeys > 1 ? slot.data() : nullptr, keys.data(), c.keylen, ivs.data(), 8);
        for (uint32_t i = 0; i < n; i++) memcpy(&exp[out_off[i]], &len[i], 4);  // htole32 (little-endian host)
    } else {
        ao_package_batch(1, plain.data(), exp.data(), n, 0, 0, in_off.data(), out_off.data(), len.data(),
                         c.nkeys > 1 ? slot.data() : nullptr, keys.data(), c.keylen, ivs.data(), 8);
    }
    fpnn_aes_keyset *ks = nullptr;
    int rc = fpnn_aes_keyset_create(e, c.nkeys, c.keylen, keys.data(), ivs.data(), 1, &ks);
    if (rc) {
        why = std::string("keyset_create: ") + fpnn_aes_last_error();
        return rc;
    }
    Guarded g_in(in_bytes, at_end), g_out(out_bytes, at_end), g_ioff(8 * (size_t)n, at_end),
        g_ooff(8 * (size_t)n, at_end), g_len(4 * (size_t)n, at_end), g_slot(4 * (size_t)n, at_end);
    if (!g_in.put(plain.data()) || !g_out.put(dst0.data()) || !g_ioff.put(in_off.data()) ||
        !g_ooff.put(out_off.data()) || !g_len.put(len.data()) || !g_slot.put(slot.data())) {
        why = "upload read back differently (HIP copy path)";
        fpnn_aes_keyset_destroy(ks);
        return -102;
    }
    std::unique_ptr<Guarded> g_iv, g_pos;
    fpnn_aes_batch b;
    memset(&b, 0, sizeof b);
    b.in = g_in.ptr;
    b.out = g_out.ptr;
    b.count = n;
    b.in_off = reinterpret_cast<const uint64_t *>(g_ioff.ptr);
    b.out_off = reinterpret_cast<const uint64_t *>(g_ooff.ptr);
    b.len = reinterpret_cast<const uint32_t *>(g_len.ptr);
    b.key_slot = (c.nkeys > 1) ? reinterpret_cast<const uint32_t *>(g_slot.ptr) : nullptr;
    b.keys = ks;
    b.flags = wire ? FPNN_AES_F_WIRE_PREFIX : 0u;
    b.max_len = c.maxlen;
    if (c.kind == 2) {
        g_iv.reset(new Guarded(iv_state.size(), at_end));
        g_pos.reset(new Guarded(4 * (size_t)n, at_end));
        if (!g_iv->put(iv_state.data()) || !g_pos->put(pos_state.data())) {
            why = "upload read back differently (HIP copy path)";
            fpnn_aes_keyset_destroy(ks);
            return -102;
        }
        if ((uintptr_t)g_iv->ptr & 15) {  // (iv_state must be 16-byte aligned: n * 16 bytes end on the grid)
            why = "iv_state misaligned";
            return -100;
        }
        rc = fpnn_aes_stream_encrypt(e, &b, g_iv->ptr, reinterpret_cast<uint32_t *>(g_pos->ptr));
    } else {
        rc = fpnn_aes_package_encrypt(e, &b);
    }
    if (rc == FPNN_AES_OK) rc = fpnn_aes_engine_sync(e);
    if (rc != FPNN_AES_OK) {
        why = fpnn_aes_last_error();
        fpnn_aes_keyset_destroy(ks);
        return rc;
    }
    std::vector<uint8_t> got(out_bytes);
    g_out.get(got.data());
    size_t bad = 0, first = 0;
    for (size_t i = 0; i < out_bytes; i++)
        if (got[i] != exp[i] && !bad++) first = i;
    if (c.kind == 2) {
        std::vector<uint8_t> giv(iv_state.size());
        std::vector<uint32_t> gpos(n);
        g_iv->get(giv.data());
        g_pos->get(gpos.data());
        if (giv != iv_exp || gpos != pos_exp) bad += 1000000000;
    }
    fpnn_aes_keyset_destroy(ks);
    if (bad) {
        // which frames: the first bad one's descriptor and where in it the bytes differ
        uint32_t nbadf = 0, fi = n;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t o = out_off[i], e = o + len[i] + (wire ? 4 : 0);
            bool fb = false;
            for (uint64_t k = o; k < e && !fb; k++) fb = got[k] != exp[k];
            if (fb && !nbadf++) fi = i;
        }
        char m[400];
        if (fi < n) {
            const uint64_t o = out_off[fi], e = o + len[fi] + (wire ? 4 : 0);
            uint64_t k0 = e, k1 = o;
            for (uint64_t k = o; k < e; k++)
                if (got[k] != exp[k]) {
                    k0 = std::min(k0, k);
                    k1 = k + 1;
                }
            snprintf(m, sizeof m,
                     "%zu bytes differ, first at %zu; %u frames bad, first frame %u (in_off %llu out_off %llu len %u "
                     "slot %u): bytes [%llu, %llu) of it; in at 0x%llx out at 0x%llx",
                     bad, first, nbadf, fi, (unsigned long long)in_off[fi], (unsigned long long)o, len[fi], slot[fi],
                     (unsigned long long)(k0 - o), (unsigned long long)(k1 - o),
                     (unsigned long long)(uintptr_t)(g_in.ptr + in_off[fi]), (unsigned long long)(uintptr_t)(g_out.ptr + o));
        } else {
            snprintf(m, sizeof m, "%zu bytes differ, first at %zu (outside every frame; state arrays: %s)", bad, first,
                     bad >= 1000000000 ? "differ" : "equal");
        }
        why = m;
        return -101;
    }
    return FPNN_AES_OK;
}

}  // namespace

int main(int argc, char **argv) {
    const char *filter = "";
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--direct-copy")) g_direct_copy = true;
        else if (!strcmp(argv[i], "--malloc")) g_malloc = true;
        else if (!strcmp(argv[i], "--keep-going")) g_keep_going = true;
        else if (!strcmp(argv[i], "--reuse-va")) g_reuse_va = true;
        else filter = argv[i];
    }
    int vmm = 0;
    HIPCHK(hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, 0));
    if (!vmm) {
        printf("guard_pages: device 0 has no HIP virtual memory management\n");
        return 4;
    }
    hipMemAllocationProp prop;
    memset(&prop, 0, sizeof prop);
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    HIPCHK(hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityMinimum));
    printf("granularity %zu B, %s, library %s\n", g_gran,
           g_malloc ? "hipMalloc arrays" : g_direct_copy ? "array-range copies" : "whole-page copies", fpnn_aes_version());
    printf("mappings %s\n", g_reuse_va ? "released after each case (addresses reused)" : "kept until exit (no address reused)");
    int failed = 0, ran = 0;
    for (const EngineKind &k : kEngines) {
        for (const auto &kv : k.env)
            if (kv[0]) setenv(kv[0], kv[1], 1);
        fpnn_aes_engine *e = nullptr;
        const int rc = fpnn_aes_engine_create(0, FPNN_AES_OWN_STREAM, &e);
        for (const auto &kv : k.env)
            if (kv[0]) unsetenv(kv[0]);
        if (rc) {
            printf("engine %s: create failed: %s\n", k.name, fpnn_aes_last_error());
            return 5;
        }
        for (const Case &c : kCases) {
            if (*filter && !strstr(c.name, filter) && !strstr(k.name, filter)) continue;
            if (c.kind == 3 && strcmp(k.name, "engine") != 0) continue;  // (K2 under max_len: default settings)
            for (int at_end = 1; at_end >= 0; at_end--) {
                std::string why;
                const int r = run_case(c, e, at_end != 0, 0x5eed0000u + 977u * (uint32_t)(&c - kCases), why);
                ran++;
                printf("%-22s %-20s %-5s %s%s\n", c.name, k.name, at_end ? "end" : "start", r ? "FAIL " : "ok",
                       r ? why.c_str() : "");
                fflush(stdout);
                if (r) failed++;
                if (r && !g_keep_going) {  // one failure tells its story; the next run could start from its debris
                    printf("stopping at the first failure (--keep-going runs on)\n");
                    return 1;
                }
            }
        }
        fpnn_aes_engine_destroy(e);
    }
    printf("%d of %d runs failed\n", failed, ran);
    return failed ? 1 : 0;
}
