// encryptor.cpp -- fpnn::PackageEncryptor / StreamEncryptor and the rijndael.h
// subset, implemented over the C-ABI (fpnn_aes.h).  Mirrors core/Encryptor.cpp:10-70
// call for call; the CFB work itself runs in the HIP kernels.
#include <endian.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/Encryptor.h"
#include "../../include/EncryptorBatch.h"
#include "../../include/fpnn_aes.h"
#include "fail_policy.hpp"
#include "thread_engine.hpp"

namespace {

using fpnn_aes::thread_engine;

std::string describe(int rc) {
    std::string s = fpnn_aes_strerror(rc);
    const char *d = fpnn_aes_last_error();
    if (d && *d) s += std::string(": ") + d;
    return s;
}

int cfb(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16],
        size_t *p_num) {
    int rc;
    const fpnn_aes::Lease lease = thread_engine(&rc);
    fpnn_aes_engine *e = lease.engine();
    if (!e) return rc ? rc : FPNN_AES_ERR_NODEV;
    static_assert(sizeof(rijndael_context) == sizeof(fpnn_aes_schedule), "context layout");
    return fpnn_aes_cfb_host(e, reinterpret_cast<const fpnn_aes_schedule *>(ctx), encrypt ? 1 : 0, in, out, len, ivec,
                             p_num);
}

// rijndael.h has no error path: report and abort (never a CPU fallback)
void or_abort(int rc, const char *fn) {
    if (rc == FPNN_AES_OK) return;
    fprintf(stderr, "%s (fpnn_aes, MI355X): %s\n", fn, describe(rc).c_str());
    abort();
}

// the calling thread's engine, locked while the returned lease lives
fpnn_aes::Lease engine_or_abort(const char *fn) {
    int rc;
    fpnn_aes::Lease lease = thread_engine(&rc);
    if (!lease.engine()) or_abort(rc ? rc : FPNN_AES_ERR_NODEV, fn);
    return lease;
}

const fpnn_aes_schedule *sched(const rijndael_context *ctx) {
    return reinterpret_cast<const fpnn_aes_schedule *>(ctx);
}

void cfb_or_fail(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                  uint8_t ivec[16], size_t *p_num) {
    const int rc = cfb(ctx, encrypt, in, out, len, ivec, p_num);
    if (rc != FPNN_AES_OK) fpnn_aes::device_failure("GPU CFB failed: " + describe(rc));  // (fail_policy.hpp)
}

}  // namespace

extern "C" {

bool rijndael_setup_encrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen) {
    return fpnn_aes_setup_encrypt(reinterpret_cast<fpnn_aes_schedule *>(ctx), key, keylen) == FPNN_AES_OK;
}

bool rijndael_setup_decrypt(rijndael_context *ctx, const uint8_t *key, size_t keylen) {
    return fpnn_aes_setup_decrypt(reinterpret_cast<fpnn_aes_schedule *>(ctx), key, keylen) == FPNN_AES_OK;
}

void rijndael_encrypt(const rijndael_context *ctx, const uint8_t plain[16], uint8_t cipher[16]) {
    or_abort(fpnn_aes_ecb_host(engine_or_abort("rijndael_encrypt").engine(), sched(ctx), 1, plain, cipher, 1),
             "rijndael_encrypt");
}

void rijndael_decrypt(const rijndael_context *ctx, const uint8_t cipher[16], uint8_t plain[16]) {
    or_abort(fpnn_aes_ecb_host(engine_or_abort("rijndael_decrypt").engine(), sched(ctx), 0, cipher, plain, 1),
             "rijndael_decrypt");
}

void rijndael_cbc_encrypt(const rijndael_context *ctx, const uint8_t *plain, uint8_t *cipher, size_t len,
                          uint8_t ivec[16]) {
    or_abort(fpnn_aes_cbc_host(engine_or_abort("rijndael_cbc_encrypt").engine(), sched(ctx), 1, plain, cipher, len, ivec),
             "rijndael_cbc_encrypt");
}

void rijndael_cbc_decrypt(const rijndael_context *ctx, const uint8_t *cipher, uint8_t *plain, size_t len,
                          uint8_t ivec[16]) {
    or_abort(fpnn_aes_cbc_host(engine_or_abort("rijndael_cbc_decrypt").engine(), sched(ctx), 0, cipher, plain, len, ivec),
             "rijndael_cbc_decrypt");
}

void rijndael_cfb_encrypt(const rijndael_context *ctx, bool encrypt, const uint8_t *in, uint8_t *out, size_t len,
                          uint8_t ivec[16], size_t *p_num) {
    or_abort(cfb(ctx, encrypt, in, out, len, ivec, p_num), "rijndael_cfb_encrypt");
}

void rijndael_ofb_encrypt(const rijndael_context *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16],
                          size_t *p_num) {
    or_abort(fpnn_aes_ofb_host(engine_or_abort("rijndael_ofb_encrypt").engine(), sched(ctx), in, out, len, ivec, p_num),
             "rijndael_ofb_encrypt");
}

}  // extern "C"

namespace fpnn {

void PackageEncryptor::decrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:10-20
    if (len <= 0) return;
    uint8_t iv[16];
    memcpy(iv, _iv, 16);
    size_t pos = 0;
    cfb_or_fail(&_ctx, false, src, dest, (size_t)len, iv, &pos);
}

void PackageEncryptor::encrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:22-32
    if (len <= 0) return;
    uint8_t iv[16];
    memcpy(iv, _iv, 16);
    size_t pos = 0;
    cfb_or_fail(&_ctx, true, src, dest, (size_t)len, iv, &pos);
}

void PackageEncryptor::encrypt(std::string *buffer) {  // core/Encryptor.cpp:34-51
    const size_t n = buffer->length();
    std::string framed(n + sizeof(uint32_t), '\0');
    const uint32_t le = htole32((uint32_t)n);
    memcpy(&framed[0], &le, sizeof le);
    if (n) {
        uint8_t iv[16];
        memcpy(iv, _iv, 16);
        size_t pos = 0;
        cfb_or_fail(&_ctx, true, reinterpret_cast<const uint8_t *>(buffer->data()),
                     reinterpret_cast<uint8_t *>(&framed[sizeof(uint32_t)]), n, iv, &pos);
    }
    buffer->swap(framed);
}

void StreamEncryptor::decrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:53-56
    if (len <= 0) return;
    cfb_or_fail(&_ctx, false, src, dest, (size_t)len, _iv, &_pos);
}

void StreamEncryptor::encrypt(uint8_t *dest, uint8_t *src, int len) {  // core/Encryptor.cpp:58-61
    if (len <= 0) return;
    cfb_or_fail(&_ctx, true, src, dest, (size_t)len, _iv, &_pos);
}

void StreamEncryptor::encrypt(std::string *buffer) {  // core/Encryptor.cpp:63-70
    const size_t n = buffer->length();
    if (!n) return;
    std::string out(n, '\0');
    cfb_or_fail(&_ctx, true, reinterpret_cast<const uint8_t *>(buffer->data()), reinterpret_cast<uint8_t *>(&out[0]),
                 n, _iv, &_pos);
    buffer->swap(out);
}

// ---- EncryptorBatch (include/EncryptorBatch.h) ------------------------------------------

void EncryptorBatch::add(Encryptor *enc, bool encrypt, uint8_t *dest, const uint8_t *src, int len,
                         std::string *buffer) {
    if (!enc) throw EncryptorError("EncryptorBatch: null encryptor");
    if (enc->_kind != 1 && enc->_kind != 2) throw EncryptorError("EncryptorBatch: unsupported Encryptor subclass");
    if (!buffer && len <= 0) return;  // the per-call methods do nothing for len <= 0
    _ops.push_back({enc, dest, src, buffer ? (uint32_t)buffer->size() : (uint32_t)len, encrypt, buffer});
    _bytes += _ops.back().len;
}

void EncryptorBatch::encrypt(Encryptor *enc, std::string *buffer) {
    if (!buffer) throw EncryptorError("EncryptorBatch: null buffer");
    add(enc, true, nullptr, nullptr, 0, buffer);
}

void EncryptorBatch::encrypt(Encryptor *enc, uint8_t *dest, uint8_t *src, int len) {
    add(enc, true, dest, src, len, nullptr);
}

void EncryptorBatch::decrypt(Encryptor *enc, uint8_t *dest, uint8_t *src, int len) {
    add(enc, false, dest, src, len, nullptr);
}

namespace {

// Serials retired by ~Encryptor / Encryptor::operator=, delivered only to the key tables
// that hold a slot for them (each drops them from its slot map at its next flush): a
// table's inbox never holds more serials than the table registered, however many
// Encryptors the process creates and destroys.
struct RetireInbox {
    std::vector<uint64_t> serials;
};
struct RetireRegistry {
    std::mutex mu;
    std::unordered_map<uint64_t, std::vector<RetireInbox *>> held;  // serial -> tables holding it
    std::atomic<size_t> n{0};                                       // live key tables
};
RetireRegistry &registry() {
    static RetireRegistry *r = new RetireRegistry();  // never destroyed: Encryptors may die at exit
    return *r;
}

}  // namespace

uint64_t encryptor_serial() {
    static std::atomic<uint64_t> next{1};
    return next.fetch_add(1, std::memory_order_relaxed);
}

void encryptor_retire(uint64_t serial) {
    RetireRegistry &r = registry();
    if (r.n.load(std::memory_order_acquire) == 0) return;  // no EncryptorBatch key table exists
    std::lock_guard<std::mutex> lk(r.mu);
    auto it = r.held.find(serial);
    if (it == r.held.end()) return;
    for (RetireInbox *b : it->second) b->serials.push_back(serial);
    r.held.erase(it);
}

// Persistent per-key-length table: slot per Encryptor serial, uploaded once
// (fpnn_aes_keyset_set).  Stream state of the touched slots is staged in iv/pos, sized
// like the table, so a flush never touches more than its own connections.  The table
// belongs to one engine, identified by its id.
// Key-table generations: an Encryptor caches (tag, slot) of the table it was last given a
// slot in (Encryptor::_batchCache, one atomic word); a table takes a new tag whenever it starts
// over, so no stale slot is ever used.  Flush ids mark the stream encryptors a flush lists.
uint64_t next_batch_tag() {
    static std::atomic<uint64_t> n{1};
    return n.fetch_add(1, std::memory_order_relaxed);
}

struct EncryptorBatch::KeyTable {
    uint64_t engine_id = 0;
    uint64_t tag = next_batch_tag();
    fpnn_aes_keyset *ks = nullptr;
    std::unordered_map<uint64_t, uint32_t> slot;
    uint32_t next = 0;
    std::vector<uint8_t> iv;
    std::vector<uint32_t> pos;
    RetireInbox inbox;
    std::unordered_map<uint64_t, bool> registered;  // serials whose retirement reaches this inbox
    KeyTable() { registry().n.fetch_add(1, std::memory_order_release); }
    ~KeyTable() {
        {
            RetireRegistry &r = registry();
            std::lock_guard<std::mutex> lk(r.mu);
            for (const auto &kv : registered) {
                auto it = r.held.find(kv.first);
                if (it == r.held.end()) continue;
                auto &v = it->second;
                v.erase(std::remove(v.begin(), v.end(), &inbox), v.end());
                if (v.empty()) r.held.erase(it);
            }
            r.n.fetch_sub(1, std::memory_order_release);
        }
        if (ks) fpnn_aes_keyset_destroy(ks);
    }
    // ask to hear of these serials' retirement (slots just handed out)
    void watch(const std::vector<uint64_t> &serials) {
        RetireRegistry &r = registry();
        std::lock_guard<std::mutex> lk(r.mu);
        for (uint64_t sr : serials)
            if (registered.emplace(sr, true).second) r.held[sr].push_back(&inbox);
    }
    // forget the slots of retired encryptors; true when most slots are dead, so the table
    // should start over (slots are handed out in order and never reused in place)
    bool collect() {
        std::vector<uint64_t> dead;
        {
            std::lock_guard<std::mutex> lk(registry().mu);
            dead.swap(inbox.serials);
        }
        for (uint64_t sr : dead) {
            slot.erase(sr);
            registered.erase(sr);
        }
        return next >= kTableMinReset && next > 2 * (uint32_t)slot.size();
    }
    static constexpr uint32_t kTableMinReset = 1024;
};

namespace {

// A table past this many slots starts over whatever is live.
constexpr uint32_t kTableMaxSlots = 1u << 20;
// Encryptor::_batchCache = (table tag: 40 bits) << 24 | slot (24 bits)
constexpr unsigned kCacheSlotBits = 24;
constexpr uint64_t kCacheSlotMask = (1ull << kCacheSlotBits) - 1;
constexpr uint64_t kCacheTagMask = (1ull << (64 - kCacheSlotBits)) - 1;

}  // namespace

EncryptorBatch::~EncryptorBatch() {
    for (KeyTable *&t : _tables) {
        delete t;
        t = nullptr;
    }
}

namespace {
// FPNN_AES_BATCH_STATS=1: per flush, where the host time goes (stderr)
struct BatchStats {
    bool on = getenv("FPNN_AES_BATCH_STATS") != nullptr;
    double t0 = 0, table = 0, frames = 0, call = 0, post = 0;
    static double now() {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
};
}  // namespace

void EncryptorBatch::flush() {
    std::vector<Op> ops;
    ops.swap(_ops);
    _bytes = 0;
    if (ops.empty()) return;
    BatchStats bs;
    if (bs.on) bs.t0 = BatchStats::now();
    struct Report {
        BatchStats &s;
        size_t n;
        ~Report() {
            if (s.on)
                fprintf(stderr, "[fpnn_aes batch] %zu ops: %.3f ms (table %.3f, frames %.3f, device call %.3f, post %.3f)\n",
                        n, 1e3 * (BatchStats::now() - s.t0), 1e3 * s.table, 1e3 * s.frames, 1e3 * s.call, 1e3 * s.post);
        }
    } report{bs, ops.size()};
    int rc;
    const fpnn_aes::Lease lease = thread_engine(&rc);
    fpnn_aes_engine *e = lease.engine();
    const uint64_t eid = lease.id();
    if (!e) fpnn_aes::device_failure("engine unavailable: " + describe(rc ? rc : FPNN_AES_ERR_NODEV));
    // group by (mode, direction, wire prefix, rounds); queue order is kept inside a group
    struct Group {
        bool stream, encrypt, prefix;
        int nrounds;
        std::vector<size_t> idx;
        // stream groups: each encryptor once, first use first, with its position in idx
        std::vector<std::pair<StreamEncryptor *, size_t>> members;
    };
    std::vector<Group> groups;
    static std::atomic<uint64_t> flush_ids{1};
    const uint64_t fid = flush_ids.fetch_add(1, std::memory_order_relaxed);
    size_t g = 0;  // (consecutive ops usually share a group)
    for (size_t i = 0; i < ops.size(); i++) {
        const Op &op = ops[i];
        const bool stream = op.enc->_kind == 2;
        StreamEncryptor *se = stream ? static_cast<StreamEncryptor *>(op.enc) : nullptr;
        const bool prefix = !stream && op.buffer != nullptr;
        const int nr = stream ? se->_ctx.nrounds : static_cast<PackageEncryptor *>(op.enc)->_ctx.nrounds;
        bool first = false;
        if (stream) {  // _batchSeen = flush id << 1 | direction
            // StreamEncryptor::encrypt(std::string*) of "" does nothing (core/Encryptor.cpp:63-70):
            // it is not grouped, so it must not mark the encryptor as listed either -- its
            // first grouped op has to stage the stream's (iv, pos) and take the result back
            const bool empty = op.buffer && op.buffer->empty();
            if ((se->_batchSeen >> 1) == fid) {
                if ((se->_batchSeen & 1) != (uint64_t)op.encrypt)
                    throw EncryptorError("EncryptorBatch: a StreamEncryptor used in both directions in one batch");
            } else if (!empty) {
                se->_batchSeen = fid << 1 | (uint64_t)op.encrypt;
                first = true;
            }
            if (empty) continue;
        }
        if (!(g < groups.size() && groups[g].stream == stream && groups[g].encrypt == op.encrypt &&
              groups[g].prefix == prefix && groups[g].nrounds == nr)) {
            g = 0;
            while (g < groups.size() && !(groups[g].stream == stream && groups[g].encrypt == op.encrypt &&
                                          groups[g].prefix == prefix && groups[g].nrounds == nr))
                g++;
            if (g == groups.size()) groups.push_back({stream, op.encrypt, prefix, nr, {}, {}});
        }
        if (first) groups[g].members.emplace_back(se, groups[g].idx.size());
        groups[g].idx.push_back(i);
    }
    for (const Group &gr : groups) {
        const double tg = bs.on ? BatchStats::now() : 0;
        // ---- this key length's table: new connections get slots, uploaded in one copy ----
        KeyTable *&tp = _tables[(gr.nrounds - 10) / 2];
        if (tp && tp->engine_id != eid) {  // flushed from another thread (engine): start a table there
            delete tp;
            tp = nullptr;
        }
        if (!tp) {
            tp = new KeyTable();
            tp->engine_id = eid;
            rc = fpnn_aes_keyset_reserve(e, 1024, gr.nrounds, &tp->ks);
            if (rc != FPNN_AES_OK) {
                delete tp;
                tp = nullptr;
                fpnn_aes::device_failure("EncryptorBatch: key table: " + describe(rc));
            }
        }
        KeyTable &t = *tp;
        if (t.collect()) {  // mostly dead connections: start over (live ones re-add below or later)
            t.slot.clear();
            t.next = 0;
            t.tag = next_batch_tag();
        }
        std::vector<uint32_t> slots(gr.idx.size());
        for (int attempt = 0;; attempt++) {
            std::vector<fpnn_aes_schedule> scheds;
            std::vector<uint8_t> ivs;
            std::vector<uint64_t> fresh;
            const uint32_t first_new = t.next;
            for (size_t k = 0; k < gr.idx.size(); k++) {
                Encryptor *enc = ops[gr.idx[k]].enc;
                const uint64_t c = enc->_batchCache.load(std::memory_order_relaxed);
                if (c != 0 && (c >> kCacheSlotBits) == (t.tag & kCacheTagMask)) {  // a connection this table holds
                    slots[k] = (uint32_t)(c & kCacheSlotMask);
                    continue;
                }
                auto ins = t.slot.emplace(enc->_serial, t.next);
                if (ins.second) {
                    const rijndael_context &ctx = gr.stream ? static_cast<const StreamEncryptor *>(enc)->_ctx
                                                            : static_cast<const PackageEncryptor *>(enc)->_ctx;
                    scheds.push_back(*reinterpret_cast<const fpnn_aes_schedule *>(&ctx));
                    ivs.insert(ivs.end(), enc->_iv, enc->_iv + 16);
                    fresh.push_back(enc->_serial);
                    t.next++;
                }
                slots[k] = ins.first->second;
                // (slots past the 24-bit field are found through the map every time)
                enc->_batchCache.store(slots[k] <= kCacheSlotMask
                                           ? (t.tag & kCacheTagMask) << kCacheSlotBits | slots[k] : 0u,
                                       std::memory_order_relaxed);
            }
            if (t.next > kTableMaxSlots && attempt == 0) {  // start over with this group's connections only
                t.slot.clear();
                t.next = 0;
                t.tag = next_batch_tag();
                continue;
            }
            rc = fpnn_aes_keyset_set(t.ks, first_new, (uint32_t)scheds.size(), scheds.data(), ivs.data());
            if (rc != FPNN_AES_OK) {
                // the slots handed out above were not uploaded: forget the table
                delete tp;
                tp = nullptr;
                fpnn_aes::device_failure("EncryptorBatch: key table upload: " + describe(rc));
            }
            t.watch(fresh);
            break;
        }
        double tt = bs.on ? BatchStats::now() : 0;
        if (bs.on) bs.table += tt - tg;
        std::vector<fpnn_aes_host_frame> frames(gr.idx.size());
        // package std::string outputs (len + 4), swapped in after the call.  (Growing the
        // buffer in place by 4 bytes instead -- a realloc for FPNN's exact-capacity frames --
        // measured slower: 1.43 against 0.6-0.9 ms per 8 192 frames, gpurun_out r05c/r05d.)
        std::vector<std::string> framed;
        if (gr.prefix) framed.resize(gr.idx.size());
        for (size_t k = 0; k < gr.idx.size(); k++) {
            Op &op = ops[gr.idx[k]];
            fpnn_aes_host_frame &f = frames[k];
            f.len = op.len;
            f.key_slot = slots[k];
            if (op.buffer) {
                f.src = reinterpret_cast<const uint8_t *>(op.buffer->data());
                if (gr.prefix) {
                    framed[k].assign(op.len + sizeof(uint32_t), '\0');
                    f.dst = reinterpret_cast<uint8_t *>(&framed[k][0]);
                } else {
                    f.dst = reinterpret_cast<uint8_t *>(&(*op.buffer)[0]);  // in place, same length
                }
            } else {
                f.src = op.src;
                f.dst = op.dest;
            }
        }
        if (bs.on) {
            const double t = BatchStats::now();
            bs.frames += t - tt;
            tt = t;
        }
        if (!gr.stream) {
            rc = fpnn_aes_package_host(e, gr.encrypt ? 1 : 0, frames.data(), (uint32_t)frames.size(), t.ks,
                                       gr.prefix ? FPNN_AES_F_WIRE_PREFIX : 0);
            if (rc != FPNN_AES_OK) fpnn_aes::device_failure("EncryptorBatch: package batch: " + describe(rc));
            if (bs.on) {
                const double t = BatchStats::now();
                bs.call += t - tt;
                tt = t;
            }
            if (gr.prefix)
                for (size_t k = 0; k < gr.idx.size(); k++) ops[gr.idx[k]].buffer->swap(framed[k]);
            if (bs.on) bs.post += BatchStats::now() - tt;
        } else {
            const uint32_t cnt = fpnn_aes_keyset_count(t.ks);
            if (t.pos.size() < cnt) {
                t.iv.resize(16 * (size_t)cnt);
                t.pos.resize(cnt);
            }
            for (const auto &m : gr.members) {  // the touched streams' current (iv, pos)
                const uint32_t sl = slots[m.second];
                memcpy(&t.iv[16 * (size_t)sl], m.first->_iv, 16);
                t.pos[sl] = (uint32_t)m.first->_pos;
            }
            rc = fpnn_aes_stream_host(e, gr.encrypt ? 1 : 0, frames.data(), (uint32_t)frames.size(), t.ks,
                                      t.iv.data(), t.pos.data());
            if (rc != FPNN_AES_OK) fpnn_aes::device_failure("EncryptorBatch: stream batch: " + describe(rc));
            for (const auto &m : gr.members) {
                const uint32_t sl = slots[m.second];
                memcpy(m.first->_iv, &t.iv[16 * (size_t)sl], 16);
                m.first->_pos = t.pos[sl];
            }
        }
    }
}

}  // namespace fpnn
