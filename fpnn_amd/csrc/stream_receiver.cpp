// stream_receiver.cpp -- fpnn::StreamReceiverBatch (include/StreamReceiverBatch.h): the
// receive side of many stream-mode connections per IO cycle in one device pass,
// EncryptedStreamReceiver::recvPackage + fetch (core/EncryptedStreamReceiver.cpp:72-163)
// over fpnn_aes_stream_recv.  Host work: lay out each connection's region (plaintext carry
// ‖ new ciphertext) in pinned staging, one H2D, the call, one D2H, hand out the messages.
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/StreamReceiverBatch.h"
#include "../../include/fpnn_aes.h"
#include "fail_policy.hpp"
#include "thread_engine.hpp"

namespace fpnn {

namespace {

std::string describe(int rc) {
    std::string s = fpnn_aes_strerror(rc);
    const char *d = fpnn_aes_last_error();
    if (d && *d) s += std::string(": ") + d;
    return s;
}

void check(int rc, const char *what) {
    if (rc != FPNN_AES_OK) fpnn_aes::device_failure(std::string("StreamReceiverBatch: ") + what + ": " + describe(rc));
}

size_t align16(size_t n) { return (n + 15) & ~(size_t)15; }

}  // namespace

// Device and pinned buffers of one batch, on the engine of the thread that flushes it
// (grown, kept), through the C-ABI's memory calls (this file is built without HIP).
// Pool engines are never destroyed (thread_engine.hpp), so the cached engine stays valid
// when the batch is destroyed or flushed by another thread after the first has exited --
// but another thread may hold that engine's lease by then, so release() runs under the
// engine's mutex (with_engine_locked), never beside a call on it.
struct StreamReceiverBatch::Dev {
    fpnn_aes::PooledEngine *pe = nullptr;
    fpnn_aes_engine *e = nullptr;
    uint64_t eid = 0;
    fpnn_aes_keyset *ks[3] = {nullptr, nullptr, nullptr};  // per key length
    uint8_t *d = nullptr, *h = nullptr;  // regions | descriptors | results
    size_t cap_d = 0, cap_h = 0;

    void release() {
        if (e) (void)fpnn_aes_engine_sync(e);  // a pass that threw may have left copies queued
        for (fpnn_aes_keyset *&k : ks) {
            if (k) fpnn_aes_keyset_destroy(k);
            k = nullptr;
        }
        if (d) (void)fpnn_aes_device_free(e, d);
        if (h) (void)fpnn_aes_pinned_free(e, h);
        d = h = nullptr;
        cap_d = cap_h = 0;
    }
    void reserve(size_t need) {
        if (need > cap_d || need > cap_h) check(fpnn_aes_engine_sync(e), "sync");
        if (need > cap_d) {
            size_t n = std::max<size_t>(cap_d * 2, std::max<size_t>(need, 1 << 20));
            if (d) (void)fpnn_aes_device_free(e, d);
            d = nullptr;
            cap_d = 0;
            void *p = nullptr;
            check(fpnn_aes_device_alloc(e, n, &p), "device buffer");
            d = static_cast<uint8_t *>(p);
            cap_d = n;
        }
        if (need > cap_h) {
            size_t n = std::max<size_t>(cap_h * 2, std::max<size_t>(need, 1 << 20));
            if (h) (void)fpnn_aes_pinned_free(e, h);
            h = nullptr;
            cap_h = 0;
            void *p = nullptr;
            check(fpnn_aes_pinned_alloc(e, n, &p), "pinned buffer");
            h = static_cast<uint8_t *>(p);
            cap_h = n;
        }
    }
};

StreamReceiverBatch::StreamReceiverBatch(uint32_t max_len, uint32_t max_frames)
    : _max_len(max_len), _max_frames(std::max<uint32_t>(1, max_frames)) {}

StreamReceiverBatch::~StreamReceiverBatch() {
    if (_dev) {
        fpnn_aes::with_engine_locked(_dev->pe, [&](fpnn_aes_engine *) { _dev->release(); });
        delete _dev;
    }
}

int StreamReceiverBatch::open(StreamEncryptor *enc) {
    if (!enc) throw EncryptorError("StreamReceiverBatch: null encryptor");
    int id;
    if (!_free.empty()) {
        id = _free.back();
        _free.pop_back();
    } else {
        id = (int)_conns.size();
        _conns.emplace_back();
    }
    Conn &c = _conns[id];
    c = Conn();
    c.enc = enc;
    c.open = true;
    return id;
}

void StreamReceiverBatch::close(int conn) {
    if (conn < 0 || conn >= (int)_conns.size() || !_conns[conn].open) return;
    _conns[conn] = Conn();
    _free.push_back(conn);
}

void StreamReceiverBatch::received(int conn, const uint8_t *data, size_t len) {
    if (conn < 0 || conn >= (int)_conns.size() || !_conns[conn].open)
        throw EncryptorError("StreamReceiverBatch: no such connection");
    Conn &c = _conns[conn];
    if (c.status != FPNN_AES_SCAN_OK || !len) return;  // a connection in error takes nothing more
    c.in.append(reinterpret_cast<const char *>(data), len);
}

const std::vector<std::string> &StreamReceiverBatch::messages(int conn) const { return _conns.at(conn).msgs; }
int StreamReceiverBatch::status(int conn) const { return _conns.at(conn).status; }
size_t StreamReceiverBatch::pending(int conn) const { return _conns.at(conn).carry.size(); }

void StreamReceiverBatch::flush() {
    // flushed from a thread with another engine: free the buffers on the old one first,
    // under its mutex, before this thread locks its own (one engine mutex at a time)
    fpnn_aes::PooledEngine *mine = fpnn_aes::thread_pooled_engine();
    if (_dev && _dev->pe != mine) {
        fpnn_aes::with_engine_locked(_dev->pe, [&](fpnn_aes_engine *) { _dev->release(); });
        delete _dev;
        _dev = nullptr;
    }
    int rc;
    const fpnn_aes::Lease lease = fpnn_aes::thread_engine(&rc);
    fpnn_aes_engine *e = lease.engine();
    const uint64_t eid = lease.id();
    if (!e) fpnn_aes::device_failure("engine unavailable: " + describe(rc ? rc : FPNN_AES_ERR_NODEV));
    if (!_dev) {
        _dev = new Dev();
        _dev->pe = lease.pe;
        _dev->e = e;
        _dev->eid = eid;
    }
    for (Conn &c : _conns) c.msgs.clear();
    // passes until no connection stopped at max_frames; one pass per key length
    for (bool first = true;; first = false) {
        std::vector<int> ids[3];
        for (int i = 0; i < (int)_conns.size(); i++) {
            Conn &c = _conns[i];
            if (!c.open || c.status != FPNN_AES_SCAN_OK) continue;
            if (first ? (c.in.empty() && !c.more) : !c.more) continue;
            ids[(c.enc->_ctx.nrounds - 10) / 2].push_back(i);
        }
        bool any = false;
        for (int k = 0; k < 3; k++)
            if (!ids[k].empty()) {
                pass(ids[k], 10 + 2 * k);
                any = true;
            }
        if (!any) break;
    }
}

void StreamReceiverBatch::pass(const std::vector<int> &ids, int nrounds) {
    Dev &D = *_dev;
    const uint32_t n = (uint32_t)ids.size();
    const uint32_t mf = _max_frames;
    // region i: carry (plaintext, already "decrypted") ‖ new ciphertext, 16-aligned starts
    std::vector<uint64_t> seg(n);
    size_t at = 0;
    for (uint32_t i = 0; i < n; i++) {
        const Conn &c = _conns[ids[i]];
        at = align16(at);
        seg[i] = at + c.carry.size();
        at = seg[i] + c.in.size();
    }
    const size_t rbytes = align16(at + 16);
    // descriptors: in_off u64 | len u32 | slot u32 | carry u32 | pos u32 | iv 16 B |
    // results: frame_off u64 [n*mf] | frame_len u32 [n*mf] | scan 16 B [n]
    const size_t o_off = rbytes, o_len = o_off + 8 * (size_t)n, o_slot = o_len + 4 * (size_t)n,
                 o_carry = o_slot + 4 * (size_t)n, o_pos = o_carry + 4 * (size_t)n,
                 o_iv = align16(o_pos + 4 * (size_t)n), o_foff = o_iv + 16 * (size_t)n,
                 o_flen = o_foff + 8 * (size_t)n * mf, o_scan = align16(o_flen + 4 * (size_t)n * mf),
                 total = o_scan + 16 * (size_t)n;
    D.reserve(total);
    uint8_t *h = D.h;
    std::vector<fpnn_aes_schedule> scheds(n);
    for (uint32_t i = 0; i < n; i++) {
        const Conn &c = _conns[ids[i]];
        memcpy(h + seg[i] - c.carry.size(), c.carry.data(), c.carry.size());
        memcpy(h + seg[i], c.in.data(), c.in.size());
        reinterpret_cast<uint64_t *>(h + o_off)[i] = seg[i];
        reinterpret_cast<uint32_t *>(h + o_len)[i] = (uint32_t)c.in.size();
        reinterpret_cast<uint32_t *>(h + o_slot)[i] = i;
        reinterpret_cast<uint32_t *>(h + o_carry)[i] = (uint32_t)c.carry.size();
        reinterpret_cast<uint32_t *>(h + o_pos)[i] = (uint32_t)c.enc->_pos;
        memcpy(h + o_iv + 16 * (size_t)i, c.enc->_iv, 16);
        memcpy(&scheds[i], &c.enc->_ctx, sizeof(fpnn_aes_schedule));
    }
    fpnn_aes_keyset *&ks = D.ks[(nrounds - 10) / 2];
    if (!ks) check(fpnn_aes_keyset_reserve(D.e, std::max<uint32_t>(n, 256), nrounds, &ks), "key table");
    check(fpnn_aes_keyset_set(ks, 0, n, scheds.data(), nullptr), "key table upload");
    check(fpnn_aes_copy_async(D.e, D.d, h, o_foff), "upload");
    fpnn_aes_batch b;
    memset(&b, 0, sizeof b);
    b.in = D.d;
    b.out = D.d;  // in place: carry bytes sit in front of each segment
    b.count = n;
    b.in_off = reinterpret_cast<const uint64_t *>(D.d + o_off);
    b.len = reinterpret_cast<const uint32_t *>(D.d + o_len);
    b.key_slot = reinterpret_cast<const uint32_t *>(D.d + o_slot);
    b.keys = ks;
    check(fpnn_aes_stream_recv(D.e, &b, D.d + o_iv, reinterpret_cast<uint32_t *>(D.d + o_pos),
                               reinterpret_cast<const uint32_t *>(D.d + o_carry), _max_len, mf,
                               reinterpret_cast<uint64_t *>(D.d + o_foff), reinterpret_cast<uint32_t *>(D.d + o_flen),
                               reinterpret_cast<fpnn_aes_frame_scan *>(D.d + o_scan)),
          "stream_recv");
    check(fpnn_aes_copy_async(D.e, h, D.d, at), "download");
    check(fpnn_aes_copy_async(D.e, h + o_pos, D.d + o_pos, total - o_pos), "download");
    check(fpnn_aes_engine_sync(D.e), "sync");
    for (uint32_t i = 0; i < n; i++) {
        Conn &c = _conns[ids[i]];
        const uint8_t *region = h + seg[i] - c.carry.size();
        const uint64_t rlen = c.carry.size() + c.in.size();
        memcpy(c.enc->_iv, h + o_iv + 16 * (size_t)i, 16);  // state advanced over every byte
        c.enc->_pos = reinterpret_cast<const uint32_t *>(h + o_pos)[i];
        const fpnn_aes_frame_scan &sc = reinterpret_cast<const fpnn_aes_frame_scan *>(h + o_scan)[i];
        for (uint32_t j = 0; j < sc.frames; j++) {
            const uint64_t fo = reinterpret_cast<const uint64_t *>(h + o_foff)[(size_t)i * mf + j];
            const uint32_t fl = reinterpret_cast<const uint32_t *>(h + o_flen)[(size_t)i * mf + j];
            c.msgs.emplace_back(reinterpret_cast<const char *>(region + fo), fl);
        }
        c.more = sc.status == FPNN_AES_SCAN_FULL;
        c.status = c.more ? FPNN_AES_SCAN_OK : (int)sc.status;
        c.carry.assign(reinterpret_cast<const char *>(region + sc.consumed), rlen - sc.consumed);
        c.in.clear();
    }
}

}  // namespace fpnn
