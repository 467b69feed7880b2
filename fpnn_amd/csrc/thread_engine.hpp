// thread_engine.hpp -- the engines behind the reference-shaped C++ classes (Encryptor,
// EncryptorBatch, StreamReceiverBatch, ECCKeyExchange).  Internal; not installed.
//
// An Encryptor is used by one thread at a time (core/IOBuffer.h:49-62,
// core/IOBuffer.cpp:219-245) and may migrate between IO and worker threads.  Each calling
// thread leases an engine (HIP stream + pinned staging) from a process-wide pool:
//   * engine k of the pool lives on device devices[k % n] -- round-robin over every GPU of
//     the node (hipGetDeviceCount), or over FPNN_AES_DEVICES="0,3,..." / the one device
//     FPNN_AES_DEVICE names -- so FPNN's IO threads (core/GlobalIOPool.h:58-114) spread
//     over the node, one stream and its staging per GPU;
//   * the pool holds at most FPNN_AES_MAX_ENGINES engines (default 16 per device); a
//     thread arriving when all are leased shares one (calls serialise on its mutex);
//   * a thread's lease returns to the pool when the thread exits, and the next new thread
//     takes that engine over.  Engines are never destroyed, so anything that cached an
//     engine or its stream (a batch's key tables, StreamReceiverBatch's buffers) stays
//     valid after the thread that created it has gone.
#pragma once

#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fpnn_aes.h"

namespace fpnn_aes {

// Engine identity for caches keyed by engine (EncryptorBatch's key tables).
inline uint64_t next_engine_id() {
    static std::atomic<uint64_t> n{1};
    return n.fetch_add(1, std::memory_order_relaxed);
}

struct PooledEngine {
    fpnn_aes_engine *e = nullptr;
    int status = FPNN_AES_OK;
    int device = 0;
    uint64_t id = next_engine_id();
    std::mutex mu;     // held for the duration of each call on this engine
    unsigned users = 0;  // threads holding a lease (guarded by the pool mutex)
};

class EnginePool {
public:
    static EnginePool &get() {
        static EnginePool *p = new EnginePool();  // never destroyed: threads may exit after main
        return *p;
    }

    PooledEngine *acquire() {
        std::lock_guard<std::mutex> lk(mu_);
        for (PooledEngine *pe : slots_)  // an engine a finished thread left behind
            if (pe->users == 0 && pe->e) {
                pe->users = 1;
                return pe;
            }
        int ndev = 0;
        if (fpnn_aes_device_count(&ndev) != FPNN_AES_OK) ndev = 0;
        const unsigned cap = (unsigned)fpnn_aes_max_thread_engines(ndev);
        if (slots_.size() < cap || slots_.empty()) {
            PooledEngine *pe = new PooledEngine();
            pe->device = fpnn_aes_thread_engine_device((uint32_t)slots_.size(), ndev);
            pe->status = pe->device < 0 ? FPNN_AES_ERR_NODEV
                                        : fpnn_aes_engine_create(pe->device, FPNN_AES_OWN_STREAM, &pe->e);
            pe->users = 1;
            if (pe->e) slots_.push_back(pe);
            return pe;  // a failed slot is handed out once (its status reports why) and dropped
        }
        PooledEngine *best = slots_[0];  // all leased: share the least shared one
        for (PooledEngine *pe : slots_)
            if (pe->users < best->users) best = pe;
        best->users++;
        return best;
    }

    void release(PooledEngine *pe) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!pe->e) {
            delete pe;  // never entered the pool
            return;
        }
        if (pe->users) pe->users--;
    }

private:
    std::mutex mu_;
    std::vector<PooledEngine *> slots_;
};

// The calling thread's engine, locked for as long as the Lease lives.
struct Lease {
    PooledEngine *pe = nullptr;
    std::unique_lock<std::mutex> lk;
    fpnn_aes_engine *engine() const { return pe ? pe->e : nullptr; }
    uint64_t id() const { return pe ? pe->id : 0; }
};

struct ThreadLease {
    PooledEngine *pe = nullptr;
    ~ThreadLease() {
        if (pe) EnginePool::get().release(pe);
    }
};

// The calling thread's pool entry (leased on first use), not locked.
inline PooledEngine *thread_pooled_engine() {
    thread_local ThreadLease tl;
    if (!tl.pe) tl.pe = EnginePool::get().acquire();
    return tl.pe;
}

inline Lease thread_engine(int *status) {
    Lease l;
    l.pe = thread_pooled_engine();
    *status = l.pe->status;
    if (l.pe->e) l.lk = std::unique_lock<std::mutex>(l.pe->mu);
    return l;
}

// Work on an engine some other thread may hold the lease of (a batch object that cached
// it): under that engine's mutex, as every call on it is.  Callers hold no other engine's
// mutex meanwhile (no lock-order cycle between two engines).
template <class F>
void with_engine_locked(PooledEngine *pe, F &&f) {
    std::lock_guard<std::mutex> lk(pe->mu);
    f(pe->e);
}

}  // namespace fpnn_aes
