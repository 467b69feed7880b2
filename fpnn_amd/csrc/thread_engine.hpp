// thread_engine.hpp -- the per-thread engine behind the reference-shaped C++ classes
// (Encryptor, EncryptorBatch, ECCKeyExchange).  Internal; not installed.
#pragma once

#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "../../include/fpnn_aes.h"

namespace fpnn_aes {

// One engine (HIP stream + pinned staging) per calling thread: an Encryptor is used
// by one thread at a time (core/IOBuffer.h:49-62, core/IOBuffer.cpp:219-245), and
// may migrate between IO and worker threads, which then use their own engines.
// Engine identity for caches keyed by engine (EncryptorBatch's key tables): a thread's
// engine dies with the thread, and a later one may be allocated at the same address.
inline uint64_t next_engine_id() {
    static std::atomic<uint64_t> n{1};
    return n.fetch_add(1, std::memory_order_relaxed);
}

struct ThreadEngine {
    fpnn_aes_engine *e = nullptr;
    int status = FPNN_AES_OK;
    uint64_t id = next_engine_id();
    ThreadEngine() {
        const char *dev = getenv("FPNN_AES_DEVICE");
        status = fpnn_aes_engine_create(dev ? atoi(dev) : 0, FPNN_AES_OWN_STREAM, &e);
    }
    ~ThreadEngine() { fpnn_aes_engine_destroy(e); }
};

inline fpnn_aes_engine *thread_engine(int *status, uint64_t *id = nullptr) {
    thread_local ThreadEngine te;
    *status = te.status;
    if (id) *id = te.id;
    return te.e;
}

}  // namespace fpnn_aes
