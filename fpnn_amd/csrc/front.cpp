// front.cpp -- libfpnn_aes.so, the library callers link (the fpnn:: classes live beside it
// in encryptor.cpp, stream_receiver.cpp, keyexchange.cpp).  It has no HIP dependency: on
// the first C-ABI call it loads libfpnn_aes_gpu.so -- the HIP kernels, the engine and the
// HIP runtime behind them -- and every fpnn_aes_* / fpnn_ecdh_* entry point forwards to
// the same-named function there (front_fwd.inc, generated from the headers).
//
// Why the split.  FPNN starts threads with 16 KiB stacks (base/msec.c:72-74, the clock
// thread every FPMessage timestamp starts).  glibc carves the static TLS of every library
// loaded at program start out of each new thread's stack, and the HIP runtime's
// dependencies carry about 30 KiB of it (librocprofiler-register): with the runtime linked
// at start-up, pthread_create refused that stack and FPNN aborted on its first message --
// found by running the reference's own receivers on this library
// (tests/test_gpu_dropin.py).  A library loaded later with dlopen keeps its TLS out of the
// static block.
#include <dlfcn.h>
#include <errno.h>
#include <stdlib.h>

#include <mutex>
#include <string>

#include "../../include/fpnn_aes.h"
#include "../../include/fpnn_ecdh.h"

namespace {

std::once_flag g_once;
void *g_gpu = nullptr;
std::string g_load_error;

void load_gpu_library() {
    std::call_once(g_once, [] {
        std::string path;
        if (const char *p = getenv("FPNN_AES_GPU_LIB")) {
            path = p;
        } else {  // beside this library
            Dl_info info;
            if (dladdr(reinterpret_cast<void *>(&load_gpu_library), &info) && info.dli_fname) {
                path = info.dli_fname;
                const size_t slash = path.rfind('/');
                path = slash == std::string::npos ? std::string() : path.substr(0, slash + 1);
            }
            path += "libfpnn_aes_gpu.so";
        }
        g_gpu = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!g_gpu) {
            const char *e = dlerror();
            g_load_error = std::string("cannot load the GPU library ") + path + ": " + (e ? e : "?");
        }
    });
}

template <class F>
F gpu_symbol(const char *name) {
    load_gpu_library();
    return g_gpu ? reinterpret_cast<F>(dlsym(g_gpu, name)) : nullptr;
}

}  // namespace

// Every entry point leaves errno as it found it.  The reference's cipher never touches
// errno, and FPNN's receivers rely on that: after a short read() they test errno
// (core/EncryptedStreamReceiver.cpp:31-55) although a decrypt call ran since the socket
// call that set it -- the HIP runtime's calls in between would otherwise make a partial
// body read look like a failed socket and close the connection (found by
// tests/test_gpu_dropin.py, stream fixtures fed in 7-byte pieces).
namespace {
struct ErrnoKeep {
    int saved = errno;
    ~ErrnoKeep() { errno = saved; }
};
}  // namespace

#define FPNN_FWD(RET, NAME, PARAMS, ARGS, FAIL)                        \
    extern "C" RET NAME PARAMS {                                       \
        using fn_t = RET(*) PARAMS;                                    \
        ErrnoKeep keep;                                                \
        static const fn_t f = gpu_symbol<fn_t>(#NAME);                 \
        if (!f) return FAIL;                                           \
        return f ARGS;                                                 \
    }
#include "front_fwd.inc"
#undef FPNN_FWD

extern "C" {

const char *fpnn_aes_strerror(int status) {
    switch (status) {
        case FPNN_AES_OK: return "ok";
        case FPNN_AES_ERR_KEYLEN: return "key length must be 16, 24 or 32 bytes";
        case FPNN_AES_ERR_ARG: return "invalid argument";
        case FPNN_AES_ERR_RANGE: return "batch too large";
        case FPNN_AES_ERR_HIP: return "HIP runtime error";
        case FPNN_AES_ERR_NODEV: return "no usable gfx950 device";
        case FPNN_AES_ERR_DEVICE: return "device-side check failed";
        default: return "unknown status";
    }
}

const char *fpnn_aes_last_error(void) {
    using fn_t = const char *(*)(void);
    ErrnoKeep keep;
    static const fn_t f = gpu_symbol<fn_t>("fpnn_aes_last_error");
    return f ? f() : g_load_error.c_str();
}

}  // extern "C"
