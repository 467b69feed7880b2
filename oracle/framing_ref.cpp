// TEST INFRASTRUCTURE ONLY -- drives the reference's own receivers to produce the framing
// golden fixtures (tests/golden/framing_cases.json); never part of the product.
//
// The reference's EncryptedPackageReceiver (core/EncryptedPackageReceiver.cpp:14-150) and
// EncryptedStreamReceiver (core/EncryptedStreamReceiver.cpp:8-163), compiled where they lie
// under /root/reference together with their real dependencies (Encryptor, rijndael,
// FPMessage + msgpack, Config, FPLog, Setting, ...; oracle/Makefile target `framing`), are
// fed a wire byte stream over a non-blocking socketpair exactly as the epoll loop feeds
// them: recvPackage() whenever bytes may be readable, fetch() whenever a package is
// complete (core/ServerIOWorker.cpp / ClientIOWorker.cpp call pattern).  Every event is
// written as one JSON object per line:
//   {"frame": k, "total": _total, "fetch": 0|1, "kind": "quest"|"answer", "raw": hex}
//   {"end": "incomplete"|"closed"|"exception", "curr": _curr, "total": _total}
// "raw" is FPQuest::raw() / FPAnswer::raw() of the decoded message, i.e. the plaintext
// the receiver decrypted.  The probe subclasses read Receiver::_curr / _total (protected
// members of the reference class) -- nothing of the reference is modified.
//
// usage: framing_ref <case.bin> <out.jsonl>
//   case.bin: "FRG1" u32 mode (0 package, 1 stream) u32 keylen key[keylen] iv[16]
//             i32 max_len u32 piece u64 wire_len wire[wire_len]   (little endian)
#include <errno.h>
#include <execinfo.h>
#include <signal.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "Config.h"
#include "FPLog.h"
#include "Receiver.h"
#include "Setting.h"

using namespace fpnn;

namespace {

struct PackageProbe : EncryptedPackageReceiver {
    PackageProbe(uint8_t *k, size_t kl, uint8_t *iv) : EncryptedPackageReceiver(k, kl, iv) {}
    int curr() const { return _curr; }
    int total() const { return _total; }
};
struct StreamProbe : EncryptedStreamReceiver {
    StreamProbe(uint8_t *k, size_t kl, uint8_t *iv) : EncryptedStreamReceiver(k, kl, iv) {}
    int curr() const { return _curr; }
    int total() const { return _total; }
};

std::string hex(const std::string &s) {
    static const char *d = "0123456789abcdef";
    std::string o;
    o.reserve(2 * s.size());
    for (unsigned char c : s) {
        o.push_back(d[c >> 4]);
        o.push_back(d[c & 15]);
    }
    return o;
}

template <class R>
int run(R &r, int rfd, int wfd, const uint8_t *wire, uint64_t n, uint32_t piece, FILE *out) {
    uint64_t pos = 0;
    int frame = 0;
    while (true) {
        if (pos < n) {  // feed the next piece (non-blocking: the receiver drains the socket)
            const uint64_t want = n - pos < piece ? n - pos : piece;
            const ssize_t w = ::write(wfd, wire + pos, want);
            if (w > 0) pos += (uint64_t)w;
        }
        bool need = true;
        bool ok;
        errno = 0;
        try {
            ok = r.recvPackage(rfd, need);
        } catch (const std::exception &) {
            fprintf(out, "{\"end\": \"exception\", \"curr\": %d, \"total\": %d}\n", r.curr(), r.total());
            return 0;
        }
        if (!ok) {
            fprintf(out, "{\"end\": \"closed\", \"curr\": %d, \"total\": %d}\n", r.curr(), r.total());
            return 0;
        }
        if (!need) {
            const int total = r.total();
            FPQuestPtr q;
            FPAnswerPtr a;
            bool http = false;
            bool f;
            try {  // the reference Encryptor cannot throw here; the drop-in reports GPU failures this way
                f = r.fetch(q, a, http);
            } catch (const std::exception &ex) {
                fprintf(stderr, "fetch threw: %s\n", ex.what());
                fprintf(out, "{\"end\": \"fetch_exception\", \"curr\": %d, \"total\": %d}\n", r.curr(), r.total());
                return 4;
            }
            std::string raw;
            const char *kind = "none";
            if (f && q) {
                kind = "quest";
                raw = *std::unique_ptr<std::string>(q->raw());
            } else if (f && a) {
                kind = "answer";
                raw = *std::unique_ptr<std::string>(a->raw());
            }
            fprintf(out, "{\"frame\": %d, \"total\": %d, \"fetch\": %d, \"kind\": \"%s\", \"raw\": \"%s\"}\n", frame,
                    total, f ? 1 : 0, kind, hex(raw).c_str());
            frame++;
            continue;
        }
        int avail = 0;
        ioctl(rfd, FIONREAD, &avail);
        if (pos == n && avail == 0) {
            fprintf(out, "{\"end\": \"incomplete\", \"curr\": %d, \"total\": %d}\n", r.curr(), r.total());
            return 0;
        }
    }
}

}  // namespace

// a crash prints its stack to stderr (the drop-in build runs on a GPU box without a debugger)
static void on_fatal(int sig) {
    void *frames[64];
    const int n = backtrace(frames, 64);
    fprintf(stderr, "fatal signal %d, stack:\n", sig);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char **argv) {
    signal(SIGABRT, on_fatal);
    signal(SIGSEGV, on_fatal);
    signal(SIGBUS, on_fatal);
    if (argc != 3) {
        fprintf(stderr, "usage: %s case.bin out.jsonl\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    fclose(f);
    const uint8_t *p = buf.data();
    if (buf.size() < 8 || memcmp(p, "FRG1", 4) != 0) return 2;
    p += 4;
    auto u32 = [&]() { uint32_t v; memcpy(&v, p, 4); p += 4; return v; };
    const uint32_t mode = u32();
    const uint32_t keylen = u32();
    uint8_t key[32], iv[16];
    memcpy(key, p, keylen);
    p += keylen;
    memcpy(iv, p, 16);
    p += 16;
    const int32_t max_len = (int32_t)u32();
    const uint32_t piece = u32();
    uint64_t n;
    memcpy(&n, p, 8);
    p += 8;
    const uint8_t *wire = p;

    // FPLog resolves the local address once for its records; pin it so that the lookup
    // never reaches the cloud-metadata client (base/ServerInfo.cpp:152-158).
    Setting::set("FP.server.local.ip4", "127.0.0.1");
    Config::_max_recv_package_length = max_len;

    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 3;
    fcntl(sv[0], F_SETFL, fcntl(sv[0], F_GETFL) | O_NONBLOCK);
    fcntl(sv[1], F_SETFL, fcntl(sv[1], F_GETFL) | O_NONBLOCK);
    FILE *out = fopen(argv[2], "w");
    if (!out) return 2;
    int rc;
    if (mode == 0) {
        PackageProbe r(key, keylen, iv);
        rc = run(r, sv[0], sv[1], wire, n, piece, out);
    } else {
        StreamProbe r(key, keylen, iv);
        rc = run(r, sv[0], sv[1], wire, n, piece, out);
    }
    fclose(out);
    close(sv[0]);
    close(sv[1]);
    fflush(stdout);
    _exit(rc);  // the logger's consumer thread is not joined
}
