// TEST INFRASTRUCTURE ONLY -- SURVEY.md section 8f row 1 inside FPNN's own IO plumbing
// (VERDICT r04 item 3): many encrypted connections, each a reference SendBuffer
// (core/IOBuffer.cpp) + receiver pair per side, driven by IO threads that each loop over
// their connections the way an FPNN IO worker serves its ready connections
// (core/ServerIOWorker.cpp:148-276: recvPackage until a frame is complete, fetch, deliver;
// answers go out through SendBuffer::send).  Every connection has its own key and IV (as
// ECDH gives them, core/KeyExchange.cpp:87-127); a client keeps `window` quests in flight.
//
// One source, three builds (oracle/Makefile `multi`):
//   _ref/io_multi_ref      reference IO code + the reference Encryptor/rijndael: one CPU
//                          cipher call per frame (the baseline);
//   _ref/io_multi_dropin   reference IO code UNCHANGED on libfpnn_aes.so: one GPU call per
//                          frame (the drop-in of INTEGRATION.md section 1);
//   _ref/io_multi_batched  reference IO code with INTEGRATION.md section 2a applied by
//                          oracle/collect_patch.py (SendBuffer::encryptData and
//                          EncryptedPackageReceiver::fetch queue into the IO thread's
//                          fpnn::EncryptorBatch), on libfpnn_aes.so, -DFPNN_IO_COLLECT
//                          -DFPNN_IO_GPU: per loop cycle and direction ONE flush for all of
//                          a thread's connections.  Stream mode receives through
//                          fpnn::StreamReceiverBatch: the
//                          stream receiver's header-then-body decrypt pair per message
//                          cannot be deferred (the body length is in the decrypted header).
// The cycle is the same in all three; in the unbatched builds the flushes are no-ops.
// A fourth build, _ref/io_multi_cpucollect (-DFPNN_IO_COLLECT only), runs the patched
// plumbing on the reference cipher through a CPU stand-in queue (io_collect_cpu.cpp): it
// checks the patch's deferral and ordering on any machine (stream mode then receives
// through the reference receiver, per call).
// Each prints one JSON line: echoes/s, and FNV-1a digests of the bytes every SendBuffer
// wrote (write() is wrapped at link time, -Wl,--wrap=write), per connection and direction,
// folded in connection order -- the three builds must agree byte for byte.
//
// With first_clear = 1 every client connection starts the way TCPClient does
// (core/TCPClient.cpp:238-243, 464-472): its SendBuffer is told encryptAfterFirstPackage()
// (core/IOBuffer.h:126) and its first frame is a "*key" quest that goes out in the clear
// (SendBuffer::encryptData skips it, core/IOBuffer.cpp:36-45); every later frame is
// encrypted.  The server reads that frame as plaintext, answers it -- encrypted, as
// ServerIOWorker::processECDH's answer is (core/ServerIOWorker.cpp:306-309) -- and only then
// hands the connection's bytes to its encrypted receiver.  In the batched build this runs
// the collect patch's first-package count (collect_patch.py, NEW_REALSEND) over a cycle
// whose collected frames start with the plaintext one.
//
// usage: io_multi <mode 0 package|1 stream> <keylen> <conns> <quests per conn> <payload>
//                 <window> [threads] [tcp 1|0] [first_clear 0|1]
#include <arpa/inet.h>
#include <errno.h>
#include <execinfo.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <exception>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "Decoder.h"
#include "FPLog.h"
#include "IOBuffer.h"
#include "Setting.h"
#ifdef FPNN_IO_COLLECT
#include "io_collect.h"
#endif
#ifdef FPNN_IO_GPU
#include "StreamReceiverBatch.h"
#include "fpnn_aes.h"
#endif

using namespace fpnn;

// ---- wire digests: every write() the IO objects make, per fd ---------------------------
namespace {
constexpr int kMaxFd = 1 << 16;
uint64_t g_fd_hash[kMaxFd];
uint64_t g_fd_bytes[kMaxFd];
uint64_t fnv(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
    return h;
}
}  // namespace

extern "C" ssize_t __real_write(int fd, const void *buf, size_t n);
extern "C" ssize_t __wrap_write(int fd, const void *buf, size_t n) {
    const ssize_t r = __real_write(fd, buf, n);
    if (r > 0 && fd >= 0 && fd < kMaxFd) {  // each fd belongs to one IO thread
        g_fd_hash[fd] = fnv(g_fd_hash[fd], static_cast<const uint8_t *>(buf), (size_t)r);
        g_fd_bytes[fd] += (uint64_t)r;
    }
    return r;
}

namespace {

void nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

// a listening loopback TCP socket; connected pairs are made from it
struct Loopback {
    int l = -1;
    sockaddr_in a;
    bool open() {
        l = socket(AF_INET, SOCK_STREAM, 0);
        if (l < 0) return false;
        memset(&a, 0, sizeof a);
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t al = sizeof a;
        return bind(l, (sockaddr *)&a, sizeof a) == 0 && listen(l, 4096) == 0 &&
               getsockname(l, (sockaddr *)&a, &al) == 0;
    }
    bool pair(int &c, int &s) {
        c = socket(AF_INET, SOCK_STREAM, 0);
        if (c < 0 || connect(c, (sockaddr *)&a, sizeof a) != 0) return false;
        s = accept(l, nullptr, nullptr);
        if (s < 0) return false;
        int one = 1;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        return true;
    }
};

// the client's "*key" quest (core/TCPClient.cpp:469-472: {publicKey, streamMode, bits} as a
// msgpack map), sent in the clear; its sequence number keeps its answer apart from the echoes
constexpr uint32_t kKeySeq = 0x7fffff00u;
std::string key_quest_raw(uint32_t conn, bool stream, int keylen) {
    std::string m("\x83\xa9publicKey\xd9\x40", 13);
    for (int k = 0; k < 64; k++) m += (char)(0x40 + ((conn * 7 + (uint32_t)k * 13) & 0x3f));
    m += std::string("\xaastreamMode", 11) + (stream ? '\xc3' : '\xc2');
    m += std::string("\xa4" "bits\xcd\x01\x00", 8);
    if (keylen != 32) m[m.size() - 2] = '\x00', m[m.size() - 1] = '\x80';
    FPQuest q("*key");
    q.setSeqNum(kKeySeq);
    q.setPayload(m);
    q.setPayloadSize((uint32_t)m.size());
    std::string *raw = q.raw();
    std::string r(*raw);
    delete raw;
    return r;
}

// Reads one plaintext FPNN frame (12-byte header + FPMessage::BodyLen) from a non-blocking
// fd into acc, never a byte more: 1 complete, 0 more to come, -1 closed / error.
int read_plain_frame(int fd, std::string &acc) {
    for (;;) {
        const size_t want = acc.size() < 12 ? 12 - acc.size() : 12 + FPMessage::BodyLen(acc.data()) - acc.size();
        if (want == 0) return 1;
        char buf[4096];
        const ssize_t r = ::read(fd, buf, std::min(want, sizeof buf));
        if (r > 0) {
            acc.append(buf, (size_t)r);
            continue;
        }
        if (r == 0) return -1;
        if (errno == EINTR) continue;
        return (errno == EAGAIN || errno == EWOULDBLOCK) ? 0 : -1;
    }
}

std::string payload_of(uint32_t conn, uint32_t i, int len) {
    std::string p((size_t)len, '\0');
    uint64_t x = 0x9E3779B97F4A7C15ull ^ ((uint64_t)i * 0xD1B54A32D192ED03ull) ^ ((uint64_t)conn << 40);
    for (int k = 0; k < len; k++) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        p[(size_t)k] = (char)x;
    }
    return p;
}

double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Conn {
    uint32_t id = 0;
    int cfd = -1, sfd = -1;
    uint8_t key[32], iv[16];
    std::mutex mc, ms;
    std::unique_ptr<SendBuffer> csend, ssend;
    std::unique_ptr<Receiver> crecv, srecv;  // the object RecvBuffer::entryEncryptMode installs
    int crx = -1, srx = -1;                  // (batched stream mode) StreamReceiverBatch ids
    uint32_t sent = 0, answered = 0, served = 0, bad = 0;
    // first_clear: the "*key" quest's state (client sent it / server still reading it /
    // client got its answer) and the server's plaintext bytes of it
    bool key_sent = false, key_pending = false, key_answered = false;
    std::string key_acc;
};

struct Params {
    bool stream;
    int keylen;
    uint32_t quests;
    int plen;
    uint32_t window;
    bool first_clear;
};

struct ThreadResult {
    bool ok = true;
    std::string err;
    double flush_s = 0, end = 0;
    uint64_t flushes = 0, cycles = 0;
};

// The IO threads warm up (engine creation, kernel loading: once per process in a server),
// then wait here until the clock starts.
struct Start {
    std::mutex mu;
    std::condition_variable cv;
    uint32_t ready = 0;
    bool go = false;
    void arrive() {
        std::unique_lock<std::mutex> lk(mu);
        ready++;
        cv.notify_all();
        cv.wait(lk, [this] { return go; });
    }
    void release(uint32_t n) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return ready == n; });
        go = true;
        cv.notify_all();
    }
};

// A frame a receiver completed this cycle, decoded after the flush.
struct Pending {
    Conn *c;
    bool server;
    char *buf;
    int len;
};

#ifdef FPNN_IO_COLLECT
#define COLLECT(batch) fpnn_io::Collect collect_phase_((batch).get())
#else
#define COLLECT(batch) (void)0
#endif

// Warm-up on a dummy connection's cipher objects, before the clock: the same kinds of calls
// (and, batched, of flushes) as a cycle makes.  Touches no connection: the wire is unchanged.
template <class Q>
void warm_up(const Params &P, Q *batch) {
    uint8_t key[32], iv[16];
    for (int k = 0; k < 32; k++) key[k] = (uint8_t)(3 * k + 1);
    for (int k = 0; k < 16; k++) iv[k] = (uint8_t)(5 * k + 2);
    std::unique_ptr<Encryptor> enc(P.stream ? (Encryptor *)new StreamEncryptor(key, (size_t)P.keylen, iv)
                                            : (Encryptor *)new PackageEncryptor(key, (size_t)P.keylen, iv));
    std::unique_ptr<Encryptor> dec(P.stream ? (Encryptor *)new StreamEncryptor(key, (size_t)P.keylen, iv)
                                            : (Encryptor *)new PackageEncryptor(key, (size_t)P.keylen, iv));
    for (int rep = 0; rep < 3; rep++) {
        std::vector<std::string> frames(256, std::string((size_t)P.plen + 40, 'w'));
        std::vector<std::string> plain(frames.size());
#ifdef FPNN_IO_COLLECT
        {
            fpnn_io::Collect phase(batch);
            for (auto &f : frames) fpnn_io::encrypt(enc.get(), &f);
        }
        batch->flush();
        {
            fpnn_io::Collect phase(batch);
            for (size_t i = 0; i < frames.size(); i++) {
                const size_t off = P.stream ? 0 : 4;
                plain[i].assign(frames[i].size() - off, '\0');
                fpnn_io::decrypt(dec.get(), reinterpret_cast<uint8_t *>(&plain[i][0]),
                                 reinterpret_cast<uint8_t *>(&frames[i][off]), (int)plain[i].size());
            }
        }
        batch->flush();
#else
        (void)batch;
        for (size_t i = 0; i < 16; i++) {
            enc->encrypt(&frames[i]);
            const size_t off = P.stream ? 0 : 4;
            plain[i].assign(frames[i].size() - off, '\0');
            dec->decrypt(reinterpret_cast<uint8_t *>(&plain[i][0]), reinterpret_cast<uint8_t *>(&frames[i][off]),
                         (int)plain[i].size());
        }
#endif
    }
}

void io_thread(std::vector<Conn *> conns, const Params P, ThreadResult *res, Start *start) {
    bool nw, act;
#ifdef FPNN_IO_COLLECT
    std::unique_ptr<fpnn_io::Queue> batch(fpnn_io::make_queue());
#ifdef FPNN_IO_GPU
    std::unique_ptr<StreamReceiverBatch> rx;
    if (P.stream) {
        rx.reset(new StreamReceiverBatch());
        for (Conn *c : conns) {
            c->crx = rx->open(new StreamEncryptor(c->key, (size_t)P.keylen, c->iv));
            c->srx = rx->open(new StreamEncryptor(c->key, (size_t)P.keylen, c->iv));
        }
    }
#endif
    auto flush = [&]() {
        if (!batch->size()) return;
        const double t = now();
        batch->flush();
        res->flush_s += now() - t;
        res->flushes++;
        fpnn_io::release_deferred();  // the received ciphertexts the decrypts read
    };
#else
    int batch = 0;
    (void)batch;
    auto flush = [&]() {};
#endif
#ifdef FPNN_IO_COLLECT
    warm_up(P, batch.get());
#ifdef FPNN_IO_GPU
    if (P.stream) {  // the receive pass too: one valid message on a dummy stream
        uint8_t key[32], iv[16];
        for (int k = 0; k < 32; k++) key[k] = (uint8_t)(7 * k + 5);
        for (int k = 0; k < 16; k++) iv[k] = (uint8_t)(9 * k + 4);
        StreamEncryptor tx(key, (size_t)P.keylen, iv);
        const int id = rx->open(new StreamEncryptor(key, (size_t)P.keylen, iv));
        FPQuest q("warm");
        q.setPayload(std::string((size_t)P.plen, 'q'));
        q.setPayloadSize((uint32_t)P.plen);
        std::string *raw = q.raw();
        tx.encrypt(raw);
        rx->received(id, reinterpret_cast<const uint8_t *>(raw->data()), raw->size());
        delete raw;
        rx->flush();
        rx->close(id);
    }
#endif
#else
    warm_up(P, (void *)nullptr);
#endif
    start->arrive();
    std::vector<Pending> pend;
    uint64_t left = 0;
    for (Conn *c : conns) left += P.quests;
    auto fail = [&](const char *what, Conn *c) {
        res->ok = false;
        res->err = std::string(what) + " on connection " + std::to_string(c->id);
    };
    // an answer on the client: the "*key" answer (first_clear) or the next echo
    auto client_answer = [&](Conn *c, const FPAnswerPtr &a) {
        if (P.first_clear && a->seqNum() == kKeySeq && !c->key_answered) {
            c->key_answered = true;
            return;
        }
        const uint32_t i = a->seqNum() - 1;
        if (i != c->answered || a->payload() != payload_of(c->id, i, P.plen)) c->bad++;
        c->answered++;
        left--;
    };
    // server, first_clear: the plaintext "*key" frame of each connection that still owes it,
    // answered (encrypted) through the connection's SendBuffer; false on a broken frame
    auto key_frames = [&]() -> bool {
        if (!P.first_clear) return true;
        COLLECT(batch);  // (the answers' encryption goes to the send flush)
        for (Conn *c : conns) {
            if (!c->key_pending) continue;
            const int r = read_plain_frame(c->sfd, c->key_acc);
            if (r < 0) {
                fail("plaintext *key frame", c);
                return false;
            }
            if (r == 0) continue;
            FPQuestPtr q = Decoder::decodeQuest(c->key_acc.data(), (int)c->key_acc.size());
            if (!q || q->method() != "*key") {
                fail("first frame is not a plaintext *key quest", c);
                return false;
            }
            FPAnswer reply(q);
            reply.setPayload(std::string("\x80", 1));  // {} (core/ServerIOWorker.cpp:306-309)
            reply.setPayloadSize(1);
            c->ssend->send(c->sfd, nw, act, reply.raw());
            c->key_pending = false;
        }
        return true;
    };
    // a complete frame on receiver r: staged for decode after the flush (batched) or fetched now
    auto take = [&](Conn *c, bool server) -> bool {
        Receiver *r = server ? c->srecv.get() : c->crecv.get();
#ifdef FPNN_IO_COLLECT
        if (!P.stream) {
            char *buf = nullptr;
            int len = 0;
            if (!static_cast<EncryptedPackageReceiver *>(r)->fetchStage(buf, len)) return false;
            pend.push_back(Pending{c, server, buf, len});
            return true;
        }
#endif
        FPQuestPtr q;
        FPAnswerPtr a;
        bool http = false;
        if (!r->fetch(q, a, http)) return false;
        if (server) {
            if (!q) return false;
            FPAnswer reply(q);
            reply.setPayload(q->payload());
            reply.setPayloadSize((uint32_t)q->payload().size());
            c->ssend->send(c->sfd, nw, act, reply.raw());
            c->served++;
        } else {
            if (!a) return false;
            client_answer(c, a);
        }
        return true;
    };
    // decode the staged frames (batched package mode) -- the reference's own decode
    auto decode = [&](bool server) -> bool {
#ifdef FPNN_IO_COLLECT
        for (const Pending &p : pend) {
            FPQuestPtr q;
            FPAnswerPtr a;
            bool http = false;
            Receiver *r = server ? p.c->srecv.get() : p.c->crecv.get();
            if (!static_cast<EncryptedPackageReceiver *>(r)->fetchDecode(p.buf, p.len, q, a, http)) return false;
            if (server) {
                if (!q) return false;
                FPAnswer reply(q);
                reply.setPayload(q->payload());
                reply.setPayloadSize((uint32_t)q->payload().size());
                p.c->ssend->send(p.c->sfd, nw, act, reply.raw());
                p.c->served++;
            } else {
                if (!a) return false;
                client_answer(p.c, a);
            }
        }
#endif
        pend.clear();
        (void)server;
        return true;
    };
    // receive side of one direction for every connection
    auto receive = [&](bool server) -> bool {
#ifdef FPNN_IO_GPU
        if (P.stream) {  // StreamReceiverBatch: read what the sockets hold, one device pass
            char buf[65536];
            std::vector<Conn *> got;
            if (server && !key_frames()) return false;
            for (Conn *c : conns) {
                if (server && c->key_pending) continue;  // its plaintext frame is not complete yet
                const int fd = server ? c->sfd : c->cfd;
                bool any = false;
                for (;;) {
                    const ssize_t n = ::read(fd, buf, sizeof buf);
                    if (n <= 0) break;
                    rx->received(server ? c->srx : c->crx, reinterpret_cast<const uint8_t *>(buf), (size_t)n);
                    any = true;
                }
                if (any) got.push_back(c);
            }
            if (got.empty()) return true;
            const double t = now();
            rx->flush();
            res->flush_s += now() - t;
            res->flushes++;
            COLLECT(batch);  // the answers' encryption goes to the send flush
            for (Conn *c : got) {
                const int id = server ? c->srx : c->crx;
                if (rx->status(id) != FPNN_AES_SCAN_OK) {
                    fail("stream receive", c);
                    return false;
                }
                for (const std::string &m : rx->messages(id)) {
                    if (server) {
                        FPQuestPtr q = FPMessage::isQuest(m.data()) ? Decoder::decodeQuest(m.data(), (int)m.size())
                                                                   : nullptr;
                        if (!q) return false;
                        FPAnswer reply(q);
                        reply.setPayload(q->payload());
                        reply.setPayloadSize((uint32_t)q->payload().size());
                        c->ssend->send(c->sfd, nw, act, reply.raw());
                        c->served++;
                    } else {
                        FPAnswerPtr a = Decoder::decodeAnswer(m.data(), (int)m.size());
                        if (!a) return false;
                        client_answer(c, a);
                    }
                }
            }
            return true;
        }
#endif
        if (server && !key_frames()) return false;
        {
            COLLECT(batch);  // package mode: fetchStage queues the decrypts
            for (Conn *c : conns) {
                if (server && c->key_pending) continue;  // its plaintext frame is not complete yet
                Receiver *r = server ? c->srecv.get() : c->crecv.get();
                const int fd = server ? c->sfd : c->cfd;
                for (;;) {
                    bool need = true;
                    if (!r->recvPackage(fd, need)) {
                        fail("recvPackage", c);
                        return false;
                    }
                    if (need) break;
                    if (!take(c, server)) {
                        fail("fetch", c);
                        return false;
                    }
                }
            }
        }
        flush();  // the cycle's decrypts
        COLLECT(batch);  // (server) the answers' encryption goes to the send flush
        if (!decode(server)) {
            res->ok = false;
            res->err = "decode";
            return false;
        }
        return true;
    };
    // write phase of one side: frames collected and encrypted by the flush go out
    auto write_out = [&](bool server) {
        flush();
        for (Conn *c : conns) {
            if (server)
                c->ssend->send(c->sfd, nw, act);
            else
                c->csend->send(c->cfd, nw, act);
        }
    };
    while (left) {
        res->cycles++;
        {
            COLLECT(batch);  // client: the next quests (their encryption is queued)
            for (Conn *c : conns) {
                if (P.first_clear && !c->key_sent) {  // TCPClient's "*key" quest goes first, in the clear
                    c->csend->send(c->cfd, nw, act, new std::string(key_quest_raw(c->id, P.stream, P.keylen)));
                    c->key_sent = true;
                }
                while (c->sent < P.quests && c->sent - c->answered < P.window) {
                    FPQuest q("echo");
                    q.setSeqNum(c->sent + 1);
                    q.setPayload(payload_of(c->id, c->sent, P.plen));
                    q.setPayloadSize((uint32_t)P.plen);
                    c->csend->send(c->cfd, nw, act, q.raw());
                    c->sent++;
                }
            }
        }
        write_out(false);
        if (!receive(true)) return;  // server: quests -> answers (queued)
        write_out(true);
        if (!receive(false)) return;  // client: answers
        if (res->cycles > 100000000ull) {
            res->ok = false;
            res->err = "no progress";
            return;
        }
    }
    res->end = now();
}

}  // namespace

static int run(int argc, char **argv);

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
    signal(SIGPIPE, SIG_IGN);
    try {
        return run(argc, argv);
    } catch (const std::exception &ex) {
        fprintf(stderr, "io_multi: %s\n", ex.what());
        fflush(stderr);
        _exit(9);
    }
}

static int run(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s mode keylen conns quests payload window [threads] [tcp] [first_clear]\n", argv[0]);
        return 2;
    }
    Params P;
    P.stream = atoi(argv[1]) != 0;
    P.keylen = atoi(argv[2]);
    const uint32_t nconn = (uint32_t)atoi(argv[3]);
    P.quests = (uint32_t)atoi(argv[4]);
    P.plen = atoi(argv[5]);
    P.window = (uint32_t)atoi(argv[6]);
    const uint32_t nthr = argc > 7 ? std::max(1, atoi(argv[7])) : 1u;
    bool tcp = argc > 8 ? atoi(argv[8]) != 0 : true;
    P.first_clear = argc > 9 && atoi(argv[9]) != 0;
    Setting::set("FP.server.local.ip4", "127.0.0.1");  // FPLog never asks the cloud-metadata client

    rlimit rl;
    if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur < rl.rlim_max) {
        rl.rlim_cur = rl.rlim_max;
        setrlimit(RLIMIT_NOFILE, &rl);
    }
    Loopback lb;
    if (tcp && !lb.open()) tcp = false;
    std::vector<std::unique_ptr<Conn>> conns;
    for (uint32_t i = 0; i < nconn; i++) {
        std::unique_ptr<Conn> c(new Conn());
        c->id = i;
        for (int k = 0; k < 32; k++) c->key[k] = (uint8_t)(11 * k + 7 * i + 3 + (i >> 8));
        for (int k = 0; k < 16; k++) c->iv[k] = (uint8_t)(29 * k + 13 * i + 7 + (i >> 8));
        bool ok = tcp && lb.pair(c->cfd, c->sfd);
        if (!ok) {
            if (tcp) {  // out of loopback ports or fds: the whole run goes over socketpairs
                fprintf(stderr, "io_multi: tcp pair %u failed (%s); using socketpairs\n", i, strerror(errno));
                return 3;
            }
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) {
                fprintf(stderr, "io_multi: socketpair %u: %s\n", i, strerror(errno));
                return 3;
            }
            c->cfd = sv[0];
            c->sfd = sv[1];
        }
        if (c->cfd >= kMaxFd || c->sfd >= kMaxFd) return 3;
        nonblock(c->cfd);
        nonblock(c->sfd);
        c->csend.reset(new SendBuffer(&c->mc));
        c->ssend.reset(new SendBuffer(&c->ms));
        if (!c->csend->entryEncryptMode(c->key, (size_t)P.keylen, c->iv, P.stream) ||
            !c->ssend->entryEncryptMode(c->key, (size_t)P.keylen, c->iv, P.stream))
            return 4;
        if (P.first_clear) {  // TCPClient::configEncryptedConnection (core/TCPClient.cpp:238-243)
            c->csend->encryptAfterFirstPackage();
            c->key_pending = true;
        }
        auto make = [&]() -> Receiver * {
            return P.stream ? (Receiver *)new EncryptedStreamReceiver(c->key, (size_t)P.keylen, c->iv)
                            : (Receiver *)new EncryptedPackageReceiver(c->key, (size_t)P.keylen, c->iv);
        };
        c->crecv.reset(make());
        c->srecv.reset(make());
        conns.push_back(std::move(c));
    }
    if (lb.l >= 0) close(lb.l);

    std::vector<ThreadResult> res(nthr);
    std::vector<std::thread> th;
    Start start;
    for (uint32_t t = 0; t < nthr; t++) {
        std::vector<Conn *> mine;
        for (uint32_t i = t; i < nconn; i += nthr) mine.push_back(conns[i].get());
        th.emplace_back(io_thread, mine, P, &res[t], &start);
    }
    start.release(nthr);  // every thread warmed up: the clock starts
    const double t0 = now();
    for (auto &x : th) x.join();
    double t1 = t0;
    for (auto &r : res) t1 = std::max(t1, r.end);
    const double dt = t1 - t0;

    bool ok = true;
    std::string err;
    double flush_s = 0;
    uint64_t flushes = 0, cycles = 0;
    for (auto &r : res) {
        ok = ok && r.ok;
        if (!r.ok && err.empty()) err = r.err;
        flush_s += r.flush_s;
        flushes += r.flushes;
        cycles += r.cycles;
    }
    uint64_t h_c2s = 0xcbf29ce484222325ull, h_s2c = 0xcbf29ce484222325ull, b_c2s = 0, b_s2c = 0;
    uint32_t bad = 0, served = 0, answered = 0;
    for (auto &c : conns) {
        if (P.first_clear && (c->key_pending || !c->key_answered)) bad++;  // the *key exchange must complete
        h_c2s = fnv(h_c2s, reinterpret_cast<const uint8_t *>(&g_fd_hash[c->cfd]), 8);
        h_s2c = fnv(h_s2c, reinterpret_cast<const uint8_t *>(&g_fd_hash[c->sfd]), 8);
        b_c2s += g_fd_bytes[c->cfd];
        b_s2c += g_fd_bytes[c->sfd];
        bad += c->bad;
        served += c->served;
        answered += c->answered;
    }
    const uint64_t echoes = (uint64_t)nconn * P.quests;
#if defined(FPNN_IO_COLLECT) && defined(FPNN_IO_GPU)
    const char *build = "batched";
#elif defined(FPNN_IO_COLLECT)
    const char *build = "cpucollect";
#elif defined(FPNN_IO_DROPIN)
    const char *build = "dropin";
#else
    const char *build = "reference";
#endif
    printf("{\"build\": \"%s\", \"transport\": \"%s\", \"mode\": \"%s\", \"keylen\": %d, \"conns\": %u, "
           "\"quests_per_conn\": %u, \"payload\": %d, \"window\": %u, \"threads\": %u, \"first_clear\": %s, "
           "\"ok\": %s, \"error\": \"%s\", "
           "\"seconds\": %.4f, \"echo_per_s\": %.1f, \"us_per_echo\": %.3f, \"answers_ok\": %s, \"served\": %u, "
           "\"answered\": %u, \"cycles\": %llu, \"flushes\": %llu, \"flush_s\": %.4f, "
           "\"wire_c2s_bytes\": %llu, \"wire_c2s_fnv\": \"%016llx\", \"wire_s2c_bytes\": %llu, "
           "\"wire_s2c_fnv\": \"%016llx\"}\n",
           build, tcp ? "tcp-loopback" : "socketpair", P.stream ? "stream" : "package", P.keylen, nconn, P.quests,
           P.plen, P.window, nthr, P.first_clear ? "true" : "false", ok ? "true" : "false", err.c_str(), dt, echoes / dt, 1e6 * dt / echoes,
           bad == 0 && ok ? "true" : "false", served, answered, (unsigned long long)cycles,
           (unsigned long long)flushes, flush_s, (unsigned long long)b_c2s, (unsigned long long)h_c2s,
           (unsigned long long)b_s2c, (unsigned long long)h_s2c);
    fflush(stdout);
    _exit(ok && bad == 0 ? 0 : 1);
}
