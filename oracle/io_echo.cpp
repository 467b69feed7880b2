// TEST INFRASTRUCTURE ONLY -- config C1 (BASELINE.json configs[0]: "Loopback TCP encrypted
// echo, AES-256/package-mode, 1 KiB payload x 10k quests") through the reference's OWN IO
// plumbing, never part of the product:
//   client SendBuffer  (core/IOBuffer.cpp:36-45,55-116,257-278: entryEncryptMode,
//                       send -> encryptData -> Encryptor::encrypt(std::string*))
//   server receiver    EncryptedPackageReceiver / EncryptedStreamReceiver::recvPackage +
//                       fetch (+ Decoder) -- the object RecvBuffer::entryEncryptMode
//                       creates (core/IOBuffer.cpp:13-25; RecvBuffer itself is not linked:
//                       its constructor's StandardReceiver pulls in the curl-based
//                       HttpClient, whose headers this image lacks)
//   server SendBuffer  the answer (FPAnswer of the decoded quest, same payload)
//   client receiver    the answer, checked against what was sent
// over a loopback TCP connection (127.0.0.1; a socketpair if the box refuses TCP), one
// epoll-style non-blocking loop on one thread.  Messages are the reference's own FPQuest /
// FPAnswer (proto/FPMessage.cpp); sequence numbers are set explicitly so the wire bytes are
// a function of the inputs alone.
//
// The same source is linked twice (oracle/Makefile):
//   _ref/io_echo_ref     with the reference's core/Encryptor.cpp + base/rijndael.c, and
//   _ref/io_echo_dropin  with every reference file compiled UNCHANGED against this repo's
//                        include/Encryptor.h + include/rijndael.h (a header overlay of
//                        symlinks) and libfpnn_aes.so -- the
//                        north-star "drops unchanged into the IOWorker send/recv plumbing".
// Both print one JSON line with FNV-1a checksums of every byte each direction carried on the
// wire; the two builds must agree byte for byte.
//
// usage: io_echo <mode 0 package|1 stream> <keylen> <quests> <payload bytes> [window]
//   window: quests in flight (1 = strict ping-pong, the per-call latency shape)
#include <arpa/inet.h>
#include <errno.h>
#include <execinfo.h>
#include <signal.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <exception>
#include <string>
#include <vector>

#include "FPLog.h"
#include "IOBuffer.h"
#include "Setting.h"

using namespace fpnn;

namespace {

uint64_t fnv(uint64_t h, const char *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
    return h;
}

void nonblock(int fd) { fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

// a connected loopback TCP pair (client, server); false if the host refuses
bool tcp_pair(int &c, int &s) {
    int l = socket(AF_INET, SOCK_STREAM, 0);
    if (l < 0) return false;
    sockaddr_in a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t al = sizeof a;
    if (bind(l, (sockaddr *)&a, sizeof a) != 0 || listen(l, 1) != 0 || getsockname(l, (sockaddr *)&a, &al) != 0) {
        close(l);
        return false;
    }
    c = socket(AF_INET, SOCK_STREAM, 0);
    if (c < 0 || connect(c, (sockaddr *)&a, sizeof a) != 0) {
        close(l);
        return false;
    }
    s = accept(l, nullptr, nullptr);
    close(l);
    if (s < 0) return false;
    int one = 1;
    setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return true;
}

// bytes a SendBuffer wrote into a socketpair, recorded and forwarded to the TCP socket
struct Tap {
    int from, to;
    std::string pending;
    uint64_t hash = 0xcbf29ce484222325ull, bytes = 0;
    Tap(int f, int t) : from(f), to(t) {}
    void pump() {
        char buf[65536];
        for (;;) {
            const ssize_t r = ::read(from, buf, sizeof buf);
            if (r <= 0) break;
            hash = fnv(hash, buf, (size_t)r);
            bytes += (uint64_t)r;
            pending.append(buf, (size_t)r);
        }
        while (!pending.empty()) {
            const ssize_t w = ::write(to, pending.data(), pending.size());
            if (w <= 0) break;
            pending.erase(0, (size_t)w);
        }
    }
};

std::string payload_of(uint32_t i, int len) {
    std::string p((size_t)len, '\0');
    uint64_t x = 0x9E3779B97F4A7C15ull ^ ((uint64_t)i * 0xD1B54A32D192ED03ull);
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

}  // namespace

static int run(int argc, char **argv);

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
    try {  // the reference Encryptor cannot throw; the drop-in reports GPU failures this way
        return run(argc, argv);
    } catch (const std::exception &ex) {
        fprintf(stderr, "io_echo: %s\n", ex.what());
        fflush(stderr);
        _exit(9);
    }
}

static int run(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s mode keylen quests payload [window]\n", argv[0]);
        return 2;
    }
    const bool stream = atoi(argv[1]) != 0;
    const int keylen = atoi(argv[2]);
    const uint32_t quests = (uint32_t)atoi(argv[3]);
    const int plen = atoi(argv[4]);
    const uint32_t window = argc > 5 ? (uint32_t)atoi(argv[5]) : 1u;
    Setting::set("FP.server.local.ip4", "127.0.0.1");  // FPLog never asks the cloud-metadata client

    uint8_t key[32], iv[16];
    for (int i = 0; i < 32; i++) key[i] = (uint8_t)(11 * i + 3);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)(29 * i + 7);

    int tc = -1, ts = -1;
    bool tcp = tcp_pair(tc, ts);
    if (!tcp) {
        int sv[2];
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 3;
        tc = sv[0];
        ts = sv[1];
    }
    int a[2], b[2];  // SendBuffer -> tap socketpairs
    if (socketpair(AF_UNIX, SOCK_STREAM, 0, a) != 0 || socketpair(AF_UNIX, SOCK_STREAM, 0, b) != 0) return 3;
    for (int fd : {tc, ts, a[0], a[1], b[0], b[1]}) nonblock(fd);

    std::mutex mc, ms;
    SendBuffer csend(&mc), ssend(&ms);
    if (!csend.entryEncryptMode(key, keylen, iv, stream) || !ssend.entryEncryptMode(key, keylen, iv, stream)) return 4;
    // what RecvBuffer::entryEncryptMode(key, key_len, iv, streamMode) installs
    Receiver *crecv = stream ? (Receiver *)new EncryptedStreamReceiver(key, keylen, iv)
                             : (Receiver *)new EncryptedPackageReceiver(key, keylen, iv);
    Receiver *srecv = stream ? (Receiver *)new EncryptedStreamReceiver(key, keylen, iv)
                             : (Receiver *)new EncryptedPackageReceiver(key, keylen, iv);
    Tap c2s(a[0], tc), s2c(b[0], ts);

    uint32_t sent = 0, answered = 0, served = 0, bad = 0;
    const double t0 = now();
    bool needWait, actual;
    while (answered < quests) {
        while (sent < quests && sent - answered < window) {  // client: next quest
            FPQuest q("echo");
            q.setSeqNum(sent + 1);
            q.setPayload(payload_of(sent, plen));
            q.setPayloadSize((uint32_t)plen);
            csend.send(a[1], needWait, actual, q.raw());
            sent++;
        }
        csend.send(a[1], needWait, actual);
        c2s.pump();
        for (;;) {  // server: every complete quest -> its answer
            bool need = true;
            if (!srecv->recvPackage(ts, need)) return 5;
            if (need) break;
            FPQuestPtr q;
            FPAnswerPtr ans;
            bool http = false;
            if (!srecv->fetch(q, ans, http) || !q) return 6;
            FPAnswer reply(q);
            reply.setPayload(q->payload());
            reply.setPayloadSize((uint32_t)q->payload().size());
            ssend.send(b[1], needWait, actual, reply.raw());
            served++;
        }
        ssend.send(b[1], needWait, actual);
        s2c.pump();
        for (;;) {  // client: answers, checked against the quests
            bool need = true;
            if (!crecv->recvPackage(tc, need)) return 7;
            if (need) break;
            FPQuestPtr q;
            FPAnswerPtr ans;
            bool http = false;
            if (!crecv->fetch(q, ans, http) || !ans) return 8;
            const uint32_t i = ans->seqNum() - 1;
            if (i != answered || ans->payload() != payload_of(i, plen)) bad++;
            answered++;
        }
    }
    const double dt = now() - t0;
    printf("{\"transport\": \"%s\", \"mode\": \"%s\", \"keylen\": %d, \"quests\": %u, \"payload\": %d, "
           "\"window\": %u, \"us_per_echo\": %.3f, \"echo_per_s\": %.1f, \"answers_ok\": %s, \"served\": %u, "
           "\"wire_c2s_bytes\": %llu, \"wire_c2s_fnv\": \"%016llx\", \"wire_s2c_bytes\": %llu, "
           "\"wire_s2c_fnv\": \"%016llx\"}\n",
           tcp ? "tcp-loopback" : "socketpair", stream ? "stream" : "package", keylen, quests, plen, window,
           1e6 * dt / quests, quests / dt, bad == 0 ? "true" : "false", served, (unsigned long long)c2s.bytes,
           (unsigned long long)c2s.hash, (unsigned long long)s2c.bytes, (unsigned long long)s2c.hash);
    fflush(stdout);
    _exit(bad == 0 ? 0 : 1);  // the logger's consumer thread is not joined
}
