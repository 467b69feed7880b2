/*
 * StreamReceiverBatch.h -- the receive side of many stream-mode connections in one GPU
 * pass per IO cycle.
 *
 * The reference's EncryptedStreamReceiver (core/EncryptedStreamReceiver.cpp:72-163) reads
 * a connection's 12-byte header, decrypts it with the connection's StreamEncryptor to
 * learn FPMessage::BodyLen (proto/FPMessage.cpp:27-44), reads the body, and decrypts it
 * in fetch(): two dependent decrypt calls per message.  Through the drop-in Encryptor
 * (include/Encryptor.h) those are two synchronous GPU round trips per message.
 *
 * Here an IO loop hands over, per cycle, the bytes each connection read from its socket;
 * flush() decrypts all of them in one pass (fpnn_aes_stream_recv: the stream state of
 * every connection's StreamEncryptor advanced over every byte, exactly as one decrypt
 * call per read would) and splits each connection's plaintext into FPNN messages on the
 * device with the reference's checks.  A message split across cycles is carried as
 * plaintext (the tail after the last complete message) into the next flush.
 *
 *   fpnn::StreamReceiverBatch rx;                 // one per IO thread (its engine)
 *   int c = rx.open(&conn->recvEncryptor);        // at connection set-up
 *   ...per epoll cycle, per readable connection:
 *   n = read(fd, buf, sizeof buf); rx.received(c, buf, n);
 *   ...once per cycle:
 *   rx.flush();
 *   for (const std::string &m : rx.messages(c))  // what fetch() hands to Decoder
 *       dispatch(Decoder::decodeQuest(m.data(), m.size()) ...);
 *   if (rx.status(c) != FPNN_AES_SCAN_OK) close(fd);   // recvPackage returned false
 *
 * Errors throw fpnn::EncryptorError; there is no CPU fallback.
 */
#ifndef FPNN_AMD_STREAM_RECEIVER_BATCH_H
#define FPNN_AMD_STREAM_RECEIVER_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "Encryptor.h"

namespace fpnn {

class StreamReceiverBatch {
public:
    /* max_len: Config::_max_recv_package_length (8 MiB by default); max_frames: messages
       reported per connection and device pass (a connection with more takes another pass
       inside the same flush). */
    explicit StreamReceiverBatch(uint32_t max_len = 8u << 20, uint32_t max_frames = 64);
    ~StreamReceiverBatch();
    StreamReceiverBatch(const StreamReceiverBatch &) = delete;
    StreamReceiverBatch &operator=(const StreamReceiverBatch &) = delete;

    /* A connection whose received bytes are decrypted by enc (its receive-direction
       StreamEncryptor; flush() advances its state).  Returns the connection id. */
    int open(StreamEncryptor *enc);
    /* Forget a connection (its id may be reused by a later open). */
    void close(int conn);
    /* Ciphertext read from the connection's socket, in arrival order. */
    void received(int conn, const uint8_t *data, size_t len);
    /* One GPU pass over every connection's bytes received since the last flush. */
    void flush();

    /* Complete messages (12-byte header + body, plaintext) found by the last flush. */
    const std::vector<std::string> &messages(int conn) const;
    /* FPNN_AES_SCAN_OK, or why the reference would close the connection
       (FPNN_AES_SCAN_TOO_LARGE / _BAD_MAGIC / _BAD_MTYPE / _BAD_LENGTH).  A connection
       in error takes no further bytes. */
    int status(int conn) const;
    /* Plaintext bytes of an incomplete message carried into the next flush. */
    size_t pending(int conn) const;

private:
    struct Conn {
        StreamEncryptor *enc = nullptr;
        std::string in;     // ciphertext received since the last flush
        std::string carry;  // plaintext of an incomplete message
        std::vector<std::string> msgs;
        int status = 0;
        bool open = false;
        bool more = false;  // the last pass stopped at max_frames
    };
    std::vector<Conn> _conns;
    std::vector<int> _free;
    uint32_t _max_len, _max_frames;
    struct Dev;
    Dev *_dev = nullptr;
    void pass(const std::vector<int> &ids, int nrounds);
};

}  // namespace fpnn

#endif
