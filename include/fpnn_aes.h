/*
 * fpnn_aes.h -- C-ABI of the MI355X AES-CFB packet-encryption path.
 *
 * Replaces, for batches of independent packets/streams, the CPU path
 *   core/Encryptor.cpp:10-70  (PackageEncryptor / StreamEncryptor)
 *     -> base/rijndael.c:1171-1201 (rijndael_cfb_encrypt)
 *        -> base/rijndael.c:852-959 (rijndael_encrypt)
 * of the reference (highras/fpnn v1.3.1).  Plain pointers and sizes only;
 * no exceptions and no C++/torch types cross this boundary.  Every call
 * returns an int status (the reference functions are void; see
 * FPNN_AES_ERR_* below for what is now reported instead of being undefined).
 *
 * Device pointers ("dev") are HIP device addresses on the engine's GPU; host
 * pointers ("host") are ordinary process memory.  All device work is queued on
 * the engine's HIP stream; calls return after queuing unless they say otherwise.
 * Results are bit-identical to the reference for every key length (16/24/32),
 * payload length (including 0 and non-multiples of 16) and CFB position.
 *
 * Library layout: libfpnn_aes.so (what callers link) carries these entry points, the
 * C++ classes (Encryptor.h, EncryptorBatch.h, StreamReceiverBatch.h, KeyExchange.h) and
 * no HIP dependency of its own; on first use it loads libfpnn_aes_gpu.so from its own
 * directory (FPNN_AES_GPU_LIB overrides the path) -- the HIP kernels and the engine --
 * and forwards every call there.  Loading the HIP runtime late keeps its static TLS
 * (about 30 KiB, rocprofiler-register) out of every thread's stack: FPNN starts threads
 * with 16 KiB stacks (base/msec.c:72-74), which the runtime linked at start-up made
 * pthread_create refuse.  If the GPU library cannot be loaded every call returns
 * FPNN_AES_ERR_NODEV (fpnn_aes_last_error says why).
 */
#ifndef FPNN_AES_H
#define FPNN_AES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------- */
#define FPNN_AES_OK            0
#define FPNN_AES_ERR_KEYLEN   -1  /* key length not 16/24/32 (reference: setup returns false
                                     and the cipher then runs with nrounds = 0, rijndael.c:797) */
#define FPNN_AES_ERR_ARG      -2  /* NULL pointer, bad descriptor, mixed key lengths */
#define FPNN_AES_ERR_RANGE    -3  /* batch too large (more than 2^32-1 16-byte blocks or packets) */
#define FPNN_AES_ERR_HIP      -4  /* HIP runtime error (message: fpnn_aes_last_error) */
#define FPNN_AES_ERR_NODEV    -5  /* no usable gfx950 device / kernels not loadable */
#define FPNN_AES_ERR_DEVICE   -6  /* a queued kernel's own consistency check failed (reported by
                                     the next fpnn_aes_engine_sync or synchronous call) */

const char *fpnn_aes_strerror(int status);
/* Thread-local text of the last HIP error seen by this thread (or ""). */
const char *fpnn_aes_last_error(void);

/* ---- key schedule ------------------------------------------------------------ */
/* Layout identical to rijndael_context (base/rijndael.h:13-16). */
typedef struct {
    int nrounds;
    uint32_t rk[60];
} fpnn_aes_schedule;

/* Host key expansion.  Mirrors rijndael_setup_encrypt (base/rijndael.c:712-799):
 * same big-endian rk[] words, same nrounds; returns FPNN_AES_OK or
 * FPNN_AES_ERR_KEYLEN (and sets nrounds = 0, like the reference). */
int fpnn_aes_setup_encrypt(fpnn_aes_schedule *ctx, const uint8_t *key, size_t keylen);

/* Decryption key schedule.  Mirrors rijndael_setup_decrypt (base/rijndael.c:805-850):
 * the encryption schedule with the round keys reversed and InvMixColumns applied to all
 * but the first and last -- the same rk[] words as the reference. */
int fpnn_aes_setup_decrypt(fpnn_aes_schedule *ctx, const uint8_t *key, size_t keylen);

/* ---- engine: one GPU, one HIP stream ---------------------------------------- */
typedef struct fpnn_aes_engine fpnn_aes_engine;
#define FPNN_AES_OWN_STREAM ((void *)(intptr_t)-1)

int fpnn_aes_device_count(int *count);
/* hip_stream: the hipStream_t to queue on (e.g. torch's current stream); NULL is
 * the device's null stream, as everywhere in HIP; FPNN_AES_OWN_STREAM creates a
 * private non-blocking stream owned by the engine.  The engine is not thread-safe; use one
 * engine per submitting thread (the reference's per-connection token discipline,
 * core/IOBuffer.h:49-62, makes each Encryptor single-threaded in the same way). */
int fpnn_aes_engine_create(int device, void *hip_stream, fpnn_aes_engine **out);
int fpnn_aes_engine_destroy(fpnn_aes_engine *e);
int fpnn_aes_engine_sync(fpnn_aes_engine *e);
void *fpnn_aes_engine_stream(fpnn_aes_engine *e);
/* Pre-size scratch for batches of up to max_segments packets/streams and
 * max_blocks total 16-byte blocks, so later device-batch calls of that size never
 * allocate or memset.  They are then graph-safe: a call captured on the engine's stream
 * (hipStreamBeginCapture) may be replayed with new data, offsets and lengths in the same
 * device arrays, because every piece of cross-call scratch state (the block map's
 * look-back epoch and tickets, the length-order block and K2h's tickets) is reset on the
 * device by the kernels that use it (tests/test_gpu_graph.py). */
int fpnn_aes_engine_reserve(fpnn_aes_engine *e, uint64_t max_segments, uint64_t max_blocks);

/* Placement of the engines behind the C++ classes (Encryptor, EncryptorBatch,
 * StreamReceiverBatch, ECCKeyExchange): one pool per process, engine k created on the
 * device returned here for (k, ndev = fpnn_aes_device_count) -- k % ndev, or the k-th
 * entry (cyclically) of the comma list FPNN_AES_DEVICES, or FPNN_AES_DEVICE alone;
 * -1 when no device is usable.  Pure functions of their arguments and the environment
 * (no HIP call), so the plan can be checked without a GPU. */
int fpnn_aes_thread_engine_device(uint32_t k, int ndev);
/* Engines the pool creates before calling threads start to share one (calls on a shared
 * engine serialise): FPNN_AES_MAX_ENGINES, default 16 per usable device, at least 1. */
int fpnn_aes_max_thread_engines(int ndev);

/* ---- key sets: the per-connection (key, IV) table on the device -------------- */
/* A key set holds `count` expanded keys of ONE key length plus one 16-byte IV each
 * (the connection IV of package mode, core/Encryptor.h:14).  keys: count*keylen
 * bytes, ivs: count*16 bytes (NULL => zero IVs).  keys_on_host != 0 means keys/ivs
 * are host pointers (copied), otherwise device pointers.  Expansion runs on the GPU. */
typedef struct fpnn_aes_keyset fpnn_aes_keyset;

int fpnn_aes_keyset_create(fpnn_aes_engine *e, uint32_t count, size_t keylen, const uint8_t *keys,
                           const uint8_t *ivs, int keys_on_host, fpnn_aes_keyset **out);
/* Same, from host schedules already expanded by fpnn_aes_setup_encrypt /
 * rijndael_setup_encrypt (all with the same nrounds). */
int fpnn_aes_keyset_from_schedules(fpnn_aes_engine *e, uint32_t count, const fpnn_aes_schedule *ctx,
                                   const uint8_t *ivs, fpnn_aes_keyset **out);
/* A key table updated in place -- the collector's persistent per-connection table
 * (fpnn::EncryptorBatch): `capacity` slots of one key length (nrounds 10/12/14), all zero.
 * fpnn_aes_keyset_set writes host schedules (+ IVs, NULL => zero) into slots
 * [first, first + count), growing the table when needed (contents kept); it is queued on
 * the engine stream through pinned staging, so a flush that adds a few connections
 * costs one small copy and no allocation.  The key set's count becomes
 * max(count, first + count). */
int fpnn_aes_keyset_reserve(fpnn_aes_engine *e, uint32_t capacity, int nrounds, fpnn_aes_keyset **out);
int fpnn_aes_keyset_set(fpnn_aes_keyset *ks, uint32_t first, uint32_t count, const fpnn_aes_schedule *ctx,
                        const uint8_t *ivs);
uint32_t fpnn_aes_keyset_count(const fpnn_aes_keyset *ks);
int fpnn_aes_keyset_destroy(fpnn_aes_keyset *ks);
int fpnn_aes_keyset_nrounds(const fpnn_aes_keyset *ks);
/* Copy the expanded schedule of slot i back to the host (rijndael_context layout). */
int fpnn_aes_keyset_get_schedule(fpnn_aes_keyset *ks, uint32_t slot, fpnn_aes_schedule *out);

/* ---- batch descriptor ---------------------------------------------------------- */
/* A batch is `count` independent segments.  Segment i reads len_i bytes at
 * in + in_off[i] and writes len_i bytes at out + out_off[i]:
 *   in_off  == NULL -> in_off[i]  = i * stride
 *   out_off == NULL -> out_off[i] = in_off[i]
 *   len     == NULL -> len_i      = uniform_len
 *   key_slot== NULL -> slot_i     = 0            (index into the key set)
 * Offsets/lengths/slots are device arrays.  `in` and `out` may be the same
 * buffer with identical offsets (in-place: in == out as pointers); any other overlap
 * -- including in != out pointers whose ranges meet -- is undefined. */
typedef struct {
    const uint8_t *in;          /* dev */
    uint8_t *out;               /* dev */
    uint32_t count;
    uint32_t uniform_len;
    uint64_t stride;
    const uint64_t *in_off;     /* dev, optional */
    const uint64_t *out_off;    /* dev, optional */
    const uint32_t *len;        /* dev, optional */
    const uint32_t *key_slot;   /* dev, optional */
    const fpnn_aes_keyset *keys;
    uint32_t flags;             /* FPNN_AES_F_* */
    uint32_t max_len;           /* optional: an upper bound on every len_i in bytes, 0 = unknown.
                                   Ragged package encrypts of many short frames (max_len <=
                                   2048, count >= 1 chain per GPU lane, i.e. 256 CUs x 1024)
                                   then run one lane per chain in grid-stride order (K2;
                                   with max_len <= 175, FPNN's quests, K2s-DB: each frame
                                   loaded, ciphered and stored whole in one pass, the next
                                   one loading meanwhile; package decrypts with that bound
                                   likewise, D2s);
                                   without the bound, or with fewer chains, the
                                   length-ordered hybrid (K2h), whose work queue also balances
                                   Zipf-like lengths.  (Was `reserved`, 0: same layout.) */
} fpnn_aes_batch;

/* Package encrypt only: write the wire frame of PackageEncryptor::encrypt(std::string*)
 * (core/Encryptor.cpp:34-51): htole32(len) at out + out_off[i], ciphertext at +4. */
#define FPNN_AES_F_WIRE_PREFIX 0x1u

/* ---- package mode (core/Encryptor.cpp:10-51) ------------------------------------- */
/* Every segment starts a fresh CFB chain from its key slot's IV at position 0,
 * exactly as PackageEncryptor re-copies _iv and re-expands the key per call.
 * Decrypt runs one GPU lane per 16-byte block; encrypt one lane per packet chain. */
int fpnn_aes_package_encrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b);
int fpnn_aes_package_decrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b);

/* ---- stream mode (core/Encryptor.cpp:53-70) ---------------------------------------- */
/* Segment i continues the CFB stream whose state is (iv_state[16*i .. +16],
 * pos_state[i]) -- StreamEncryptor::_iv and ::_pos -- with key slot slot_i; the
 * state is updated in place (dev arrays).  A given stream must appear at most once
 * per call; successive frames of a stream go in successive calls. */
int fpnn_aes_stream_encrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state,
                            uint32_t *pos_state);
int fpnn_aes_stream_decrypt(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state,
                            uint32_t *pos_state);

/* ---- single call from host memory (the per-frame drop-in) --------------------------- */
/* Exactly rijndael_cfb_encrypt(ctx, encrypt, in, out, len, ivec, p_num)
 * (base/rijndael.c:1171-1201) with host buffers: stages through pinned memory,
 * runs the GPU kernels, copies back and updates ivec/p_num.  Synchronous. */
int fpnn_aes_cfb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt,
                      const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16], size_t *p_num);

/* ---- the rest of rijndael.h, single calls from host memory (synchronous) ------------------ */
/* ECB: nblocks independent 16-byte blocks through the forward cipher (encrypt != 0,
 * ctx from fpnn_aes_setup_encrypt; rijndael_encrypt, base/rijndael.c:852-959) or the
 * inverse cipher (ctx from fpnn_aes_setup_decrypt; rijndael_decrypt, :961-1068).
 * in == out allowed. */
int fpnn_aes_ecb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt, const uint8_t *in, uint8_t *out,
                      size_t nblocks);
/* CBC exactly as rijndael_cbc_encrypt / _decrypt (base/rijndael.c:1070-1153): encrypt
 * zero-pads a partial last block and writes 16*ceil(len/16) bytes; decrypt reads
 * 16*ceil(len/16) bytes and writes len; ivec is updated to the last ciphertext block.
 * Decrypt takes the setup_decrypt schedule.  in == out allowed. */
int fpnn_aes_cbc_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, int encrypt, const uint8_t *in, uint8_t *out,
                      size_t len, uint8_t ivec[16]);
/* OFB exactly as rijndael_ofb_encrypt (base/rijndael.c:1155-1169), (ivec, *p_num) carried. */
int fpnn_aes_ofb_host(fpnn_aes_engine *e, const fpnn_aes_schedule *ctx, const uint8_t *in, uint8_t *out, size_t len,
                      uint8_t ivec[16], size_t *p_num);

/* ---- many frames from host memory (the cross-connection batch path, §8f row 1) ------- */
/* One entry per frame.  src/dst are host pointers (dst may equal src for in-place;
 * with FPNN_AES_F_WIRE_PREFIX, dst receives htole32(len) || ciphertext and must hold
 * len + 4 bytes and not overlap src).  key_slot indexes `keys`. */
typedef struct {
    const uint8_t *src;
    uint8_t *dst;
    uint32_t len;
    uint32_t key_slot;
} fpnn_aes_host_frame;

/* Package-mode encrypt (encrypt != 0) or decrypt of n host frames: the frames are
 * gathered into pinned staging by a few host threads, and chunks are pipelined
 * (H2D of chunk i+1 || kernel of chunk i || D2H of chunk i-1) over the engine's
 * streams.  Results equal n PackageEncryptor calls.  Synchronous. */
int fpnn_aes_package_host(fpnn_aes_engine *e, int encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                          const fpnn_aes_keyset *keys, uint32_t flags);

/* Stream-mode encrypt/decrypt of n host frames (StreamEncryptor::encrypt/decrypt,
 * core/Encryptor.cpp:53-70, one call per frame in the reference).  key_slot names the
 * stream: its key slot in `keys` AND its state (iv_state[16*slot .. +16], pos_state[slot],
 * host arrays of keys->count entries, StreamEncryptor::_iv/_pos), updated in place.  A
 * stream may appear many times: its frames are processed in array order, exactly as
 * that many successive calls.  Synchronous. */
int fpnn_aes_stream_host(fpnn_aes_engine *e, int encrypt, const fpnn_aes_host_frame *frames, uint32_t n,
                         const fpnn_aes_keyset *keys, uint8_t *iv_state, uint32_t *pos_state);

/* One host-frame batch over several engines -- e.g. one per GPU of the node, each
 * with its own copy of the key set (keys[k] created on engines[k], same count and key
 * length).  Package mode splits the frames into byte-balanced contiguous ranges; stream
 * mode gives whole streams (all frames of a key slot, in order) to engines, longest first
 * onto the least-loaded one.  Every engine runs its share through its own pipeline in
 * its own host thread; results are as from one call of fpnn_aes_package_host /
 * fpnn_aes_stream_host.  Synchronous. */
int fpnn_aes_package_host_multi(fpnn_aes_engine *const *engines, const fpnn_aes_keyset *const *keys, int n_engines,
                                int encrypt, const fpnn_aes_host_frame *frames, uint32_t n, uint32_t flags);
int fpnn_aes_stream_host_multi(fpnn_aes_engine *const *engines, const fpnn_aes_keyset *const *keys, int n_engines,
                               int encrypt, const fpnn_aes_host_frame *frames, uint32_t n, uint8_t *iv_state,
                               uint32_t *pos_state);

/* ---- host-mapped frames (zero-copy host-frame path) --------------------------------- */
/* Register [ptr, ptr + len) of host memory -- e.g. the arena a server allocates its
 * connections' socket buffers from -- with every GPU (hipHostRegister, portable + mapped;
 * the pages are locked).  fpnn_aes_package_host / _multi calls whose frames all lie in
 * registered memory (src: len bytes, dst: len (+4 with the wire prefix) bytes) are then
 * moved by the GPU itself over PCIe: no host gather/scatter and no pinned bounce copy;
 * the host threads only write 40 bytes of descriptor per frame.  A call whose frames
 * leave registered memory from frame k on runs frames [k, n) through the staged path;
 * calls that start outside it are staged entirely.  Ranges must not overlap; registration is process-wide.
 * Unregister only while no call uses the range. */
int fpnn_aes_host_register(void *ptr, size_t len);
int fpnn_aes_host_unregister(void *ptr);
/* 1 if [ptr, ptr + len) lies inside one registered range, else 0. */
int fpnn_aes_host_is_mapped(const void *ptr, size_t len);

/* ---- receive side: wire framing on the device (§8f row 3) --------------------------- */
/* Per received segment (the bytes one connection delivered), the outcome of walking its
 * frames: `frames` complete frames cover the first `consumed` bytes; the rest is an
 * incomplete frame to keep for the next call, unless status says the connection is bad. */
typedef struct {
    uint32_t frames;
    uint32_t status;   /* FPNN_AES_SCAN_* */
    uint64_t consumed;
} fpnn_aes_frame_scan;
#define FPNN_AES_SCAN_OK         0 /* stopped at the end of the data (maybe mid-frame) */
#define FPNN_AES_SCAN_FULL       1 /* max_frames frames recorded; call again from `consumed` */
#define FPNN_AES_SCAN_TOO_LARGE  2 /* frame above max_len: the reference closes the connection */
#define FPNN_AES_SCAN_BAD_MAGIC  3 /* stream: header magic is not "FPNN" */
#define FPNN_AES_SCAN_BAD_MTYPE  4 /* stream: mtype not 0/1/2 (FPMessage::BodyLen throws) */
#define FPNN_AES_SCAN_BAD_LENGTH 5 /* stream: message length <= 0 by the reference's int arithmetic */

/* Package-mode receive: EncryptedPackageReceiver::recvPackage + fetch
 * (core/EncryptedPackageReceiver.cpp:60-118) for many connections at once.  Segment i of
 * b (b->in + in_off[i], len_i bytes, key slot slot_i) starts at a frame boundary and holds
 * [htole32(n)][n bytes ciphertext] wire frames.  The complete frames' bodies are
 * decrypted (fresh chain each, like PackageEncryptor::decrypt) to b->out at the same
 * offsets (b->out_off must be NULL; in place when b->out == b->in); prefixes and the
 * trailing incomplete frame are not written.  Frame j of segment i is reported at
 * [i*max_frames + j]: frame_off = body offset within the segment, frame_len = n
 * (dev arrays; scan[count] dev).  max_len: Config::_max_recv_package_length (8 MiB). */
int fpnn_aes_package_recv(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint32_t max_len, uint32_t max_frames,
                          uint64_t *frame_off, uint32_t *frame_len, fpnn_aes_frame_scan *scan);

/* Stream-mode receive: EncryptedStreamReceiver (core/EncryptedStreamReceiver.cpp:72-163).
 * Segment i is the ciphertext newly received on stream i; it is decrypted exactly as
 * fpnn_aes_stream_decrypt (state advanced over every byte) and the plaintext, preceded
 * by carry[i] bytes already in b->out (the previous call's incomplete message, NULL = 0),
 * is split into FPNN messages: 12-byte header + FPMessage::BodyLen (proto/FPMessage.cpp:27-44).
 * frame_off is relative to the region start (out + out_off[i] - carry[i]), frame_len is the
 * whole message length (what fetch() hands to the decoder). */
int fpnn_aes_stream_recv(fpnn_aes_engine *e, const fpnn_aes_batch *b, uint8_t *iv_state, uint32_t *pos_state,
                         const uint32_t *carry, uint32_t max_len, uint32_t max_frames, uint64_t *frame_off,
                         uint32_t *frame_len, fpnn_aes_frame_scan *scan);

/* ---- memory on an engine's device, for callers built without HIP headers ------------ */
/* (StreamReceiverBatch uses these: libfpnn_aes.so itself has no HIP dependency, see the
 * library layout note at the top.)  device_free waits for the device; copy_async queues a
 * copy of `bytes` between any two of host-pinned / device memory on the engine stream. */
int fpnn_aes_device_alloc(fpnn_aes_engine *e, size_t bytes, void **out);
int fpnn_aes_device_free(fpnn_aes_engine *e, void *p);
int fpnn_aes_pinned_alloc(fpnn_aes_engine *e, size_t bytes, void **out);
int fpnn_aes_pinned_free(fpnn_aes_engine *e, void *p);
int fpnn_aes_copy_async(fpnn_aes_engine *e, void *dst, const void *src, size_t bytes);

/* NUMA placement of the engine's host side: `node` the node its pinned
 * arenas (pinned_alloc, the host-frame staging) are allocated on and its copy threads run
 * on (-1: none); `device_node` the GPU's node from sysfs (-1: unknown); `ncpus` the node's
 * CPUs the copy threads are pinned to (0: unpinned).  fpnn_aes_last_error() then holds one
 * line saying how the placement was chosen.  FPNN_AES_NUMA=auto|off|<node>. */
int fpnn_aes_engine_numa(fpnn_aes_engine *e, int *node, int *device_node, int *ncpus);

/* ---- synthetic data (bench/tests utility, not part of the cipher) ------------------ */
/* dst[k] = byte (off+k)&7 of splitmix64((off+k)>>3 + seed*0xD1B54A32D192ED03), LE. */
int fpnn_aes_fill_synthetic(fpnn_aes_engine *e, uint8_t *dst, uint64_t nbytes, uint64_t seed,
                            uint64_t byte_offset);

/* ---- instrumentation ---------------------------------------------------------------- */
/* When enabled, every batch call records HIP events around its main kernel on the
 * engine stream; fpnn_aes_engine_kernel_stats returns the count and summed milliseconds
 * of the main-kernel launches since the last reset (synchronizes the stream). */
int fpnn_aes_engine_set_timing(fpnn_aes_engine *e, int enable);
int fpnn_aes_engine_kernel_stats(fpnn_aes_engine *e, int which /* FPNN_AES_K_* */, uint64_t *launches,
                                 double *total_ms);
int fpnn_aes_engine_reset_stats(fpnn_aes_engine *e);
/* Name of the kernel variant the last call queued as its main kernel for that direction
 * ("cfb_decrypt_dense", "cfb_encrypt_queue", ...; "" before any call).  Static storage. */
const char *fpnn_aes_engine_last_kernel(fpnn_aes_engine *e, int which);
#define FPNN_AES_K_DECRYPT 0
#define FPNN_AES_K_ENCRYPT 1
#define FPNN_AES_K_HOST 2 /* last_kernel only: the last host-frame call's path, "host_mapped",
                           "host_staged" or "host_mapped+staged" */

/* Version string of the built library (kernel variant + build flags). */
const char *fpnn_aes_version(void);

#ifdef __cplusplus
}
#endif

#endif /* FPNN_AES_H */
