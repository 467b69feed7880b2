// kernels.hpp -- internal launch interface between the C-ABI (engine.hip) and the
// HIP kernels (k_encrypt.hip, k_decrypt.hip, k_support.hip).  Not installed; the public boundary is include/fpnn_aes.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aes_common.hpp"
#include "audit.hpp"

namespace fpnn_aes {

constexpr uint32_t F_WIRE_PREFIX = 0x1u;
constexpr uint32_t F_ALIGN_CHUNKS = 0x100u;  // internal (engine -> K2): line-align the chunks of each chain

// Kernel-side view of one batch (passed by value as the kernel argument).
struct KBatch {
    const uint8_t *in;
    uint8_t *out;
    uint64_t count;
    uint64_t stride;
    uint32_t uniform_len;
    uint32_t flags;
    const uint64_t *in_off;
    const uint64_t *out_off;
    const uint32_t *len;
    const uint32_t *key_slot;
    const DevKey *keys;
    uint8_t *iv_state;    // stream mode: 16 B per segment (in/out)
    uint32_t *pos_state;  // stream mode: CFB position per segment (in/out)
    const uint32_t *t0le; // 1 KiB T0 source for the LDS image
    // block map (decrypt)
    uint64_t total_blocks;   // uniform layout: exact; general: copy of *total_ptr
    uint32_t nb_uniform;     // uniform layout: blocks per segment
    uint32_t runs;           // K1r: interior runs on (Variant::k1r_runs)
    uint64_t magic;          // ceil(2^64 / nb_uniform)
    const uint64_t *bstart;  // general: first virtual block of each segment (count + 1)
    const uint4 *boundary;   // in-place: Cx block preceding each 64-block chunk
    // stream decrypt: the (iv, pos) state as it was when the call was queued.  The
    // kernel writes the new state into iv_state/pos_state while other waves may still
    // be reading the old one, so every read goes to this snapshot.
    const uint4 *iv_snap;
    const uint32_t *pos_snap;
    // encrypt of ragged batches: segment visiting order (longest first), or null
    const uint32_t *perm;
    // package mode: E_k(IV) per key slot (the first keystream block of every chain of the
    // slot, fpnn_aes_keyset.d_eiv), or null (then computed)
    const uint4 *eiv;
    // the address-audit build's extent table (audit.hpp; null in the product build)
    AuditTable *aud;
};

// UNIFORM: segment i at i*stride, uniform_len bytes, key slot 0.  FULL: the same with
// uniform_len % 16 == 0 in package mode, so no block is partial (decrypt skips the
// byte-granular head/tail paths); with KEY_LANE, FULL also means dense (stride ==
// uniform_len) with key_slot[] holding one slot per packet (K1d keyed when
// uniform_len % 1024 == 0, else K1k).
// GENERAL: offset/length/slot arrays (decrypt: K1r, k_ragged.hip).
enum Layout { LAYOUT_UNIFORM = 0, LAYOUT_GENERAL = 1, LAYOUT_FULL = 2 };
enum KeyMode { KEY_UNIFORM = 0, KEY_LANE = 1 };

// Per-engine dispatch settings that tests set (tests/conftest.py) so that small batches
// reach every session of the shipped kernels.  Round 4 removed the measured-and-rejected
// kernel variants (2-table LDS image, 1/4-block encrypt chunks, unfenced rounds, K2q, K1 on
// dense batches, the separate K1r plan launch for out-of-place batches); round 6 the A/B
// switches whose other side was measured slower (K2h's lane-session wire funnel, the K2c
// threshold, E_k(IV) off, K2's ragged / short-frame / fence / 4-block-chunk / line-
// alignment switches, the three-launch block map) -- their numbers stay in DESIGN.md.
struct Variant {
    // K2h: chains of at least hyb_long blocks (bucket-rounded) go to quads; hyb_quad_waves
    // of a workgroup's 16 waves start on them.  Round-3 sweep on C4 (profiles/r03/
    // sweep_c4_r03x.json): 1024 / 12 at 790-799 GiB/s against 738 for 512 / 8.
    int hyb_long = 1024;
    int hyb_quad_waves = 12;
    int hyb_force = 0;  // every ragged batch of more than one chain takes K2h (tests)
    // tests only: the next poison_order ragged encrypts find their length-order block's
    // counts dirty (FPNN_AES_DEBUG_POISON_ORDER), to check that the device reports it
    int poison_order = 0;
    // K1r: chunks inside one segment's interior take the lean loop (k_ragged.hip); 0 runs
    // every chunk through the general path (FPNN_AES_K1R_RUNS=0: tests reach the general
    // path at every chunk position)
    int k1r_runs = 1;
};

// Base name ("cfb_decrypt_dense", ...) of the main kernel the last launch_* call on this
// thread queued (the variant the dispatch actually chose; instrumentation and bench labels).
const char *last_launched();
void set_launched(const char *name);
// threads = workgroup size (64..1024, multiple of 64): few chains are spread over all
// CUs with small workgroups instead of packed into a few full ones.
// Frame scan of received segments (framing.hip).
enum : uint32_t { SCAN_OK = 0, SCAN_FULL = 1, SCAN_TOO_LARGE = 2, SCAN_BAD_MAGIC = 3, SCAN_BAD_MTYPE = 4,
                  SCAN_BAD_LENGTH = 5 };
struct ScanResult {  // == fpnn_aes_frame_scan
    uint32_t frames, status;
    uint64_t consumed;
};
struct KScan {
    const uint8_t *buf;       // package: received bytes; stream: decrypted plaintext
    uint64_t count;
    const uint64_t *off;      // segment starts (NULL: i * stride)
    uint64_t stride;
    const uint32_t *len;      // segment lengths (NULL: uniform_len)
    uint32_t uniform_len;
    uint32_t max_len;
    const uint32_t *carry;    // stream: plaintext bytes before each segment (NULL: 0)
    const uint32_t *key_slot; // package: segment key slots (NULL: 0)
    uint32_t max_frames;
    uint32_t pad;
    uint64_t *frame_off;      // [count * max_frames], relative to the segment (region) start
    uint32_t *frame_len;
    ScanResult *scan;         // [count]
    uint64_t *abs_off;        // package: absolute body offsets, for the decrypt batch
    uint32_t *abs_slot;       // package: key slot per frame slot (NULL: one key)
};

hipError_t launch_scan_frames(const KScan &s, bool stream, int num_cus, hipStream_t st);
hipError_t launch_encrypt_chains(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool stream, int grid,
                                 int threads, hipStream_t st);
// K2s-DB (k_encrypt.hip): ragged package batches of short frames -- every len <=
// kFrameMaxBytes (the caller's fpnn_aes_batch.max_len) -- one lane per chain, the whole frame
// loaded, ciphered and stored at once while the lane's next frame loads; wire = the 4-byte
// length prefix (FPNN_AES_F_WIRE_PREFIX); grid = one workgroup per CU.
constexpr int kFrameMaxBlocks = 10;
constexpr uint32_t kFrameMaxBytes = 16u * kFrameMaxBlocks + 15u;  // 175: FPNN's 145-B quests and shorter
hipError_t launch_encrypt_frames(const KBatch &b, int nrounds, KeyMode km, bool wire, int grid, hipStream_t st);
// D2s: the same pipeline for package decrypts of short frames (one lane per frame, its
// blocks' AES passes independent of each other); grid = one workgroup per CU
hipError_t launch_decrypt_frames(const KBatch &b, int nrounds, KeyMode km, int grid, hipStream_t st);
// K2c: one 4-lane quad per chain (few / long chains); threads = workgroup size.
hipError_t launch_encrypt_coop(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool stream, int grid,
                               int threads, hipStream_t st);
// K2h (k_hybrid.hip): ragged batches with more chains than quads.  Chains of perm[]
// in length buckets <= long_bucket run on quads (K2c's cipher), the rest one per lane
// (K2's); quad_waves waves per workgroup start on the long ones.  ctr: the 2 ticket
// words of the call's length-order block; buckets: its counts.
// A length-order block (launch_length_order): 128 bucket counts, 128 cursors, then
// (wire-prefix batches) a flag word, nonzero when some frame starts off the 4-byte grid,
// then K2h's two ticket counters, then a count of finished workgroups.  The block starts
// zeroed and its LAST reader zeroes it again once every workgroup is done with it: the
// bucket scatter's last workgroup when K2c follows, K2h's when K2h follows.  No memset
// launch per call, and a call captured in a graph finds the block zeroed on every replay.
constexpr int kWireFlagWord = 256;
constexpr int kTicketWords = 257;
constexpr int kDoneWord = 259;
constexpr int kLengthOrderWords = 260;

struct HybridArgs {
    uint32_t *ctr;
    const uint32_t *buckets;  // the call's length-order block
    uint32_t long_bucket;
    uint32_t quad_waves;
    uint4 *sink;      // 2 x uint4 per wave (grid * kThreads / 64 waves): stores with nothing to store
};
hipError_t launch_encrypt_hybrid(const KBatch &b, const HybridArgs &h, int nrounds, KeyMode km, bool stream, int grid,
                                 hipStream_t st);
// length bucket of a block count (descending: bucket 0 = longest), as launch_length_order
uint32_t length_bucket_of(uint64_t nblocks);
// Ragged batches: perm[] = segment indices ordered by block count, longest first
// (quarter-octave buckets).  block: the length-order block (zero on entry); zero_after:
// nothing reads it after the scatter (K2c follows), so the scatter's last workgroup zeroes
// it; otherwise K2h does.  fault: as for the block map below -- gets kFaultLengthOrder when
// the bucket counts do not add up to b.count (a block not zero on entry); the scatter then
// writes no perm[] entry past the batch and K2h clamps what it reads, so a bad block gives
// FPNN_AES_ERR_DEVICE at the next sync instead of wild addresses.
hipError_t launch_length_order(const KBatch &b, bool stream, uint32_t *perm, uint32_t *block, bool zero_after,
                               uint32_t *fault, hipStream_t st);
// K1 / K1d / K1k for uniform and dense layouts (every segment's block count known on the host).
hipError_t launch_decrypt_blocks(const KBatch &b, int nrounds, Layout layout, KeyMode km, bool inplace, int grid,
                                 hipStream_t st);
// K1r (k_ragged.hip): ragged decrypt with no host round trip.  b.bstart[0..count] from
// launch_block_map_onepass / _small (bstart[count] = total blocks, device only); plan: one entry per
// wave of the grid (grid * kThreads / 64), filled by the plan kernel queued first.
struct RaggedPlan {
    uint64_t s0;  // segment holding the wave's first block
    uint64_t pad;
    uint4 fill;   // ciphertext block before it (same segment), saved before any write
};
// b.in_off, b.out_off and b.len must be device arrays (launch_ragged_desc writes the missing
// ones from stride / uniform_len; out_off may be in_off).
// sink: 2 x uint4 per wave of the grid, written by lanes with nothing to store, never read.
hipError_t launch_decrypt_ragged(const KBatch &b, int nrounds, KeyMode km, bool stream, RaggedPlan *plan, uint4 *sink,
                                 bool plan_launch, int grid, hipStream_t st);
hipError_t launch_ragged_desc(uint64_t count, uint64_t stride, uint32_t uniform_len, uint64_t *in_off, uint32_t *len,
                              hipStream_t st);
// In-place K1 / K1d: save the ciphertext block before every 64-block chunk.
hipError_t launch_boundary_save(const KBatch &b, uint4 *boundary, uint64_t nchunks, hipStream_t st);
// General-layout block map: bstart[0..count], the exclusive scan of per-segment block counts
// (bstart[count] = *total = total blocks, both device), in one launch (decoupled
// look-back); lb = block_map_onepass_words(count) words
// (lb_words = the buffer's capacity), zero when first used.  Everything the next launch
// needs is kept by the kernel itself -- tickets reset and the tile-status epoch advanced by
// its last workgroup -- so a launch captured in a graph and replayed stays correct.
// fault: a device-visible word (pinned host) that gets kFaultLookback if a look-back ever
// gave up waiting (the host reports FPNN_AES_ERR_DEVICE at the next sync).
constexpr uint32_t kFaultLookback = 1u;
constexpr uint32_t kFaultLengthOrder = 2u;
uint64_t block_map_onepass_words(uint64_t count);
hipError_t launch_block_map_onepass(const KBatch &b, bool stream, uint64_t *bstart, uint64_t *lb, uint64_t lb_words,
                                    uint32_t *fault, uint64_t *total, hipStream_t st);
// The same for count <= block_map_small_max() in one workgroup; stream batches also
// copy (iv_state, pos_state) into the snapshot (snap_iv / snap_pos) on the way.
hipError_t launch_block_map_small(const KBatch &b, bool stream, const uint8_t *iv_state, const uint32_t *pos_state,
                                  uint4 *snap_iv, uint32_t *snap_pos, uint64_t *bstart, uint64_t *total,
                                  hipStream_t st);
uint64_t block_map_small_max();
// The rest of rijndael.h (k_modes.hip): ECB / CBC / OFB over one host call's buffers.
enum : int { MODE_ECB_ENC = 0, MODE_ECB_DEC = 1, MODE_CBC_ENC = 2, MODE_CBC_DEC = 3, MODE_OFB = 4 };
struct ModeArgs {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nblocks;      // whole 16-byte blocks to process (ECB, CBC)
    uint64_t len;          // OFB: bytes
    const DevKey *key;     // encryption schedule, or the decryption schedule (ECB/CBC decrypt)
    uint8_t *iv;           // 16 B, in/out (CBC encrypt, OFB); CBC decrypt reads it
    uint32_t *pos;         // OFB position, in/out
    const uint32_t *t0le, *td0le;
    const uint8_t *isbox;
};
hipError_t launch_block_modes(const ModeArgs &a, int nrounds, int mode, int num_cus, hipStream_t st);
// K0 (k_small.hip): one synchronous CFB call of up to kSmallMaxBytes bytes, in place in
// pinned host staging: body at io + kSmallBodyAt (16-aligned), the head's bytes (pos != 0)
// right before it.  state (pinned): [ivec 16 B][pos u32][seq u32], the kernel stores seq
// last (system-scope release) once everything else is visible to the host.
constexpr uint32_t kSmallMaxBytes = 16384;
constexpr uint32_t kSmallBodyAt = 32;
struct SmallArgs {
    uint8_t *io;
    uint32_t len;   // bytes in the call (head + body)
    uint32_t head;  // min(len, (16 - pos) % 16): bytes finishing the current keystream block
    uint32_t pos;   // *p_num on entry
    uint32_t seq;
    uint4 iv;       // ivec on entry
    uint32_t rk[60];
    const uint32_t *t0le;
    uint32_t *state;
};
hipError_t launch_cfb_single(const SmallArgs &a, int nrounds, bool encrypt, hipStream_t st);
// K0s (k_small.hip): the resident form of K0 behind a mailbox in pinned host memory.  The
// host fills req (seq last, release), the server serves each new seq and stores it into
// resp.done after the results (io in place, resp.state = ivec + pos); it leaves after
// idle_ticks without a request, after life_ticks in any case, or when req.stop is set,
// storing its epoch into resp.exited.  Ticks of the device wall clock (wall_clock64).
struct alignas(16) SmallReq {
    uint32_t seq, op, len, head, pos, nrounds, stop, pad;  // op bit 0: encrypt
    uint32_t iv[4];
    uint32_t rk[60];  // block byte order
};
struct alignas(64) SmallResp {
    uint32_t done, exited, pad[2];
    uint32_t state[8];  // ivec (4 words), pos
};
struct SmallMailbox {
    SmallReq req;
    SmallResp resp;
    alignas(64) uint8_t io[kSmallBodyAt + kSmallMaxBytes + 64];
};
// yield: the device's batch-activity word (pinned host memory), y0 its value when the host
// launched the server: the host bumps it before it queues batch kernels; a server that sees
// it differ from y0 leaves after its current request (also one that only started after the
// bump), so no batch workgroup waits for a CU (or a hardware queue) a server holds.
hipError_t launch_cfb_server(SmallMailbox *mb, const uint32_t *t0le, uint32_t epoch, uint64_t idle_ticks,
                             uint64_t life_ticks, const uint32_t *yield, uint32_t y0, hipStream_t st);
// E_k(IV) of key slots [first, first + count) into eiv[first ...] (k_small.hip)
hipError_t launch_slot_eiv(const DevKey *keys, uint32_t first, uint32_t count, int nrounds, const uint32_t *t0le,
                           uint4 *eiv, hipStream_t st);
hipError_t launch_expand_keys(const uint8_t *keys, uint32_t keylen, const uint8_t *ivs, uint32_t count,
                              const uint8_t *sbox, DevKey *out, hipStream_t st);
// Host-mapped frame moves: a job copies n segments, segment i from address sbase + soff[i]
// to dbase + doff[i], len[i] + extra bytes (soff/doff/len device arrays; either side may be
// mapped host memory; a base of 0 makes the offsets absolute device-visible addresses).
// One launch runs two jobs concurrently (n = 0: none).
struct MoveJob {
    uint64_t sbase;
    const uint64_t *soff;
    uint64_t dbase;
    const uint64_t *doff;
    const uint32_t *len;
    uint32_t extra;
    uint32_t n;
};
hipError_t launch_move_segments(const MoveJob &a, const MoveJob &b, hipStream_t st);
hipError_t launch_fill_synthetic(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, int grid,
                                 hipStream_t st);

}  // namespace fpnn_aes
