/*
 * aes_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker), never shipped.
 *
 * A clean-room, plain-C restatement of the reference algorithm for FPNN's AES
 * packet-encryption path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (as liboracle.so via ctypes); the product path in
 * fpnn_amd/ has no CPU cipher and no dependency on this file.
 *
 * What it restates (reference = /root/reference, FPNN v1.3.1):
 *   - T-table AES forward cipher: Te0..Te3 = SubBytes o MixColumns, pre-rotated,
 *     and the final round's S-box masks (base/rijndael.c:8-346, 852-959).  The
 *     tables are *generated* here from GF(2^8) arithmetic, not copied.
 *   - FIPS-197 key expansion with big-endian words (base/rijndael.c:696-799).
 *   - CFB-128 byte loop with the (ivec, *p_num) carry (base/rijndael.c:1171-1201).
 *   - The rest of the rijndael.h surface: the decryption key schedule (reversed round
 *     keys with InvMixColumns, base/rijndael.c:805-850), the inverse cipher (Td0..Td4,
 *     :348-686, 961-1068), CBC with its zero-padded / partial last block (:1070-1153)
 *     and OFB with the (ivec, *p_num) carry (:1155-1169).
 *   - PackageEncryptor / StreamEncryptor call semantics (core/Encryptor.cpp:10-70).
 *
 * Parity pinned by (tests/test_oracle.py):
 *   - FIPS-197 C.1/C.3 and SP 800-38A F.3.13/F.3.17 known-answer vectors;
 *   - the JSON fixtures in tests/golden/ produced by oracle/gen_golden.py, which runs the
 *     reference sources compiled by oracle/Makefile into oracle/_ref/;
 *   - when oracle/_ref/libfpnn_ref.so is present, a live randomized comparison.
 */
#include "aes_oracle.h"

#include <pthread.h>
#include <string.h>
#include <stdlib.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* Table generation (equivalent of the static tables at base/rijndael.c:8-346) */

static uint8_t g_sbox[256];
static uint8_t g_isbox[256];
static uint32_t g_te[4][256];
static uint32_t g_td[4][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static uint8_t gf_mul2(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0x00)); }

static uint8_t rotl8(uint8_t v, int n) { return (uint8_t)((v << n) | (v >> (8 - n))); }

static uint32_t ror32(uint32_t v, int n) { return n ? (v >> n) | (v << (32 - n)) : v; }

static void build_tables(void)
{
    /* exp/log tables over generator 0x03 of GF(2^8) mod x^8+x^4+x^3+x+1 */
    uint8_t exp_t[255], log_t[256];
    uint8_t a = 1;
    for (int i = 0; i < 255; i++) {
        exp_t[i] = a;
        log_t[a] = (uint8_t)i;
        a = (uint8_t)(a ^ gf_mul2(a)); /* a *= 3 */
    }
    for (int x = 0; x < 256; x++) {
        uint8_t inv = x ? exp_t[(255 - log_t[x]) % 255] : 0;
        uint8_t s = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
        g_sbox[x] = s;
    }
    for (int x = 0; x < 256; x++) {
        uint8_t s = g_sbox[x], s2 = gf_mul2(s), s3 = (uint8_t)(s2 ^ s);
        /* column (2s, s, s, 3s) as a big-endian word */
        uint32_t t0 = ((uint32_t)s2 << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | s3;
        for (int k = 0; k < 4; k++)
            g_te[k][x] = ror32(t0, 8 * k);
        g_isbox[s] = (uint8_t)x;
    }
    /* inverse tables: InvSubBytes o InvMixColumns, column (14i, 9i, 13i, 11i) */
    for (int x = 0; x < 256; x++) {
        uint8_t i1 = g_isbox[x], i2 = gf_mul2(i1), i4 = gf_mul2(i2), i8 = gf_mul2(i4);
        uint8_t i9 = (uint8_t)(i8 ^ i1), i11 = (uint8_t)(i8 ^ i2 ^ i1), i13 = (uint8_t)(i8 ^ i4 ^ i1),
                i14 = (uint8_t)(i8 ^ i4 ^ i2);
        uint32_t t0 = ((uint32_t)i14 << 24) | ((uint32_t)i9 << 16) | ((uint32_t)i13 << 8) | i11;
        for (int k = 0; k < 4; k++)
            g_td[k][x] = ror32(t0, 8 * k);
    }
}

static void ensure_tables(void) { pthread_once(&g_once, build_tables); }

static uint32_t load_be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void store_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

static uint32_t sub_word(uint32_t w)
{
    return ((uint32_t)g_sbox[w >> 24] << 24) | ((uint32_t)g_sbox[(w >> 16) & 0xff] << 16) |
           ((uint32_t)g_sbox[(w >> 8) & 0xff] << 8) | g_sbox[w & 0xff];
}

/* ------------------------------------------------------------------------- */
/* Key expansion: base/rijndael.c:712-799 (FIPS-197 section 5.2)              */

int ao_setup_encrypt(ao_ctx *ctx, const uint8_t *key, size_t keylen)
{
    ensure_tables();
    int nk, nr;
    switch (keylen) {
    case 16: nk = 4; nr = 10; break;
    case 24: nk = 6; nr = 12; break;
    case 32: nk = 8; nr = 14; break;
    default: ctx->nrounds = 0; return 0; /* reference: nrounds = 0, return false (:797-798) */
    }
    uint32_t *w = ctx->rk;
    for (int i = 0; i < nk; i++)
        w[i] = load_be32(key + 4 * i);
    uint32_t rcon = 0x01;
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = sub_word((t << 8) | (t >> 24)) ^ (rcon << 24);
            rcon = gf_mul2((uint8_t)rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = sub_word(t);
        }
        w[i] = w[i - nk] ^ t;
    }
    ctx->nrounds = nr;
    return nr;
}

/* ------------------------------------------------------------------------- */
/* Forward cipher: base/rijndael.c:852-959                                    */

void ao_encrypt_block(const ao_ctx *ctx, const uint8_t in[16], uint8_t out[16])
{
    const uint32_t *rk = ctx->rk;
    const int nr = ctx->nrounds;
    uint32_t s[4], t[4];
    for (int i = 0; i < 4; i++)
        s[i] = load_be32(in + 4 * i) ^ rk[i];
    /* one full round per iteration, columns written out (same arithmetic as the
       indexed form t[i] = Te0[s_i] ^ Te1[s_i+1] ^ Te2[s_i+2] ^ Te3[s_i+3] ^ rk) */
#define AO_COL(i0, i1, i2, i3, k)                                                            \
    (g_te[0][s[i0] >> 24] ^ g_te[1][(s[i1] >> 16) & 0xff] ^ g_te[2][(s[i2] >> 8) & 0xff] ^ \
     g_te[3][s[i3] & 0xff] ^ rk[k])
    for (int r = 1; r < nr; r++) {
        t[0] = AO_COL(0, 1, 2, 3, 4 * r);
        t[1] = AO_COL(1, 2, 3, 0, 4 * r + 1);
        t[2] = AO_COL(2, 3, 0, 1, 4 * r + 2);
        t[3] = AO_COL(3, 0, 1, 2, 4 * r + 3);
        s[0] = t[0]; s[1] = t[1]; s[2] = t[2]; s[3] = t[3];
    }
#undef AO_COL
    for (int i = 0; i < 4; i++) {
        uint32_t v = ((uint32_t)g_sbox[s[i] >> 24] << 24) |
                     ((uint32_t)g_sbox[(s[(i + 1) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t)g_sbox[(s[(i + 2) & 3] >> 8) & 0xff] << 8) |
                     (uint32_t)g_sbox[s[(i + 3) & 3] & 0xff];
        store_be32(out + 4 * i, v ^ rk[4 * nr + i]);
    }
}

/* ------------------------------------------------------------------------- */
/* Decryption key schedule: base/rijndael.c:805-850 -- the encryption schedule with
   the round-key order reversed and InvMixColumns applied to every round key but the
   first and the last (InvMixColumns(w) = Td0[S[b0]] ^ Td1[S[b1]] ^ Td2[S[b2]] ^ Td3[S[b3]]) */

int ao_setup_decrypt(ao_ctx *ctx, const uint8_t *key, size_t keylen)
{
    if (!ao_setup_encrypt(ctx, key, keylen))
        return 0;
    const int nr = ctx->nrounds;
    uint32_t *rk = ctx->rk;
    for (int i = 0, j = 4 * nr; i < j; i += 4, j -= 4)
        for (int k = 0; k < 4; k++) {
            uint32_t t = rk[i + k];
            rk[i + k] = rk[j + k];
            rk[j + k] = t;
        }
    for (int r = 1; r < nr; r++)
        for (int k = 0; k < 4; k++) {
            uint32_t w = rk[4 * r + k];
            rk[4 * r + k] = g_td[0][g_sbox[w >> 24]] ^ g_td[1][g_sbox[(w >> 16) & 0xff]] ^
                            g_td[2][g_sbox[(w >> 8) & 0xff]] ^ g_td[3][g_sbox[w & 0xff]];
        }
    return nr;
}

/* Inverse cipher: base/rijndael.c:961-1068 (equivalent inverse cipher, FIPS-197 5.3.5):
   column c takes rows 0..3 from state columns c, c-1, c-2, c-3. */
void ao_decrypt_block(const ao_ctx *ctx, const uint8_t in[16], uint8_t out[16])
{
    const uint32_t *rk = ctx->rk;
    const int nr = ctx->nrounds;
    uint32_t s[4], t[4];
    for (int i = 0; i < 4; i++)
        s[i] = load_be32(in + 4 * i) ^ rk[i];
    for (int r = 1; r < nr; r++) {
        for (int i = 0; i < 4; i++)
            t[i] = g_td[0][s[i] >> 24] ^ g_td[1][(s[(i + 3) & 3] >> 16) & 0xff] ^
                   g_td[2][(s[(i + 2) & 3] >> 8) & 0xff] ^ g_td[3][s[(i + 1) & 3] & 0xff] ^ rk[4 * r + i];
        memcpy(s, t, sizeof s);
    }
    for (int i = 0; i < 4; i++) {
        uint32_t v = ((uint32_t)g_isbox[s[i] >> 24] << 24) |
                     ((uint32_t)g_isbox[(s[(i + 3) & 3] >> 16) & 0xff] << 16) |
                     ((uint32_t)g_isbox[(s[(i + 2) & 3] >> 8) & 0xff] << 8) |
                     (uint32_t)g_isbox[s[(i + 1) & 3] & 0xff];
        store_be32(out + 4 * i, v ^ rk[4 * nr + i]);
    }
}

/* CBC: base/rijndael.c:1070-1153.  Encrypt: a partial last block is the plaintext
   zero-padded to 16 bytes (out[i] = iv[i] for i >= len, i.e. 0 ^ iv), so 16 bytes are
   written; ivec := the last ciphertext block.  Decrypt: the last (partial) block is
   deciphered from 16 input bytes but only `len` bytes are written; ivec := the last
   16 input bytes. */
void ao_cbc_encrypt(const ao_ctx *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16])
{
    uint8_t iv[16], blk[16];
    memcpy(iv, ivec, 16);
    for (size_t off = 0; off < len; off += 16) {
        size_t n = len - off < 16 ? len - off : 16;
        for (size_t i = 0; i < 16; i++)
            blk[i] = (uint8_t)((i < n ? in[off + i] : 0) ^ iv[i]);
        ao_encrypt_block(ctx, blk, out + off);
        memcpy(iv, out + off, 16);
    }
    memcpy(ivec, iv, 16);
}

void ao_cbc_decrypt(const ao_ctx *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16])
{
    uint8_t iv[16], c[16], p[16];
    memcpy(iv, ivec, 16);
    for (size_t off = 0; off < len; off += 16) {
        size_t n = len - off < 16 ? len - off : 16;
        memcpy(c, in + off, 16); /* whole block: the cipher buffer is a multiple of 16 */
        ao_decrypt_block(ctx, c, p);
        for (size_t i = 0; i < n; i++)
            out[off + i] = (uint8_t)(p[i] ^ iv[i]);
        memcpy(iv, c, 16);
    }
    memcpy(ivec, iv, 16);
}

/* OFB: base/rijndael.c:1155-1169 -- keystream ivec := E(ivec) at n == 0, never fed back
   from the data. */
void ao_ofb(const ao_ctx *ctx, const uint8_t *in, uint8_t *out, size_t len, uint8_t ivec[16], size_t *num)
{
    size_t n = *num;
    for (size_t k = 0; k < len; k++) {
        if (n == 0)
            ao_encrypt_block(ctx, ivec, ivec);
        out[k] = (uint8_t)(in[k] ^ ivec[n]);
        n = (n + 1) & 15;
    }
    *num = n;
}

/* ------------------------------------------------------------------------- */
/* CFB-128: base/rijndael.c:1171-1201                                         */

void ao_cfb(const ao_ctx *ctx, int encrypt, const uint8_t *in, uint8_t *out, size_t len,
            uint8_t ivec[16], size_t *num)
{
    size_t n = *num;
    for (size_t k = 0; k < len; k++) {
        if (n == 0)
            ao_encrypt_block(ctx, ivec, ivec); /* keystream block = E(previous ciphertext) */
        uint8_t c = in[k];
        uint8_t o = (uint8_t)(c ^ ivec[n]);
        out[k] = o;
        ivec[n] = encrypt ? o : c; /* feedback is always the ciphertext byte (:1182, :1195) */
        n = (n + 1) & 15;
    }
    *num = n;
}

/* ------------------------------------------------------------------------- */
/* Encryptor semantics: core/Encryptor.cpp                                    */

void ao_package_crypt(const uint8_t *key, size_t keylen, const uint8_t iv[16], int encrypt,
                      const uint8_t *src, uint8_t *dst, size_t len)
{
    ao_ctx ctx;
    uint8_t ivec[16];
    size_t pos = 0;
    memcpy(ivec, iv, 16);                 /* :12, :24 -- the connection IV is never advanced */
    ao_setup_encrypt(&ctx, key, keylen);  /* :17, :29 -- fresh schedule per call */
    ao_cfb(&ctx, encrypt, src, dst, len, ivec, &pos);
}

size_t ao_package_encrypt_frame(const uint8_t *key, size_t keylen, const uint8_t iv[16],
                                const uint8_t *src, size_t len, uint8_t *dst)
{
    uint32_t l = (uint32_t)len;           /* :47 htole32(len) */
    dst[0] = (uint8_t)l; dst[1] = (uint8_t)(l >> 8); dst[2] = (uint8_t)(l >> 16); dst[3] = (uint8_t)(l >> 24);
    ao_package_crypt(key, keylen, iv, 1, src, dst + 4, len);
    return len + 4;
}

void ao_stream_init(ao_stream *s, const uint8_t *key, size_t keylen, const uint8_t iv[16])
{
    ao_setup_encrypt(&s->ctx, key, keylen); /* core/Encryptor.h:53 */
    memcpy(s->iv, iv, 16);
    s->pos = 0;
}

void ao_stream_crypt(ao_stream *s, int encrypt, const uint8_t *src, uint8_t *dst, size_t len)
{
    ao_cfb(&s->ctx, encrypt, src, dst, len, s->iv, &s->pos); /* core/Encryptor.cpp:53-70 */
}

/* ------------------------------------------------------------------------- */
/* Batches (pthread fan-out over contiguous packet ranges)                   */

typedef struct {
    int encrypt, stream;
    const uint8_t *in;
    uint8_t *out;
    uint32_t begin, end;
    uint64_t stride;
    uint32_t uniform_len;
    const uint64_t *in_off, *out_off;
    const uint32_t *len, *key_slot;
    const uint8_t *keys;
    size_t keylen;
    const uint8_t *ivs;
    uint8_t *iv_state;
    uint32_t *pos_state;
} batch_job;

static void *batch_worker(void *arg)
{
    const batch_job *j = (const batch_job *)arg;
    for (uint32_t i = j->begin; i < j->end; i++) {
        uint64_t io = j->in_off ? j->in_off[i] : (uint64_t)i * j->stride;
        uint64_t oo = j->out_off ? j->out_off[i] : io;
        uint32_t l = j->len ? j->len[i] : j->uniform_len;
        uint32_t ks = j->key_slot ? j->key_slot[i] : 0;
        const uint8_t *key = j->keys + (size_t)ks * j->keylen;
        if (!j->stream) {
            ao_package_crypt(key, j->keylen, j->ivs + 16 * (size_t)ks, j->encrypt, j->in + io, j->out + oo, l);
        } else {
            ao_ctx ctx;
            size_t pos = j->pos_state[i];
            ao_setup_encrypt(&ctx, key, j->keylen);
            ao_cfb(&ctx, j->encrypt, j->in + io, j->out + oo, l, j->iv_state + 16 * (size_t)i, &pos);
            j->pos_state[i] = (uint32_t)pos;
        }
    }
    return NULL;
}

static void run_batch(batch_job *proto, uint32_t count, int threads)
{
    ensure_tables();
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > count) threads = count ? (int)count : 1;
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    batch_job *jobs = (batch_job *)calloc((size_t)threads, sizeof(batch_job));
    for (int t = 0; t < threads; t++) {
        jobs[t] = *proto;
        jobs[t].begin = (uint32_t)((uint64_t)count * t / threads);
        jobs[t].end = (uint32_t)((uint64_t)count * (t + 1) / threads);
        if (t) pthread_create(&tid[t], NULL, batch_worker, &jobs[t]);
    }
    batch_worker(&jobs[0]);
    for (int t = 1; t < threads; t++)
        pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
}

void ao_package_batch(int encrypt, const uint8_t *in, uint8_t *out, uint32_t count,
                      uint64_t stride, uint32_t uniform_len,
                      const uint64_t *in_off, const uint64_t *out_off, const uint32_t *len,
                      const uint32_t *key_slot, const uint8_t *keys, size_t keylen,
                      const uint8_t *ivs, int threads)
{
    batch_job j;
    memset(&j, 0, sizeof j);
    j.encrypt = encrypt; j.in = in; j.out = out; j.stride = stride; j.uniform_len = uniform_len;
    j.in_off = in_off; j.out_off = out_off; j.len = len; j.key_slot = key_slot;
    j.keys = keys; j.keylen = keylen; j.ivs = ivs;
    run_batch(&j, count, threads);
}

void ao_stream_batch(int encrypt, const uint8_t *in, uint8_t *out, uint32_t count,
                     const uint64_t *in_off, const uint64_t *out_off, const uint32_t *len,
                     const uint32_t *key_slot, const uint8_t *keys, size_t keylen,
                     uint8_t *iv_state, uint32_t *pos_state, int threads)
{
    batch_job j;
    memset(&j, 0, sizeof j);
    j.encrypt = encrypt; j.stream = 1; j.in = in; j.out = out;
    j.in_off = in_off; j.out_off = out_off; j.len = len; j.key_slot = key_slot;
    j.keys = keys; j.keylen = keylen; j.iv_state = iv_state; j.pos_state = pos_state;
    run_batch(&j, count, threads);
}

/* ------------------------------------------------------------------------- */
/* Synthetic data (counter-based splitmix64)                                  */

uint64_t ao_synth_word(uint64_t seed, uint64_t i)
{
    uint64_t z = i + seed * 0xD1B54A32D192ED03ULL;
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

typedef struct {
    uint8_t *dst;
    uint64_t begin, end, seed, base;
} synth_job;

static void *synth_worker(void *arg)
{
    const synth_job *j = (const synth_job *)arg;
    for (uint64_t k = j->begin; k < j->end;) {
        uint64_t g = j->base + k;
        uint64_t w = ao_synth_word(j->seed, g >> 3);
        if ((g & 7) == 0 && k + 8 <= j->end) {
            for (int b = 0; b < 8; b++) j->dst[k + b] = (uint8_t)(w >> (8 * b));
            k += 8;
        } else {
            j->dst[k] = (uint8_t)(w >> (8 * (g & 7)));
            k++;
        }
    }
    return NULL;
}

void ao_synth_fill(uint8_t *dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset, int threads)
{
    if (threads < 1) threads = 1;
    pthread_t tid[256];
    synth_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t].dst = dst; jobs[t].seed = seed; jobs[t].base = byte_offset;
        jobs[t].begin = nbytes * (uint64_t)t / (uint64_t)threads;
        jobs[t].end = nbytes * (uint64_t)(t + 1) / (uint64_t)threads;
        if (t) pthread_create(&tid[t], NULL, synth_worker, &jobs[t]);
    }
    synth_worker(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
}

/* ------------------------------------------------------------------------- */

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double ao_time_package_roundtrip(const uint8_t *in, uint8_t *tmp, uint8_t *out, uint32_t count,
                                 uint32_t len, const uint8_t *key, size_t keylen,
                                 const uint8_t iv[16], int threads, int reps)
{
    double t0 = now_s();
    for (int r = 0; r < reps; r++) {
        ao_package_batch(1, in, tmp, count, len, len, NULL, NULL, NULL, NULL, key, keylen, iv, threads);
        ao_package_batch(0, tmp, out, count, len, len, NULL, NULL, NULL, NULL, key, keylen, iv, threads);
    }
    return now_s() - t0;
}

/* ------------------------------------------------------------------------- */
/* Receive-side framing                                                        */

static uint32_t le32_at(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

void ao_scan_package(const uint8_t *seg, uint64_t len, uint32_t max_len, uint32_t max_frames, uint64_t *off,
                     uint32_t *flen, ao_scan *res)
{
    uint64_t pos = 0;
    uint32_t f = 0, status = AO_SCAN_OK;
    while (len - pos >= 4) {                      /* _packageLen read complete (:62-71) */
        uint32_t n = le32_at(seg + pos);          /* le32toh(_packageLen) (:76) */
        if (n > max_len) { status = AO_SCAN_TOO_LARGE; break; }   /* (:77-81) */
        if (len - pos - 4 < n) break;             /* body still incomplete (:62-71 again) */
        if (f == max_frames) { status = AO_SCAN_FULL; break; }
        off[f] = pos + 4;
        flen[f] = n;
        f++;
        pos += 4 + (uint64_t)n;
    }
    res->frames = f;
    res->status = status;
    res->consumed = pos;
}

void ao_scan_stream(const uint8_t *plain, uint64_t len, uint32_t max_len, uint32_t max_frames, uint64_t *off,
                    uint32_t *flen, ao_scan *res)
{
    uint64_t pos = 0;
    uint32_t f = 0, status = AO_SCAN_OK;
    while (len - pos >= 12) {                     /* 12 header bytes received and decrypted (:87-89) */
        const uint8_t *h = plain + pos;
        uint32_t mtype, ss, psize, body;
        int64_t length;
        if (memcmp(h, "FPNN", 4) != 0) { status = AO_SCAN_BAD_MAGIC; break; }  /* isTCP (:11) */
        mtype = h[6];                             /* Header{magic, version, flag, mtype, ss, psize} */
        ss = h[7];
        psize = le32_at(h + 8);
        if (mtype == 1) body = psize + ss + 4u;   /* FP_MT_TWOWAY (FPMessage.cpp:31-34) */
        else if (mtype == 2) body = psize + 4u;   /* FP_MT_ANSWER (:35-37) */
        else if (mtype == 0) body = psize + ss;   /* FP_MT_ONEWAY (:38-40) */
        else { status = AO_SCAN_BAD_MTYPE; break; }  /* throws FpnnProtoError (:41-42) */
        /* remainDataLen (:12): (int)(sizeof(Header) + BodyLen) - _curr, _curr == 12 */
        length = (int64_t)(int32_t)(uint32_t)(12u + body) - 12;
        if (length <= 0) { status = AO_SCAN_BAD_LENGTH; break; }          /* (:92, :106-110) */
        if (12 + length > (int64_t)max_len) { status = AO_SCAN_TOO_LARGE; break; }  /* (:94-98) */
        if (len - pos < 12 + (uint64_t)length) break;   /* body still incomplete */
        if (f == max_frames) { status = AO_SCAN_FULL; break; }
        off[f] = pos;
        flen[f] = (uint32_t)(12 + length);
        f++;
        pos += 12 + (uint64_t)length;
    }
    res->frames = f;
    res->status = status;
    res->consumed = pos;
}
