/* openssl_cfb.c -- TEST / BASELINE INFRASTRUCTURE ONLY (never the product).
 *
 * A stronger CPU comparator than the reference (SURVEY.md 8(d) "optionally also
 * OpenSSL EVP cfb128 (AES-NI)"): FPNN's package mode -- a fresh CFB-128 chain per
 * packet from the connection IV, core/Encryptor.cpp:10-32 -- run through the host's
 * OpenSSL (EVP_aes_{128,192,256}_cfb128, AES-NI).  The survey checked that EVP cfb128
 * equals the reference's rijndael_cfb_encrypt byte for byte; bench.py checks this
 * comparator's output against the GPU's on the sample it times.
 *
 * Build: make -C oracle ossl  ->  oracle/libossl_cfb.so  (-lcrypto)
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

static const EVP_CIPHER *cipher_for(size_t keylen)
{
    return keylen == 16 ? EVP_aes_128_cfb128() : keylen == 24 ? EVP_aes_192_cfb128() : EVP_aes_256_cfb128();
}

typedef struct {
    int enc;
    const uint8_t *in;
    uint8_t *out;
    uint32_t first, last, len;
    const uint8_t *key;
    size_t keylen;
    const uint8_t *iv;
    int rc;
} job;

static void *run(void *arg)
{
    job *j = (job *)arg;
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new(), *tmpl = EVP_CIPHER_CTX_new();
    const EVP_CIPHER *ci = cipher_for(j->keylen);
    j->rc = 0;
    /* key schedule once per thread into a template context (the reference re-expands
       per packet); per packet a copy of the template = the IV reset of package mode.
       Copying measured 1.4x faster than re-initialising the IV through the EVP
       provider on OpenSSL 3.0 at 1 KiB packets. */
    if (!c || !tmpl || EVP_CipherInit_ex(tmpl, ci, NULL, j->key, j->iv, j->enc) != 1) { j->rc = -1; goto done; }
    for (uint32_t i = j->first; i < j->last; i++) {
        int n = 0;
        const uint64_t o = (uint64_t)i * j->len;
        if (EVP_CIPHER_CTX_copy(c, tmpl) != 1 ||
            EVP_CipherUpdate(c, j->out + o, &n, j->in + o, (int)j->len) != 1) { j->rc = -1; break; }
    }
done:
    EVP_CIPHER_CTX_free(c);
    EVP_CIPHER_CTX_free(tmpl);
    return NULL;
}

static int batch(int enc, const uint8_t *in, uint8_t *out, uint32_t count, uint32_t len, const uint8_t *key,
                 size_t keylen, const uint8_t *iv, int threads)
{
    pthread_t th[256];
    job jobs[256];
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job){enc, in, out, (uint32_t)((uint64_t)count * t / threads),
                        (uint32_t)((uint64_t)count * (t + 1) / threads), len, key, keylen, iv, 0};
        pthread_create(&th[t], NULL, run, &jobs[t]);
    }
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        rc |= jobs[t].rc;
    }
    return rc;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* encrypt in -> tmp, decrypt tmp -> out, `reps` times; returns seconds (< 0 on error) */
double ossl_time_package_roundtrip(const uint8_t *in, uint8_t *tmp, uint8_t *out, uint32_t count, uint32_t len,
                                   const uint8_t *key, size_t keylen, const uint8_t iv[16], int threads, int reps)
{
    double t0 = now_s();
    for (int r = 0; r < reps; r++) {
        if (batch(1, in, tmp, count, len, key, keylen, iv, threads) ||
            batch(0, tmp, out, count, len, key, keylen, iv, threads))
            return -1.0;
    }
    return now_s() - t0;
}
