// rijndael_link.cpp -- calls every function base/rijndael.h declares, through
// include/rijndael.h, linked against libfpnn_aes.so with no rijndael.o
// (tests/test_abi.py::test_rijndael_surface_links_without_reference_object checks with nm
// that each rijndael_* symbol is undefined here and defined by libfpnn_aes.so).
// Run on a GPU box it prints FIPS-197 / SP 800-38A results for tests/test_gpu_modes.py.
#include <stdio.h>
#include <string.h>

#include "rijndael.h"

static void hex(const char *name, const uint8_t *p, size_t n) {
    printf("%s ", name);
    for (size_t i = 0; i < n; i++) printf("%02x", p[i]);
    printf("\n");
}

int main() {
    uint8_t key[32], pt[16], ct[16], back[16], iv[16], buf[64], out[64];
    for (int i = 0; i < 32; i++) key[i] = (uint8_t)i;
    for (int i = 0; i < 16; i++) pt[i] = (uint8_t)(0x11 * i);
    rijndael_context enc, dec;
    if (!rijndael_setup_encrypt(&enc, key, 32) || !rijndael_setup_decrypt(&dec, key, 32)) return 2;
    rijndael_encrypt(&enc, pt, ct);  // FIPS-197 C.3: 8ea2b7ca516745bfeafc49904b496089
    rijndael_decrypt(&dec, ct, back);
    hex("ecb_encrypt", ct, 16);
    hex("ecb_decrypt", back, 16);
    for (int i = 0; i < 64; i++) buf[i] = (uint8_t)(3 * i + 1);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)i;
    rijndael_cbc_encrypt(&enc, buf, out, 50, iv);  // 4 blocks out, the last zero-padded
    hex("cbc_encrypt", out, 64);
    hex("cbc_iv", iv, 16);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)i;
    rijndael_cbc_decrypt(&dec, out, out, 50, iv);  // in place
    hex("cbc_decrypt", out, 50);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)i;
    size_t num = 0;
    rijndael_ofb_encrypt(&enc, buf, out, 37, iv, &num);
    hex("ofb", out, 37);
    printf("ofb_num %zu\n", num);
    for (int i = 0; i < 16; i++) iv[i] = (uint8_t)i;
    num = 0;
    rijndael_cfb_encrypt(&enc, true, buf, out, 37, iv, &num);
    hex("cfb", out, 37);
    return memcmp(back, pt, 16) == 0 ? 0 : 1;
}
