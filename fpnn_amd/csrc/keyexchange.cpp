// keyexchange.cpp -- fpnn::ECCKeyExchange / ECCKeysMaker (include/KeyExchange.h) over the
// GPU ECDH of include/fpnn_ecdh.h.  Mirrors core/KeyExchange.cpp:49-187 check for check;
// the scalar multiplications and hashes run in k_ecdh.hip.
#include <string.h>

#include <string>

#include "../../include/Encryptor.h"
#include "../../include/KeyExchange.h"
#include "../../include/fpnn_ecdh.h"
#include "thread_engine.hpp"

namespace {

// the calling thread's engine, locked while the returned lease lives
fpnn_aes::Lease engine_or_throw() {
    int rc;
    fpnn_aes::Lease lease = fpnn_aes::thread_engine(&rc);
    if (!lease.engine())
        throw fpnn::EncryptorError(std::string("fpnn_aes ECDH: no GPU engine: ") + fpnn_aes_strerror(rc));
    return lease;
}

void throw_if_error(int rc, const char *what) {
    if (rc < 0) {
        std::string m = std::string("fpnn_aes ECDH ") + what + ": " + fpnn_aes_strerror(rc);
        const char *d = fpnn_aes_last_error();
        if (d && *d) m += std::string(" (") + d + ")";
        throw fpnn::EncryptorError(m);
    }
}

const char *curve_name(int curve) { return fpnn_ecdh_curve_name(curve); }

}  // namespace

namespace fpnn {

bool ECCKeyExchange::init(const std::string &curve, const std::string &privateKey) {
    const int cv = fpnn_ecdh_curve(curve.c_str());
    if (cv < 0) return false;  // "Unsupported ECC curve."
    _curve = cv;
    _secertLen = fpnn_ecdh_secret_len(cv);
    if ((int)privateKey.length() != fpnn_ecdh_private_len(cv)) return false;  // "Private length missmatched."
    _privateKey = privateKey;
    return true;
}

bool ECCKeyExchange::calcKey(uint8_t *key, uint8_t *iv, int keylen, const std::string &peerPublicKey) {
    if (_curve < 0) return false;  // "ECC Private Key Config ERROR."
    if ((int)peerPublicKey.length() != _secertLen * 2) return false;
    const int r = fpnn_ecdh_calc_key_host(engine_or_throw().engine(), curve_name(_curve),
                                          reinterpret_cast<const uint8_t *>(_privateKey.data()), _privateKey.size(),
                                          reinterpret_cast<const uint8_t *>(peerPublicKey.data()),
                                          peerPublicKey.size(), keylen, key, iv);
    throw_if_error(r, "calcKey");
    return r == 1;
}

bool ECCKeyExchange::calcKeys(size_t count, const uint8_t *peerPublicKeys, int keylen, uint8_t *keys, uint8_t *ivs,
                              uint8_t *ok) {
    if (_curve < 0 || (keylen != 16 && keylen != 32)) return false;
    if ((int)_privateKey.size() != fpnn_ecdh_private_len(_curve)) {
        memset(ok, 0, count);
        return true;
    }
    const int rc = fpnn_ecdh_calc_keys_host(engine_or_throw().engine(), _curve,
                                            reinterpret_cast<const uint8_t *>(_privateKey.data()), peerPublicKeys,
                                            (uint32_t)count, keylen, keys, ivs, ok);
    throw_if_error(rc, "calcKeys");
    return true;
}

bool ECCKeysMaker::setCurve(const std::string &curve) {
    const int cv = fpnn_ecdh_curve(curve.c_str());
    if (cv < 0) return false;
    _curve = cv;
    _secertLen = fpnn_ecdh_secret_len(cv);
    _publicKey.clear();
    _privateKey.clear();
    return true;
}

std::string ECCKeysMaker::publicKey(bool reGen) {
    if (_curve < 0) return std::string();  // "ECC Private Key Config ERROR."
    if (_publicKey.empty() || reGen) {
        // uECC_make_key (core/micro-ecc/uECC.c:1004-1032): up to 64 draws of a private key
        // whose public key is not the point at infinity
        const fpnn_aes::Lease lease = engine_or_throw();
        fpnn_aes_engine *e = lease.engine();
        uint8_t priv[32], pub[64];
        for (int tries = 0; tries < 64; tries++) {
            if (!fpnn_ecdh_random_private(_curve, priv)) return std::string();  // "Gen public key & private key failed."
            const int r = fpnn_ecdh_public_key_host(e, _curve, priv, pub);
            throw_if_error(r, "publicKey");
            if (r == 1) {
                _publicKey.assign(reinterpret_cast<char *>(pub), _secertLen * 2);
                _privateKey.assign(reinterpret_cast<char *>(priv), _secertLen);
                return _publicKey;
            }
        }
        return std::string();
    }
    return _publicKey;
}

}  // namespace fpnn
