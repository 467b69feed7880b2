// KeyExchange.h -- drop-in for the reference's core/KeyExchange.h (ECCKeyExchange /
// ECCKeysMaker, core/KeyExchange.h:25-71), computed by libfpnn_aes.so on the GPU
// (include/fpnn_ecdh.h).  Same class names, members and return values:
//   ECCKeyExchange::init(curve, privateKey)             core/KeyExchange.cpp:49-85
//   ECCKeyExchange::calcKey(key, iv, keylen, peerPub)   core/KeyExchange.cpp:87-127
//   ECCKeysMaker::setCurve / publicKey / calcKey        core/KeyExchange.cpp:130-187
// plus ECCKeyExchange::calcKeys, the batch form a server uses for many accepted
// connections at once.
//
// init() and init(const char* proto) are declared (FPNN's servers call them,
// core/TCPEpollServer.epoll.cpp:126, core/UDPEpollServer.epoll.cpp:84) but defined by
// FPNN itself: they read its Setting and key file and call init(curve, privateKey) --
// keep core/KeyExchange.cpp:10-47.  The curve is held as an index
// instead of a uECC_Curve.
// Failures of the device itself throw fpnn::EncryptorError (Encryptor.h) -- there is no
// CPU fallback.
#ifndef FPNN_AMD_KeyExchange_h
#define FPNN_AMD_KeyExchange_h

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace fpnn {

class ECCKeyExchange  //-- Server using.
{
protected:
    int _secertLen;
    int _curve;  // FPNN_ECDH_* (fpnn_ecdh.h); -1: not initialised
    std::string _privateKey;

public:
    ECCKeyExchange() : _secertLen(0), _curve(-1) {}
    virtual ~ECCKeyExchange() {}

    bool init();                    // defined by FPNN (core/KeyExchange.cpp:10-26)
    bool init(const char *proto);   // defined by FPNN (core/KeyExchange.cpp:28-47)
    bool init(const std::string &curve, const std::string &privateKey);
    /*
        key: OUT. Key buffer length is equal to keylen.
        iv: OUT. iv buffer length is 16 bytes.
        keylen: IN. 16 or  32.
        peerPublicKey: IN.
    */
    bool calcKey(uint8_t *key, uint8_t *iv, int keylen, const std::string &peerPublicKey);
    /* Batch: count peers (host buffer, count * 2*secretLen bytes, each the peer's public
       key as calcKey takes it).  keys: count*keylen, ivs: count*16, ok: count (calcKey's
       return per peer).  Returns false only for a bad keylen / an uninitialised object
       (calcKey's own false for every peer). */
    bool calcKeys(size_t count, const uint8_t *peerPublicKeys, int keylen, uint8_t *keys, uint8_t *ivs,
                  uint8_t *ok);
};

//-- Client using.
class ECCKeysMaker : public ECCKeyExchange {
    std::string _publicKey;
    std::string _peerPublicKey;

public:
    ECCKeysMaker() {}
    void setPeerPublicKey(const std::string &peerPublicKey) { _peerPublicKey = peerPublicKey; }
    bool setCurve(const std::string &curve);
    std::string publicKey(bool reGen = false);

    inline bool calcKey(uint8_t *key, uint8_t *iv, int keylen) {
        return ECCKeyExchange::calcKey(key, iv, keylen, _peerPublicKey);
    }
};

}  // namespace fpnn

#endif
