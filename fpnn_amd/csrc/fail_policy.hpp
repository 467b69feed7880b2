// fail_policy.hpp -- what the drop-in classes do when the GPU fails under a caller that has
// no error path.  Internal to the front library; not installed.
//
// The reference Encryptor cannot fail: its methods return void (core/Encryptor.cpp:10-70),
// and FPNN's callers do not expect an exception.  One that escaped
//   * EncryptedPackageReceiver::fetch would leave at :110, before its try (leaking `buf`,
//     core/EncryptedPackageReceiver.cpp:108-124), then TCPServerIOWorker::read with the
//     receive token still held (core/ServerIOWorker.cpp:153-182), and the IO pool swallows
//     it (base/ParamTemplateThreadPool.h:372-375);
//   * SendBuffer::realSend would lose the send token the same way;
// so the connection would never read, send or close again, and nothing would be logged.
// The default is therefore fail-stop, as rijndael_cfb_encrypt already does: the message
// goes to stderr and the process aborts (a supervisor restarts the server; every peer sees
// its connections close).  FPNN_AES_ON_ERROR=throw raises fpnn::EncryptorError instead, for
// callers that catch it and close the connection themselves.
#pragma once

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../../include/Encryptor.h"

namespace fpnn_aes {

enum class OnError { Abort, Throw };

inline OnError on_error_policy() {
    static const OnError p = [] {
        const char *v = getenv("FPNN_AES_ON_ERROR");
        return (v && strcmp(v, "throw") == 0) ? OnError::Throw : OnError::Abort;
    }();
    return p;
}

// A device failure on a data path of the C++ classes: abort (default) or throw.
[[noreturn]] inline void device_failure(const std::string &what) {
    if (on_error_policy() == OnError::Throw) throw fpnn::EncryptorError(what);
    fprintf(stderr, "fpnn_aes: %s -- aborting (FPNN_AES_ON_ERROR=abort; =throw raises fpnn::EncryptorError)\n",
            what.c_str());
    fflush(stderr);
    abort();
}

}  // namespace fpnn_aes
