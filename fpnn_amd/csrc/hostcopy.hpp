// hostcopy.hpp -- streaming host copies of the host-frame path (hostcopy.cpp).
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace fpnn_aes {

// dst <- src (non-overlapping), non-temporal stores where that pays (>= 256 bytes, AVX2).
void copy_streaming(uint8_t *dst, const uint8_t *src, size_t n);
// Orders a thread's streaming stores before anything it signals afterwards.
void copy_fence();

}  // namespace fpnn_aes
