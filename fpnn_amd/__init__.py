"""fpnn_amd -- MI355X-native AES-CFB packet encryption for FPNN.

A drop-in for FPNN's link-encryption hot path (base/rijndael.c driven by
core/Encryptor.{h,cpp}): hand-written gfx950 HIP kernels behind the C-ABI in
include/fpnn_aes.h, the source-compatible fpnn::Encryptor classes in
include/Encryptor.h, and this thin Python host layer.
"""
from ._lib import (LIB_PATH, FpnnAesError, Schedule, build, check, lib, OK, ERR_ARG, ERR_HIP, ERR_KEYLEN, ERR_NODEV,
                   ERR_RANGE, F_WIRE_PREFIX, K_DECRYPT, K_ENCRYPT, K_HOST)
from .engine import (Engine, KeySet, PackageEncryptor, StreamEncryptor, device_count, host_is_mapped, host_register,
                     host_unregister, package_host_multi, setup_decrypt, setup_encrypt, stream_host_multi)

__all__ = [
    "LIB_PATH", "FpnnAesError", "Schedule", "build", "check", "lib", "Engine", "KeySet", "PackageEncryptor",
    "StreamEncryptor", "device_count", "setup_decrypt", "setup_encrypt", "OK", "ERR_ARG", "ERR_HIP", "ERR_KEYLEN", "ERR_NODEV",
    "ERR_RANGE", "F_WIRE_PREFIX", "K_DECRYPT", "K_ENCRYPT", "K_HOST", "host_register", "host_unregister",
    "host_is_mapped", "package_host_multi",
]


def version() -> str:
    return lib.fpnn_aes_version().decode()
