"""Loader for libfpnn_aes.so (the C-ABI of include/fpnn_aes.h).

torch is imported first so that its bundled HIP runtime (same SONAME
libamdhip64.so.7) is the one the library binds to: tensors allocated by torch and
kernels launched by the library then share one runtime, one device context and
one stream namespace.

There is no fallback: if the shared library is missing or cannot be loaded the
import raises, and the C-ABI itself returns FPNN_AES_ERR_NODEV on a machine
without a gfx950 GPU.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# FPNN_AES_LIB: another build of the library (A/B of two builds in one session; tools only)
LIB_PATH = os.environ.get("FPNN_AES_LIB") or os.path.join(PKG_DIR, "libfpnn_aes.so")
CSRC = os.path.join(PKG_DIR, "csrc")

OK = 0
ERR_KEYLEN = -1
ERR_ARG = -2
ERR_RANGE = -3
ERR_HIP = -4
ERR_NODEV = -5
ERR_DEVICE = -6

F_WIRE_PREFIX = 0x1
SCAN_OK, SCAN_FULL, SCAN_TOO_LARGE, SCAN_BAD_MAGIC, SCAN_BAD_MTYPE, SCAN_BAD_LENGTH = range(6)
MAX_RECV_PACKAGE_LENGTH = 8 * 1024 * 1024  # FPNN_DEFAULT_MAX_PACKAGE_LEN, core/Config.h:14
K_DECRYPT = 0
K_ENCRYPT = 1
K_HOST = 2  # last_kernel only: "host_mapped" / "host_staged"


class FpnnAesError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(what)


class Schedule(C.Structure):
    """fpnn_aes_schedule == rijndael_context (base/rijndael.h:13-16)."""

    _fields_ = [("nrounds", C.c_int), ("rk", C.c_uint32 * 60)]


class HostFrame(C.Structure):
    """fpnn_aes_host_frame (include/fpnn_aes.h)."""

    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("len", C.c_uint32), ("key_slot", C.c_uint32)]


class BatchDesc(C.Structure):
    """fpnn_aes_batch (include/fpnn_aes.h)."""

    _fields_ = [
        ("in_", C.c_void_p),
        ("out", C.c_void_p),
        ("count", C.c_uint32),
        ("uniform_len", C.c_uint32),
        ("stride", C.c_uint64),
        ("in_off", C.c_void_p),
        ("out_off", C.c_void_p),
        ("len", C.c_void_p),
        ("key_slot", C.c_void_p),
        ("keys", C.c_void_p),
        ("flags", C.c_uint32),
        ("max_len", C.c_uint32),
    ]


_vp = C.c_void_p
_u8p = C.POINTER(C.c_uint8)

# name -> (restype, argtypes); every function declared in include/fpnn_aes.h
SIGNATURES = {
    "fpnn_aes_strerror": (C.c_char_p, [C.c_int]),
    "fpnn_aes_last_error": (C.c_char_p, []),
    "fpnn_aes_version": (C.c_char_p, []),
    "fpnn_aes_setup_encrypt": (C.c_int, [C.POINTER(Schedule), _u8p, C.c_size_t]),
    "fpnn_aes_setup_decrypt": (C.c_int, [C.POINTER(Schedule), _u8p, C.c_size_t]),
    "fpnn_aes_ecb_host": (C.c_int, [_vp, C.POINTER(Schedule), C.c_int, _vp, _vp, C.c_size_t]),
    "fpnn_aes_cbc_host": (C.c_int, [_vp, C.POINTER(Schedule), C.c_int, _vp, _vp, C.c_size_t, _u8p]),
    "fpnn_aes_ofb_host": (C.c_int, [_vp, C.POINTER(Schedule), _vp, _vp, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]),
    "fpnn_aes_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "fpnn_aes_engine_create": (C.c_int, [C.c_int, _vp, C.POINTER(_vp)]),
    "fpnn_aes_engine_destroy": (C.c_int, [_vp]),
    "fpnn_aes_engine_sync": (C.c_int, [_vp]),
    "fpnn_aes_engine_stream": (_vp, [_vp]),
    "fpnn_aes_thread_engine_device": (C.c_int, [C.c_uint32, C.c_int]),
    "fpnn_aes_max_thread_engines": (C.c_int, [C.c_int]),
    "fpnn_aes_device_alloc": (C.c_int, [_vp, C.c_size_t, C.POINTER(_vp)]),
    "fpnn_aes_device_free": (C.c_int, [_vp, _vp]),
    "fpnn_aes_pinned_alloc": (C.c_int, [_vp, C.c_size_t, C.POINTER(_vp)]),
    "fpnn_aes_pinned_free": (C.c_int, [_vp, _vp]),
    "fpnn_aes_copy_async": (C.c_int, [_vp, _vp, _vp, C.c_size_t]),
    "fpnn_aes_engine_numa": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "fpnn_aes_engine_reserve": (C.c_int, [_vp, C.c_uint64, C.c_uint64]),
    "fpnn_aes_keyset_create": (C.c_int, [_vp, C.c_uint32, C.c_size_t, _vp, _vp, C.c_int, C.POINTER(_vp)]),
    "fpnn_aes_keyset_from_schedules": (C.c_int, [_vp, C.c_uint32, C.POINTER(Schedule), _vp, C.POINTER(_vp)]),
    "fpnn_aes_keyset_destroy": (C.c_int, [_vp]),
    "fpnn_aes_keyset_reserve": (C.c_int, [_vp, C.c_uint32, C.c_int, C.POINTER(_vp)]),
    "fpnn_aes_keyset_set": (C.c_int, [_vp, C.c_uint32, C.c_uint32, C.POINTER(Schedule), _vp]),
    "fpnn_aes_keyset_count": (C.c_uint32, [_vp]),
    "fpnn_aes_keyset_nrounds": (C.c_int, [_vp]),
    "fpnn_aes_keyset_get_schedule": (C.c_int, [_vp, C.c_uint32, C.POINTER(Schedule)]),
    "fpnn_aes_package_encrypt": (C.c_int, [_vp, C.POINTER(BatchDesc)]),
    "fpnn_aes_package_decrypt": (C.c_int, [_vp, C.POINTER(BatchDesc)]),
    "fpnn_aes_stream_encrypt": (C.c_int, [_vp, C.POINTER(BatchDesc), _vp, _vp]),
    "fpnn_aes_stream_decrypt": (C.c_int, [_vp, C.POINTER(BatchDesc), _vp, _vp]),
    "fpnn_aes_cfb_host": (C.c_int, [_vp, C.POINTER(Schedule), C.c_int, _vp, _vp, C.c_size_t, _u8p,
                                    C.POINTER(C.c_size_t)]),
    "fpnn_aes_package_host": (C.c_int, [_vp, C.c_int, C.POINTER(HostFrame), C.c_uint32, _vp, C.c_uint32]),
    "fpnn_aes_stream_host": (C.c_int, [_vp, C.c_int, C.POINTER(HostFrame), C.c_uint32, _vp, _vp, _vp]),
    "fpnn_aes_package_host_multi": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.POINTER(HostFrame), C.c_uint32,
                                              C.c_uint32]),
    "fpnn_aes_stream_host_multi": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.POINTER(HostFrame), C.c_uint32, _vp,
                                             _vp]),
    "fpnn_aes_host_register": (C.c_int, [_vp, C.c_size_t]),
    "fpnn_aes_host_unregister": (C.c_int, [_vp]),
    "fpnn_aes_host_is_mapped": (C.c_int, [_vp, C.c_size_t]),
    "fpnn_aes_package_recv": (C.c_int, [_vp, C.POINTER(BatchDesc), C.c_uint32, C.c_uint32, _vp, _vp, _vp]),
    "fpnn_aes_stream_recv": (C.c_int, [_vp, C.POINTER(BatchDesc), _vp, _vp, _vp, C.c_uint32, C.c_uint32, _vp, _vp,
                                       _vp]),
    "fpnn_aes_fill_synthetic": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64]),
    "fpnn_aes_engine_set_timing": (C.c_int, [_vp, C.c_int]),
    "fpnn_aes_engine_kernel_stats": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    "fpnn_aes_engine_reset_stats": (C.c_int, [_vp]),
    "fpnn_aes_engine_last_kernel": (C.c_char_p, [_vp, C.c_int]),
    # fpnn_ecdh.h (include/fpnn_ecdh.h)
    "fpnn_ecdh_curve": (C.c_int, [C.c_char_p]),
    "fpnn_ecdh_secret_len": (C.c_int, [C.c_int]),
    "fpnn_ecdh_private_len": (C.c_int, [C.c_int]),
    "fpnn_ecdh_curve_name": (C.c_char_p, [C.c_int]),
    "fpnn_ecdh_random_private": (C.c_int, [C.c_int, C.c_char_p]),
    "fpnn_ecdh_calc_keys": (C.c_int, [_vp, C.c_int, C.c_char_p, _vp, C.c_uint32, C.c_int, _vp, _vp, _vp]),
    "fpnn_ecdh_calc_keys_client": (C.c_int, [_vp, C.c_int, _vp, C.c_char_p, C.c_uint32, C.c_int, _vp, _vp, _vp]),
    "fpnn_ecdh_public_keys": (C.c_int, [_vp, C.c_int, _vp, C.c_uint32, _vp, _vp]),
    "fpnn_ecdh_keyset": (C.c_int, [_vp, C.c_int, C.c_char_p, _vp, C.c_uint32, C.c_int, _vp, C.POINTER(_vp)]),
    "fpnn_ecdh_calc_keys_host": (C.c_int, [_vp, C.c_int, C.c_char_p, C.c_char_p, C.c_uint32, C.c_int, _vp, _vp,
                                           _vp]),
    "fpnn_ecdh_calc_key_host": (C.c_int, [_vp, C.c_char_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_int,
                                          _vp, _vp]),
    "fpnn_ecdh_public_key_host": (C.c_int, [_vp, C.c_int, C.c_char_p, _vp]),
    # rijndael.h (include/rijndael.h)
    "rijndael_setup_encrypt": (C.c_bool, [C.POINTER(Schedule), _u8p, C.c_size_t]),
    "rijndael_setup_decrypt": (C.c_bool, [C.POINTER(Schedule), _u8p, C.c_size_t]),
    "rijndael_encrypt": (None, [C.POINTER(Schedule), _vp, _vp]),
    "rijndael_decrypt": (None, [C.POINTER(Schedule), _vp, _vp]),
    "rijndael_cbc_encrypt": (None, [C.POINTER(Schedule), _vp, _vp, C.c_size_t, _u8p]),
    "rijndael_cbc_decrypt": (None, [C.POINTER(Schedule), _vp, _vp, C.c_size_t, _u8p]),
    "rijndael_ofb_encrypt": (None, [C.POINTER(Schedule), _vp, _vp, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]),
    "rijndael_cfb_encrypt": (None, [C.POINTER(Schedule), C.c_bool, _vp, _vp, C.c_size_t, _u8p,
                                    C.POINTER(C.c_size_t)]),
}


def build(force: bool = False) -> str:
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        jobs = str(min(8, os.cpu_count() or 1))
        subprocess.run(["make", "-C", CSRC, "-j", jobs], check=True)
    return LIB_PATH


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {CSRC}` or __graft_entry__.build(). "
            "fpnn_amd has no CPU fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status: int, what: str = "") -> None:
    if status != OK:
        detail = lib.fpnn_aes_last_error().decode(errors="replace")
        msg = lib.fpnn_aes_strerror(status).decode()
        raise FpnnAesError(status, f"{what}: {msg}" + (f" ({detail})" if detail else ""))
