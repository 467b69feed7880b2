"""ctypes bindings for the parity checkers -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  Two interchangeable back ends expose the same Python surface:

* ``Oracle("port")``      -> oracle/liboracle.so, the clean-room C restatement
  (oracle/aes_oracle.c) of base/rijndael.c + core/Encryptor.cpp;
* ``Oracle("reference")`` -> oracle/_ref/libfpnn_ref.so, the reference's own
  sources compiled by oracle/Makefile (present wherever it was built; it travels
  to the GPU box as a built artefact, the reference sources do not).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libfpnn_ref.so")

_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


class Ctx(C.Structure):
    """rijndael_context / ao_ctx layout (base/rijndael.h:13-16)."""

    _fields_ = [("nrounds", C.c_int), ("rk", C.c_uint32 * 60)]


def _ptr(a, t=_u8p):
    if a is None:
        return None
    return a.ctypes.data_as(t)


def _bytes_ptr(b: bytes):
    return C.cast(C.c_char_p(b), _u8p)


def build_port() -> str:
    if not os.path.exists(PORT_LIB):
        subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True, capture_output=True)
    return PORT_LIB


def ref_available() -> bool:
    return os.path.exists(REF_LIB)


class Oracle:
    """Checker facade; ``kind`` is "port" (restatement) or "reference" (compiled ref)."""

    def __init__(self, kind: str = "port"):
        self.kind = kind
        if kind == "port":
            lib = C.CDLL(build_port())
            p = "ao_"
            self._setup = lib.ao_setup_encrypt
            self._block = lib.ao_encrypt_block
            self._cfb = lib.ao_cfb
            self._pkg = lib.ao_package_crypt
            self._frame = lib.ao_package_encrypt_frame
            self._pbatch = lib.ao_package_batch
            self._sbatch = lib.ao_stream_batch
            self._time = lib.ao_time_package_roundtrip
        elif kind == "reference":
            if not ref_available():
                raise FileNotFoundError(REF_LIB + " (build with `make -C oracle ref` where /root/reference exists)")
            lib = C.CDLL(REF_LIB)
            p = "ref_"
            self._setup = lib.ref_setup_encrypt
            self._block = lib.ref_encrypt_block
            self._cfb = lib.ref_cfb
            self._pkg = lib.ref_package_crypt
            self._frame = lib.ref_package_encrypt_frame
            self._pbatch = lib.ref_package_batch
            self._sbatch = lib.ref_stream_batch
            self._time = lib.ref_time_package_roundtrip
            self._snew = lib.ref_stream_new
            self._snew.restype = C.c_void_p
            self._snew.argtypes = [_u8p, C.c_size_t, _u8p]
            self._scrypt = lib.ref_stream_crypt
            self._scrypt.argtypes = [C.c_void_p, C.c_int, _u8p, _u8p, C.c_size_t]
            self._sstr = lib.ref_stream_encrypt_string
            self._sstr.argtypes = [C.c_void_p, _u8p, C.c_size_t, _u8p]
            self._sfree = lib.ref_stream_free
            self._sfree.argtypes = [C.c_void_p]
        else:
            raise ValueError(kind)
        self.lib = lib
        self._prefix = p
        self._setup.argtypes = [C.POINTER(Ctx), _u8p, C.c_size_t]
        self._setup.restype = C.c_int
        self._block.argtypes = [C.POINTER(Ctx), _u8p, _u8p]
        self._cfb.argtypes = [C.POINTER(Ctx), C.c_int, _u8p, _u8p, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]
        self._pkg.argtypes = [_u8p, C.c_size_t, _u8p, C.c_int, _u8p, _u8p, C.c_size_t]
        self._frame.argtypes = [_u8p, C.c_size_t, _u8p, _u8p, C.c_size_t, _u8p]
        self._frame.restype = C.c_size_t
        self._pbatch.argtypes = [C.c_int, _u8p, _u8p, C.c_uint32, C.c_uint64, C.c_uint32,
                                 _u64p, _u64p, _u32p, _u32p, _u8p, C.c_size_t, _u8p, C.c_int]
        self._sbatch.argtypes = [C.c_int, _u8p, _u8p, C.c_uint32, _u64p, _u64p, _u32p, _u32p,
                                 _u8p, C.c_size_t, _u8p, _u32p, C.c_int]
        self._time.argtypes = [_u8p, _u8p, _u8p, C.c_uint32, C.c_uint32, _u8p, C.c_size_t, _u8p,
                               C.c_int, C.c_int]
        self._time.restype = C.c_double

    # -- rijndael.h level -------------------------------------------------------
    def setup_encrypt(self, key: bytes) -> Ctx:
        ctx = Ctx()
        self._setup(C.byref(ctx), _bytes_ptr(key), len(key))
        return ctx

    def encrypt_block(self, key: bytes, block: bytes) -> bytes:
        ctx = self.setup_encrypt(key)
        out = (C.c_uint8 * 16)()
        self._block(C.byref(ctx), _bytes_ptr(block), out)
        return bytes(out)

    # -- the rest of rijndael.h (base/rijndael.c:805-850, 961-1068, 1070-1169) ---------
    def _fn(self, port_name, ref_name):
        return getattr(self.lib, port_name if self.kind == "port" else ref_name)

    def setup_decrypt(self, key: bytes) -> Ctx:
        ctx = Ctx()
        f = self._fn("ao_setup_decrypt", "ref_setup_decrypt")
        f.argtypes = [C.POINTER(Ctx), _u8p, C.c_size_t]
        f(C.byref(ctx), _bytes_ptr(key), len(key))
        return ctx

    def decrypt_block(self, key: bytes, block: bytes) -> bytes:
        ctx = self.setup_decrypt(key)
        f = self._fn("ao_decrypt_block", "ref_decrypt_block")
        f.argtypes = [C.POINTER(Ctx), _u8p, _u8p]
        out = (C.c_uint8 * 16)()
        f(C.byref(ctx), _bytes_ptr(block), out)
        return bytes(out)

    def cbc(self, key: bytes, encrypt: bool, data: bytes, ivec: bytes, length=None):
        """rijndael_cbc_encrypt / _decrypt of `length` bytes (default len(data)); returns
        (out, new_ivec).  Encrypt output is 16*ceil(len/16) bytes; decrypt reads that many
        input bytes (data is zero-extended here) and writes len."""
        ctx = self.setup_encrypt(key) if encrypt else self.setup_decrypt(key)
        n = len(data) if length is None else length
        padded = (n + 15) // 16 * 16
        src = bytes(data[:padded]) + bytes(max(0, padded - len(data)))
        out = (C.c_uint8 * max(1, padded))()
        iv = (C.c_uint8 * 16)(*ivec)
        if self.kind == "port":
            f = self.lib.ao_cbc_encrypt if encrypt else self.lib.ao_cbc_decrypt
            f.argtypes = [C.POINTER(Ctx), _u8p, _u8p, C.c_size_t, _u8p]
            f(C.byref(ctx), _bytes_ptr(src), out, n, iv)
        else:
            f = self.lib.ref_cbc
            f.argtypes = [C.POINTER(Ctx), C.c_int, _u8p, _u8p, C.c_size_t, _u8p]
            f(C.byref(ctx), int(encrypt), _bytes_ptr(src), out, n, iv)
        return bytes(out)[: padded if encrypt else n], bytes(iv)

    def ofb(self, key: bytes, data: bytes, ivec: bytes, num: int = 0):
        """rijndael_ofb_encrypt; returns (out, new_ivec, new_num)."""
        ctx = self.setup_encrypt(key)
        f = self._fn("ao_ofb", "ref_ofb")
        f.argtypes = [C.POINTER(Ctx), _u8p, _u8p, C.c_size_t, _u8p, C.POINTER(C.c_size_t)]
        iv = (C.c_uint8 * 16)(*ivec)
        n = C.c_size_t(num)
        out = (C.c_uint8 * max(1, len(data)))()
        f(C.byref(ctx), _bytes_ptr(data), out, len(data), iv, C.byref(n))
        return bytes(out)[: len(data)], bytes(iv), n.value

    def cfb(self, key: bytes, encrypt: bool, data: bytes, ivec: bytes, num: int = 0):
        """One rijndael_cfb_encrypt call; returns (out, new_ivec, new_num)."""
        ctx = self.setup_encrypt(key)
        iv = (C.c_uint8 * 16)(*ivec)
        n = C.c_size_t(num)
        out = (C.c_uint8 * max(1, len(data)))()
        self._cfb(C.byref(ctx), int(encrypt), _bytes_ptr(data), out, len(data), iv, C.byref(n))
        return bytes(out)[: len(data)], bytes(iv), n.value

    # -- Encryptor level -----------------------------------------------------------
    def package(self, key: bytes, iv: bytes, encrypt: bool, data: bytes) -> bytes:
        out = (C.c_uint8 * max(1, len(data)))()
        self._pkg(_bytes_ptr(key), len(key), _bytes_ptr(iv), int(encrypt), _bytes_ptr(data), out, len(data))
        return bytes(out)[: len(data)]

    def package_frame(self, key: bytes, iv: bytes, data: bytes) -> bytes:
        out = (C.c_uint8 * (len(data) + 4))()
        n = self._frame(_bytes_ptr(key), len(key), _bytes_ptr(iv), _bytes_ptr(data), len(data), out)
        return bytes(out)[:n]

    # -- batches (numpy) -------------------------------------------------------------
    def package_batch(self, encrypt: bool, inp: np.ndarray, out: np.ndarray, count: int, *,
                      stride: int = 0, uniform_len: int = 0, in_off=None, out_off=None, lens=None,
                      key_slot=None, keys: np.ndarray, keylen: int, ivs: np.ndarray, threads: int = 1):
        self._pbatch(int(encrypt), _ptr(inp), _ptr(out), count, stride, uniform_len,
                     _ptr(in_off, _u64p), _ptr(out_off, _u64p), _ptr(lens, _u32p), _ptr(key_slot, _u32p),
                     _ptr(keys), keylen, _ptr(ivs), threads)

    def stream_batch(self, encrypt: bool, inp: np.ndarray, out: np.ndarray, count: int, *,
                     in_off, out_off, lens, key_slot, keys: np.ndarray, keylen: int,
                     iv_state: np.ndarray, pos_state: np.ndarray, threads: int = 1):
        self._sbatch(int(encrypt), _ptr(inp), _ptr(out), count, _ptr(in_off, _u64p), _ptr(out_off, _u64p),
                     _ptr(lens, _u32p), _ptr(key_slot, _u32p), _ptr(keys), keylen, _ptr(iv_state),
                     _ptr(pos_state, _u32p), threads)

    def time_package_roundtrip(self, inp, tmp, out, count, length, key: bytes, iv: bytes, threads, reps=1):
        return self._time(_ptr(inp), _ptr(tmp), _ptr(out), count, length, _bytes_ptr(key), len(key),
                          _bytes_ptr(iv), threads, reps)


class StreamOracle:
    """StreamEncryptor restated on top of ``Oracle.cfb`` semantics (state carried)."""

    def __init__(self, oracle: Oracle, key: bytes, iv: bytes):
        self.o, self.key, self.iv, self.pos = oracle, key, bytes(iv), 0

    def crypt(self, encrypt: bool, data: bytes) -> bytes:
        out, self.iv, self.pos = self.o.cfb(self.key, encrypt, data, self.iv, self.pos)
        return out


# -- synthetic data (same generator as fpnn_amd's device fill) ----------------------
_port_lib = None


def _plib():
    global _port_lib
    if _port_lib is None:
        _port_lib = C.CDLL(build_port())
        _port_lib.ao_synth_fill.argtypes = [_u8p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int]
        _port_lib.ao_synth_word.argtypes = [C.c_uint64, C.c_uint64]
        _port_lib.ao_synth_word.restype = C.c_uint64
    return _port_lib


def synth_bytes(nbytes: int, seed: int, offset: int = 0, threads: int = 8) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        _plib().ao_synth_fill(_ptr(out), nbytes, seed, offset, threads)
    return out


def synth_word(seed: int, i: int) -> int:
    return int(_plib().ao_synth_word(seed, i))


# -- receive-side framing (restated, see aes_oracle.h) --------------------------------
class _Scan(C.Structure):
    _fields_ = [("frames", C.c_uint32), ("status", C.c_uint32), ("consumed", C.c_uint64)]


SCAN_OK, SCAN_FULL, SCAN_TOO_LARGE, SCAN_BAD_MAGIC, SCAN_BAD_MTYPE, SCAN_BAD_LENGTH = range(6)


def _scan(fn_name, data: bytes, max_len: int, max_frames: int):
    lib = _plib()
    fn = getattr(lib, fn_name)
    fn.argtypes = [C.c_char_p, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64),
                   C.POINTER(C.c_uint32), C.POINTER(_Scan)]
    off = (C.c_uint64 * max(1, max_frames))()
    ln = (C.c_uint32 * max(1, max_frames))()
    res = _Scan()
    fn(data, len(data), max_len, max_frames, off, ln, C.byref(res))
    return [(int(off[i]), int(ln[i])) for i in range(res.frames)], int(res.status), int(res.consumed)


def scan_package(data: bytes, max_len: int, max_frames: int):
    """[(body_offset, n)], status, consumed for [htole32(n)][n] wire frames."""
    return _scan("ao_scan_package", data, max_len, max_frames)


def scan_stream(plain: bytes, max_len: int, max_frames: int):
    """[(offset, message_length)], status, consumed for FPNN messages in stream plaintext."""
    return _scan("ao_scan_stream", plain, max_len, max_frames)
