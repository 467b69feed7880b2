"""Python host layer over the C-ABI (include/fpnn_aes.h).

Mirrors the reference's interface for this path so the parity tests read like the
reference's own usage:

* :func:`setup_encrypt`  -- rijndael_setup_encrypt (base/rijndael.c:712-799)
* :meth:`Engine.cfb`     -- rijndael_cfb_encrypt (base/rijndael.c:1171-1201), host bytes
* :class:`PackageEncryptor` / :class:`StreamEncryptor` -- core/Encryptor.h:32-61
* :meth:`Engine.package_encrypt` / ``package_decrypt`` / ``stream_encrypt`` /
  ``stream_decrypt`` -- the batched device-resident form (the hot path).

Device buffers are torch uint8 tensors on the engine's GPU; torch is used for
memory and streams only, every payload byte is transformed by the HIP kernels.
"""
from __future__ import annotations

import atexit
import ctypes as C
import weakref
from typing import Optional

import numpy as np

import torch

from ._lib import (BatchDesc, FpnnAesError, HostFrame, Schedule, check, lib, F_WIRE_PREFIX, K_DECRYPT, K_ENCRYPT,
                   ERR_KEYLEN, OK)


def _buf(b: bytes):
    return C.cast(C.c_char_p(b), C.POINTER(C.c_uint8))


# Live handles, released (key sets first) at interpreter exit while the HIP runtime
# is still up -- finalizers that run during runtime teardown must not call into HIP.
_live_keysets: "weakref.WeakSet" = weakref.WeakSet()
_live_engines: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _release_all():
    for ks in list(_live_keysets):
        ks.close()
    for e in list(_live_engines):
        e.close()


# numpy mirror of fpnn_aes_host_frame for building large frame lists without a Python loop
HOST_FRAME_DTYPE = np.dtype([("src", np.uint64), ("dst", np.uint64), ("len", np.uint32),
                             ("key_slot", np.uint32)])
assert HOST_FRAME_DTYPE.itemsize == C.sizeof(HostFrame)


def setup_encrypt(key: bytes) -> Schedule:
    """rijndael_setup_encrypt: host key expansion, reference rk[] layout."""
    ctx = Schedule()
    rc = lib.fpnn_aes_setup_encrypt(C.byref(ctx), _buf(key), len(key))
    if rc == ERR_KEYLEN:
        raise FpnnAesError(rc, f"key length {len(key)} (must be 16, 24 or 32)")
    check(rc, "setup_encrypt")
    return ctx


def setup_decrypt(key: bytes) -> Schedule:
    """rijndael_setup_decrypt: host decryption schedule, reference rk[] layout."""
    ctx = Schedule()
    rc = lib.fpnn_aes_setup_decrypt(C.byref(ctx), _buf(key), len(key))
    if rc == ERR_KEYLEN:
        raise FpnnAesError(rc, f"key length {len(key)} (must be 16, 24 or 32)")
    check(rc, "setup_decrypt")
    return ctx


def device_count() -> int:
    n = C.c_int(0)
    rc = lib.fpnn_aes_device_count(C.byref(n))
    return n.value if rc == OK else 0


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("device array expected (torch tensor on a HIP device)")
    if not t.is_contiguous():
        raise ValueError("contiguous tensor expected")
    return C.c_void_p(t.data_ptr())


class Engine:
    """One GPU + one HIP stream (default: torch's current stream on that device)."""

    def __init__(self, device: int = 0, stream: Optional[torch.cuda.Stream] = None):
        self.device = device
        if stream is None:
            stream = torch.cuda.current_stream(device)
        self.torch_stream = stream
        h = C.c_void_p()
        check(lib.fpnn_aes_engine_create(device, C.c_void_p(stream.cuda_stream), C.byref(h)), "engine_create")
        self._h = h
        _live_engines.add(self)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            lib.fpnn_aes_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(lib.fpnn_aes_engine_sync(self._h), "sync")

    def reserve(self, max_segments: int, max_blocks: int):
        check(lib.fpnn_aes_engine_reserve(self._h, max_segments, max_blocks), "reserve")

    # -- timing -----------------------------------------------------------------------
    def set_timing(self, enable: bool):
        check(lib.fpnn_aes_engine_set_timing(self._h, int(enable)), "set_timing")

    def kernel_stats(self, which: int):
        n = C.c_uint64()
        ms = C.c_double()
        check(lib.fpnn_aes_engine_kernel_stats(self._h, which, C.byref(n), C.byref(ms)), "kernel_stats")
        return n.value, ms.value

    def reset_stats(self):
        check(lib.fpnn_aes_engine_reset_stats(self._h), "reset_stats")

    def last_kernel(self, which: int) -> str:
        """Base name of the kernel variant the last call queued for that direction."""
        return lib.fpnn_aes_engine_last_kernel(self._h, which).decode()

    def numa(self) -> dict:
        """The engine's NUMA placement (fpnn_aes_engine_numa): node of its pinned arenas and
        copy threads, the GPU's node from sysfs, CPUs the threads are pinned to, and why."""
        node, dnode, ncpus = C.c_int(), C.c_int(), C.c_int()
        check(lib.fpnn_aes_engine_numa(self._h, C.byref(node), C.byref(dnode), C.byref(ncpus)), "engine_numa")
        return {"node": node.value, "device_node": dnode.value, "ncpus": ncpus.value,
                "why": lib.fpnn_aes_last_error().decode()}

    # -- synthetic data ------------------------------------------------------------------
    def fill_synthetic(self, dst: torch.Tensor, seed: int, byte_offset: int = 0, nbytes: Optional[int] = None):
        n = dst.numel() * dst.element_size() if nbytes is None else nbytes
        check(lib.fpnn_aes_fill_synthetic(self._h, _ptr(dst), n, seed, byte_offset), "fill_synthetic")

    # -- single host call (drop-in for rijndael_cfb_encrypt) ------------------------------
    def cfb(self, ctx: Schedule, encrypt: bool, data: bytes, ivec: bytes, num: int = 0):
        iv = (C.c_uint8 * 16)(*ivec)
        n = C.c_size_t(num)
        out = C.create_string_buffer(max(1, len(data)))
        check(lib.fpnn_aes_cfb_host(self._h, C.byref(ctx), int(encrypt), C.c_char_p(data), out, len(data), iv,
                                    C.byref(n)), "cfb_host")
        return out.raw[: len(data)], bytes(iv), n.value

    # -- the rest of rijndael.h (synchronous, host bytes) ----------------------------------------
    def ecb(self, ctx: Schedule, encrypt: bool, data: bytes) -> bytes:
        """rijndael_encrypt / rijndael_decrypt over len(data)/16 blocks."""
        if len(data) % 16:
            raise ValueError("ECB takes whole 16-byte blocks")
        out = C.create_string_buffer(max(1, len(data)))
        check(lib.fpnn_aes_ecb_host(self._h, C.byref(ctx), int(encrypt), C.c_char_p(data), out, len(data) // 16),
              "ecb_host")
        return out.raw[: len(data)]

    def cbc(self, ctx: Schedule, encrypt: bool, data: bytes, ivec: bytes, length: Optional[int] = None):
        """rijndael_cbc_encrypt / _decrypt; returns (out, new_ivec).  length defaults to
        len(data); decrypt reads 16*ceil(length/16) bytes of data."""
        n = len(data) if length is None else length
        whole = (n + 15) // 16 * 16
        src = bytes(data) + bytes(max(0, whole - len(data)))
        iv = (C.c_uint8 * 16)(*ivec)
        out = C.create_string_buffer(max(1, whole))
        check(lib.fpnn_aes_cbc_host(self._h, C.byref(ctx), int(encrypt), C.c_char_p(src), out, n, iv), "cbc_host")
        return out.raw[: whole if encrypt else n], bytes(iv)

    def ofb(self, ctx: Schedule, data: bytes, ivec: bytes, num: int = 0):
        """rijndael_ofb_encrypt; returns (out, new_ivec, new_num)."""
        iv = (C.c_uint8 * 16)(*ivec)
        n = C.c_size_t(num)
        out = C.create_string_buffer(max(1, len(data)))
        check(lib.fpnn_aes_ofb_host(self._h, C.byref(ctx), C.c_char_p(data), out, len(data), iv, C.byref(n)),
              "ofb_host")
        return out.raw[: len(data)], bytes(iv), n.value

    # -- many frames in host memory (the cross-connection batch path) ----------------------
    def package_host(self, encrypt: bool, frames, keys: "KeySet", wire_prefix: bool = False):
        """frames: sequence of (src, dst, key_slot) with src/dst contiguous uint8 numpy
        arrays in host memory (dst may be src; with wire_prefix dst holds len + 4)."""
        arr = (HostFrame * max(1, len(frames)))()
        for i, (src, dst, slot) in enumerate(frames):
            arr[i].src = src.ctypes.data if src.size else None
            arr[i].dst = dst.ctypes.data if dst.size else None
            arr[i].len = src.size
            arr[i].key_slot = slot
        check(lib.fpnn_aes_package_host(self._h, int(encrypt), arr, len(frames), keys.handle,
                                        F_WIRE_PREFIX if wire_prefix else 0), "package_host")

    def package_host_array(self, encrypt: bool, frames_np, keys: "KeySet", wire_prefix: bool = False):
        """frames_np: numpy structured array with HOST_FRAME_DTYPE (vectorized form)."""
        ptr = C.cast(C.c_void_p(frames_np.ctypes.data), C.POINTER(HostFrame))
        check(lib.fpnn_aes_package_host(self._h, int(encrypt), ptr, len(frames_np), keys.handle,
                                        F_WIRE_PREFIX if wire_prefix else 0), "package_host")

    def stream_host(self, encrypt: bool, frames, keys: "KeySet", iv_state: np.ndarray, pos_state: np.ndarray):
        """Stream-mode host frames.  frames: sequence of (src, dst, stream_slot); a stream's
        frames are processed in sequence order.  iv_state: uint8 [keys.count, 16] and
        pos_state: uint32 [keys.count] host arrays, updated in place."""
        arr = (HostFrame * max(1, len(frames)))()
        for i, (src, dst, slot) in enumerate(frames):
            arr[i].src = src.ctypes.data if src.size else None
            arr[i].dst = dst.ctypes.data if dst.size else None
            arr[i].len = src.size
            arr[i].key_slot = slot
        self._stream_host(encrypt, arr, len(frames), keys, iv_state, pos_state)

    def stream_host_array(self, encrypt: bool, frames_np, keys: "KeySet", iv_state: np.ndarray,
                          pos_state: np.ndarray):
        ptr = C.cast(C.c_void_p(frames_np.ctypes.data), C.POINTER(HostFrame))
        self._stream_host(encrypt, ptr, len(frames_np), keys, iv_state, pos_state)

    def _stream_host(self, encrypt, arr, n, keys, iv_state, pos_state):
        if iv_state.dtype != np.uint8 or pos_state.dtype != np.uint32:
            raise TypeError("iv_state must be uint8, pos_state uint32")
        if iv_state.size < 16 * keys.count or pos_state.size < keys.count:
            raise ValueError("state arrays must hold keys.count streams")
        if not (iv_state.flags.c_contiguous and pos_state.flags.c_contiguous):
            raise ValueError("state arrays must be contiguous")
        check(lib.fpnn_aes_stream_host(self._h, int(encrypt), arr, n, keys.handle,
                                       iv_state.ctypes.data, pos_state.ctypes.data), "stream_host")

    # -- receive side: framing on the device -------------------------------------------------
    @staticmethod
    def _scan_buffers(count, max_frames, device):
        off = torch.empty(count * max_frames, dtype=torch.int64, device=device)
        ln = torch.empty(count * max_frames, dtype=torch.int32, device=device)
        scan = torch.empty(count * 2, dtype=torch.int64, device=device)  # fpnn_aes_frame_scan[count]
        return off, ln, scan

    @staticmethod
    def decode_scan(scan: torch.Tensor):
        """fpnn_aes_frame_scan[count] -> numpy (frames, status, consumed) columns."""
        a = scan.cpu().numpy().view(np.uint32).reshape(-1, 4)
        return a[:, 0].copy(), a[:, 1].copy(), scan.cpu().numpy().reshape(-1, 2)[:, 1].copy()

    def package_recv(self, inp, out, count, keys: "KeySet", max_len: int, max_frames: int, **kw):
        """fpnn_aes_package_recv: returns device tensors (frame_off, frame_len, scan)."""
        d = self._desc(inp, out, count, keys, **kw)
        off, ln, scan = self._scan_buffers(count, max_frames, inp.device)
        check(lib.fpnn_aes_package_recv(self._h, C.byref(d), max_len, max_frames, _ptr(off), _ptr(ln), _ptr(scan)),
              "package_recv")
        return off, ln, scan

    def stream_recv(self, inp, out, count, keys: "KeySet", iv_state, pos_state, max_len: int, max_frames: int,
                    carry: Optional[torch.Tensor] = None, **kw):
        """fpnn_aes_stream_recv: returns device tensors (frame_off, frame_len, scan)."""
        d = self._desc(inp, out, count, keys, **kw)
        off, ln, scan = self._scan_buffers(count, max_frames, inp.device)
        check(lib.fpnn_aes_stream_recv(self._h, C.byref(d), _ptr(iv_state), _ptr(pos_state), _ptr(carry), max_len,
                                       max_frames, _ptr(off), _ptr(ln), _ptr(scan)), "stream_recv")
        return off, ln, scan

    # -- ECDH key derivation (include/fpnn_ecdh.h) -------------------------------------------
    @staticmethod
    def ecdh_curve(name: str) -> int:
        cv = lib.fpnn_ecdh_curve(name.encode())
        if cv < 0:
            raise ValueError(f"unsupported ECC curve {name!r}")
        return cv

    def ecdh_calc_keys(self, curve: str, private_key: bytes, peer_public: torch.Tensor, keylen: int):
        """Server side, many peers (ECCKeyExchange::calcKey per connection) -> device
        tensors (keys [n, keylen], ivs [n, 16], ok [n] uint8).  Queued, no host wait."""
        cv = self.ecdh_curve(curve)
        n = peer_public.numel() // (2 * lib.fpnn_ecdh_secret_len(cv))
        keys = torch.empty((n, keylen), dtype=torch.uint8, device=peer_public.device)
        ivs = torch.empty((n, 16), dtype=torch.uint8, device=peer_public.device)
        ok = torch.empty(n, dtype=torch.uint8, device=peer_public.device)
        check(lib.fpnn_ecdh_calc_keys(self._h, cv, bytes(private_key), _ptr(peer_public), n, keylen, _ptr(keys),
                                      _ptr(ivs), _ptr(ok)), "ecdh_calc_keys")
        return keys, ivs, ok

    def ecdh_calc_keys_client(self, curve: str, private_keys: torch.Tensor, server_public: bytes, keylen: int):
        """Client side (ECCKeysMaker::calcKey) for many clients of one server."""
        cv = self.ecdh_curve(curve)
        n = private_keys.numel() // lib.fpnn_ecdh_private_len(cv)
        keys = torch.empty((n, keylen), dtype=torch.uint8, device=private_keys.device)
        ivs = torch.empty((n, 16), dtype=torch.uint8, device=private_keys.device)
        ok = torch.empty(n, dtype=torch.uint8, device=private_keys.device)
        check(lib.fpnn_ecdh_calc_keys_client(self._h, cv, _ptr(private_keys), bytes(server_public), n, keylen,
                                             _ptr(keys), _ptr(ivs), _ptr(ok)), "ecdh_calc_keys_client")
        return keys, ivs, ok

    def ecdh_public_keys(self, curve: str, private_keys: torch.Tensor):
        """Public keys (x || y) of many private keys -> (public [n, 2*secret_len], ok [n])."""
        cv = self.ecdh_curve(curve)
        n = private_keys.numel() // lib.fpnn_ecdh_private_len(cv)
        pub = torch.empty((n, 2 * lib.fpnn_ecdh_secret_len(cv)), dtype=torch.uint8, device=private_keys.device)
        ok = torch.empty(n, dtype=torch.uint8, device=private_keys.device)
        check(lib.fpnn_ecdh_public_keys(self._h, cv, _ptr(private_keys), n, _ptr(pub), _ptr(ok)),
              "ecdh_public_keys")
        return pub, ok

    def ecdh_keyset(self, curve: str, private_key: bytes, peer_public: torch.Tensor, keylen: int):
        """Derive every connection's (key, iv) and expand them into a KeySet -> (KeySet, ok)."""
        cv = self.ecdh_curve(curve)
        n = peer_public.numel() // (2 * lib.fpnn_ecdh_secret_len(cv))
        ok = torch.empty(n, dtype=torch.uint8, device=peer_public.device)
        h = C.c_void_p()
        check(lib.fpnn_ecdh_keyset(self._h, cv, bytes(private_key), _ptr(peer_public), n, keylen, _ptr(ok),
                                   C.byref(h)), "ecdh_keyset")
        return KeySet.adopt(self, h, n, keylen), ok

    def ecdh_calc_key_host(self, curve: str, private_key: bytes, peer_public: bytes, keylen: int):
        """One connection, exactly ECCKeyExchange::init + calcKey -> (ok, key, iv)."""
        key, iv = C.create_string_buffer(32), C.create_string_buffer(16)
        r = lib.fpnn_ecdh_calc_key_host(self._h, curve.encode(), bytes(private_key), len(private_key),
                                        bytes(peer_public), len(peer_public), keylen, key, iv)
        if r < 0:
            check(r, "ecdh_calc_key_host")
        return (True, key.raw[:keylen], iv.raw) if r == 1 else (False, b"", b"")

    # -- batches ----------------------------------------------------------------------------
    def _desc(self, inp, out, count, keys, *, stride=0, uniform_len=0, in_off=None, out_off=None, lens=None,
              key_slot=None, flags=0, max_len=0) -> BatchDesc:
        d = BatchDesc()
        d.in_ = _ptr(inp).value if inp is not None else None
        d.out = _ptr(out).value if out is not None else None
        d.count = count
        d.uniform_len = uniform_len
        d.stride = stride
        for name, t, dt in (("in_off", in_off, torch.int64), ("out_off", out_off, torch.int64),
                            ("len", lens, torch.int32), ("key_slot", key_slot, torch.int32)):
            if t is not None:
                if t.dtype not in (dt, torch.uint64 if dt == torch.int64 else torch.uint32):
                    raise TypeError(f"{name}: dtype {t.dtype}, expected {dt}")
                if t.numel() < count:
                    raise ValueError(f"{name}: {t.numel()} entries for {count} segments")
                setattr(d, name, _ptr(t).value)
        d.keys = keys.handle.value
        d.flags = flags
        d.max_len = max_len  # optional bound on every length (fpnn_aes.h: picks K2 for many short frames)
        return d

    def package_encrypt(self, inp, out, count, keys: "KeySet", wire_prefix: bool = False, **kw):
        d = self._desc(inp, out, count, keys, flags=F_WIRE_PREFIX if wire_prefix else 0, **kw)
        check(lib.fpnn_aes_package_encrypt(self._h, C.byref(d)), "package_encrypt")

    def package_decrypt(self, inp, out, count, keys: "KeySet", **kw):
        d = self._desc(inp, out, count, keys, **kw)
        check(lib.fpnn_aes_package_decrypt(self._h, C.byref(d)), "package_decrypt")

    def stream_encrypt(self, inp, out, count, keys: "KeySet", iv_state: torch.Tensor, pos_state: torch.Tensor, **kw):
        d = self._desc(inp, out, count, keys, **kw)
        check(lib.fpnn_aes_stream_encrypt(self._h, C.byref(d), _ptr(iv_state), _ptr(pos_state)), "stream_encrypt")

    def stream_decrypt(self, inp, out, count, keys: "KeySet", iv_state: torch.Tensor, pos_state: torch.Tensor, **kw):
        d = self._desc(inp, out, count, keys, **kw)
        check(lib.fpnn_aes_stream_decrypt(self._h, C.byref(d), _ptr(iv_state), _ptr(pos_state)), "stream_decrypt")


def host_register(buf: np.ndarray):
    """fpnn_aes_host_register over a numpy buffer's memory (e.g. a socket-buffer arena):
    package_host calls whose frames all lie in registered memory are then moved by the GPU
    over PCIe (no host gather/scatter).  Keep `buf` alive until host_unregister(buf)."""
    check(lib.fpnn_aes_host_register(C.c_void_p(buf.ctypes.data), buf.nbytes), "host_register")


def host_unregister(buf: np.ndarray):
    check(lib.fpnn_aes_host_unregister(C.c_void_p(buf.ctypes.data)), "host_unregister")


def host_is_mapped(addr: int, nbytes: int) -> bool:
    return bool(lib.fpnn_aes_host_is_mapped(C.c_void_p(addr), nbytes))


def package_host_multi(engines, keysets, encrypt: bool, frames_np, wire_prefix: bool = False):
    """fpnn_aes_package_host_multi: one host-frame batch split byte-balanced over engines
    (keysets[k] on engines[k])."""
    n = len(engines)
    eh = (C.c_void_p * n)(*[e.handle.value for e in engines])
    kh = (C.c_void_p * n)(*[k.handle.value for k in keysets])
    ptr = C.cast(C.c_void_p(frames_np.ctypes.data), C.POINTER(HostFrame))
    check(lib.fpnn_aes_package_host_multi(eh, kh, n, int(encrypt), ptr, len(frames_np),
                                          F_WIRE_PREFIX if wire_prefix else 0), "package_host_multi")


def stream_host_multi(engines, keysets, encrypt: bool, frames_np, iv_state: np.ndarray, pos_state: np.ndarray):
    """fpnn_aes_stream_host_multi: whole streams to engines, state arrays updated in place."""
    n = len(engines)
    eh = (C.c_void_p * n)(*[e.handle.value for e in engines])
    kh = (C.c_void_p * n)(*[k.handle.value for k in keysets])
    ptr = C.cast(C.c_void_p(frames_np.ctypes.data), C.POINTER(HostFrame))
    check(lib.fpnn_aes_stream_host_multi(eh, kh, n, int(encrypt), ptr, len(frames_np), iv_state.ctypes.data,
                                         pos_state.ctypes.data), "stream_host_multi")


class KeySet:
    """Per-connection (key, IV) table on the device, expanded by the GPU."""

    def __init__(self, engine: Engine, keys, keylen: int, ivs=None):
        h = C.c_void_p()
        if isinstance(keys, (bytes, bytearray)):
            count = len(keys) // keylen
            kb = bytes(keys)
            ib = bytes(ivs) if ivs is not None else None
            rc = lib.fpnn_aes_keyset_create(engine.handle, count, keylen, C.c_char_p(kb),
                                            C.c_char_p(ib) if ib is not None else None, 1, C.byref(h))
        else:  # device tensors
            count = keys.numel() // keylen
            rc = lib.fpnn_aes_keyset_create(engine.handle, count, keylen, _ptr(keys),
                                            _ptr(ivs) if ivs is not None else None, 0, C.byref(h))
        check(rc, "keyset_create")
        self._h = h
        _live_keysets.add(self)
        self.count = count
        self.keylen = keylen
        self.engine = engine

    @classmethod
    def reserve(cls, engine: Engine, capacity: int, keylen: int) -> "KeySet":
        """An updatable table (fpnn_aes_keyset_reserve): slots are written with set()."""
        h = C.c_void_p()
        check(lib.fpnn_aes_keyset_reserve(engine.handle, capacity, keylen // 4 + 6, C.byref(h)), "keyset_reserve")
        return cls.adopt(engine, h, 0, keylen)

    def set(self, first: int, keys, ivs=None):
        """fpnn_aes_keyset_set: slots [first, first + len(keys)) get these keys (host key
        expansion, as EncryptorBatch does) and IVs; queued on the creating engine's stream."""
        keys = [bytes(k) for k in keys]
        n = len(keys)
        ctx = (Schedule * n)(*[setup_encrypt(k) for k in keys])
        ib = b"".join(bytes(v) for v in ivs) if ivs is not None else None
        check(lib.fpnn_aes_keyset_set(self._h, first, n, ctx, C.c_char_p(ib) if ib is not None else None), "keyset_set")
        self.count = max(self.count, first + n)

    @classmethod
    def adopt(cls, engine: Engine, h, count: int, keylen: int) -> "KeySet":
        """Wrap a key set the library created (e.g. fpnn_ecdh_keyset)."""
        ks = cls.__new__(cls)
        ks._h = h
        _live_keysets.add(ks)
        ks.count, ks.keylen, ks.engine = count, keylen, engine
        return ks

    @property
    def handle(self):
        return self._h

    @property
    def nrounds(self) -> int:
        return lib.fpnn_aes_keyset_nrounds(self._h)

    def schedule(self, slot: int) -> Schedule:
        s = Schedule()
        check(lib.fpnn_aes_keyset_get_schedule(self._h, slot, C.byref(s)), "keyset_get_schedule")
        return s

    def close(self):
        if getattr(self, "_h", None):
            lib.fpnn_aes_keyset_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# -- Encryptor surface (core/Encryptor.h:11-61) -------------------------------------------------

class Encryptor:
    def __init__(self, engine: Engine, key: bytes, iv: bytes):
        self._engine = engine
        self._key = bytes(key)
        self._iv = bytes(iv[:16])
        self._ctx = setup_encrypt(self._key)


class PackageEncryptor(Encryptor):
    """core/Encryptor.cpp:10-51: each call is a fresh chain from the connection IV."""

    def decrypt(self, src: bytes) -> bytes:
        return self._engine.cfb(self._ctx, False, src, self._iv, 0)[0]

    def encrypt(self, src: bytes) -> bytes:
        return self._engine.cfb(self._ctx, True, src, self._iv, 0)[0]

    def encrypt_frame(self, src: bytes) -> bytes:
        """encrypt(std::string*): htole32(len) || ciphertext."""
        return len(src).to_bytes(4, "little") + (self.encrypt(src) if src else b"")


class StreamEncryptor(Encryptor):
    """core/Encryptor.cpp:53-70: (iv, pos) carried across calls."""

    def __init__(self, engine: Engine, key: bytes, iv: bytes):
        super().__init__(engine, key, iv)
        self._pos = 0

    def _run(self, enc: bool, src: bytes) -> bytes:
        if not src:
            return b""
        out, self._iv, self._pos = self._engine.cfb(self._ctx, enc, src, self._iv, self._pos)
        return out

    def decrypt(self, src: bytes) -> bytes:
        return self._run(False, src)

    def encrypt(self, src: bytes) -> bytes:
        return self._run(True, src)

    @property
    def state(self):
        return self._iv, self._pos
