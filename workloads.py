"""Synthetic workload definitions for BASELINE.json's configs (shared by bench.py,
tests/ and oracle/gen_golden.py).

Data generator: counter-based splitmix64.  Byte k of stream(seed) is byte (k & 7)
(little-endian) of splitmix64((k >> 3) + seed * 0xD1B54A32D192ED03).  The same
definition is implemented by the device fill (fpnn_aes_fill_synthetic) and by the
oracle (ao_synth_fill); tests check all three agree.

Keys/IVs: single-key configs take key = stream(key_seed)[0:keylen] and
iv = stream(key_seed)[32:48]; many-key configs take slot k's key from
stream(key_seed)[48k : 48k+keylen] and its IV from [48k+32 : 48k+48].
"""
from __future__ import annotations

import numpy as np

GOLDEN_MUL = np.uint64(0xD1B54A32D192ED03)

C1 = dict(name="C1", mode="package", keylen=32, packets=10_000, length=1024, key_seed=1001, payload_seed=1,
          note="loopback TCP encrypted echo, CPU-only reference case (not a GPU bench line)")
C2 = dict(name="C2", mode="package", keylen=32, packets=1 << 20, length=1024, key_seed=1002, payload_seed=2,
          note="1M x 1 KiB AES-256 package-mode encrypt+decrypt, one key/IV -- the bench workload")
C3 = dict(name="C3", mode="stream", keylen=16, streams=4096, length=4 << 20, key_seed=1003, payload_seed=3,
          split_seed=3003, note="4096 streams x 4 MiB AES-128 stream mode, random frame splits")
C4 = dict(name="C4", mode="package", keylen=32, total_bytes=4 << 30, zipf_s=1.1, zipf_max=1024, unit=64,
          key_seed=1004, payload_seed=4, size_seed=4004, note="Zipf 64 B-64 KiB AES-256 package mode")
C5 = dict(name="C5", mode="package", keylen=32, packets=65536, length=4096, key_seed=1005, payload_seed=5,
          note="65536 keys x 4 KiB AES-256, per-key IV")
# UDP v2 shape: MTU-sized datagrams (1472 = 1500 - IP - UDP headers,
# core/UDP.v2/UDPIOBuffer.v2.h:14) of many connections, whole-datagram package encryption
# (UDPEncryptor::packageEncrypt, core/UDP.v2/UDPCommon.v2.cpp:197-205), AES-128 (the
# non-reinforced key length).  Datagram i belongs to connection i % connections.
U1 = dict(name="U1", mode="package", keylen=16, packets=1 << 20, length=1472, connections=16384, key_seed=2001,
          payload_seed=21, note="1M x 1472 B UDP datagrams over 16384 connections, AES-128 package mode")
CONFIGS = {c["name"]: c for c in (C1, C2, C3, C4, C5, U1)}


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_words(seed: int, start: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        base = np.uint64(start) + np.uint64(seed) * GOLDEN_MUL
        return _splitmix(base + np.arange(n, dtype=np.uint64))


def synth_bytes(nbytes: int, seed: int, offset: int = 0) -> np.ndarray:
    """Bytes [offset, offset + nbytes) of stream(seed) (numpy; for small/medium sizes)."""
    w0 = offset >> 3
    w1 = (offset + nbytes + 7) >> 3
    words = synth_words(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    s = offset - (w0 << 3)
    return b[s:s + nbytes].copy()


def single_key(cfg: dict):
    s = synth_bytes(48, cfg["key_seed"])
    return s[:cfg["keylen"]].tobytes(), s[32:48].tobytes()


def many_keys(cfg: dict):
    n = cfg.get("connections", cfg.get("packets", cfg.get("streams")))
    s = synth_bytes(48 * n, cfg["key_seed"]).reshape(n, 48)
    keys = np.ascontiguousarray(s[:, :cfg["keylen"]]).reshape(-1)
    ivs = np.ascontiguousarray(s[:, 32:48]).reshape(-1)
    return keys, ivs


def zipf_sizes(cfg: dict = C4) -> np.ndarray:
    """C4 packet sizes: unit * r, r ~ Zipf(s) on 1..zipf_max by inverse CDF on 53-bit
    uniforms from stream(size_seed), drawn until the total reaches total_bytes."""
    r = np.arange(1, cfg["zipf_max"] + 1, dtype=np.float64)
    cdf = np.cumsum(r ** -cfg["zipf_s"])
    cdf /= cdf[-1]
    thresholds = np.floor(cdf * float(1 << 53)).astype(np.uint64)
    mean = cfg["unit"] * float((r * (r ** -cfg["zipf_s"])).sum() / (r ** -cfg["zipf_s"]).sum())
    n_est = int(cfg["total_bytes"] / mean * 1.2) + 1024
    u = synth_words(cfg["size_seed"], 0, n_est) >> np.uint64(11)
    idx = np.searchsorted(thresholds, u, side="right")
    sizes = (np.minimum(idx, cfg["zipf_max"] - 1) + 1).astype(np.uint64) * np.uint64(cfg["unit"])
    csum = np.cumsum(sizes)
    n = int(np.searchsorted(csum, np.uint64(cfg["total_bytes"]), side="left")) + 1
    return sizes[:n].astype(np.uint32)


def stream_splits(cfg: dict, stream: int, max_frame: int = 65536) -> np.ndarray:
    """C3 frame lengths for one stream: 1 B .. max_frame from stream(split_seed + 7919*stream)."""
    L = cfg["length"]
    nw = 1024
    while True:
        w = synth_words(cfg["split_seed"] + 7919 * stream, 0, nw)
        lens = (w % np.uint64(max_frame)).astype(np.int64) + 1
        c = np.cumsum(lens)
        if c[-1] >= L:
            break
        nw *= 4
    n = int(np.searchsorted(c, L, side="left")) + 1
    out = lens[:n].copy()
    out[-1] -= int(c[n - 1] - L)
    return out


def describe() -> dict:
    return {k: {kk: vv for kk, vv in v.items()} for k, v in CONFIGS.items()}
