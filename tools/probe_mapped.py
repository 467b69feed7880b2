#!/usr/bin/env python3
"""Probe: fpnn_aes_package_host over registered host arenas (the mapped path) on C2's
shape -- 1M x 1 KiB frames at shuffled arena positions.  Prints GiB/s per direction."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import workloads as W  # noqa: E402


def page_aligned(nbytes):
    raw = np.empty(nbytes + 4096, dtype=np.uint8)
    return raw[(-raw.ctypes.data) % 4096:][:nbytes]


def main():
    import fpnn_amd
    P, L = 1 << 20, 1024
    key, iv = W.single_key(W.C2)
    import torch
    eng = fpnn_amd.Engine(0, stream=torch.cuda.Stream() if os.environ.get("OWN_STREAM") else None)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    src, dst = page_aligned(P * L), page_aligned(P * L)
    src[:] = 7
    t0 = time.perf_counter()
    fpnn_amd.host_register(src)
    fpnn_amd.host_register(dst)
    treg = time.perf_counter() - t0
    perm = np.random.default_rng(1).permutation(P).astype(np.uint64)
    fm = np.zeros(P, dtype=fpnn_amd.engine.HOST_FRAME_DTYPE)
    fm["src"] = src.ctypes.data + perm * L
    fm["dst"] = dst.ctypes.data + perm[::-1] * L
    fm["len"] = L
    res = []
    for enc in (True, False):
        eng.package_host_array(enc, fm, ks)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.package_host_array(enc, fm, ks)
            ts.append(time.perf_counter() - t0)
        res.append(round(P * L / min(ts) / 2**30, 2))
    print({"own_stream": bool(os.environ.get("OWN_STREAM")), "chunk_MB": os.environ.get("FPNN_AES_MAP_CHUNK_MB", "64"), "encrypt_GiBs": res[0], "decrypt_GiBs": res[1],
           "register_2GiB_ms": round(treg * 1e3, 1), "path": eng.last_kernel(fpnn_amd.K_HOST)}, flush=True)


if __name__ == "__main__":
    main()
