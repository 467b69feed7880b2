#!/usr/bin/env python3
"""Probe: K1r (ragged decrypt) on C2's 1M x 1 KiB packets with every segment at a 16-B
aligned offset vs shifted by 1..15 bytes (stream frames start at arbitrary CFB positions,
so their blocks are unaligned in memory), AES-128 and AES-256, kernel time per call."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import fpnn_amd
    P, L = 1 << 20, 1024
    eng = fpnn_amd.Engine(0)
    a = torch.empty(P * L + 64, dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(a, 2)
    r = torch.empty_like(a)
    lens = torch.full((P,), L, dtype=torch.int32, device="cuda")
    for keylen in (16, 32):
        ks = fpnn_amd.KeySet(eng, bytes(range(keylen)), keylen, bytes(16))
        for shift in (0, 1, 5, 8, 15):
            offs = torch.arange(P, dtype=torch.int64, device="cuda") * L + shift
            for _ in range(3):
                eng.package_decrypt(a, r, P, ks, in_off=offs, lens=lens)
            eng.reset_stats()
            eng.set_timing(True)
            for _ in range(10):
                eng.package_decrypt(a, r, P, ks, in_off=offs, lens=lens)
            eng.set_timing(False)
            n, ms = eng.kernel_stats(fpnn_amd.K_DECRYPT)
            print({"keylen": keylen, "shift": shift, "kernel": eng.last_kernel(fpnn_amd.K_DECRYPT),
                   "GiBs": round(P * L / (ms / n / 1e3) / 2**30, 1)}, flush=True)


if __name__ == "__main__":
    main()
