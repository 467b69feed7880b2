#!/usr/bin/env python3
"""Probe: K1r kernel throughput on 1M x 1 KiB segments (AES-128) by feature -- package vs
stream mode, one key vs one key slot per segment, CFB position 0 vs random -- to find what
costs K1r its speed on C3's framed calls (stream mode, per-stream keys, random positions)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import fpnn_amd
    P, L = int(os.environ.get("P", 1 << 20)), int(os.environ.get("L", 1024))
    eng = fpnn_amd.Engine(0)
    a = torch.empty(P * L + 64, dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(a, 2)
    r = torch.empty_like(a)
    lens = torch.full((P,), L, dtype=torch.int32, device="cuda")
    offs = torch.arange(P, dtype=torch.int64, device="cuda") * L
    g = torch.Generator(device="cuda").manual_seed(1)
    for nkeys in (1, P):
        ks = fpnn_amd.KeySet(eng, bytes(range(16)) * nkeys, 16, bytes(16 * nkeys))
        slots = torch.arange(P, dtype=torch.int32, device="cuda") % nkeys
        for mode in ("package", "stream0", "streamR"):
            iv = torch.zeros(P * 16, dtype=torch.uint8, device="cuda")
            pos = torch.zeros(P, dtype=torch.int32, device="cuda")

            def call():
                if mode == "package":
                    eng.package_decrypt(a, r, P, ks, in_off=offs, lens=lens, key_slot=slots if nkeys > 1 else None)
                else:
                    if mode == "streamR":
                        pos.copy_(torch.randint(0, 16, (P,), device="cuda", generator=g, dtype=torch.int32))
                    else:
                        pos.zero_()
                    eng.stream_decrypt(a, r, P, ks, iv, pos, in_off=offs, lens=lens,
                                       key_slot=slots if nkeys > 1 else None)
            for _ in range(3):
                call()
            eng.reset_stats()
            eng.set_timing(True)
            for _ in range(10):
                call()
            eng.set_timing(False)
            n, ms = eng.kernel_stats(fpnn_amd.K_DECRYPT)
            print({"P": P, "L": L, "keys": nkeys, "mode": mode, "kernel": eng.last_kernel(fpnn_amd.K_DECRYPT),
                   "GiBs": round(P * L / (ms / n / 1e3) / 2**30, 1)}, flush=True)


if __name__ == "__main__":
    main()
