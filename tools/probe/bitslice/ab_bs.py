#!/usr/bin/env python3
"""A/B of the bitsliced decrypt share (FPNN_AES_BITSLICE_FRAC) on C2, interleaved rounds
in one process; prints median decrypt time per fraction."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import workloads as W  # noqa: E402


def main():
    import fpnn_amd
    fracs = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0 0.15 0.25 0.35 0.5 1.0").split()]
    P, L = 1 << 20, 1024
    key, iv = W.single_key(W.C2)
    engines = []
    for f in fracs:
        os.environ["FPNN_AES_BITSLICE_FRAC"] = str(f)
        e = fpnn_amd.Engine(0)
        engines.append((f, e, fpnn_amd.KeySet(e, key, 32, iv)))
    plain = torch.empty(P * L, dtype=torch.uint8, device="cuda")
    engines[0][1].fill_synthetic(plain, 2)
    cipher, back = torch.empty_like(plain), torch.empty_like(plain)
    engines[0][1].package_encrypt(plain, cipher, P, engines[0][2], stride=L, uniform_len=L)
    res = {f: [] for f in fracs}
    for r in range(7):
        for f, e, ks in engines:
            e.reset_stats()
            e.set_timing(True)
            for _ in range(3):
                e.package_decrypt(cipher, back, P, ks, stride=L, uniform_len=L)
            e.set_timing(False)
            n, ms = e.kernel_stats(fpnn_amd.K_DECRYPT)
            torch.cuda.synchronize()
            assert torch.equal(back, plain), f
            if r:
                res[f].append(ms / n)
    print(json.dumps({str(f): {"median_ms": round(statistics.median(v), 4),
                               "GiBs": round(P * L / (statistics.median(v) / 1e3) / 2**30, 1)}
                      for f, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
