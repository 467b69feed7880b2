#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (guide §5.4 rule 24).

Each variant is an engine created under its own FPNN_AES_* environment; rounds
alternate between variants; per-kernel HIP-event times are collected per round.
Usage: python tools/ab.py [--rounds 8] [--variants "FPNN_AES_DEC_FULL=0;FPNN_AES_DEC_FULL=1"] [--keylen 32]
(a variant is a comma-separated list of NAME=VALUE settings; variants are ';'-separated)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="FPNN_AES_DEC_FULL=0;FPNN_AES_DEC_FULL=1")
    ap.add_argument("--packets", type=int, default=1 << 20)
    ap.add_argument("--length", type=int, default=1024)
    ap.add_argument("--keylen", type=int, default=32)
    args = ap.parse_args()
    import fpnn_amd

    P, L = args.packets, args.length
    key, iv = W.single_key(W.C2)
    key = key[:args.keylen]
    plain = torch.empty(P * L, dtype=torch.uint8, device="cuda")
    cipher = torch.empty_like(plain)
    back = torch.empty_like(plain)
    variants = []
    for v in args.variants.split(";"):
        saved = dict(os.environ)
        for kv in v.split(","):
            if kv.strip():
                k, val = kv.strip().split("=")
                os.environ[k] = val
        e = fpnn_amd.Engine(0)
        os.environ.clear()
        os.environ.update(saved)
        ks = fpnn_amd.KeySet(e, key, len(key), iv)
        variants.append((v, e, ks))
    variants[0][1].fill_synthetic(plain, 2)
    ref = None
    res = {v: {"enc": [], "dec": []} for v, _, _ in variants}
    for r in range(args.rounds + 1):
        for v, e, ks in variants:
            e.reset_stats()
            e.set_timing(True)
            for _ in range(args.reps):
                e.package_encrypt(plain, cipher, P, ks, stride=L, uniform_len=L)
                e.package_decrypt(cipher, back, P, ks, stride=L, uniform_len=L)
            e.set_timing(False)
            ne, me = e.kernel_stats(fpnn_amd.K_ENCRYPT)
            nd, md = e.kernel_stats(fpnn_amd.K_DECRYPT)
            torch.cuda.synchronize()
            assert torch.equal(back, plain), v
            h = int(cipher[::4099].to(torch.int64).sum())
            ref = h if ref is None else ref
            assert h == ref, f"variant {v} produced different ciphertext"
            if r:  # round 0 = warmup
                res[v]["enc"].append(me / ne)
                res[v]["dec"].append(md / nd)
    out = {}
    for v in res:
        enc, dec = res[v]["enc"], res[v]["dec"]
        out[v] = {k: {"median_ms": round(statistics.median(x), 4), "min_ms": round(min(x), 4),
                      "GiBs_median": round(P * L / (statistics.median(x) / 1e3) / 2**30, 1)}
                  for k, x in (("encrypt", enc), ("decrypt", dec))}
    print(json.dumps({"P": P, "L": L, "keylen": args.keylen, "variants": out}, indent=1))


if __name__ == "__main__":
    main()
