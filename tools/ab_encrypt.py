#!/usr/bin/env python3
"""Interleaved A/B of encrypt-kernel variants on one ragged config, in ONE process.

Each variant is an engine created under its own FPNN_AES_* settings (';'-separated
variants, ','-separated NAME=VALUE inside one); rounds alternate over the variants and
the per-launch HIP-event kernel time is collected per round.  Every variant's output must
equal the first variant's, byte for byte.

  C4   Zipf 64 B..64 KiB, 4 GiB, AES-256 package (workloads.C4)
  R1   send side of R1: 16384 x 64 bodies of 1 KiB -> htole32(len) || C wire frames
       (frames back to back: body offsets 4, 8, 12, 0 mod 16)
  R1A  the same with 16-byte aligned bodies (1040-byte frame pitch)
  C2R  C2's 1M x 1 KiB packets as a ragged batch (offset / length arrays)
With --decrypt the package configs also decrypt the output back (timed, round trip checked).
Usage: python tools/ab_encrypt.py --config C4 --variants "FPNN_AES_HYB_LONG=512;FPNN_AES_HYB_LONG=1024"
"""
import argparse
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402


def make_engine(spec):
    import fpnn_amd
    saved = dict(os.environ)
    for kv in spec.split(","):
        if kv.strip():
            k, v = kv.strip().split("=")
            os.environ[k] = v
    try:
        return fpnn_amd.Engine(0)
    finally:
        os.environ.clear()
        os.environ.update(saved)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--variants", default="FPNN_AES_HYB_LONG=512;FPNN_AES_HYB_LONG=1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--decrypt", action="store_true", help="also time decrypting the output back (package batches)")
    args = ap.parse_args()
    import fpnn_amd

    if args.config == "C4":
        c = W.C4
        sizes = W.zipf_sizes(c)
        n = len(sizes)
        offs = np.concatenate([[0], np.cumsum(sizes[:-1].astype(np.int64))]).astype(np.int64)
        total = int(offs[-1] + sizes[-1])
        key, iv = W.single_key(c)
        src = torch.empty(total, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        kw = dict(in_off=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(sizes.astype(np.int32)).cuda())
        nbytes = total
        fill_seed = c["payload_seed"]
    elif args.config == "R1":
        NC, F, L = 16384, 64, 1024
        n = NC * F
        key, iv = W.single_key(W.C2)
        src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dst = torch.empty(n * (L + 4), dtype=torch.uint8, device="cuda")
        kw = dict(in_off=torch.arange(n, dtype=torch.int64, device="cuda") * L,
                  out_off=torch.arange(n, dtype=torch.int64, device="cuda") * (L + 4),
                  lens=torch.full((n,), L, dtype=torch.int32, device="cuda"), wire_prefix=True)
        nbytes = n * L
        fill_seed = 7
    elif args.config == "R1A":  # R1 with 16-byte aligned bodies (frames of 1040 B, prefix at +12)
        NC, F, L = 16384, 64, 1024
        n = NC * F
        key, iv = W.single_key(W.C2)
        src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dst = torch.empty(n * (L + 16), dtype=torch.uint8, device="cuda")
        kw = dict(in_off=torch.arange(n, dtype=torch.int64, device="cuda") * L,
                  out_off=torch.arange(n, dtype=torch.int64, device="cuda") * (L + 16) + 12,
                  lens=torch.full((n,), L, dtype=torch.int32, device="cuda"), wire_prefix=True)
        nbytes = n * L
        fill_seed = 7
    elif args.config == "C2R":  # C2's packets as a ragged batch (offset / length arrays)
        c = W.C2
        n, L = c["packets"], c["length"]
        key, iv = W.single_key(c)
        src = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        kw = dict(in_off=torch.arange(n, dtype=torch.int64, device="cuda") * L,
                  lens=torch.full((n,), L, dtype=torch.int32, device="cuda"))
        nbytes = n * L
        fill_seed = c["payload_seed"]
    else:
        raise SystemExit(f"unknown config {args.config}")
    decrypt = args.decrypt and "wire_prefix" not in kw
    back = torch.empty_like(src) if decrypt else None

    variants = []
    for spec in args.variants.split(";"):
        e = make_engine(spec)
        variants.append((spec, e, fpnn_amd.KeySet(e, key, len(key), iv)))
    variants[0][1].fill_synthetic(src, fill_seed)
    torch.cuda.synchronize()
    res = {spec: [] for spec, _, _ in variants}
    dres = {spec: [] for spec, _, _ in variants}
    digest, kernel, dkernel, rt = {}, {}, {}, {}
    for r in range(args.rounds + 1):
        for spec, e, ks in variants:
            e.reset_stats()
            e.set_timing(True)
            for _ in range(args.reps):
                e.package_encrypt(src, dst, n, ks, **kw)
                if decrypt:
                    e.package_decrypt(dst, back, n, ks, **kw)
            torch.cuda.synchronize()
            e.set_timing(False)
            cnt, ms = e.kernel_stats(fpnn_amd.K_ENCRYPT)
            kernel[spec] = e.last_kernel(fpnn_amd.K_ENCRYPT)
            dcnt, dms = e.kernel_stats(fpnn_amd.K_DECRYPT)
            dkernel[spec] = e.last_kernel(fpnn_amd.K_DECRYPT)
            if r == 0:  # warm-up round: clocks, scratch growth; record the output digest
                digest[spec] = hashlib.sha256(dst.cpu().numpy().tobytes()).hexdigest()
                rt[spec] = bool(torch.equal(back, src)) if decrypt else None
                continue
            res[spec].append(nbytes / (ms / max(1, cnt) / 1e3) / 2**30)
            if decrypt:
                dres[spec].append(nbytes / (dms / max(1, dcnt) / 1e3) / 2**30)
    first = variants[0][0]

    def row(spec, v):
        d = {"env": spec, "kernel": kernel[spec], "median_GiBs": round(statistics.median(v), 1),
             "min_GiBs": round(min(v), 1), "max_GiBs": round(max(v), 1),
             "output_equals_first": digest[spec] == digest[first]}
        if decrypt:
            dv = dres[spec]
            d.update(decrypt_kernel=dkernel[spec], decrypt_median_GiBs=round(statistics.median(dv), 1),
                     decrypt_min_GiBs=round(min(dv), 1), roundtrip_ok=rt[spec])
        return d
    out = {"config": args.config, "chains": n, "bytes": nbytes, "rounds": args.rounds, "reps": args.reps,
           "variants": [row(spec, v) for spec, v in res.items()]}
    print(json.dumps(out), flush=True)
    bad = [v["env"] for v in out["variants"] if not v["output_equals_first"] or v.get("roundtrip_ok") is False]
    if bad:
        raise SystemExit(f"outputs differ from {first!r}: {bad}")


if __name__ == "__main__":
    main()
