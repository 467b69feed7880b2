#!/usr/bin/env python3
"""Probe timing of the short-frame kernels on Q1 / Q1s (bench_configs' shapes) through
whatever GPU library FPNN_AES_GPU_LIB names, WITHOUT checking the output (for probe builds
that skip work, e.g. -DFPNN_PROBE_NOSTORE).  Prints one JSON line per config: kernel GiB/s
of the encrypt and the decrypt, and whether the round trip still held.

  FPNN_AES_GPU_LIB=$PWD/fpnn_amd/libfpnn_aes_gpu_X.so python tools/probe/q1_time.py [--configs Q1,Q1s]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import workloads as W  # noqa: E402
from bench_configs import gib, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="Q1,Q1s,Q1w")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import fpnn_amd
    E, D = fpnn_amd.K_ENCRYPT, fpnn_amd.K_DECRYPT
    eng = fpnn_amd.Engine(0)
    for name in args.configs.split(","):
        P, L, NC = 2 << 20, 145, 16384
        kl = 32 if name == "Q1" else 16  # (Q1w: Q1s as wire frames, htole32(len) || C; encrypt only)
        keys, ivs = W.many_keys(dict(W.U1, connections=NC, keylen=kl))
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), kl, ivs.tobytes())
        kw = dict(in_off=torch.arange(P, dtype=torch.int64, device="cuda") * L,
                  lens=torch.full((P,), L, dtype=torch.int32, device="cuda"),
                  key_slot=(torch.arange(P, dtype=torch.int32, device="cuda") % NC).contiguous())
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 11)
        b, r = torch.empty_like(a), torch.empty_like(a)
        if name == "Q1w":
            w = torch.empty(P * (L + 4), dtype=torch.uint8, device="cuda")
            ow = torch.arange(P, dtype=torch.int64, device="cuda") * (L + 4)
            _, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, w, P, ks, max_len=L, out_off=ow, wire_prefix=True,
                                                                 **kw), args.reps)
            print(json.dumps({name: {"encrypt_kernel_GiBs": gib(P * L, ke), "kernels": [eng.last_kernel(E)]}}),
                  flush=True)
            del a, b, r, w
            continue
        _, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, max_len=L, **kw), args.reps)
        kname_e = eng.last_kernel(E)
        _, kd, _ = timed(eng, D, lambda: eng.package_decrypt(b, r, P, ks, max_len=L, **kw), args.reps)
        kname_d = eng.last_kernel(D)
        print(json.dumps({name: {"encrypt_kernel_GiBs": gib(P * L, ke), "decrypt_kernel_GiBs": gib(P * L, kd),
                                 "kernels": [kname_e, kname_d], "roundtrip_ok": bool(torch.equal(r, a))}}),
              flush=True)
        del a, b, r


if __name__ == "__main__":
    main()
