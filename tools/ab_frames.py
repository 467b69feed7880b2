#!/usr/bin/env python3
"""Same-box A/B of the short-frame encrypt (round 6): FPNN's 145-B quests
from 16 384 keyed connections (bench_configs' Q1 / Q1s, and Q1w: Q1s as wire frames,
htole32(len) || C) through K2s (k_cfb_encrypt_frames, chosen by max_len <= 175) and through
K2 (the same batch with max_len = 2048), alternating, the ciphertexts compared.  Kernel-time
GiB/s of payload (steady state, tools/bench_configs.timed).

  python tools/ab_frames.py [--rounds 2] [--configs Q1,Q1s,Q1w]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import workloads as W  # noqa: E402
from bench_configs import gib, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--configs", default="Q1,Q1s,Q1w")
    args = ap.parse_args()
    import fpnn_amd
    E = fpnn_amd.K_ENCRYPT
    eng = fpnn_amd.Engine(0)
    out = {}
    for name in args.configs.split(","):
        P, L, NC = 2 << 20, 145, 16384
        kl = 32 if name == "Q1" else 16
        wire = name == "Q1w"
        keys, ivs = W.many_keys(dict(W.U1, connections=NC, keylen=kl))
        ks = fpnn_amd.KeySet(eng, keys.tobytes(), kl, ivs.tobytes())
        offs = torch.arange(P, dtype=torch.int64, device="cuda") * L
        lens = torch.full((P,), L, dtype=torch.int32, device="cuda")
        slots = (torch.arange(P, dtype=torch.int32, device="cuda") % NC).contiguous()
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, 11)
        kw = dict(in_off=offs, lens=lens, key_slot=slots)
        if wire:
            kw["out_off"] = torch.arange(P, dtype=torch.int64, device="cuda") * (L + 4)
            kw["wire_prefix"] = True
        outs = {}
        res = {"frames": P, "frame_bytes": L, "keylen": kl, "wire": wire}
        for r in range(args.rounds):
            for label, bound in (("K2s", L), ("K2", 2048)):
                b = torch.empty(P * (L + 4 if wire else L), dtype=torch.uint8, device="cuda")
                _, ke, _ = timed(eng, E, lambda: eng.package_encrypt(a, b, P, ks, max_len=bound, **kw), args.reps)
                kname = eng.last_kernel(E)
                res.setdefault(label, []).append(gib(P * L, ke))
                res[label + "_kernel"] = kname
                outs[label] = b
        assert torch.equal(outs["K2s"], outs["K2"]), name
        res["same_ciphertext"] = True
        out[name] = res
        print(json.dumps({name: res}), flush=True)
        del a, outs
    print(json.dumps({"ab_frames": out}))


if __name__ == "__main__":
    main()
