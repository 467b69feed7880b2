#!/usr/bin/env python3
"""why tools/bench_configs.py read the C2 kernels 12-15 % below
bench.py on the same box.  Runs, in ONE process on one engine and one C2 batch, the two
harnesses' timing loops in alternation:

  bench     bench.py's step loop: W warm-up steps, then K steps of encrypt + decrypt
            back to back, HIP events per launch (eng.set_timing) over the timed region
  configs   tools/bench_configs.py's timed(): 2 warm-up calls, then 3 rounds of `reps`
            calls of ONE direction back to back, median round
  enc_only  bench.py's loop with encrypt only (isolates "same kernel back to back")

and prints one JSON line per pass plus a summary.

  python tools/timer_probe.py [--passes 2]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import fpnn_amd
    from bench_configs import timed
    E, D = fpnn_amd.K_ENCRYPT, fpnn_amd.K_DECRYPT
    eng = fpnn_amd.Engine(0)
    c = W.C2
    P, L = c["packets"], c["length"]
    key, iv = W.single_key(c)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(a, c["payload_seed"])
    b, r = torch.empty_like(a), torch.empty_like(a)
    kw = dict(stride=L, uniform_len=L)
    enc = lambda: eng.package_encrypt(a, b, P, ks, **kw)  # noqa: E731
    dec = lambda: eng.package_decrypt(b, r, P, ks, **kw)  # noqa: E731
    gib = lambda s: round(P * L / s / 2**30, 1)  # noqa: E731

    def bench_loop(fns, warm=5):
        for _ in range(warm):
            for f in fns:
                f()
        torch.cuda.synchronize()
        eng.reset_stats()
        eng.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            for f in fns:
                f()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        eng.set_timing(False)
        out = {"wall_ms_per_step": round(wall / args.steps * 1e3, 4)}
        for name, which in (("enc", E), ("dec", D)):
            n, ms = eng.kernel_stats(which)
            if n:
                out[f"{name}_kernel_GiBs"] = gib(ms / n / 1e3)
        return out

    res = []
    for p in range(args.passes):
        for mode in ("bench", "configs", "enc_only"):
            if mode == "bench":
                d = bench_loop([enc, dec])
            elif mode == "enc_only":
                d = bench_loop([enc])
            else:
                we, ke, _ = timed(eng, E, enc, args.reps)
                wd, kd, _ = timed(eng, D, dec, args.reps)
                d = {"enc_kernel_GiBs": gib(ke), "dec_kernel_GiBs": gib(kd), "enc_wall_GiBs": gib(we),
                     "dec_wall_GiBs": gib(wd)}
            d = {"pass": p, "mode": mode, **d}
            print(json.dumps(d), flush=True)
            res.append(d)
    assert torch.equal(r, a)
    summ = {}
    for mode in ("bench", "configs", "enc_only"):
        for k in ("enc_kernel_GiBs", "dec_kernel_GiBs"):
            v = [d[k] for d in res if d["mode"] == mode and k in d]
            if v:
                summ[f"{mode}.{k}"] = statistics.median(v)
    print(json.dumps({"timer_probe": summ}), flush=True)


if __name__ == "__main__":
    main()
