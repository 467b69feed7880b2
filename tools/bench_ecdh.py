#!/usr/bin/env python3
"""ECDH key-derivation throughput (§8f row 4): fpnn_ecdh_calc_keys on the GPU -- one
server private key against N peer public keys, i.e. ECCKeyExchange::calcKey for N
accepted connections (config C5's 65 536-connection key table) -- against the reference's
own calcKey (core/KeyExchange.cpp + core/micro-ecc, oracle/_ref/ecdh_ref) on the host
cores, one process per core.

  python tools/bench_ecdh.py [--n 65536] [--reps 5] [--cpu-seconds 3]
Prints one JSON object (derivations/s per curve).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
ECDH_REF = os.path.join(ROOT, "oracle", "_ref", "ecdh_ref")


def gpu_rate(engine, curve: str, n: int, reps: int):
    import numpy as np
    import torch
    import fpnn_amd
    lib = fpnn_amd.lib
    cv = engine.ecdh_curve(curve)
    pl = lib.fpnn_ecdh_private_len(cv)
    rng = np.random.default_rng(n)
    privs = torch.from_numpy(rng.integers(0, 256, (n, pl), dtype=np.uint8)).to("cuda:0")
    privs[:, 0] &= 0x7F
    peers, ok = engine.ecdh_public_keys(curve, privs)  # setup, not timed
    server = bytes(rng.integers(1, 255, pl, dtype=np.uint8))
    torch.cuda.synchronize()
    engine.ecdh_calc_keys(curve, server, peers, 32)  # warm-up
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        keys, ivs, ok = engine.ecdh_calc_keys(curve, server, peers, 32)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    assert bool(ok.all())
    return n / best, best * 1e3


def gpu_percall(engine, curve: str, calls: int):
    """The drop-in per-call form (ECCKeyExchange::calcKey through fpnn_ecdh_calc_key_host:
    one peer, host buffers, synchronous): median microseconds per call."""
    import statistics
    import numpy as np
    import torch
    import fpnn_amd
    cv = engine.ecdh_curve(curve)
    pl = fpnn_amd.lib.fpnn_ecdh_private_len(cv)
    rng = np.random.default_rng(77)
    privs = torch.from_numpy(rng.integers(0, 256, (calls, pl), dtype=np.uint8)).to("cuda:0")
    privs[:, 0] &= 0x7F
    peers, _ = engine.ecdh_public_keys(curve, privs)
    peers = peers.cpu().numpy()
    server = bytes(rng.integers(1, 255, pl, dtype=np.uint8))
    engine.ecdh_calc_key_host(curve, server, peers[0].tobytes(), 32)  # warm-up (scratch)
    times = []
    for i in range(calls):
        p = peers[i].tobytes()
        t0 = time.perf_counter()
        engine.ecdh_calc_key_host(curve, server, p, 32)
        times.append(time.perf_counter() - t0)
    return statistics.median(times) * 1e6


def cpu_rate(curve: str, procs: int, seconds: float):
    """calcKey/s of the reference, `procs` processes in parallel (one per core)."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "ecdh_cases.json")))
    cv = next(c for c in g["curves"] if c["curve"] == curve)
    req = f"T {curve} {cv['server_private']} {cv['clients'][0]['public']} 50\n"
    t0 = time.perf_counter()
    r = subprocess.run([ECDH_REF], input=req, capture_output=True, text=True, check=True)
    one = float([ln for ln in r.stdout.splitlines() if ln.startswith("R ")][0].split()[1]) / 50
    reps = max(20, int(seconds / one))
    req = f"T {curve} {cv['server_private']} {cv['clients'][0]['public']} {reps}\n"
    t0 = time.perf_counter()
    ps = [subprocess.Popen([ECDH_REF], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True) for _ in range(procs)]
    for p in ps:
        p.stdin.write(req)
        p.stdin.close()
    for p in ps:
        p.wait()
    wall = time.perf_counter() - t0
    return procs * reps / wall, reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--curves", default="secp256k1,secp256r1,secp224r1,secp192r1")
    ap.add_argument("--no-cpu", action="store_true", help="skip the reference CPU legs (profiling runs)")
    ap.add_argument("--percall", type=int, default=0, help="also time this many single-peer calcKey calls")
    args = ap.parse_args()
    import fpnn_amd
    eng = fpnn_amd.Engine(0)
    cores = len(os.sched_getaffinity(0))
    try:
        quota = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota[0] != "max":
            cores = min(cores, max(1, int(int(quota[0]) / int(quota[1]))))
    except OSError:
        pass
    out = {"metric": "ECDH calcKey derivations/s", "n": args.n, "host_cores_used": cores, "curves": {}}
    for curve in args.curves.split(","):
        g, ms = gpu_rate(eng, curve, args.n, args.reps)
        row = {"gpu_per_s": round(g), "gpu_ms_per_batch": round(ms, 3)}
        if args.percall:
            row["gpu_percall_us_median"] = round(gpu_percall(eng, curve, args.percall), 1)
        if os.path.exists(ECDH_REF) and not args.no_cpu:
            c1, _ = cpu_rate(curve, 1, args.cpu_seconds)
            cn, _ = cpu_rate(curve, cores, args.cpu_seconds)
            row.update({"reference_1core_per_s": round(c1), f"reference_{cores}cores_per_s": round(cn),
                        "gpu_over_reference_all_cores": round(g / cn, 1)})
            if args.percall:
                row["reference_percall_us"] = round(1e6 / c1, 1)
        out["curves"][curve] = row
        print(json.dumps({curve: row}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
