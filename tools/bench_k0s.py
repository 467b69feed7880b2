#!/usr/bin/env python3
"""The resident small-call server (K0s, k_small.hip) beside batch kernels, both ways
(more engines than the box's GPU_MAX_HW_QUEUES = 4).

  * batch time with servers resident: N threads (N = 0, 1, 4, 16), each with its own engine
    and stream, keep issuing 1 KiB per-call decrypts (PackageEncryptor's shape through
    fpnn_aes_cfb_host, so each keeps a K0s server alive) while the main thread times C2
    (1M x 1 KiB AES-256) and C4 (Zipf, 1 GiB here) encrypt + decrypt calls on its own
    engine: wall time per call, host clock around call + stream sync (a kernel queued
    behind a server on a shared hardware queue waits there, so the engine's event timing
    would not see it);
  * per-call latency during batch flushes: one thread times 1 KiB per-call decrypts while
    the main thread runs C4 encrypt calls back to back, against the same thread alone.

  python tools/bench_k0s.py [--servers 0,1,4,16] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--servers", default="0,1,4,16")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--c4-bytes", type=int, default=1 << 30)
    args = ap.parse_args()
    import fpnn_amd

    main_stream = torch.cuda.Stream()
    eng = fpnn_amd.Engine(0, stream=main_stream)
    c2 = W.C2
    P, L = c2["packets"], c2["length"]
    key, iv = W.single_key(c2)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    with torch.cuda.stream(main_stream):
        a = torch.empty(P * L, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a, c2["payload_seed"])
        b, r = torch.empty_like(a), torch.empty_like(a)
    sizes = W.zipf_sizes(dict(W.C4, total_bytes=args.c4_bytes))
    n4 = len(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1].astype(np.int64))]).astype(np.int64)
    t4 = int(offs[-1] + sizes[-1])
    with torch.cuda.stream(main_stream):
        a4 = torch.empty(t4, dtype=torch.uint8, device="cuda")
        eng.fill_synthetic(a4, 4)
        b4, r4 = torch.empty_like(a4), torch.empty_like(a4)
        kw4 = dict(in_off=torch.from_numpy(offs).cuda(), lens=torch.from_numpy(sizes.astype(np.int32)).cuda())
    main_stream.synchronize()

    calls = {
        "C2_encrypt": lambda: eng.package_encrypt(a, b, P, ks, stride=L, uniform_len=L),
        "C2_decrypt": lambda: eng.package_decrypt(b, r, P, ks, stride=L, uniform_len=L),
        "C4_encrypt": lambda: eng.package_encrypt(a4, b4, n4, ks, **kw4),
        "C4_decrypt": lambda: eng.package_decrypt(b4, r4, n4, ks, **kw4),
    }

    def wall(fn, reps):
        fn()
        main_stream.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            main_stream.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    # warm-up: clocks up, scratch grown
    t_end = time.perf_counter() + 0.5
    while time.perf_counter() < t_end:
        for fn in calls.values():
            fn()
        main_stream.synchronize()

    stop = threading.Event()

    def per_call_loop(lat, ready):
        st = torch.cuda.Stream()
        e = fpnn_amd.Engine(0, stream=st)
        ctx = fpnn_amd.setup_encrypt(bytes(range(32)))
        data = bytes(np.random.default_rng(len(lat)).integers(0, 256, 1024, dtype=np.uint8))
        ivb = bytes(16)
        e.cfb(ctx, False, data, ivb)
        ready.set()
        while not stop.is_set():
            t0 = time.perf_counter()
            e.cfb(ctx, False, data, ivb)
            lat.append(time.perf_counter() - t0)
        e.close()

    def with_servers(n, body):
        stop.clear()
        lats = [[] for _ in range(n)]
        readies = [threading.Event() for _ in range(n)]
        th = [threading.Thread(target=per_call_loop, args=(lats[i], readies[i])) for i in range(n)]
        for t in th:
            t.start()
        for rd in readies:
            rd.wait()
        time.sleep(0.01)
        try:
            out = body()
        finally:
            stop.set()
            for t in th:
                t.join()
        return out, lats

    res = {"what": "batch call wall time (ms, median of reps) with N threads keeping K0s servers busy",
           "rows": []}
    base = {}
    for n in [int(x) for x in args.servers.split(",")]:
        row, lats = with_servers(n, lambda: {k: round(1e3 * wall(fn, args.reps), 3) for k, fn in calls.items()})
        row = {"servers": n, **row}
        if n == 0:
            base = dict(row)
        else:
            row["slowdown_vs_none"] = {k: round(row[k] / base[k], 3) for k in calls if k in base}
            allc = [x for l in lats for x in l]
            row["per_call_us_meanwhile"] = {"n": len(allc), "p50": round(1e6 * np.percentile(allc, 50), 1),
                                            "p99": round(1e6 * np.percentile(allc, 99), 1)} if allc else {}
        res["rows"].append(row)
        print(json.dumps(row), flush=True)

    # per-call latency alone, then during back-to-back C4 encrypt flushes
    def lat_only():
        time.sleep(0.5)
        return None

    _, alone = with_servers(1, lat_only)

    def flushing():
        t_end = time.perf_counter() + 0.5
        k = 0
        while time.perf_counter() < t_end:
            calls["C4_encrypt"]()
            k += 1
        main_stream.synchronize()
        return k

    nflush, during = with_servers(1, flushing)
    q = lambda v: {"n": len(v), "p50": round(1e6 * np.percentile(v, 50), 1),  # noqa: E731
                   "p90": round(1e6 * np.percentile(v, 90), 1), "p99": round(1e6 * np.percentile(v, 99), 1),
                   "max": round(1e6 * max(v), 1)}
    res["per_call_decrypt_us"] = {"alone": q(alone[0]), "during_C4_encrypt_flushes": q(during[0]),
                                  "c4_flushes": nflush, "c4_encrypt_ms": base.get("C4_encrypt")}
    print(json.dumps({"per_call_decrypt_us": res["per_call_decrypt_us"]}), flush=True)
    print(json.dumps({"k0s_interference": res}))


if __name__ == "__main__":
    main()
