#!/usr/bin/env python3
"""Echoes/s through FPNN's own IO plumbing with many connections (oracle/io_multi.cpp):
the reference build (CPU cipher per frame) and the batched build (INTEGRATION.md 2a applied,
one EncryptorBatch flush per loop cycle and direction) on the same box, same configs,
alternating; both must carry identical wire bytes (tests/golden/multi_cases.json).
Prints one JSON line per run and a summary line.  VERDICT r04 item 3 asks for this pair.

usage: python tools/bench_io_multi.py [--reps 2] [--cases M1,M4] [--threads 1,4] [--dropin]
"""
import argparse
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")


def run(exe, c, threads, timeout=900):
    args = [os.path.join(REF, exe), "1" if c["mode"] == "stream" else "0", str(c["keylen"]), str(c["conns"]),
            str(c["quests_per_conn"]), str(c["payload"]), str(c["window"]), str(threads)]
    out = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    if out.returncode != 0:
        raise SystemExit(f"{exe} failed ({out.returncode}): {out.stderr[-2000:]}")
    d = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("wire_c2s_fnv", "wire_s2c_fnv"):
        if d[k] != c[k]:
            raise SystemExit(f"{exe} {c['name']}: {k} {d[k]} != reference {c[k]}")
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--cases", default="M1,M4")
    ap.add_argument("--threads", default="1,4")
    ap.add_argument("--dropin", action="store_true", help="also the unchanged drop-in (one GPU call per frame)")
    args = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "multi_cases.json")) as f:
        cases = {c["name"]: c for c in json.load(f)["cases"]}
    summary = []
    for name in args.cases.split(","):
        c = cases[name]
        for thr in (int(t) for t in args.threads.split(",")):
            best = {}
            builds = ["io_multi_ref", "io_multi_batched"] + (["io_multi_dropin"] if args.dropin else [])
            for _ in range(args.reps):
                for exe in builds:
                    d = run(exe, c, thr)
                    print(json.dumps({"case": name, **d}), flush=True)
                    best[exe] = max(best.get(exe, 0.0), d["echo_per_s"])
            row = {"case": name, "mode": c["mode"], "keylen": c["keylen"], "conns": c["conns"],
                   "window": c["window"], "payload": c["payload"], "threads": thr,
                   "reference_echo_per_s": best["io_multi_ref"], "batched_echo_per_s": best["io_multi_batched"],
                   "batched_over_reference": round(best["io_multi_batched"] / best["io_multi_ref"], 3)}
            if args.dropin:
                row["dropin_echo_per_s"] = best["io_multi_dropin"]
            summary.append(row)
    print(json.dumps({"io_multi": summary, "timing": f"best of {args.reps} alternating runs per build; "
                      "wire bytes of every run equal the reference build's"}))


if __name__ == "__main__":
    main()
