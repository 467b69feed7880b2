#!/usr/bin/env python3
"""Per-call latency of the drop-in PackageEncryptor (config C1's shape: 10 000 x 1 KiB
frames, AES-256, one call per frame) on the GPU library against the reference's own
Encryptor on one host core (oracle/_ref/percall_ref), plus the same frames through one
EncryptorBatch flush.  Both builds of oracle/percall.cpp print a checksum of all outputs;
they must agree.

  python tools/bench_percall.py [--frames 10000] [--len 1024]
"""
import argparse
import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--len", type=int, default=1024)
    args = ap.parse_args()
    libdir = os.path.join(ROOT, "fpnn_amd")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "percall_gpu")
        subprocess.run(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "oracle", "percall.cpp"), "-o", exe, "-L", libdir, "-lfpnn_aes",
                        f"-Wl,-rpath,{libdir}"], check=True)
        gpu = json.loads(subprocess.run([exe, str(args.frames), str(args.len)], capture_output=True, text=True,
                                        check=True, timeout=600).stdout.strip().splitlines()[-1])
    out = {"metric": "PackageEncryptor per-call latency (us per 1 KiB frame)", "gpu_dropin": gpu}
    ref = os.path.join(ROOT, "oracle", "_ref", "percall_ref")
    if os.path.exists(ref):
        r = json.loads(subprocess.run([ref, str(args.frames), str(args.len)], capture_output=True, text=True,
                                      check=True, timeout=600).stdout.strip().splitlines()[-1])
        out["reference_1core"] = r
        out["checksums_match"] = r["checksum"] == gpu["checksum"]
        out["per_call_slowdown_vs_reference"] = round(gpu["us_per_encrypt"] / r["us_per_encrypt"], 2)
        out["batched_speedup_vs_reference_per_call"] = round(r["us_per_encrypt"] / gpu["us_per_frame_batched"], 2)
    # C1 itself: the reference's SendBuffer + encrypted receivers, encrypted echo over loopback
    # TCP (oracle/io_echo.cpp), on the reference's Encryptor and on the drop-in
    echo = {}
    for name in ("io_echo_ref", "io_echo_dropin"):
        exe = os.path.join(ROOT, "oracle", "_ref", name)
        if not os.path.exists(exe):
            continue
        for mode, kl, win in (("0", "32", "1"), ("0", "32", "64"), ("1", "16", "1")):
            r = subprocess.run([exe, mode, kl, str(args.frames), str(args.len), win], capture_output=True, text=True,
                               timeout=600)
            if r.returncode == 0:
                d = json.loads(r.stdout.strip().splitlines()[-1])
                echo.setdefault(f"{d['mode']}_aes{8 * int(kl)}_window{win}", {})[name] = {
                    k: d[k] for k in ("us_per_echo", "echo_per_s", "answers_ok", "wire_c2s_fnv", "wire_s2c_fnv")}
            else:
                echo.setdefault(f"mode{mode}_window{win}", {})[name] = {"rc": r.returncode, "stderr": r.stderr[-300:]}
    if echo:
        for v in echo.values():
            if "io_echo_ref" in v and "io_echo_dropin" in v and "wire_c2s_fnv" in v["io_echo_ref"]:
                v["wire_matches"] = all(v["io_echo_ref"][k] == v["io_echo_dropin"].get(k)
                                        for k in ("wire_c2s_fnv", "wire_s2c_fnv"))
        out["c1_echo"] = echo
    print(json.dumps(out))


if __name__ == "__main__":
    main()
