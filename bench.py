#!/usr/bin/env python3
"""bench.py -- AES-256 GiB/s on a device-resident packet batch (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): 1 M x 1 KiB random payloads, AES-256
package mode, one connection key/IV.  One step = encrypt the whole batch (K2,
one lane per packet chain) + decrypt it back (K1d, one lane per 16-byte block),
inputs resident in HBM before timing starts.

value = payload bytes processed by all ranks (P*L encrypted + P*L decrypted per
rank per step) / wall time of K steps (barrier + synchronize on both sides, max over
ranks), in GiB/s -- i.e. the per-direction payload rate of the whole job.

Multi-GPU: one process per GPU (torchrun); rank r encrypts/decrypts packets
[r*P, (r+1)*P) of one global synthetic batch (weak scaling, no data-path collective;
torch.distributed only for the barrier and the max-time reduction).

Also reported: "roofline" for the dominant kernel (algorithmic bytes per launch /
its mean HIP-event duration vs the 8 TB/s HBM peak) and "cpu_baseline" (the
reference's own Encryptor compiled into oracle/_ref, timed on this host's cores).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import workloads as W  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=W.C2["packets"])
    ap.add_argument("--length", type=int, default=W.C2["length"])
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="target wall time of the multi-thread CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--pcie", action="store_true", help="also time pinned H2D + kernels + D2H (for DESIGN.md)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL; default) or gloo (rehearsal)")
    ap.add_argument("--workload", choices=["C2", "C4", "C5"], default="C2",
                    help="C2 = the bench line (default); C4 / C5 = the BASELINE.json sharded configs")
    ap.add_argument("--only", choices=["encrypt", "decrypt"], default=None,
                    help="profiling aid: run one direction only (not a bench line)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())  # == local on a node with one GPU per rank
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(args.dist_backend)
    return world, rank, dev


def sum_over_ranks(value: int, world: int, device=None) -> int:
    if world <= 1:
        return int(value)
    import torch.distributed as dist
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def load_traffic(kernel: str):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_*.json), if any."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(plain_host: np.ndarray, P: int, L: int, key: bytes, iv: bytes, target_s: float, gpu_cipher):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle, ref_available
    kind = "reference" if ref_available() else "port"
    o = Oracle(kind)
    threads = max(1, min(16, os.cpu_count() or 1))
    # calibrate on a small sample, then size the sample (packets x repetitions) to
    # ~target_s of wall time on `threads` threads (target_s * threads s of CPU work)
    n = min(P, 8192)
    tmp = np.empty(n * L, np.uint8)
    out = np.empty(n * L, np.uint8)
    t = o.time_package_roundtrip(plain_host[:n * L], tmp, out, n, L, key, iv, threads, 1)
    want = n * target_s / max(t, 1e-6)
    n = int(min(P, max(n, want)))
    reps = max(1, int(round(want / n)))
    tmp = np.empty(n * L, np.uint8)
    out = np.empty(n * L, np.uint8)
    t = o.time_package_roundtrip(plain_host[:n * L], tmp, out, n, L, key, iv, threads, reps)
    ok = bool(np.array_equal(tmp, gpu_cipher[:n * L])) and bool(np.array_equal(out, plain_host[:n * L]))
    gib = 2.0 * n * L * reps / t / 2**30
    # one core, as SURVEY.md 8(d) asks for both: ~1 s on a prefix of the same batch
    n1 = min(n, 16384)
    t1 = o.time_package_roundtrip(plain_host[:n1 * L], tmp[:n1 * L], out[:n1 * L], n1, L, key, iv, 1, 1)
    n1 = int(min(n, max(n1, n1 * 1.0 / max(t1, 1e-6))))
    t1 = o.time_package_roundtrip(plain_host[:n1 * L], tmp[:n1 * L], out[:n1 * L], n1, L, key, iv, 1, 1)
    src = "oracle/_ref: reference base/rijndael.c + core/Encryptor.cpp (-O2)" if kind == "reference" \
        else "oracle/aes_oracle.c restatement (-O2)"
    return {"value": round(gib, 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"{n} x {L} B packets (first {n} of the C2 batch) x {reps} passes, "
                      f"PackageEncryptor::encrypt then ::decrypt per packet, {threads} threads; {src}; "
                      f"{t:.2f} s wall = {t * threads:.1f} s of CPU work; matches GPU output: {ok}",
            "single_core": {"value": round(2.0 * n1 * L / t1 / 2**30, 4), "cores": 1,
                            "sample": f"first {n1} packets, {t1:.2f} s"},
            "openssl_aesni": openssl_baseline(plain_host, P, L, key, iv, threads, gpu_cipher),
            "cpu_model": _cpu_model()}


def openssl_baseline(plain_host, P, L, key, iv, threads, gpu_cipher, target_s=1.0):
    """The stronger CPU comparator SURVEY.md 8(d) names: the same package-mode work
    through the host's OpenSSL EVP cfb128 (AES-NI) -- oracle/libossl_cfb.so, built by
    `make -C oracle ossl`.  None when it was not built."""
    import ctypes as C
    lib_path = os.path.join(ROOT, "oracle", "libossl_cfb.so")
    if not os.path.exists(lib_path):
        return None
    lib = C.CDLL(lib_path)
    f = lib.ossl_time_package_roundtrip
    u8 = C.POINTER(C.c_uint8)
    f.argtypes = [u8, u8, u8, C.c_uint32, C.c_uint32, C.c_char_p, C.c_size_t, C.c_char_p, C.c_int, C.c_int]
    f.restype = C.c_double
    ptr = lambda a: a.ctypes.data_as(u8)  # noqa: E731
    n = min(P, 65536)
    tmp, out = np.empty(n * L, np.uint8), np.empty(n * L, np.uint8)
    t = f(ptr(plain_host), ptr(tmp), ptr(out), n, L, key, len(key), iv, threads, 1)
    if t <= 0:
        return None
    n = int(min(P, max(n, n * target_s / t)))
    tmp, out = np.empty(n * L, np.uint8), np.empty(n * L, np.uint8)
    t = f(ptr(plain_host), ptr(tmp), ptr(out), n, L, key, len(key), iv, threads, 1)
    ok = bool(np.array_equal(tmp, gpu_cipher[:n * L])) and bool(np.array_equal(out, plain_host[:n * L]))
    return {"value": round(2.0 * n * L / t / 2**30, 3), "unit": "GiB/s", "cores": threads,
            "sample": f"{n} x {L} B packets, EVP_aes_256_cfb128 encrypt then decrypt per packet (IV reset per "
                      f"packet), {threads} threads, {t:.2f} s; matches GPU output: {ok}"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pcie_rate(eng, ks, P, L, steps=3):
    """Pinned host buffers -> H2D -> encrypt -> D2H (and the reverse for decrypt)."""
    n = P * L
    h_in = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(d_in, 2)
    h_in.copy_(d_in)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        d_in.copy_(h_in, non_blocking=True)
        eng.package_encrypt(d_in, d_out, P, ks, stride=L, uniform_len=L)
        h_out.copy_(d_out, non_blocking=True)
        d_in.copy_(h_out, non_blocking=True)
        eng.package_decrypt(d_in, d_out, P, ks, stride=L, uniform_len=L)
        h_out.copy_(d_out, non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = torch.equal(h_out, h_in)
    return {"value": round(2.0 * n * steps / dt / 2**30, 3), "unit": "GiB/s",
            "note": "host pinned -> H2D -> kernel -> D2H per direction, serialized on one stream", "roundtrip_ok": ok}


def setup_c2(args, eng, world, rank):
    """C2 (the bench line): P x L uniform packets per rank, one key; weak scaling."""
    import fpnn_amd
    from fpnn_amd.sharding import shard_range
    P, L = args.packets, args.length
    cfg = W.C2
    key, iv = W.single_key(cfg)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    # the global batch is world * P packets; this rank owns a contiguous packet range
    # of it (no collective on the data path)
    first, last = shard_range(P * world, world, rank)
    assert last - first == P
    plain = torch.empty(P * L, dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(plain, cfg["payload_seed"], byte_offset=first * L)
    kw = dict(stride=L, uniform_len=L)
    desc = {"workload": "C2: 1M x 1 KiB AES-256 package-mode CFB encrypt+decrypt per GPU",
            "packets_per_gpu": P, "payload_bytes": L, "key_bits": 256, "mode": "package",
            "global_packets": P * world, "parallelism": f"packet-shard x{world}"}
    digest = "C2" if (world == 1 and P == cfg["packets"] and L == cfg["length"]) else None
    return dict(plain=plain, ks=ks, kw=kw, P=P, nkeys=1, scaling="weak", config=desc, digest=digest,
                data="synthetic (counter splitmix64 payload, seed 2; key/IV from seed 1002)",
                key=key, iv=iv, L=L, uniform=True)


def setup_c4(args, eng, world, rank):
    """C4: one global Zipf batch (64 B - 64 KiB, 4 GiB), byte-balanced contiguous packet
    ranges per rank; strong scaling (the global batch is fixed)."""
    import fpnn_amd
    from fpnn_amd.sharding import shard_range
    cfg = W.C4
    sizes = W.zipf_sizes(cfg).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.int64)
    first, last = shard_range(len(sizes), world, rank, sizes)
    lo = int(offs[first])
    nbytes = int(offs[last - 1] + sizes[last - 1] - lo) if last > first else 0
    key, iv = W.single_key(cfg)
    ks = fpnn_amd.KeySet(eng, key, len(key), iv)
    plain = torch.empty(max(1, nbytes), dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(plain[:nbytes], cfg["payload_seed"], byte_offset=lo, nbytes=nbytes)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda")  # noqa: E731
    kw = dict(in_off=d(offs[first:last] - lo), lens=d(sizes[first:last].astype(np.int32)))
    desc = {"workload": "C4: Zipf(1.1) 64 B-64 KiB packets, 4 GiB global, AES-256 package-mode encrypt+decrypt",
            "packets_this_rank": last - first, "global_packets": len(sizes), "global_bytes": int(sizes.sum()),
            "key_bits": 256, "mode": "package", "parallelism": f"byte-balanced packet-shard x{world}"}
    return dict(plain=plain[:nbytes], ks=ks, kw=kw, P=last - first, nkeys=1, scaling="strong", config=desc,
                digest=None, data="synthetic (splitmix64 payload seed 4, Zipf sizes seed 4004, key/IV seed 1004)",
                key=key, iv=iv, L=None, uniform=False)


def setup_c5(args, eng, world, rank):
    """C5: 65 536 packets x 4 KiB, each with its own key and IV; the key table is
    replicated, packets split evenly (8 GPUs x 8 192 keys); strong scaling."""
    import fpnn_amd
    from fpnn_amd.sharding import shard_range
    cfg = W.C5
    Pg, L = cfg["packets"], cfg["length"]
    keys, ivs = W.many_keys(cfg)
    ks = fpnn_amd.KeySet(eng, keys.tobytes(), cfg["keylen"], ivs.tobytes())
    first, last = shard_range(Pg, world, rank)
    P = last - first
    plain = torch.empty(max(1, P * L), dtype=torch.uint8, device="cuda")
    eng.fill_synthetic(plain[:P * L], cfg["payload_seed"], byte_offset=first * L, nbytes=P * L)
    slots = torch.arange(first, last, dtype=torch.int32, device="cuda")
    kw = dict(stride=L, uniform_len=L, key_slot=slots)
    desc = {"workload": "C5: 65536 keys x 4 KiB AES-256 package-mode encrypt+decrypt, per-key IV",
            "packets_this_rank": P, "global_packets": Pg, "payload_bytes": L, "key_bits": 256, "mode": "package",
            "parallelism": f"packet-shard x{world} (key table replicated)"}
    digest = "C5" if world == 1 else None
    return dict(plain=plain[:P * L], ks=ks, kw=kw, P=P, nkeys=Pg, scaling="strong", config=desc, digest=digest,
                data="synthetic (splitmix64 payload seed 5; keys/IVs seed 1005)", key=None, iv=None, L=L,
                uniform=False)


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    import fpnn_amd
    from fpnn_amd.sharding import max_over_ranks

    eng = fpnn_amd.Engine(local)  # queues on torch's current stream of this device
    job = {"C2": setup_c2, "C4": setup_c4, "C5": setup_c5}[args.workload](args, eng, world, rank)
    plain, ks, kw, P = job["plain"], job["ks"], job["kw"], job["P"]
    nbytes = plain.numel()
    cipher = torch.empty_like(plain)
    back = torch.empty_like(plain)

    def step():
        if args.only != "decrypt":
            eng.package_encrypt(plain, cipher, P, ks, **kw)
        if args.only != "encrypt":
            eng.package_decrypt(cipher, back, P, ks, **kw)

    if args.only == "decrypt":
        eng.package_encrypt(plain, cipher, P, ks, **kw)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    eng.reset_stats()
    eng.set_timing(True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    elapsed = max_over_ranks(elapsed, world, "cuda" if args.dist_backend == "nccl" else None)
    n_enc, ms_enc = eng.kernel_stats(fpnn_amd.K_ENCRYPT)
    n_dec, ms_dec = eng.kernel_stats(fpnn_amd.K_DECRYPT)
    total_bytes = sum_over_ranks(nbytes, world, "cuda" if args.dist_backend == "nccl" else None)

    verify = {}
    if not args.no_verify:
        if args.only is None:
            verify["roundtrip_ok"] = bool(torch.equal(back, plain))
        if rank == 0 and job["digest"]:
            with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
                gold = json.load(f)[job["digest"]]
            verify["cipher_sha256_matches_reference"] = \
                hashlib.sha256(cipher.cpu().numpy()).hexdigest() == gold["cipher_sha256"]

    directions = 2 if args.only is None else 1
    payload = float(directions) * total_bytes * args.steps
    value = payload / elapsed / 2**30

    # roofline for the dominant kernel: algorithmic bytes per launch
    alg_bytes = 2.0 * nbytes + 28.0 * P + 244.0 * job["nkeys"]
    kernels = {}
    names = {"C2": ("cfb_encrypt_chains", "cfb_decrypt_dense"), "C4": ("cfb_encrypt_queue", "cfb_decrypt_blocks"),
             "C5": ("cfb_encrypt_coop", "cfb_decrypt_dense")}[args.workload]
    for name, n, ms in ((names[0], n_enc, ms_enc), (names[1], n_dec, ms_dec)):
        if n:
            avg_s = ms / n / 1e3
            ach = alg_bytes / avg_s / 1e9
            kernels[name] = {"launches": n, "avg_ms": round(ms / n, 4), "achieved_GBs": round(ach, 1),
                             "payload_GiBs": round(nbytes / avg_s / 2**30, 2)}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    ach = kernels[dom]["achieved_GBs"]
    traffic = load_traffic(dom) if args.workload == "C2" else None  # the committed PMC summary is of C2
    roofline = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
                "alg_bytes_per_launch": int(alg_bytes), "kernels": kernels}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and job["uniform"]:
        host_plain = plain.cpu().numpy()
        cpu = cpu_baseline(host_plain, P, job["L"], job["key"], job["iv"], args.cpu_seconds, cipher.cpu().numpy())

    extra = {}
    if args.pcie and rank == 0 and job["uniform"]:
        extra["pcie_inclusive"] = pcie_rate(eng, ks, P, job["L"])

    if rank == 0:
        line = {
            "metric": "AES-256 GiB/s on device-resident packet batch",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": job["scaling"],
            "vs_baseline": None,
            "dtype": "u8",
            "data": job["data"],
            "config": job["config"],
            "roofline": roofline,
            "cpu_baseline": cpu,
            "verify": verify,
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
