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
# LDS: ds_read_b32 serves a wave's 64 lanes in 2 LDS cycles = 32 T-table lookups per clock
# per CU (MI355X_MICROARCH.md, LDS table); the clock is the kernel's effective one from PMC
LDS_PEAK_LOOKUPS = 32
NOMINAL_CLOCK_GHZ = 2.4
METRIC = "AES-256 GiB/s on device-resident packet batch; 1/2/4/8-GPU scaling"  # BASELINE.json "metric"
# newest committed PMC summary of the bench command (tools/pmc_summary.py output), per workload
# (C2: this bench command under the PMC passes, `tools/gpu.sh <tag> bench_pmc`; C4 / C5:
# `tools/gpu.sh <tag> prof:C4` -- the same kernels on the same batches through tools/bench_configs.py)
PMC_SUMMARIES = {"C2": ["profiles/r06/bench/pmc_summary.json", "profiles/r05/bench/pmc_summary.json"],
                 "C4": ["profiles/r04/C4/pmc_summary.json"], "C5": ["profiles/r05/C5/pmc_summary.json"]}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 150 C2 steps = 0.3 s of load before the timed steps: the chip needs tens of ms of work
    # to reach its clock (profiles/r04/timers.json: 5 warm-up steps read 3-4 % low)
    ap.add_argument("--warmup", type=int, default=150)
    ap.add_argument("--packets", type=int, default=W.C2["packets"])
    ap.add_argument("--length", type=int, default=W.C2["length"])
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="target wall time of the multi-thread CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--pcie", action="store_true", help="also time pinned H2D + kernels + D2H (for DESIGN.md)")
    ap.add_argument("--dist-backend", default="auto",
                    help="auto (RCCL when every local rank has a GPU of its own, else gloo: RCCL refuses two ranks "
                         "on one device), nccl or gloo")
    ap.add_argument("--workload", choices=["C2", "C4", "C5"], default="C2",
                    help="C2 = the bench line (default); C4 / C5 = the BASELINE.json sharded configs")
    ap.add_argument("--only", choices=["encrypt", "decrypt"], default=None,
                    help="profiling aid: run one direction only (not a bench line)")
    ap.add_argument("--plumbing-only", action="store_true",
                    help="CPU rehearsal of the multi-rank launch/reduction/verify contract (no GPU work)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base=None):
    """Environment of each of the n rank processes of a one-node job (what torchrun
    would set): RANK = LOCAL_RANK = r, WORLD_SIZE = LOCAL_WORLD_SIZE = n, rendezvous on
    127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(argv, n: int) -> int:
    """`bench.py --gpus N` started without a launcher: start the N rank processes here
    (children of this process, before anything touches the GPU) and return the job's
    exit code -- the first non-zero rank code, or 0.  Rank 0 prints the JSON line."""
    import signal
    import subprocess
    envs = rank_envs(n, _free_port())
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + list(argv)
    procs = [subprocess.Popen(cmd, env=e) for e in envs]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # one rank failed: the others would wait forever in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU is required")
    ndev = max(1, torch.cuda.device_count())  # (counting devices does not initialise the GPU)
    dev = local % ndev  # == local on a node with one GPU per rank
    if args.dist_backend == "auto":
        # the data path has no collective; torch.distributed carries only the barrier and the
        # reductions of the timing, so ranks that share a device (a rehearsal) take gloo
        args.dist_backend = "nccl" if int(os.environ.get("LOCAL_WORLD_SIZE", str(world))) <= ndev else "gloo"
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


def load_pmc(kernel: str, workload: str):
    """The newest committed PMC summary (tools/pmc_summary.py) of this workload's bench
    command that holds `kernel`: (its per-kernel record, the file), or (None, None)."""
    for path in PMC_SUMMARIES.get(workload, []):
        try:
            with open(os.path.join(ROOT, path)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        entry = d.get(kernel)
        if entry and entry.get("hbm_bytes_per_launch") is not None:
            rec = dict(d.get("kernels", {}).get(entry.get("variant"), {}))
            rec["hbm_bytes_per_launch"] = entry["hbm_bytes_per_launch"]
            return rec, path
    return None, None


def lds_roofline(avg_s: float, lookups: int, num_cus: int, pmc, pmc_path) -> dict:
    """The LDS side of the dominant kernel: T-table lookups per clock per CU against the
    32/clk/CU ds_read_b32 peak, and the LDS-array busy fraction (SQ_LDS_IDX_ACTIVE per CU over
    active cycles).  Clocks come from the committed PMC summary of this command (the same
    kernel on the same batch): its GRBM_GUI_ACTIVE cycles per launch give lookups per cycle,
    and those cycles over this run's HIP-event time give the clock this run implies.  With no
    summary the live rate is priced at the nominal 2.4 GHz."""
    grbm = ((pmc or {}).get("counters_avg_per_dispatch") or {}).get("GRBM_GUI_ACTIVE")
    live_nominal = lookups / avg_s / num_cus / (NOMINAL_CLOCK_GHZ * 1e9)
    out = {"bound": "lds", "peak": LDS_PEAK_LOOKUPS, "unit": "lookups/clk/CU", "lookups_per_launch": lookups,
           "lookups_formula": "NR * 16 per block ciphered: decrypt kernels every 16-B block (block 0's "
                              "keystream E_k(IV) included), encrypt kernels every block but each packet's "
                              "first (the key set's precomputed E_k(IV))",
           "num_cus": num_cus, "frac_at_nominal_clock": round(live_nominal / LDS_PEAK_LOOKUPS, 4)}
    if grbm:
        cycles = grbm / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs
        per_clk = lookups / cycles / num_cus
        out.update({"achieved": round(per_clk, 2), "frac": round(per_clk / LDS_PEAK_LOOKUPS, 4),
                    "cycles_per_launch": round(cycles), "effective_clock_GHz": round(cycles / avg_s / 1e9, 3),
                    "pmc_run_clock_GHz": pmc.get("effective_clock_GHz"),
                    "lds_array_busy_frac": pmc.get("lds_array_busy_frac"), "source": pmc_path})
    else:
        out.update({"achieved": round(live_nominal, 2), "frac": round(live_nominal / LDS_PEAK_LOOKUPS, 4),
                    "effective_clock_GHz": None, "lds_array_busy_frac": None,
                    "source": f"nominal {NOMINAL_CLOCK_GHZ} GHz (no PMC summary of this kernel)"})
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """(threads this process may run on, cgroup CPU quota or None, physical cores or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    cores = None
    try:
        seen = set()
        phys = core = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                    seen.add((phys, core))
        cores = len(seen) or None
    except OSError:
        pass
    return aff, quota, cores


def _timed_legs(run, n0: int, P: int, thread_counts, target_s: float):
    """run(n, threads) -> seconds for n packets.  Per thread count: calibrate on n0
    packets, then time a sample sized to ~target_s of wall time (bounded by P)."""
    legs = {}
    for th in thread_counts:
        n = min(P, n0 * max(1, th))
        t = run(n, th)
        n = int(min(P, max(n, n * target_s / max(t, 1e-6))))
        t = run(n, th)
        legs[th] = (n, t)
    return legs


def cpu_baseline(plain_host: np.ndarray, P: int, L: int, key: bytes, iv: bytes, target_s: float, gpu_cipher):
    """The reference's own PackageEncryptor (oracle/_ref, or the restatement where it was
    not built) on 1 core, 16 threads and every CPU this process may use; value = all CPUs."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle, ref_available
    kind = "reference" if ref_available() else "port"
    o = Oracle(kind)
    aff, quota, phys = host_cpus()
    counts = sorted({1, min(16, aff), aff})
    tmp = np.empty(P * L, np.uint8)
    out = np.empty(P * L, np.uint8)

    def run(n, th):
        return o.time_package_roundtrip(plain_host[:n * L], tmp[:n * L], out[:n * L], n, L, key, iv, th, 1)

    legs = _timed_legs(run, 512, P, counts, target_s)
    gib = {th: 2.0 * n * L / t / 2**30 for th, (n, t) in legs.items()}
    best = max(counts, key=lambda th: gib[th])  # a cgroup CPU quota can make "every CPU" the slower leg
    n_b, t_b = legs[best]
    ok = bool(np.array_equal(tmp[:n_b * L], gpu_cipher[:n_b * L])) and \
        bool(np.array_equal(out[:n_b * L], plain_host[:n_b * L]))
    src = "oracle/_ref: reference base/rijndael.c + core/Encryptor.cpp (-O2)" if kind == "reference" \
        else "oracle/aes_oracle.c restatement (-O2)"
    quota_note = (f"; this process may use {quota:g} CPUs (cgroup cpu.max) of the host's {aff} hardware threads, "
                  f"so legs above {int(quota)} threads are throttled") if quota else ""
    res = {"value": round(gib[best], 4), "unit": "GiB/s", "cores": best, "kind": kind,
           "sample": f"{n_b} x {L} B packets (first {n_b} of the C2 batch), PackageEncryptor::encrypt then "
                     f"::decrypt per packet, {best} threads (the fastest of the 1 / 16 / all-CPU legs){quota_note}; "
                     f"{src}; {t_b:.2f} s wall; matches GPU output: {ok}",
           "legs": {str(th): {"value": round(gib[th], 4), "threads": th, "packets": legs[th][0],
                              "seconds": round(legs[th][1], 3)} for th in counts},
           "host": {"affinity_cpus": aff, "nproc": os.cpu_count(), "cgroup_cpu_quota": quota,
                    "physical_cores": phys, "cpu_model": _cpu_model()},
           "openssl_aesni": openssl_baseline(plain_host, P, L, key, iv, counts, gpu_cipher, target_s)}
    if phys:
        res["whole_host_projection"] = {
            "value": round(gib[1] * phys, 2), "unit": "GiB/s", "cores": phys,
            "note": "NOT measured: the 1-core rate x the host's physical cores (linear scaling assumed), for "
                    "comparison with a host that gives the reference every core"}
    return res


def openssl_baseline(plain_host, P, L, key, iv, counts, gpu_cipher, target_s=1.0):
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
    tmp, out = np.empty(P * L, np.uint8), np.empty(P * L, np.uint8)

    def run(n, th):
        return f(ptr(plain_host), ptr(tmp), ptr(out), n, L, key, len(key), iv, th, 1)

    if run(min(P, 1024), 1) <= 0:
        return None
    legs = _timed_legs(run, 1024, P, counts, target_s)
    gib = {th: 2.0 * legs[th][0] * L / legs[th][1] / 2**30 for th in counts}
    top = max(counts, key=lambda th: gib[th])
    n, t = legs[top]
    ok = bool(np.array_equal(tmp[:n * L], gpu_cipher[:n * L])) and bool(np.array_equal(out[:n * L], plain_host[:n * L]))
    return {"value": round(gib[top], 3), "unit": "GiB/s", "cores": top,
            "sample": f"{n} x {L} B packets, EVP_aes_256_cfb128 encrypt then decrypt per packet (IV reset per "
                      f"packet), {top} threads (fastest leg), {t:.2f} s; matches GPU output: {ok}",
            "legs": {str(th): {"value": round(gib[th], 3), "threads": th, "packets": legs[th][0],
                               "seconds": round(legs[th][1], 3)} for th in counts}}


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
    return dict(plain=plain, ks=ks, kw=kw, P=P, nkeys=1, scaling="weak", config=desc, blocks=P * ((L + 15) // 16),
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
                blocks=int(((sizes[first:last] + 15) // 16).sum()),
                data="synthetic (splitmix64 payload seed 4, Zipf sizes seed 4004, key/IV seed 1004)",
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
    return dict(plain=plain[:P * L], ks=ks, kw=kw, P=P, nkeys=Pg, scaling="strong", config=desc,
                blocks=P * ((L + 15) // 16),
                data="synthetic (splitmix64 payload seed 5; keys/IVs seed 1005)", key=None, iv=None, L=L,
                uniform=False)


def shard_key(workload: str, world: int, rank: int, P: int, L) -> str:
    """Key of this rank's reference digest in tests/golden/digests.json "shards"
    (oracle/gen_golden.py shard_digests)."""
    if workload == "C2":
        return f"C2/r{rank}" if (P, L) == (W.C2["packets"], W.C2["length"]) else ""
    return f"{workload}/w{world}/r{rank}"


def verify_rank(args, job, cipher, back, plain, world, rank) -> dict:
    v = {"rank": rank}
    if args.only is None:
        v["roundtrip_ok"] = bool(torch.equal(back, plain))
    key = shard_key(args.workload, world, rank, job["P"], job["L"])
    try:
        with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
            gold = json.load(f).get("shards", {}).get(key)
    except (OSError, ValueError):
        gold = None
    if gold:
        v["shard"] = key
        v["cipher_sha256_matches_reference"] = hashlib.sha256(cipher.cpu().numpy()).hexdigest() == gold
    return v


def gather_objects(obj, world):
    if world <= 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def alg_bytes_per_launch(nbytes: int, P: int, kw: dict, nkeys: int) -> int:
    """Algorithmic HBM bytes of one encrypt or decrypt launch (counting only
    what the call reads): payload in + out, the descriptor arrays actually passed
    (in_off/out_off u64, len/key_slot u32 per packet) and the key records (272 B each:
    round keys + IV)."""
    per_packet = sum(sz for name, sz in (("in_off", 8), ("out_off", 8), ("lens", 4), ("key_slot", 4))
                     if kw.get(name) is not None)
    return int(2 * nbytes + per_packet * P + 272 * nkeys)


def plumbing_only(args, world, rank):
    """CPU rehearsal of the multi-rank contract (tests/test_bench_launcher.py): the
    launcher's world/rank environment, the barrier, max-over-ranks time and the
    per-rank verify gather, with no GPU work."""
    from fpnn_amd.sharding import max_over_ranks, shard_range
    barrier(world)
    t0 = time.perf_counter()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0 + 0.001 * rank, world)
    first, last = shard_range(W.C2["packets"] * world, world, rank)
    ranks = gather_objects({"rank": rank, "world": world, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                            "packets": [first, last], "shard": shard_key("C2", world, rank, W.C2["packets"],
                                                                          W.C2["length"])}, world)
    if rank == 0:
        print(json.dumps({"plumbing_only": True, "n_gpus": world, "elapsed_max": elapsed, "ranks": ranks}),
              flush=True)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if args.plumbing_only:
        world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
        if world != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        plumbing_only(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
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
    dev = "cuda" if args.dist_backend == "nccl" else None
    elapsed = max_over_ranks(elapsed, world, dev)
    n_enc, ms_enc = eng.kernel_stats(fpnn_amd.K_ENCRYPT)
    n_dec, ms_dec = eng.kernel_stats(fpnn_amd.K_DECRYPT)
    names = (eng.last_kernel(fpnn_amd.K_ENCRYPT), eng.last_kernel(fpnn_amd.K_DECRYPT))
    total_bytes = sum_over_ranks(nbytes, world, dev)

    verify = None
    if not args.no_verify:
        ranks = gather_objects(verify_rank(args, job, cipher, back, plain, world, rank), world)
        verify = {"all_ok": all(all(v for k, v in r.items() if k.endswith("_ok") or k.startswith("cipher_"))
                                for r in ranks),
                  "every_rank_checked_against_reference": all("cipher_sha256_matches_reference" in r for r in ranks),
                  "ranks": ranks}

    directions = 2 if args.only is None else 1
    payload = float(directions) * total_bytes * args.steps
    value = payload / elapsed / 2**30

    # roofline for the dominant kernel: algorithmic bytes per launch
    alg_bytes = alg_bytes_per_launch(nbytes, P, kw, job["nkeys"])
    kernels = {}
    for name, n, ms in ((names[0], n_enc, ms_enc), (names[1], n_dec, ms_dec)):
        if n:
            avg_s = ms / n / 1e3
            ach = alg_bytes / avg_s / 1e9
            kernels[name] = {"launches": n, "avg_ms": round(ms / n, 4), "achieved_GBs": round(ach, 1),
                             "payload_GiBs": round(nbytes / avg_s / 2**30, 2)}
    dom = max(kernels, key=lambda k: kernels[k]["avg_ms"])
    ach = kernels[dom]["achieved_GBs"]
    pmc, pmc_src = load_pmc(dom, args.workload)
    avg_s = kernels[dom]["avg_ms"] / 1e3
    # SURVEY.md 8(d)'s 28*P term prices descriptor arrays; alg_bytes counts only the arrays
    # the call passes (C2 passes none: stride + uniform length, the kernels read none)
    desc_term = 28 * P
    with_desc = alg_bytes + (0 if kw.get("in_off") is not None else desc_term)
    roofline = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None, "traffic_source": pmc_src,
                "kernel": dom, "alg_bytes_per_launch": alg_bytes,
                "alg_bytes_formula": "2*payload + descriptor arrays passed per packet + 272*keys",
                "descriptor_28P": {"counted": kw.get("in_off") is not None, "bytes": desc_term,
                                   "frac_if_counted": round(with_desc / avg_s / 1e9 / HBM_PEAK_GBS, 4)},
                "lds": lds_roofline(avg_s, (job["blocks"] - (0 if "decrypt" in dom else P)) * ks.nrounds * 16,
                                    torch.cuda.get_device_properties(local).multi_processor_count, pmc, pmc_src),
                "kernels": kernels}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and job["uniform"]:
        host_plain = plain.cpu().numpy()
        cpu = cpu_baseline(host_plain, P, job["L"], job["key"], job["iv"], args.cpu_seconds, cipher.cpu().numpy())

    extra = {}
    if args.pcie and rank == 0 and job["uniform"]:
        extra["pcie_inclusive"] = pcie_rate(eng, ks, P, job["L"])

    if rank == 0:
        line = {
            "metric": METRIC,
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
