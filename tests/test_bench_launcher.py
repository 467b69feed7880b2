"""bench.py's multi-rank contract on CPU: `--gpus N` without a launcher starts N rank
processes itself (world/rank/rendezvous environment as torchrun sets it), a WORLD_SIZE
that disagrees with --gpus is refused, and the barrier / max-over-ranks / per-rank verify
gather run over a real gloo group (--plumbing-only: no GPU work)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _env_without_dist():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["PYTHONUNBUFFERED"] = "1"
    return env


def test_rank_envs_match_torchrun_layout():
    import bench
    envs = bench.rank_envs(4, 29555, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555" for e in envs)
    assert all(e["PATH"] == "/bin" for e in envs)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_ranks(n):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--plumbing-only"],
                         env=_env_without_dist(), capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(n))
    assert [r["local_rank"] for r in ranks] == list(range(n))
    assert all(r["world"] == n for r in ranks)
    # weak-scaling C2 shards tile the global batch, and each names its own reference digest
    P = 1 << 20
    assert [tuple(r["packets"]) for r in ranks] == [(i * P, (i + 1) * P) for i in range(n)]
    assert [r["shard"] for r in ranks] == [f"C2/r{i}" for i in range(n)]
    assert d["elapsed_max"] >= 0.001 * (n - 1)  # the max over ranks, not rank 0's time


def test_world_size_mismatch_refused():
    env = _env_without_dist()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--plumbing-only"],
                         env=env, capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


def test_shard_digests_cover_every_rank():
    """tests/golden/digests.json holds a reference digest for every rank the bench can run."""
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        shards = json.load(f)["shards"]
    import bench
    for r in range(8):
        assert bench.shard_key("C2", 8, r, 1 << 20, 1024) in shards
    for w in (1, 2, 4, 8):
        for r in range(w):
            assert bench.shard_key("C4", w, r, 0, None) in shards
            assert bench.shard_key("C5", w, r, 0, 4096) in shards
    # rank 0 of the weak-scaling C2 batch is the single-GPU batch
    with open(os.path.join(ROOT, "tests", "golden", "digests.json")) as f:
        d = json.load(f)
    assert shards["C2/r0"] == d["C2"]["cipher_sha256"]
    assert shards["C5/w1/r0"] == d["C5"]["cipher_sha256"]


def test_cpu_baseline_leg_runs_on_cpu():
    """bench.cpu_baseline end to end on a small sample (the leg the GPU bench runs on rank 0):
    every field of the JSON object is produced and the CPU output is checked against the
    expected ciphertext (here the oracle's, standing in for the GPU's)."""
    import numpy as np
    import bench
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle
    P, L = 256, 1024
    rng = np.random.default_rng(5)
    plain = rng.integers(0, 256, P * L, dtype=np.uint8)
    key, iv = bytes(range(32)), bytes(range(16))
    expect = np.empty_like(plain)
    o = Oracle("port")
    o.package_batch(True, plain, expect, P, in_off=np.arange(P, dtype=np.uint64) * L,
                    lens=np.full(P, L, np.uint32), key_slot=np.zeros(P, np.uint32), keys=np.frombuffer(key, np.uint8),
                    keylen=32, ivs=np.frombuffer(iv, np.uint8), threads=4)
    res = bench.cpu_baseline(plain, P, L, key, iv, 0.05, expect)
    assert res["value"] > 0 and res["cores"] >= 1 and res["kind"] in ("reference", "port")
    assert "matches GPU output: True" in res["sample"]
    assert res["host"]["cpu_model"] and res["host"]["affinity_cpus"] >= 1
    json.dumps(res)
