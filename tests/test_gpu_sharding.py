"""Row (e) on the GPU: the sharded configs through bench.py's own rank launcher.

`bench.py --gpus N` starts N rank processes (RANK = LOCAL_RANK = r, rendezvous on
127.0.0.1, before anything touches the GPU); on a one-GPU box every rank shares device 0
(LOCAL_RANK % device_count), so the sharding, the per-rank batches and the max-over-ranks
timing run exactly as on an 8-GPU node, over gloo.  Each rank encrypts its own contiguous
shard of the global C4 / C5 batch and checks the ciphertext against the reference's
digest for that shard (tests/golden/digests.json "shards", made through oracle/_ref by
oracle/gen_golden.py); the line must report every rank checked and matching.  World 8 is
the driver's 8-GPU layout rehearsed on one card (8 rank processes, within the box's limit
of 16 processes on the GPU).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("workload,world", [("C4", 2), ("C5", 2), ("C4", 4), ("C5", 4), ("C4", 8), ("C5", 8)])
def test_sharded_config_every_rank_matches_reference(workload, world):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--workload", workload,
           "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    # C4 / C5 split one fixed global batch over the ranks (bench.py: strong scaling)
    assert d["n_gpus"] == world and d["scaling"] == "strong"
    v = d["verify"]
    assert v["every_rank_checked_against_reference"], v
    ranks = sorted(v["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(world))
    assert [r["shard"] for r in ranks] == [f"{workload}/w{world}/r{i}" for i in range(world)]
    assert all(r["cipher_sha256_matches_reference"] for r in ranks), ranks
    assert all(r["roundtrip_ok"] for r in ranks), ranks
    assert v["all_ok"]
