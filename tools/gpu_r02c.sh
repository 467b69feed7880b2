#!/bin/bash
# Round-2 session C: K1r v2 parity, then the per-config throughput and profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_parity.py -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/tests_c.log 2>&1 || { tail -20 gpurun_out/tests_c.log; exit 1; }
tail -2 gpurun_out/tests_c.log
timeout -k 10 600 python tools/bench_configs.py --reps 3 --no-host --configs C3,C4,R1 > gpurun_out/configs_c.log 2>&1 || { tail -5 gpurun_out/configs_c.log; exit 1; }
grep -E '^\{' gpurun_out/configs_c.log | tail -1
CFGS="C3 C4 R1" bash tools/profile_configs.sh
