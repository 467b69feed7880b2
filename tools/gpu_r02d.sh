#!/bin/bash
# K1r iteration: parity, configs, one PMC profile (CFGS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/tests_d.log 2>&1 || { tail -30 gpurun_out/tests_d.log; exit 1; }
tail -2 gpurun_out/tests_d.log
timeout -k 10 600 python tools/bench_configs.py --reps 3 --no-host --configs ${CONFIGS:-C3,C4,R1} > gpurun_out/configs_d.log 2>&1 || { tail -5 gpurun_out/configs_d.log; exit 1; }
grep -E '^\{"configs' gpurun_out/configs_d.log
[ -n "$CFGS" ] && TAG=${TAG:-r02d} bash tools/profile_configs.sh
exit 0
