#!/bin/bash
# Round-3 session zk: validation of the final round-3 build (smoke, whole GPU suite, bench
# line) and every device config's steady-state medians (tools/bench_configs.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=r03zk NO_CONFIGS=1 bash tools/gpu_validate.sh || exit $?
echo "== configs $(date +%T)"
timeout -k 10 600 python -u tools/bench_configs.py --reps 3 --no-host --configs C2,C3,C4,C5,U1,R1 \
  > gpurun_out/r03zk_configs.log 2>&1 || { tail -5 gpurun_out/r03zk_configs.log; exit 1; }
grep -E '^\{"configs' gpurun_out/r03zk_configs.log | cut -c1-300
