#!/bin/bash
# Round-3 session y: validation of the build with the new K2h defaults -- smoke, the whole GPU
# suite, the bench line -- then every config's steady-state medians with the host legs (S1
# included) and the C4 K2h profile (trace + PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=r03y NO_CONFIGS=1 bash tools/gpu_validate.sh || exit $?
echo "== configs $(date +%T)"
timeout -k 10 900 python -u tools/bench_configs.py --reps 3 --configs C2,C3,C4,C5,U1,R1,S1 > gpurun_out/r03y_configs.log 2>&1 || { tail -5 gpurun_out/r03y_configs.log; exit 1; }
grep -E '^\{"configs' gpurun_out/r03y_configs.log | cut -c1-200
TAG=r03y CFGS="C4" bash tools/profile_configs.sh
