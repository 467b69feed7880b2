#!/bin/bash
# Round-3 session zd: final validation of the round-3 build -- smoke, the whole GPU suite, the
# default bench line -- then every config's steady-state medians (host legs, S1, R2) and the
# ECDH derivation rates with the reference's CPU legs and per-call latency.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=r03zd NO_CONFIGS=1 bash tools/gpu_validate.sh || exit $?
echo "== configs $(date +%T)"
timeout -k 10 900 python -u tools/bench_configs.py --reps 3 --configs C2,C3,C4,C5,U1,R1,R2,S1 > gpurun_out/r03zd_configs.log 2>&1 || { tail -5 gpurun_out/r03zd_configs.log; exit 1; }
grep -E '^\{"configs' gpurun_out/r03zd_configs.log | cut -c1-200
echo "== ecdh $(date +%T)"
timeout -k 10 600 python -u tools/bench_ecdh.py --percall 100 > gpurun_out/r03zd_ecdh.log 2>&1 || { tail -5 gpurun_out/r03zd_ecdh.log; exit 1; }
tail -1 gpurun_out/r03zd_ecdh.log | cut -c1-300
