#!/bin/bash
# Round-2 session e: GPU suite, K2q line-aligned steps A/B (FPNN_AES_ENC_ALIGN=0/1,
# alternating, same box) on C4 / R1 / U1, then trace + PMC passes of those configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh || exit $?
for v in 0 1 0 1; do
  echo "== FPNN_AES_ENC_ALIGN=$v"
  FPNN_AES_ENC_ALIGN=$v timeout -k 10 300 python tools/bench_configs.py --reps 3 --no-host --configs "${CONFIGS:-C4,R1,U1}" \
    > gpurun_out/e_ab_$v.log 2>&1 || { tail -5 gpurun_out/e_ab_$v.log; exit 1; }
  grep -E '^\{"configs' gpurun_out/e_ab_$v.log | cut -c1-2000
done
[ -n "$NO_PROF" ] || TAG=r02e CFGS="${PCFGS:-C4 R1 U1}" bash tools/profile_configs.sh
