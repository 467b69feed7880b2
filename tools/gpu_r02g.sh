#!/bin/bash
# Round-2 session g: ECDH parity, special-prime forms A/B (FPNN_ECDH_MONT=1 = Montgomery
# kernel for every curve, same box), then trace + PMC passes of ECDH and R1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ecdh.py > gpurun_out/g_tests.log 2>&1 || { tail -30 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
for v in 1 0 1 0; do
  echo "== FPNN_ECDH_MONT=$v"
  FPNN_ECDH_MONT=$v timeout -k 10 120 python tools/bench_ecdh.py --curves secp256k1,secp256r1,secp224r1,secp192r1 --no-cpu --reps 5 \
    > gpurun_out/g_ecdh_$v.log 2>&1 || { tail -5 gpurun_out/g_ecdh_$v.log; exit 1; }
  grep -E '^\{' gpurun_out/g_ecdh_$v.log | tail -1 | cut -c1-600
done
[ -n "$NO_PROF" ] || TAG=r02g CFGS="ECDH R1" bash tools/profile_configs.sh
