#!/bin/bash
# Round-3 session m: validation of the committed build (smoke, GPU suite, bench line),
# then ECDH A/B of two builds (ab_libs/base.so vs ab_libs/ecdh_split.so: carries in
# compiler-allocated SGPR pairs instead of vcc) at 65 536 and 262 144 connections, with
# the split build's ECDH tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03m NO_CONFIGS=1 bash tools/gpu_validate.sh || exit $?
for n in 65536 262144; do
  for v in base ecdh_split; do
    echo "== ecdh $v n=$n"
    FPNN_AES_LIB=ab_libs/$v.so timeout -k 10 120 python tools/bench_ecdh.py --n $n --no-cpu --reps 5 \
      > gpurun_out/r03m_ecdh_${v}_$n.log 2>&1 || { tail -5 gpurun_out/r03m_ecdh_${v}_$n.log; exit 1; }
    tail -1 gpurun_out/r03m_ecdh_${v}_$n.log
  done
done
FPNN_AES_LIB=ab_libs/ecdh_split.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py > gpurun_out/r03m_ecdh_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03m_ecdh_tests.log
exit $rc
