#!/bin/bash
# Round-3 session o: the carry-hazard probe (unpadded carry chains vs plain C), then ECDH
# A/B of ab_libs/base vs ab_libs/fast (carry chains via __builtin_addc/subc, column-start
# macs, three-chain secp256k1 fold) with the fast build's ECDH tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 tools/probe/carry_hazard > gpurun_out/r03o_hazard.log 2>&1; rc=$?; cat gpurun_out/r03o_hazard.log
[ $rc -eq 0 ] || exit $rc
FPNN_AES_LIB=ab_libs/fast/libfpnn_aes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py -k "not cpp" > gpurun_out/r03o_ecdh_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03o_ecdh_tests.log | head -20; tail -3 gpurun_out/r03o_ecdh_tests.log; exit 1; }
tail -1 gpurun_out/r03o_ecdh_tests.log
for n in 65536 262144; do
  for v in base fast base fast; do
    FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --n $n --no-cpu --reps 5 \
      > gpurun_out/r03o_ecdh.log 2>&1 || { tail -5 gpurun_out/r03o_ecdh.log; exit 1; }
    echo "$v $n $(tail -1 gpurun_out/r03o_ecdh.log)"
  done
done
