#!/bin/bash
# Round-3 session p: ECDH with the carry chains and product-scan columns as single asm
# blocks (ecc_chains.hpp, ab_libs/asm) -- its ECDH tests, then A/B against ab_libs/base and
# ab_libs/fast (builtin carry chains) at 65 536 and 262 144 connections.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/asm/libfpnn_aes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py -k "not cpp" > gpurun_out/r03p_ecdh_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03p_ecdh_tests.log | head -20; tail -3 gpurun_out/r03p_ecdh_tests.log; exit 1; }
tail -1 gpurun_out/r03p_ecdh_tests.log
for n in 65536 262144; do
  for v in base asm fast asm; do
    FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --n $n --no-cpu --reps 5 \
      > gpurun_out/r03p_ecdh.log 2>&1 || { tail -5 gpurun_out/r03p_ecdh.log; exit 1; }
    echo "$v $n $(tail -1 gpurun_out/r03p_ecdh.log)"
  done
done
