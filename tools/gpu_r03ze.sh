#!/bin/bash
# Round-3 session ze: secp192r1's fold as carry chains (ab_libs/p192) against the round-3
# build (ab_libs/base): ECDH tests on the new build, then derivations/s alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03ze
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/p192/libfpnn_aes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py > gpurun_out/r03ze/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03ze/tests.log | head -20; tail -3 gpurun_out/r03ze/tests.log; exit 1; }
tail -1 gpurun_out/r03ze/tests.log
for v in base p192 base p192; do
  FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --no-cpu --reps 5 \
    > gpurun_out/r03ze/ecdh.log 2>&1 || { tail -5 gpurun_out/r03ze/ecdh.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03ze/ecdh.log | cut -c1-500)"
done
