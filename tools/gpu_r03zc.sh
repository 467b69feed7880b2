#!/bin/bash
# Round-3 session zc: secp224r1's fold as carry chains (ab_libs/p224, which also has the
# secp256r1 chain fold) against ab_libs/base: ECDH tests on the new build, then
# derivations/s alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zc
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/p224/libfpnn_aes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py > gpurun_out/r03zc/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zc/tests.log | head -20; tail -3 gpurun_out/r03zc/tests.log; exit 1; }
tail -1 gpurun_out/r03zc/tests.log
for v in base p224 base p224; do
  FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --no-cpu --reps 5 \
    > gpurun_out/r03zc/ecdh.log 2>&1 || { tail -5 gpurun_out/r03zc/ecdh.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03zc/ecdh.log | cut -c1-500)"
done
