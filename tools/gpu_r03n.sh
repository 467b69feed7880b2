#!/bin/bash
# Round-3 session n: ECDH A/B of two builds (ab_libs/base vs ab_libs/dual: the ladder's field
# products in independent pairs, prod_dual/mac2) at 65 536 and 262 144 connections, the dual
# build's ECDH tests, then the GPU tests the r03m run did not reach (sharding, stream receiver).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/dual/libfpnn_aes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_ecdh.py > gpurun_out/r03n_ecdh_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03n_ecdh_tests.log | head -20; tail -3 gpurun_out/r03n_ecdh_tests.log; exit 1; }
tail -1 gpurun_out/r03n_ecdh_tests.log
for n in 65536 262144; do
  for v in base dual base dual; do
    FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --n $n --no-cpu --reps 5 \
      > gpurun_out/r03n_ecdh.log 2>&1 || { tail -5 gpurun_out/r03n_ecdh.log; exit 1; }
    echo "$v $n $(tail -1 gpurun_out/r03n_ecdh.log)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sharding.py tests/test_gpu_stream_receiver.py > gpurun_out/r03n_tests.log 2>&1; rc=$?
grep -E "^E |FAILED" gpurun_out/r03n_tests.log | head -20; tail -2 gpurun_out/r03n_tests.log
exit $rc
