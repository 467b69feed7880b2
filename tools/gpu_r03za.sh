#!/bin/bash
# Round-3 session za: K1r's interior-chunk fast path + secp256r1's chain fold (ab_libs/k1rf)
# against the committed build (ab_libs/base): the whole GPU suite on the new build, then
# ECDH and the K1r configs (C4, C2R decrypt; R1 receive) alternating between the builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03za
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/k1rf/libfpnn_aes.so timeout -k 10 900 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03za/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03za/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/r03za/tests.log | head -20; exit $rc; fi
for v in base k1rf base k1rf; do
  FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 120 python tools/bench_ecdh.py --no-cpu --reps 5 --curves secp256r1,secp256k1 \
    > gpurun_out/r03za/ecdh.log 2>&1 || { tail -5 gpurun_out/r03za/ecdh.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r03za/ecdh.log | cut -c1-300)"
  FPNN_AES_LIB=ab_libs/$v/libfpnn_aes.so timeout -k 10 300 python -u tools/bench_configs.py --configs C4,R1 --no-host --reps 3 \
    > gpurun_out/r03za/cfg.log 2>&1 || { tail -5 gpurun_out/r03za/cfg.log; exit 1; }
  echo "$v $(grep -E '^\{"configs' gpurun_out/r03za/cfg.log | cut -c1-600)"
done
