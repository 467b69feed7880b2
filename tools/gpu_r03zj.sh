#!/bin/bash
# Round-3 session zj: K1d keyed (C5 decrypt) with fenced rounds and the next step's DevKey
# prefetched by one vector load (FPNN_AES_KEYED_PF=1, default) vs fenced only (=0) vs the
# K1r-prologue build (ab_libs/k1r: unfenced, scalar key loads at each step start).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zj
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_ecdh.py -k "dense_keyed or c5 or key_table" \
  > gpurun_out/r03zj/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zj/tests.log | head -20; tail -3 gpurun_out/r03zj/tests.log; exit 1; }
tail -1 gpurun_out/r03zj/tests.log
for v in base pf0 pf1 base pf0 pf1; do
  lib=fpnn_amd/libfpnn_aes.so; [ $v = base ] && lib=ab_libs/k1r/libfpnn_aes.so
  pf=1; [ $v = pf0 ] && pf=0
  FPNN_AES_KEYED_PF=$pf FPNN_AES_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py --reps 5 --no-host --configs C5 \
    > gpurun_out/r03zj/cfg_$v.log 2>&1 || { tail -5 gpurun_out/r03zj/cfg_$v.log; exit 1; }
  echo "$v $(grep -E '^\{"C5"' gpurun_out/r03zj/cfg_$v.log | cut -c1-300)"
done
