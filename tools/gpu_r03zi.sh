#!/bin/bash
# Round-3 session zi: the package frame walk (k_scan_wave) with guesses widening 1/4/16/64
# and one wave per connection, and fenced rounds for the keyed K1d (C5 decrypt) -- tests on
# the new build, then R1 and C5 alternating against the K1r-prologue build (ab_libs/k1r).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zi
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_framing_golden.py tests/test_gpu_stream_receiver.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py \
  > gpurun_out/r03zi/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zi/tests.log | head -20; tail -3 gpurun_out/r03zi/tests.log; exit 1; }
tail -1 gpurun_out/r03zi/tests.log
for v in base new base new; do
  lib=fpnn_amd/libfpnn_aes.so; [ $v = base ] && lib=ab_libs/k1r/libfpnn_aes.so
  FPNN_AES_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py --reps 5 --no-host --configs R1,C5 \
    > gpurun_out/r03zi/cfg_$v.log 2>&1 || { tail -5 gpurun_out/r03zi/cfg_$v.log; exit 1; }
  echo "$v $(grep -E '^\{"(R1|C5)"' gpurun_out/r03zi/cfg_$v.log | tr '\n' ' ' | cut -c1-700)"
done
