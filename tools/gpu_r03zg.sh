#!/bin/bash
# Round-3 session zg: K1r prologue -- the small block-map scan as coalesced rounds with a
# wave scan (was a 1024-wide Hillis-Steele), and the per-wave plan inside the decrypt
# kernel for out-of-place batches.  GPU tests of the ragged / stream / framing paths on the
# new build, then C3 / C4 / R1 alternating against the round-3 build (ab_libs/base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zg
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ragged.py tests/test_gpu_parity.py tests/test_gpu_stream_receiver.py tests/test_gpu_framing_golden.py \
  tests/test_gpu_fuzz.py > gpurun_out/r03zg/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zg/tests.log | head -20; tail -3 gpurun_out/r03zg/tests.log; exit 1; }
tail -1 gpurun_out/r03zg/tests.log
for v in base new base new; do
  lib=fpnn_amd/libfpnn_aes.so; [ $v = base ] && lib=ab_libs/base/libfpnn_aes.so
  FPNN_AES_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --no-host --configs C3,C4,R1 \
    > gpurun_out/r03zg/cfg_$v.log 2>&1 || { tail -5 gpurun_out/r03zg/cfg_$v.log; exit 1; }
  echo "$v $(grep -E '^\{"(C3|C4|R1)"' gpurun_out/r03zg/cfg_$v.log | tr '\n' ' ' | cut -c1-900)"
done
