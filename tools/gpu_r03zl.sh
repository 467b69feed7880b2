#!/bin/bash
# Round-3 session zl: K2h with the last 16 AES round-key words in VGPRs (ab_libs/vk16:
# C4 lane session SGPR spills 69 -> 45) against the head build -- K2h tests on vk16, then
# C4 / R1 alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zl
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/vk16/libfpnn_aes.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_hybrid.py tests/test_gpu_parity.py -k "hybrid or c4 or wire or queue" \
  > gpurun_out/r03zl/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zl/tests.log | head -20; tail -3 gpurun_out/r03zl/tests.log; exit 1; }
tail -1 gpurun_out/r03zl/tests.log
for v in base vk16 base vk16 base vk16; do
  lib=fpnn_amd/libfpnn_aes.so; [ $v = vk16 ] && lib=ab_libs/vk16/libfpnn_aes.so
  FPNN_AES_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --no-host --configs C4,R1 \
    > gpurun_out/r03zl/cfg_$v.log 2>&1 || { tail -5 gpurun_out/r03zl/cfg_$v.log; exit 1; }
  echo "$v $(grep -E '^\{"(C4|R1)"' gpurun_out/r03zl/cfg_$v.log | tr '\n' ' ' | cut -c1-420)"
done
