#!/bin/bash
# Round-3 session zn: S1's mapped stream path with the frames copied in slot order before
# the quota walk (ab_libs/s1 = the tree with tools/probe/mapped_stream_sorted_copy.patch applied; FPNN_AES_MAP_SORTED=1) vs walking frames[order[i]] (=0):
# host-frame tests, then S1 alternating in fresh processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03zn
export TMPDIR=/tmp
FPNN_AES_LIB=ab_libs/s1/libfpnn_aes.so FPNN_AES_MAP_SORTED=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_hostmap.py tests/test_gpu_parity.py -k "host" \
  > gpurun_out/r03zn/tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r03zn/tests.log | head -20; tail -3 gpurun_out/r03zn/tests.log; exit 1; }
tail -1 gpurun_out/r03zn/tests.log
for v in 0 1 0 1 0 1; do
  FPNN_AES_LIB=ab_libs/s1/libfpnn_aes.so FPNN_AES_MAP_SORTED=$v FPNN_AES_HOST_STATS=1 timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --configs S1 \
    > gpurun_out/r03zn/s1_$v.log 2>&1 || { tail -5 gpurun_out/r03zn/s1_$v.log; exit 1; }
  echo "sorted=$v $(grep -E '^\{"S1"' gpurun_out/r03zn/s1_$v.log | cut -c1-260)"
done
