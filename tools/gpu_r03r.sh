#!/bin/bash
# Round-3 session r: the whole GPU suite on the build with the parallel mapped-stream chunk
# preparation and the mapped per-call path, then the per-call cost under
# FPNN_AES_PERCALL_MAPPED = 0 / 1 / 2 and the S1 stream host frames with host stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03r
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r03r/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03r/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/r03r/tests.log | head -20; exit $rc; fi
for m in 0 1 2; do
  FPNN_AES_PERCALL_MAPPED=$m timeout -k 10 300 python -u tools/bench_percall.py > gpurun_out/r03r/percall_$m.log 2>&1 || { tail -5 gpurun_out/r03r/percall_$m.log; exit 1; }
  echo "mapped=$m $(tail -1 gpurun_out/r03r/percall_$m.log | cut -c1-300)"
done
FPNN_AES_HOST_STATS=1 timeout -k 10 300 python -u tools/bench_configs.py --configs S1 > gpurun_out/r03r/s1.log 2>&1 || { tail -5 gpurun_out/r03r/s1.log; exit 1; }
grep -E "mapped stream|^\{" gpurun_out/r03r/s1.log | tail -6 | cut -c1-400
