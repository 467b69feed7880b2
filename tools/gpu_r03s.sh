#!/bin/bash
# Round-3 session s: mapped host paths with the parallel stream-order sort and the cipher
# queued before the host prepares the next chunk -- host-frame tests, then S1 and C2's
# host legs with host stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03s
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_gpu_hostmap.py \
  tests/test_gpu_parity.py -k "host or stream" > gpurun_out/r03s/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03s/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/r03s/tests.log | head -20; exit $rc; fi
FPNN_AES_HOST_STATS=1 timeout -k 10 300 python -u tools/bench_configs.py --configs S1,C2 > gpurun_out/r03s/cfg.log 2>&1 || { tail -5 gpurun_out/r03s/cfg.log; exit 1; }
grep -E "mapped|^\{" gpurun_out/r03s/cfg.log | tail -14 | cut -c1-400
