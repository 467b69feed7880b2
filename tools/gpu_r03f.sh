#!/bin/bash
# Round-3 session f: C3 decrypt regression hunt (fence on/off, pools on/off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "FPNN_AES_FENCE=1" "FPNN_AES_FENCE=0" "FPNN_AES_POOLS=0"; do
  env $v timeout -k 10 300 python tools/bench_configs.py --configs C3 --no-host --reps 5 > gpurun_out/r03f_c3.log 2>&1 || { tail -5 gpurun_out/r03f_c3.log; exit 1; }
  echo "$v $(grep '^{"C3' gpurun_out/r03f_c3.log)"
done
