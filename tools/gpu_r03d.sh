#!/bin/bash
# Round-3 session d: the rest of session c (stream receiver, hybrid/ragged/parity parity,
# fence + K2h A/B, R1 PMC), the chain-latency probe and the S1 stream host-frame rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probe/chain_latency > gpurun_out/r03d_latency.json 2>&1 || { cat gpurun_out/r03d_latency.json; exit 1; }
cat gpurun_out/r03d_latency.json
sed -i 's/^timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \\$/timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \\/' tools/gpu_r03c.sh
bash tools/gpu_r03c.sh || exit $?
timeout -k 10 300 python tools/bench_configs.py --configs S1 --reps 3 > gpurun_out/r03d_s1.log 2>&1 || { tail -5 gpurun_out/r03d_s1.log; exit 1; }
grep '^{"S1' gpurun_out/r03d_s1.log
