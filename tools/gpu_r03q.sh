#!/bin/bash
# Round-3 session q: the committed records -- every config's medians (bench_configs, host
# legs included), the per-call drop-in cost (C1's shape), ECDH with the reference's CPU legs
# and per-call latency, then rocprofv3 trace + PMC passes of C4, R1, C3 and ECDH (TAG=r03).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03q
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/r03q/$name.log" 2>&1; local rc=$?
  grep -E '^\{' "gpurun_out/r03q/$name.log" | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/r03q/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step configs 900 python -u tools/bench_configs.py --reps 5
step percall 300 python -u tools/bench_percall.py
step ecdh 300 python -u tools/bench_ecdh.py --percall 200
TAG=r03 CFGS="C4 R1 C3 ECDH" bash tools/profile_configs.sh
