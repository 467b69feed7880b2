#!/bin/bash
# Round-2 session B: K1r (sync-free ragged decrypt) parity + the configs' throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step ragged 300 python -u -m pytest tests/test_gpu_ragged.py -x -v --timeout 120 --timeout-method thread
step pytest_gpu 900 python -u -m pytest tests -q -x -m "gpu and not slow" --timeout 300 --timeout-method thread
step configs 600 python tools/bench_configs.py --reps 3
