#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> short bench.  Stops at the first
# crash/timeout (exit codes other than 0 = pass and 1 = test failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-'-m "gpu and not slow"'}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m3 -E 'gfx|Marketing' > gpurun_out/rocminfo.txt
nproc > gpurun_out/nproc.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
eval step pytest_gpu 600 python -m pytest tests -q --maxfail=20 $PYTEST_ARGS
step bench 240 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3
