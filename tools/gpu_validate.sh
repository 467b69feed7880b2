#!/bin/bash
# Full validation on one GPU box: smoke, the whole GPU suite (incl. slow), the default
# bench line, every config.  Each step has its own limit; the first crash/timeout ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-val}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run tests 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread
run bench 300 python -u bench.py
[ -n "$NO_CONFIGS" ] || run configs 600 python -u tools/bench_configs.py --reps 3 --no-host
exit 0
