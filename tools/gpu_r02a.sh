#!/bin/bash
# Round-2 session A: smoke, GPU parity tests, the default bench line, and the
# self-launched multi-rank bench (2 ranks on the box's one GPU over gloo: checks the
# launcher and every rank's reference digest, not a scaling number).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>: stop at crash/timeout, keep going on test failures
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
nproc > gpurun_out/nproc.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/nproc.txt 2>/dev/null
python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/nproc.txt
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -q -x -m "gpu and not slow" --timeout 300 --timeout-method thread
step bench 300 python bench.py
step bench_2r 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --steps 10
step bench_c4_2r 400 python bench.py --gpus 2 --dist-backend gloo --workload C4 --steps 5 --warmup 2
step bench_c5_2r 300 python bench.py --gpus 2 --dist-backend gloo --workload C5 --steps 10
