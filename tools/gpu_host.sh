#!/bin/bash
# GPU session: full GPU test suite, host-frame/config throughput (C2, C3), default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" gpurun_out/t_all.log | head -20; exit $rc; fi
timeout -k 10 500 python tools/bench_configs.py --reps 3 --configs ${CONFIGS:-C2,C3} > gpurun_out/configs_host.log 2>&1; rc=$?
grep -E '^\{"configs' gpurun_out/configs_host.log || tail -5 gpurun_out/configs_host.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
