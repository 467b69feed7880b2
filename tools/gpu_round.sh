#!/bin/bash
# Full GPU session: tests, every config's throughput, the bench line, then the
# rocprofv3 kernel trace + PMC passes (tools/profile_session.sh) under TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r01}
bash tools/gpu_tests.sh || exit $?
echo "== configs $(date +%T)"
timeout -k 10 600 python tools/bench_configs.py --reps 3 > gpurun_out/configs_all.log 2>&1; rc=$?
grep -E '^\{"configs' gpurun_out/configs_all.log > gpurun_out/configs_all.json || tail -5 gpurun_out/configs_all.log
[ $rc -eq 0 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
[ -n "$NO_PROFILE" ] && exit 0
TAG=$TAG bash tools/profile_session.sh
