#!/bin/bash
# GPU session: the whole GPU test suite (stops at the first failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x ${PYTEST_ARGS:-} > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert|FAILED" gpurun_out/t_all.log | head -30; fi
exit $rc
