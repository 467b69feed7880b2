#!/bin/bash
# Round-3 session zb: rocprofv3 kernel trace + PMC passes of the default bench command on
# the final round-3 build (profiles/r03/bench), then the default bench line once more.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=r03bench bash tools/profile_session.sh || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r03zb_bench.log 2>&1 || { tail -5 gpurun_out/r03zb_bench.log; exit 1; }
tail -1 gpurun_out/r03zb_bench.log | cut -c1-400
