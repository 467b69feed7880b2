#!/bin/bash
# Round-3 session zh: validation of the K1r-prologue build (smoke, whole GPU suite, bench
# line) and a rocprofv3 kernel trace of C3 (framed decrypt timeline: scan, K1r, gaps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=r03zh NO_CONFIGS=1 bash tools/gpu_validate.sh || exit $?
TAG=r03zh CFGS="C3" PASSES="" bash tools/profile_configs.sh
