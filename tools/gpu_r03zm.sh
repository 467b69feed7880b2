#!/bin/bash
# Round-3 session zm: the K2h VGPR-key A/B (tools/gpu_r03zl.sh), then the validation of the
# head build and every device config's steady-state medians (tools/gpu_r03zk.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r03zl.sh || exit $?
bash tools/gpu_r03zk.sh
