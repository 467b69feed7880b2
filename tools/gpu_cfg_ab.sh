#!/bin/bash
# Parity suite, then tools/bench_configs.py for CONFIGS under each ';'-separated
# environment variant in VARIANTS (one process per variant, same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
IFS=";" read -ra VS <<< "${VARIANTS:-FPNN_AES_QUEUE=0;FPNN_AES_QUEUE=1}"
for v in "${VS[@]}"; do
  echo "== $v"
  env $(echo "$v" | tr ',' ' ') timeout -k 10 300 python tools/bench_configs.py --reps 3 --configs "${CONFIGS:-C4}" \
    > gpurun_out/cfg_ab.log 2>&1 || { tail -5 gpurun_out/cfg_ab.log; exit 1; }
  grep -E '^\{"configs' gpurun_out/cfg_ab.log
done
