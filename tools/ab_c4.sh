#!/bin/bash
# Same-box A/B of two library builds (tools/probe/ablib/lib_old.so vs the tree's) on C4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do for v in old new; do
  if [ $v = old ]; then export FPNN_AES_LIB=$PWD/tools/probe/ablib/lib_old.so; else unset FPNN_AES_LIB; fi
  echo "== $v"
  timeout -k 10 300 python tools/bench_configs.py --reps 3 --no-host --configs ${CONFIGS:-C4} 2>&1 | grep '"configs"' || exit 1
done; done
