#!/bin/bash
# Profiling session on the GPU box: kernel trace + stats, then one rocprofv3 run per
# PMC group (counters never combined with sys/runtime tracing).  Outputs under
# gpurun_out/prof/<tag>/; copy the summaries worth keeping into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof/$TAG
mkdir -p "$OUT"
BENCH_ARGS=${BENCH_ARGS:-""}  # default: exactly the driver's `python bench.py`
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -n "$SLOW" ]; then
  run pytest_slow 900 python -m pytest tests -q -m slow
fi
rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $BENCH_ARGS
grep -E '^\{"metric"' "$OUT/trace.log" > "$OUT/bench_under_rocprof.json" || true
PASSES=${PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES|SQ_WAIT_INST_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE"}
i=0
IFS="|" read -ra PGROUPS <<< "$PASSES"
for g in "${PGROUPS[@]}"; do
  i=$((i+1))
  run "pmc$i" 300 rocprofv3 --kernel-trace --pmc ${g//,/ } --kernel-include-regex 'cfb_' --output-format csv -d "$OUT/pmc$i" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify
done
echo done
