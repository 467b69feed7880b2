#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes of tools/bench_configs.py, one config at a
# time (CFGS="C3 C4 ..."), under gpurun_out/prof/$TAG/<cfg>/.  Summaries:
# python tools/pmc_summary.py gpurun_out/prof/$TAG/<cfg> -o profiles/$TAG/<cfg>/pmc_summary.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
CFGS=${CFGS:-"C3 C4 C5 U1 R1"}
PASSES=${PASSES:-"FETCH_SIZE|WRITE_SIZE|SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES|SQ_WAIT_INST_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_ANY,GRBM_GUI_ACTIVE"}
run() {  # run <dir> <name> <timeout> <cmd...>
  local dir=$1 name=$2 t=$3; shift 3
  echo "== $dir/$name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$dir/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -E '^\{' "$dir/$name.log" | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -5 "$dir/$name.log"; echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for cfg in $CFGS; do
  OUT=gpurun_out/prof/$TAG/$cfg
  mkdir -p "$OUT"
  if [ "$cfg" = ECDH ]; then  # tools/bench_ecdh.py: the device ECDH derivation (k_ecdh)
    CMD="python3 tools/bench_ecdh.py --curves secp256k1 --no-cpu --reps 3"; RX='k_ecdh'
  else
    CMD="python3 tools/bench_configs.py --configs $cfg --no-host --reps 3"; RX='cfb_'
  fi
  run "$OUT" trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $CMD
  i=0
  IFS="|" read -ra PGROUPS <<< "$PASSES"
  for g in "${PGROUPS[@]}"; do
    i=$((i+1))
    run "$OUT" "pmc$i" 300 rocprofv3 --kernel-trace --pmc ${g//,/ } --kernel-include-regex "$RX" --output-format csv -d "$OUT/pmc$i" -o run -- $CMD
  done
done
echo done
