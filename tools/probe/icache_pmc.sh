#!/bin/bash
# Instruction-cache PMC pass over the short-frame kernels (Q1) and the bench kernels (C2):
#   bash tools/probe/icache_pmc.sh <tag>   ->  gpurun_out/<tag>/ic_{q1,c2}/
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
C="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex frames --output-format csv \
  -d $OUT/ic_q1 -o run -- python3 tools/probe/q1_time.py --configs Q1,Q1s > $OUT/ic_q1.log 2>&1 || exit 3
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex cfb_ --output-format csv \
  -d $OUT/ic_c2 -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > $OUT/ic_c2.log 2>&1 || exit 3
echo done
