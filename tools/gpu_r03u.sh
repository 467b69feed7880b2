#!/bin/bash
# Round-3 session u: steady-state config numbers (bench_configs' back-to-back timing) for
# the ragged configs, and the K2q / K2h A/B on C4 and R1's send side (ab_encrypt.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03u
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_configs.py --configs C4,R1,C3,C5,U1,C2 --no-host > gpurun_out/r03u/cfg.log 2>&1 || { tail -5 gpurun_out/r03u/cfg.log; exit 1; }
grep -E '^\{"configs' gpurun_out/r03u/cfg.log
for cfg in C4 R1; do
  timeout -k 10 300 python tools/ab_encrypt.py --config $cfg --rounds 4 --reps 3 --decrypt \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=0" > gpurun_out/r03u/ab_$cfg.json 2> gpurun_out/r03u/ab_$cfg.err || { tail -5 gpurun_out/r03u/ab_$cfg.err; exit 1; }
  cat gpurun_out/r03u/ab_$cfg.json
done
V="FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=8"
for l in 384 640 768 1024; do for q in 6 8 10; do V="$V;FPNN_AES_HYB_LONG=$l,FPNN_AES_HYB_QW=$q"; done; done
V="$V;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=6;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=10"
timeout -k 10 600 python tools/ab_encrypt.py --config C4 --rounds 3 --reps 3 --variants "$V" > gpurun_out/r03u/sweep_C4.json 2> gpurun_out/r03u/sweep_C4.err || { tail -5 gpurun_out/r03u/sweep_C4.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03u/sweep_C4.json'))
for v in d['variants']: print(v['env'], v['median_GiBs'], v['output_equals_first'])"
