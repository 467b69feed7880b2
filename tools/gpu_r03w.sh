#!/bin/bash
# Round-3 session w: C4 K2h threshold / quad-wave A/B with more rounds (the r03u sweep's
# leaders against the default), twice in one process each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03w
export TMPDIR=/tmp
V="FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=8;FPNN_AES_HYB_LONG=1024,FPNN_AES_HYB_QW=10;FPNN_AES_HYB_LONG=768,FPNN_AES_HYB_QW=10;FPNN_AES_HYB_LONG=384,FPNN_AES_HYB_QW=8;FPNN_AES_HYB_LONG=1024,FPNN_AES_HYB_QW=12"
for rep in 1 2; do
timeout -k 10 600 python tools/ab_encrypt.py --config C4 --rounds 8 --reps 3 --variants "$V" > gpurun_out/r03w/c4_$rep.json 2> gpurun_out/r03w/c4_$rep.err || { tail -5 gpurun_out/r03w/c4_$rep.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03w/c4_$rep.json'))
for v in d['variants']: print('$rep', v['env'], v['median_GiBs'], v['min_GiBs'], v['max_GiBs'], v['output_equals_first'])"
done
