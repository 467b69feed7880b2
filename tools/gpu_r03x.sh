#!/bin/bash
# Round-3 session x: C4 K2h sweep around the r03w leader (threshold 1024 blocks, 12 of 16
# waves starting on quads), and the same settings on R1's send side and C2R.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03x
export TMPDIR=/tmp
V="FPNN_AES_HYB_LONG=1024,FPNN_AES_HYB_QW=12"
for l in 768 1024 1536 2048; do for q in 11 12 13 14 16; do V="$V;FPNN_AES_HYB_LONG=$l,FPNN_AES_HYB_QW=$q"; done; done
timeout -k 10 900 python tools/ab_encrypt.py --config C4 --rounds 5 --reps 3 --variants "$V" > gpurun_out/r03x/c4.json 2> gpurun_out/r03x/c4.err || { tail -5 gpurun_out/r03x/c4.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03x/c4.json'))
for v in d['variants']: print(v['env'], v['median_GiBs'], v['min_GiBs'], v['max_GiBs'], v['output_equals_first'])"
for cfg in C2R; do
timeout -k 10 300 python tools/ab_encrypt.py --config $cfg --rounds 5 --reps 3 --variants "FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=8;FPNN_AES_HYB_LONG=1024,FPNN_AES_HYB_QW=12;FPNN_AES_HYB_LONG=2048,FPNN_AES_HYB_QW=14" > gpurun_out/r03x/$cfg.json 2> gpurun_out/r03x/$cfg.err || { tail -5 gpurun_out/r03x/$cfg.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03x/$cfg.json'))
for v in d['variants']: print('$cfg', v['env'], v['median_GiBs'], v['min_GiBs'], v['max_GiBs'], v['output_equals_first'])"
done
