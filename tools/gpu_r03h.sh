#!/bin/bash
# Round-3 session h: R1 on quads-only K2h, A/B of line-aligned steps and prefetch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_encrypt.py --config R1 --rounds 4 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=1;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=2;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=3;FPNN_AES_HYBRID=0" \
    > gpurun_out/r03h_ab_r1.json 2> gpurun_out/r03h_ab_r1.err || { tail -5 gpurun_out/r03h_ab_r1.err; exit 1; }
cat gpurun_out/r03h_ab_r1.json
timeout -k 10 300 python tools/ab_encrypt.py --config C4 --rounds 4 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=1;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=2" \
    > gpurun_out/r03h_ab_c4.json 2> gpurun_out/r03h_ab_c4.err || { tail -5 gpurun_out/r03h_ab_c4.err; exit 1; }
cat gpurun_out/r03h_ab_c4.json
