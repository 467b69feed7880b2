#!/bin/bash
# Round-3 session j: cheaper in-quad funnel; R1 and C4 A/B (prefetch on/off, K2q).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py \
    tests/test_gpu_framing_golden.py > gpurun_out/r03j_tests.log 2>&1 \
    || { grep -E "^E |Error|FAILED" gpurun_out/r03j_tests.log | head -30; tail -3 gpurun_out/r03j_tests.log; exit 1; }
tail -2 gpurun_out/r03j_tests.log
for cfg in R1 C4; do
timeout -k 10 300 python tools/ab_encrypt.py --config $cfg --rounds 6 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=1,FPNN_AES_HYB_QFLAGS=2;FPNN_AES_HYBRID=0" \
    > gpurun_out/r03j_ab_$cfg.json 2> gpurun_out/r03j_ab_$cfg.err || { tail -5 gpurun_out/r03j_ab_$cfg.err; exit 1; }
cat gpurun_out/r03j_ab_$cfg.json
done
