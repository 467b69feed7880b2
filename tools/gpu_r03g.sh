#!/bin/bash
# Round-3 session g: K2h quad session with line-aligned steps, prefetch and the in-quad
# funnel shift (wire frames on quads-only K2h); K1r fenced KEY_LANE without spills.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py \
    tests/test_gpu_framing_golden.py tests/test_gpu_fuzz.py > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -2 gpurun_out/r03g_tests.log
timeout -k 10 300 python tools/ab_encrypt.py --config R1 --rounds 6 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=0" > gpurun_out/r03g_ab_r1.json 2> gpurun_out/r03g_ab_r1.err || { tail -5 gpurun_out/r03g_ab_r1.err; exit 1; }
cat gpurun_out/r03g_ab_r1.json
timeout -k 10 300 python tools/ab_encrypt.py --config C4 --rounds 6 --decrypt \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=0" > gpurun_out/r03g_ab_c4.json 2> gpurun_out/r03g_ab_c4.err || { tail -5 gpurun_out/r03g_ab_c4.err; exit 1; }
cat gpurun_out/r03g_ab_c4.json
timeout -k 10 300 python tools/bench_configs.py --configs C3 --no-host --reps 5 > gpurun_out/r03g_c3.log 2>&1 || { tail -5 gpurun_out/r03g_c3.log; exit 1; }
grep '^{"C3' gpurun_out/r03g_c3.log
