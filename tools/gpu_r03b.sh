#!/bin/bash
# Round-3 session b: K2h shift path with fenced rounds (parity), fenced-round A/B on C2
# (K2 + K1d), C4 threshold sweep, R1 send side K2q vs K2h, then the C2 bench under FENCE=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_hybrid.py tests/test_gpu_parity.py -k "hybrid or wire or golden_package or uniform_layout" \
  > gpurun_out/r03b_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03b_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/r03b_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python tools/ab.py --rounds 8 --variants "FPNN_AES_FENCE=0;FPNN_AES_FENCE=1" > gpurun_out/r03b_c2fence.log 2>&1 || { tail -5 gpurun_out/r03b_c2fence.log; exit 1; }
tr -d '\n ' < gpurun_out/r03b_c2fence.log; echo
V="FPNN_AES_HYBRID=0;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=8;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=10;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=12;FPNN_AES_HYB_LONG=384,FPNN_AES_HYB_QW=10;FPNN_AES_HYB_LONG=384,FPNN_AES_HYB_QW=12;FPNN_AES_HYB_LONG=256,FPNN_AES_HYB_QW=12;FPNN_AES_HYB_LONG=256,FPNN_AES_HYB_QW=14;FPNN_AES_HYB_LONG=768,FPNN_AES_HYB_QW=10"
timeout -k 10 400 python tools/ab_encrypt.py --config C4 --rounds 4 --variants "$V" > gpurun_out/r03b_c4.log 2>&1 || { tail -5 gpurun_out/r03b_c4.log; exit 1; }
grep '^{' gpurun_out/r03b_c4.log
timeout -k 10 300 python tools/ab_encrypt.py --config R1 --variants "FPNN_AES_HYBRID=0;FPNN_AES_HYBRID=1" > gpurun_out/r03b_r1.log 2>&1 || { tail -5 gpurun_out/r03b_r1.log; exit 1; }
grep '^{' gpurun_out/r03b_r1.log
FPNN_AES_FENCE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03b_bench_fence.log 2>&1 || { tail -5 gpurun_out/r03b_bench_fence.log; exit 1; }
grep '^{' gpurun_out/r03b_bench_fence.log | cut -c1-400
