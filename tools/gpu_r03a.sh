#!/bin/bash
# Round-3 session a: K2h parity (new tests + the queue/hybrid-parametrized parity suite),
# then same-process A/B of K2q vs K2h settings on C4 and R1's send side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_hybrid.py tests/test_gpu_parity.py -k "hybrid or queue or wire or golden_package or random_package or random_stream" \
  > gpurun_out/r03a_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03a_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/r03a_tests.log | head -30; exit $rc; fi
V="FPNN_AES_HYBRID=0;FPNN_AES_HYB_LONG=2048,FPNN_AES_HYB_QW=4;FPNN_AES_HYB_LONG=1024,FPNN_AES_HYB_QW=6;FPNN_AES_HYB_LONG=512,FPNN_AES_HYB_QW=8;FPNN_AES_HYB_LONG=3000,FPNN_AES_HYB_QW=2"
timeout -k 10 300 python tools/ab_encrypt.py --config C4 --variants "$V" > gpurun_out/r03a_c4.log 2>&1 || { tail -5 gpurun_out/r03a_c4.log; exit 1; }
grep '^{' gpurun_out/r03a_c4.log
timeout -k 10 300 python tools/ab_encrypt.py --config R1 --variants "FPNN_AES_HYBRID=0;FPNN_AES_HYBRID=1" > gpurun_out/r03a_r1.log 2>&1 || { tail -5 gpurun_out/r03a_r1.log; exit 1; }
grep '^{' gpurun_out/r03a_r1.log
# then the rest of the GPU suite on this build
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  --deselect tests/test_gpu_hybrid.py > gpurun_out/r03a_all.log 2>&1; rc=$?; tail -3 gpurun_out/r03a_all.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/r03a_all.log | head -30; exit $rc; fi
