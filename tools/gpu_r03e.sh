#!/bin/bash
# Round-3 session e: mapped stream path with kChunk pipelining (S1), the wire-batch default
# (all-quad K2h) against K2q and lane-shift K2h on R1, per-config medians, ECDH per call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hostmap.py \
    > gpurun_out/r03e_tests.log 2>&1 || { tail -30 gpurun_out/r03e_tests.log; exit 1; }
tail -2 gpurun_out/r03e_tests.log
timeout -k 10 300 python tools/bench_configs.py --configs S1 --reps 3 > gpurun_out/r03e_s1.log 2>&1 || { tail -5 gpurun_out/r03e_s1.log; exit 1; }
grep '^{"S1' gpurun_out/r03e_s1.log
timeout -k 10 300 python tools/ab_encrypt.py --config R1 --rounds 6 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=0;FPNN_AES_HYBRID=1,FPNN_AES_HYB_WIRE_LANES=1" \
    > gpurun_out/r03e_ab_r1.json 2> gpurun_out/r03e_ab_r1.err || { tail -5 gpurun_out/r03e_ab_r1.err; exit 1; }
cat gpurun_out/r03e_ab_r1.json
timeout -k 10 600 python tools/bench_configs.py --configs C3,C4,R1 --reps 5 > gpurun_out/r03e_cfg.log 2>&1 || { tail -5 gpurun_out/r03e_cfg.log; exit 1; }
grep '^{' gpurun_out/r03e_cfg.log
timeout -k 10 300 python tools/bench_ecdh.py --cpu-seconds 5 --percall 200 > gpurun_out/r03e_ecdh.json 2>&1 || { tail -5 gpurun_out/r03e_ecdh.json; exit 1; }
tail -3 gpurun_out/r03e_ecdh.json
