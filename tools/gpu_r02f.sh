#!/bin/bash
# Round-2 session f: ECDH + encrypt parity, secp256k1 special reduction A/B
# (FPNN_ECDH_MONT=1 is the Montgomery kernel), R1 wire encrypt A/B (FPNN_AES_ENC_ALIGN).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ecdh.py tests/test_gpu_parity.py > gpurun_out/f_tests.log 2>&1 || { tail -30 gpurun_out/f_tests.log; exit 1; }
tail -2 gpurun_out/f_tests.log
for v in 1 0 1 0; do  # ECDH
  echo "== FPNN_ECDH_MONT=$v"
  FPNN_ECDH_MONT=$v timeout -k 10 120 python tools/bench_ecdh.py --curves secp256k1 --no-cpu --reps 5 \
    > gpurun_out/f_ecdh_$v.log 2>&1 || { tail -5 gpurun_out/f_ecdh_$v.log; exit 1; }
  grep -E '^\{' gpurun_out/f_ecdh_$v.log | tail -1 | cut -c1-600
done
for v in 0 1 0 1; do
  echo "== FPNN_AES_ENC_ALIGN=$v"
  FPNN_AES_ENC_ALIGN=$v timeout -k 10 200 python tools/bench_configs.py --reps 5 --no-host --configs R1,C4 \
    > gpurun_out/f_enc_$v.log 2>&1 || { tail -5 gpurun_out/f_enc_$v.log; exit 1; }
  grep -E '^\{"configs' gpurun_out/f_enc_$v.log | cut -c1-400
done
