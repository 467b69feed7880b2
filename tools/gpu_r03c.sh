#!/bin/bash
# Round-3 session c: fence defaults (K2h, K1r) parity + A/B on C4 / C2R enc+dec; R1 vs R1A
# vs C2R lane-mode efficiency; PMC passes (LDS, VALU, HBM bytes) of R1's send side, K2q vs K2h.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_hostmap.py tests/test_gpu_stream_receiver.py tests/test_gpu_hybrid.py tests/test_gpu_ragged.py tests/test_gpu_parity.py -k "not slow" \
  > gpurun_out/r03c_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03c_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/r03c_tests.log | head -30; exit $rc; fi
run() { local name=$1; shift; timeout -k 10 400 python tools/ab_encrypt.py "$@" > gpurun_out/r03c_$name.log 2>&1 || { tail -5 gpurun_out/r03c_$name.log; exit 1; }; grep '^{' gpurun_out/r03c_$name.log; }
run c4 --config C4 --decrypt --rounds 4 --variants "FPNN_AES_FENCE=0;FPNN_AES_FENCE=1;FPNN_AES_HYBRID=0"
run c2r --config C2R --decrypt --rounds 4 --variants "FPNN_AES_FENCE=0;FPNN_AES_FENCE=1;FPNN_AES_HYBRID=0"
run r1 --config R1 --rounds 4 --variants "FPNN_AES_HYBRID=0;FPNN_AES_HYBRID=1"
run r1a --config R1A --rounds 4 --variants "FPNN_AES_HYBRID=0;FPNN_AES_HYBRID=1"
for v in 0 1; do
  for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
    tag=$(echo "$p" | cut -d' ' -f1)
    FPNN_AES_HYBRID=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p --kernel-include-regex 'cfb_encrypt' --output-format csv \
      -d gpurun_out/prof/r03c/r1_h$v/$tag -o run -- python3 tools/ab_encrypt.py --config R1 --rounds 1 --reps 2 --variants "FPNN_AES_HYBRID=$v" \
      > gpurun_out/r03c_pmc_${v}_$tag.log 2>&1 || { tail -5 gpurun_out/r03c_pmc_${v}_$tag.log; exit 1; }
  done
done
echo pmc done
