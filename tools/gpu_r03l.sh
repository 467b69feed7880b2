#!/bin/bash
# Round-3 session l: wave-batched quad tickets (adjacent frames side by side in a wave);
# parity, R1/C4 A/B, R1 PMC (HBM bytes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hybrid.py \
    tests/test_gpu_framing_golden.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "not slow" > gpurun_out/r03l_tests.log 2>&1 \
    || { grep -E "^E |Error|FAILED" gpurun_out/r03l_tests.log | head -30; tail -3 gpurun_out/r03l_tests.log; exit 1; }
tail -2 gpurun_out/r03l_tests.log
for cfg in R1 C4; do
timeout -k 10 300 python tools/ab_encrypt.py --config $cfg --rounds 6 \
    --variants "FPNN_AES_HYBRID=1;FPNN_AES_HYBRID=0" \
    > gpurun_out/r03l_ab_$cfg.json 2> gpurun_out/r03l_ab_$cfg.err || { tail -5 gpurun_out/r03l_ab_$cfg.err; exit 1; }
cat gpurun_out/r03l_ab_$cfg.json
done
D=gpurun_out/prof/r03l/r1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex 'cfb_encrypt' --output-format csv -d $D/trace -o run \
    -- python3 tools/ab_encrypt.py --config R1 --rounds 1 --reps 3 --variants "FPNN_AES_HYBRID=1" > gpurun_out/r03l_trace.log 2>&1 \
    || { tail -5 gpurun_out/r03l_trace.log; exit 1; }
for p in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  tag=$(echo "$p" | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $p --kernel-include-regex 'cfb_encrypt' --output-format csv -d $D/pmc_$tag -o run \
    -- python3 tools/ab_encrypt.py --config R1 --rounds 1 --reps 3 --variants "FPNN_AES_HYBRID=1" > gpurun_out/r03l_pmc_$tag.log 2>&1 \
    || { tail -5 gpurun_out/r03l_pmc_$tag.log; exit 1; }
done
python3 tools/pmc_summary.py $D -o gpurun_out/r03l_r1_pmc.json | grep -E "hbm_|lds_array|clock|trace_avg|wait|valu_per"
