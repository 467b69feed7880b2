#!/bin/bash
# Parity suite, then an interleaved in-process A/B of engine variants (tools/ab.py)
# and the default bench line.  VARIANTS / AB_ARGS select what is compared.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python tools/ab.py --variants "${VARIANTS:-FPNN_AES_DEC_FULL=0;FPNN_AES_DEC_FULL=1}" ${AB_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
cat gpurun_out/ab.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], json.dumps(d['roofline']['kernels']))"
