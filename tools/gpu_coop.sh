#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|assert" gpurun_out/t_all.log | head -20; exit $rc; fi
timeout -k 10 400 python tools/bench_configs.py --reps 3 --configs C5,C4,C3 2>&1 | grep -E '^\{"configs' > gpurun_out/configs_coop.json; cat gpurun_out/configs_coop.json
FPNN_AES_COOP=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('coop C2', d['value'], d['roofline']['kernels'])"
