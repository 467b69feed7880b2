#!/bin/bash
# Multi-rank rehearsal on one GPU (gloo, 2 ranks) + all-config throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== torchrun 2 ranks (gloo)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/torchrun2.log 2>&1
rc=$?; echo "rc=$rc"; grep -E '^\{' gpurun_out/torchrun2.log | cut -c1-400
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 gpurun_out/torchrun2.log; exit $rc; fi
echo "== configs"
timeout -k 10 600 python tools/bench_configs.py --reps 5 > gpurun_out/configs.log 2>&1
rc=$?; echo "rc=$rc"; grep -E '^\{' gpurun_out/configs.log | tail -1; tail -3 gpurun_out/configs.log
exit $rc
