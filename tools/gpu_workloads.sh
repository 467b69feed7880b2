#!/bin/bash
# bench.py on the sharded BASELINE.json configs (C4, C5) at N=1, then a 2-rank gloo
# rehearsal of each on the one GPU (the 8-GPU runs are the driver's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for w in C4 C5; do
  echo "== $w N=1"
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 > gpurun_out/bench_$w.log 2>&1 || { tail -5 gpurun_out/bench_$w.log; exit 1; }
  tail -1 gpurun_out/bench_$w.log
  echo "== $w torchrun 2 ranks (gloo, one GPU)"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --workload $w --gpus 2 --steps 3 --warmup 1 --dist-backend gloo \
    > gpurun_out/bench_${w}_2r.log 2>&1 || { tail -20 gpurun_out/bench_${w}_2r.log; exit 1; }
  grep -E '^\{' gpurun_out/bench_${w}_2r.log
done
