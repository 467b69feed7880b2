#!/bin/bash
# Rehearsal of the driver's N>1 bench launch (torch.distributed.run, one rank per GPU) on a
# one-GPU box: bench.py maps LOCAL_RANK onto the visible devices, so N ranks share cuda:0.
# Never N=8 here (that run is the driver's).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r06m
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/r06m/bench_n$n.log 2>&1 || { echo "n=$n failed"; tail -20 gpurun_out/r06m/bench_n$n.log; exit 3; }
  grep '^{' gpurun_out/r06m/bench_n$n.log | cut -c1-300
done
