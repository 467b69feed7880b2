#!/bin/bash
# Host-frame pipeline probe: the host-frame parity tests, then C2/C3 host-frame rates
# with the per-call breakdown (FPNN_AES_HOST_STATS) at two copy-thread counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x -k "host_frames" > gpurun_out/t_host.log 2>&1; rc=$?; tail -2 gpurun_out/t_host.log
[ $rc -eq 0 ] || { grep -E "^E " gpurun_out/t_host.log | head; exit $rc; }
for th in 16 8; do
  FPNN_AES_HOST_STATS=1 FPNN_AES_HOST_THREADS=$th timeout -k 10 400 python tools/bench_configs.py --reps 2 --configs C2,C3 > gpurun_out/hostprobe_$th.log 2>&1 || exit $?
  echo "== threads $th"; grep -E "fpnn_aes host" gpurun_out/hostprobe_$th.log | tail -6; grep -E '^\{"configs' gpurun_out/hostprobe_$th.log
done
