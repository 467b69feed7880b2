#!/bin/bash
# Round-2 session h: host-frame tests, then the mapped path's chunk ramp A/B
# (FPNN_AES_MAP_RAMP_MB=0 = fixed 32 MiB chunks; default 4 MiB ramp), alternating, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_hostmap.py \
  tests/test_gpu_parity.py -k "host or frames or collector or udp" > gpurun_out/h_host.log 2>&1 || { tail -30 gpurun_out/h_host.log; exit 1; }
tail -2 gpurun_out/h_host.log
for v in 0 4 0 4 0 4; do
  echo "== FPNN_AES_MAP_RAMP_MB=$v"
  FPNN_AES_MAP_RAMP_MB=$v timeout -k 10 120 python tools/probe_mapped.py > gpurun_out/h_map_$v.log 2>&1 || { tail -5 gpurun_out/h_map_$v.log; exit 1; }
  tail -1 gpurun_out/h_map_$v.log
done
