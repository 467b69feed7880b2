#!/bin/bash
# Round-2 session k: ECDH throughput vs batch size (65 536 = C5's connections, one wave
# per SIMD; 262 144 = four), then trace + PMC passes of C3 / C5 / C2R on the final build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 65536 262144; do
  timeout -k 10 120 python tools/bench_ecdh.py --n $n --no-cpu --reps 5 > gpurun_out/k_ecdh_$n.log 2>&1 || { tail -5 gpurun_out/k_ecdh_$n.log; exit 1; }
  grep -E '^\{' gpurun_out/k_ecdh_$n.log | tail -1 | cut -c1-600
done
TAG=r02k CFGS="C3 C5 C2R" bash tools/profile_configs.sh
