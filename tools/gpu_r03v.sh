#!/bin/bash
# Round-3 session v: per-call forms waiting by polling (sync_spin) vs the blocking
# hipStreamSynchronize (FPNN_AES_SYNC_SPIN=0): GPU tests of those paths, then the per-call
# drop-in cost (C1's shape) and the per-call ECDH latency, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03v
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -m gpu -x --timeout 300 --timeout-method thread tests/test_gpu_modes.py \
  tests/test_gpu_ecdh.py tests/test_gpu_parity.py -k "golden or kat or modes or ecdh or dropin or cpp" > gpurun_out/r03v/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r03v/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/r03v/tests.log | head -20; exit $rc; fi
for rep in 1 2; do for s in 1 0; do
  FPNN_AES_SYNC_SPIN=$s timeout -k 10 300 python -u tools/bench_percall.py > gpurun_out/r03v/percall_$s.log 2>&1 || { tail -5 gpurun_out/r03v/percall_$s.log; exit 1; }
  echo "spin=$s $(tail -1 gpurun_out/r03v/percall_$s.log | cut -c1-260)"
done; done
for s in 1 0; do
  FPNN_AES_SYNC_SPIN=$s timeout -k 10 300 python -u tools/bench_ecdh.py --no-cpu --percall 200 --curves secp256k1,secp192r1 > gpurun_out/r03v/ecdh_$s.log 2>&1 || { tail -5 gpurun_out/r03v/ecdh_$s.log; exit 1; }
  echo "spin=$s $(tail -1 gpurun_out/r03v/ecdh_$s.log | cut -c1-400)"
done
