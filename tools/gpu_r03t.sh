#!/bin/bash
# Round-3 session t: same-box A/B of the mapped host paths (S1 stream frames, C2 package
# frames): ab_libs/base (round-2 pipeline) vs this build with FPNN_AES_MAP_PREP_FIRST=1
# (chunk t + 1 prepared before the cipher of t - 1 is queued) and =0 (cipher first), twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r03t
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "base:0" "cur:1" "cur:0"; do
    lib=${v%%:*}; pf=${v##*:}
    if [ $lib = base ]; then L=ab_libs/base/libfpnn_aes.so; else L=fpnn_amd/libfpnn_aes.so; fi
    FPNN_AES_LIB=$L FPNN_AES_MAP_PREP_FIRST=$pf timeout -k 10 300 python -u tools/bench_configs.py --configs S1 > gpurun_out/r03t/s1.log 2>&1 || { tail -5 gpurun_out/r03t/s1.log; exit 1; }
    echo "$lib prep_first=$pf $(grep -E '^\{"S1"' gpurun_out/r03t/s1.log | cut -c1-200)"
  done
done
