# Same-box A/B of builds of the GPU library (the front loads FPNN_AES_GPU_LIB):
#   bash tools/probe/ab_lib.sh <tag> <configs|bench> [variants]
# variants (default "base new"): "new" is fpnn_amd/libfpnn_aes_gpu.so, any other name X is
# fpnn_amd/libfpnn_aes_gpu_X.so beside it; each runs twice, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for i in 1 2; do
  for v in ${3:-base new}; do
    lib=$PWD/fpnn_amd/libfpnn_aes_gpu.so; [ $v != new ] && lib=$PWD/fpnn_amd/libfpnn_aes_gpu_$v.so
    if [ "$2" = bench ]; then
      FPNN_AES_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/ab_${v}_$i.log" 2>&1 || exit 3
      echo "$v #$i: $(grep -o '"value": [0-9.]*\|"payload_GiBs": [0-9.]*' "$OUT/ab_${v}_$i.log" | tr '\n' ' ')"
    else
      FPNN_AES_GPU_LIB=$lib timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --no-host --configs "$2" \
        > "$OUT/ab_${v}_$i.log" 2>&1 || exit 3
      echo "$v #$i: $(grep -h '^{"configs"' "$OUT/ab_${v}_$i.log" | cut -c1-600)"
    fi
  done
done
