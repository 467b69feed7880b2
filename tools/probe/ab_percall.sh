# Same-box A/B of per-call latency for two builds of the GPU library (FPNN_AES_GPU_LIB):
#   bash tools/probe/ab_percall.sh <tag>   with fpnn_amd/libfpnn_aes_gpu_base.so beside the build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for i in 1 2 3; do
  for v in base new; do
    lib=$PWD/fpnn_amd/libfpnn_aes_gpu.so; [ $v = base ] && lib=$PWD/fpnn_amd/libfpnn_aes_gpu_base.so
    FPNN_AES_GPU_LIB=$lib timeout -k 10 200 python -u tools/bench_percall.py > "$OUT/percall_${v}_$i.log" 2>&1 || exit 3
    echo "$v #$i: $(grep -o '"us_per_encrypt": [0-9.]*, "us_per_decrypt": [0-9.]*' "$OUT/percall_${v}_$i.log" | head -1)"
  done
done
