cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do for v in $2; do
  lib=$PWD/fpnn_amd/libfpnn_aes_gpu.so; [ $v != new ] && lib=$PWD/fpnn_amd/libfpnn_aes_gpu_$v.so
  FPNN_AES_GPU_LIB=$lib timeout -k 10 200 python -u tools/probe/q1_time.py > $OUT/q1_${v}_$i.log 2>&1 || { tail -5 $OUT/q1_${v}_$i.log; exit 3; }
  echo "$v #$i: $(grep -h '^{' $OUT/q1_${v}_$i.log | tr '\n' ' ' | cut -c1-400)"
done; done
