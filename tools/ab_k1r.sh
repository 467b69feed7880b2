cd $GRAFT_REPO_ROOT
for rep in 1 2; do for v in old new; do
  if [ $v = old ]; then export FPNN_AES_LIB=$PWD/tools/probe/ablib/lib_old.so; else unset FPNN_AES_LIB; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/probe_k1r.py 2>&1 | grep -v amdgpu.ids | grep -E "streamR|stream0" || exit 1
  timeout -k 10 300 python tools/bench_configs.py --reps 3 --no-host --configs C3,C4,R1 2>&1 | grep '"configs"' | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['configs']; print('C3 framed', d['C3']['framed_decrypt_wall_GiBs'], d['C3']['framed_decrypt_kernel_GiBs'], 'C4 dec', d['C4']['decrypt_kernel_GiBs'], 'R1', d['R1']['recv_wall_GiBs'], d['R1']['decrypt_kernel_GiBs'])" || exit 1
done; done
