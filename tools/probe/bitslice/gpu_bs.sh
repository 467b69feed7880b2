cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_bitslice.py -q -x > gpurun_out/bs_test.log 2>&1; rc=$?; tail -3 gpurun_out/bs_test.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ab_bs.py > gpurun_out/ab_bs.json 2>gpurun_out/ab_bs.err; rc=$?; cat gpurun_out/ab_bs.json; tail -2 gpurun_out/ab_bs.err; exit $rc
