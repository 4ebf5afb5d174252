cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_configs.py -k "c5" tests/test_gpu_eigen.py tests/test_gpu_predict.py tests/test_gpu_local.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r3_tests3.log 2>&1
echo rc=$?
grep -E "FAILED|passed|failed|error|compared" gpurun_out/r3_tests3.log | tail -20
timeout -k 10 300 python -u bench.py --c5 only --c5-users 2000 > gpurun_out/r3_c5_2k.log 2>&1
echo rc=$?
tail -c 3000 gpurun_out/r3_c5_2k.log
