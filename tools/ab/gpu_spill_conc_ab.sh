# Spill predictor: the k > 2048 launch beside the rest (default) vs one after the other; spill/C5/local tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_step.py -m gpu -k "spill or c5 or local or step or deterministic or fused" -x -v --timeout 500 --timeout-method thread > gpurun_out/spill_tests.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|FAILED" gpurun_out/spill_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_conc.log 2>&1 || exit 1
echo "== concurrent"; grep -E "ratings in|raw" gpurun_out/pspill_conc.log
CF_PSPILL_CONCURRENT=0 timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_seq.log 2>&1 || exit 1
echo "== sequential"; grep -E "ratings in|raw" gpurun_out/pspill_seq.log
