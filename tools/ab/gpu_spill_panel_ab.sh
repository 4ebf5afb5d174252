# Spill predictor wide LDL^T: two-level panels of CF_SPILL_LDL_PANEL columns (128 default / 256 / 64) on the C5 sample, + spill parity tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_local.py -m gpu -k "spill or c5 or local" -x -v --timeout 500 --timeout-method thread > gpurun_out/spill_tests.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|FAILED" gpurun_out/spill_tests.log | tail -4
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_cap2816.log 2>&1 || exit 1
echo "== small-kernel cap 2816"; grep -E "ratings in|raw" gpurun_out/pspill_cap2816.log
for v in NONE; do [ "$v" = NONE ] && break
  CF_MI355X_LIB=$PWD/collaborative_filtering_amd/variants/libcf_$v.so timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_$v.log 2>&1 || exit 1
  echo "== $v"; grep -E "ratings in|raw" gpurun_out/pspill_$v.log
done
