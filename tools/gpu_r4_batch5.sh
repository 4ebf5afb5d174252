# spill predictor G-mode: parity (spill + C5 tail tests), then both spill groups' timing (C5 sample)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 700 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py -k "spill or c5_tail" -v -s --timeout 600 --timeout-method thread > gpurun_out/r4_gmode_tests_$tag.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "PASSED|FAILED|vs min-norm|Error|assert" gpurun_out/r4_gmode_tests_$tag.log | head -30
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 3072 5000 > gpurun_out/r4_pspill_big_$tag.log 2>&1; echo big_rc=$?
grep -v amdgpu.ids gpurun_out/r4_pspill_big_$tag.log | head -8 | cut -c1-400
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 192 3072 > gpurun_out/r4_pspill_mid_$tag.log 2>&1; echo mid_rc=$?
grep -v amdgpu.ids gpurun_out/r4_pspill_mid_$tag.log | head -8 | cut -c1-400
