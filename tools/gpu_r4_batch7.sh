# spill tile_gemm with two staging buffers: spill / C5 / local parity, both spill groups' timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 900 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_eigen.py -k "spill or c5 or local" -v -s --timeout 600 --timeout-method thread > gpurun_out/r4_b7_tests_$tag.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|FAILED|spill rank-deficient" gpurun_out/r4_b7_tests_$tag.log | tail -8
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 3072 5000 > gpurun_out/r4_pspill_big3_$tag.log 2>&1; echo big_rc=$?
grep -v amdgpu.ids gpurun_out/r4_pspill_big3_$tag.log | head -3 | cut -c1-300
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 192 3072 > gpurun_out/r4_pspill_mid3_$tag.log 2>&1; echo mid_rc=$?
grep -v amdgpu.ids gpurun_out/r4_pspill_mid3_$tag.log | head -3 | cut -c1-300
