# Round-4 profile: rocprofv3 kernel stats of the C4 steps (no secondary legs), then the spill
# G-mode parity tests and the k > 3072 spill predictor timing on the current build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4_$tag -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pmc off --io off --c2 off --knn2 off --prep off --c5 off > gpurun_out/prof_r4_$tag.log 2>&1
echo prof_rc=$?
f=$(find gpurun_out/prof_r4_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -14 "$f" | cut -d, -f1-8
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_predict.py -k "spill" -v -s --timeout 600 --timeout-method thread > gpurun_out/r4_gmode2_tests_$tag.log 2>&1
echo tests_rc=$?; grep -E "PASSED|FAILED|spill rank-deficient" gpurun_out/r4_gmode2_tests_$tag.log | head -12
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 3072 5000 > gpurun_out/r4_pspill_big2_$tag.log 2>&1; echo big_rc=$?
grep -v amdgpu.ids gpurun_out/r4_pspill_big2_$tag.log | head -4 | cut -c1-300
