# Round 5, batch C: dense-queue predictor + MFMA/Illinois w_lim kernel: parity tests, the C2
# predictor per sort direction, the uncapped C2 local_calc leg (timing, then kernel stats)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-c1}
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py tests/test_gpu_predict.py tests/test_gpu_step.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r5/tests_$tag.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "FAILED|ERROR|passed|failed|unit n =|bisection:|HUGE layout" gpurun_out/r5/tests_$tag.log | tail -20
[ $rc -eq 0 ] || exit $rc
for s in 2 1; do
  CF_EIGEN_SORT=$s PROBE_CFG=c2 timeout -k 10 300 python -u tools/probe_c4.py 100000 > gpurun_out/r5/c2_sort${s}_$tag.log 2>&1 || { echo "probe sort $s rc=$?"; exit 1; }
  grep -E "eigen:|predict:" gpurun_out/r5/c2_sort${s}_$tag.log
done
timeout -k 10 600 python -u tools/local_leg.py c2 1 > gpurun_out/r5/local_leg_$tag.log 2>&1
echo local_rc=$?; grep -v amdgpu.ids gpurun_out/r5/local_leg_$tag.log | tail -2 | cut -c1-900
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_local_$tag -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r5/local_leg_prof_$tag.log 2>&1
echo prof_rc=$?
f=$(find gpurun_out/r5/prof_local_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r5/local_kernel_stats_$tag.csv && head -14 "$f" | cut -d, -f1-4
find gpurun_out/r5/prof_local_$tag -name "*kernel_trace.csv" -delete
