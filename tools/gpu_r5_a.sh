# Round 5, batch A: HUGE spill layout (local_calc without a neighbourhood cap) parity, the C2
# predictor per sort direction, and the kernel statistics of the uncapped C2 local_calc leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-a1}
timeout -k 10 900 python -u -m pytest tests/test_gpu_local.py tests/test_gpu_eigen.py tests/test_gpu_step.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r5/tests_$tag.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "PASSED|FAILED|ERROR|passed|failed|unit n =|HUGE layout" gpurun_out/r5/tests_$tag.log | tail -30
[ $rc -eq 0 ] || exit $rc
for s in 2 1; do
  CF_EIGEN_SORT=$s PROBE_CFG=c2 PROBE_SAVE=gpurun_out/r5/c2_sort$s.npz timeout -k 10 300 python -u tools/probe_c4.py 100000 > gpurun_out/r5/c2_sort$s.log 2>&1 || { echo "probe sort $s rc=$?"; exit 1; }
  grep -E "eigen:|predict:|phase share|fast ratings|block cycles" gpurun_out/r5/c2_sort$s.log
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_local_$tag -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r5/local_leg_$tag.log 2>&1
echo local_rc=$?
tail -1 gpurun_out/r5/local_leg_$tag.log | cut -c1-700
f=$(find gpurun_out/r5/prof_local_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -16 "$f" | cut -d, -f1-8
