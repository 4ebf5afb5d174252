# Round 6: local_calc (w_lim classes + symmetric units) and eigen stream tests, then the C2
# local_calc leg under rocprofv3 kernel stats.  usage: tools/ab/gpu_r6_local.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-a}
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_local.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r6_local_tests_$tag.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|FAILED|unit n =|bisection:" gpurun_out/r6_local_tests_$tag.log | tail -12
[ $rc -eq 0 ] || exit $rc
CF_LOCAL_VERBOSE=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_localprof_$tag -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r6_local_leg_$tag.log 2>&1
echo leg_rc=$?; tail -4 gpurun_out/r6_local_leg_$tag.log | cut -c1-600
f=$(find gpurun_out/r6_localprof_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r6_local_kernel_stats_$tag.csv && head -8 "$f" | cut -c1-160
