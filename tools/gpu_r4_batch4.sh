# local_calc parity; spill predictor G-mode parity + timings; then the C2 local_calc --pct 1 leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -v -s --timeout 500 --timeout-method thread > gpurun_out/r4_local_$tag.log 2>&1
echo local_rc=$?; grep -E "PASSED|FAILED|bisection:|spill units:|Error|assert" gpurun_out/r4_local_$tag.log | head -20
bash tools/gpu_r4_batch5.sh $tag || exit 1
timeout -k 10 900 python -u tools/local_leg.py > gpurun_out/r4_localleg_$tag.log 2>&1
echo leg_rc=$?; tail -3 gpurun_out/r4_localleg_$tag.log | cut -c1-900
