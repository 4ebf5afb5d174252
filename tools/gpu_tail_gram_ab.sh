# Gram-checked last sweep A/B: eigen parity tests with the default build, then
# the C4 125k-user eigen probe with CF_EIGEN_TAIL=0 / 1 (time, sweeps, escapes, ev error)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -k "eigen" -x -v --timeout 200 --timeout-method thread > gpurun_out/tailg_tests_$tag.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed|Error" gpurun_out/tailg_tests_$tag.log | tail -4
for t in 0 1; do
  CF_EIGEN_TAIL=$t timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/tailg${t}_$tag.log 2>&1 || { echo "probe $t failed"; tail -3 gpurun_out/tailg${t}_$tag.log; exit 1; }
  echo "tail=$t"; tail -1 gpurun_out/tailg${t}_$tag.log | cut -c1-400
done
