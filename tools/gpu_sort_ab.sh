# Sorted-sweeps A/B: eigen parity tests with the default (sorted) kernel, then the
# C4 125k-user eigen probe with CF_EIGEN_SORT=0 / 1 (time, sweeps, projector escapes, ev error)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 400 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -k "eigen" -x -v --timeout 200 --timeout-method thread > gpurun_out/sort_tests_$tag.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/sort_tests_$tag.log | tail -3
for s in 0 1; do
  CF_EIGEN_SORT=$s timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/sort${s}_$tag.log 2>&1 || exit 1
  echo "sort=$s"; tail -1 gpurun_out/sort${s}_$tag.log | cut -c1-400
done
