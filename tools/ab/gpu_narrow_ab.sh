# A/B of the narrow bucket-12 eigen layout (CF_EIGEN_NARROW=0/1) on k = 180 and the C2 mix,
# then the eigen parity tests with the narrow layout on: tools/ab/gpu_narrow_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for kf in 180 0; do
  for nw in 0 1; do
    CF_EIGEN_NARROW=$nw timeout -k 10 200 python -u tools/probe_eigen_ab.py 100000 $kf > gpurun_out/nab_k${kf}_n${nw}.log 2>&1 || { echo "AB k=$kf narrow=$nw FAILED"; tail -5 gpurun_out/nab_k${kf}_n${nw}.log; exit 1; }
    echo "k=$kf narrow=$nw: $(tail -n 1 gpurun_out/nab_k${kf}_n${nw}.log)"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_eigen.py tests/test_gpu_configs.py -m gpu > gpurun_out/narrow_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/narrow_tests.log; exit 1; }
tail -3 gpurun_out/narrow_tests.log
