# Eigen epilogue/assembly change check: k = 180 and C2-mix stage times, then every -m gpu test.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for kf in 180 0; do
  timeout -k 10 200 python -u tools/probe_eigen_ab.py 100000 $kf > gpurun_out/epi_k${kf}.log 2>&1 || { echo "AB k=$kf FAILED"; tail -5 gpurun_out/epi_k${kf}.log; exit 1; }
  echo "k=$kf: $(tail -n 1 gpurun_out/epi_k${kf}.log)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_epi.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests_epi.log; exit 1; }
tail -2 gpurun_out/gpu_tests_epi.log
