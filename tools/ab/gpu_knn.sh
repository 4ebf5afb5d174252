set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/knn_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/knn_tests.log; exit 1; }
tail -3 gpurun_out/knn_tests.log
timeout -k 10 400 python -u bench.py --knn2 only --cpu-seconds 8 > gpurun_out/knn2_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/knn2_bench.log; exit 1; }
tail -1 gpurun_out/knn2_bench.log
