set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pmc off > gpurun_out/bench_quick.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_quick.log; exit 1; }
tail -1 gpurun_out/bench_quick.log
