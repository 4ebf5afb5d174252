# round-2 first GPU pass: host info, GPU tests, C4 bench (short), logs under gpurun_out/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
{ nproc; python -c 'import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>&1; free -g | head -2; df -h /tmp | tail -1; } > gpurun_out/host_info.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --pmc off --c2 off --knn2 off --c5 off > gpurun_out/bench_c4_quick.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_c4_quick.log; exit 1; }
tail -1 gpurun_out/bench_c4_quick.log
