# round-2 full default bench (all legs) + rocprofv3 kernel stats of the C4 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --steps 3 --warmup 1 --profile-steps-only > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/bench_prof.log; exit 1; }
tail -1 gpurun_out/bench_prof.log
ls -R gpurun_out/prof_c4 | head
