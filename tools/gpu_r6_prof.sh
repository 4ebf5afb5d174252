# Round 6 profile: the default bench line (all legs), then rocprofv3 kernel stats of the C4 steps
# (bench.py --profile-steps-only: the same timed step as the line's value).
# usage: bash tools/gpu_r6_prof.sh <tag>
set -o pipefail
tag=${1:-p1}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/r6_bench_$tag.json 2> gpurun_out/r6_bench_$tag.err || { echo BENCH_FAILED; tail -20 gpurun_out/r6_bench_$tag.err; exit 1; }
tail -c 600 gpurun_out/r6_bench_$tag.json
[ -n "$NOPROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_$tag.log; exit 1; }
head -12 gpurun_out/prof_$tag/run_kernel_stats.csv | cut -c1-220
echo PROFILE_OK
