# rocprofv3 kernel trace + stats of the timed C4 steps only (no legs, no PMC, no CPU baseline).
# usage: bash tools/gpu_prof_steps.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-steps}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 -u bench.py --profile-steps-only --steps 3 --warmup 1 > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err || { echo rc=$?; tail -5 gpurun_out/prof_$tag.err; exit 1; }
tail -c 600 gpurun_out/prof_$tag.json
f=$(find gpurun_out/prof_$tag -name "*kernel_stats.csv" | head -1)
cut -c1-160 "$f" | head -12
