# Round 6 batch B: the C2 local_calc leg (w_lim class stats, kernel stats) then the hybrid A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-b1}
CF_LOCAL_VERBOSE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_localprof_$tag -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r6_local_leg_$tag.log 2>&1
echo leg_rc=$?; grep -E "^\[local\]|predictions_per_s" gpurun_out/r6_local_leg_$tag.log | cut -c1-400
f=$(find gpurun_out/r6_localprof_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r6_local_kernel_stats_$tag.csv && cut -d, -f1-4 "$f" | head -8 | cut -c1-150
bash tools/ab/gpu_r6_hybrid.sh $tag
