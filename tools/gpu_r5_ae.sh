# Round 5, batch AE: kernel stats of the C2 local_calc --pct 1 leg (79 units, n up to 10,000)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-ae1}
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_local_$tag -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r5/prof_local_$tag.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5/prof_local_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/prof_local_$tag.log | grep predictions | cut -c1-400
f=$(find gpurun_out/r5/prof_local_$tag -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5/local_kernel_stats_$tag.csv
find gpurun_out/r5/prof_local_$tag -name "*kernel_trace.csv" -delete
head -14 gpurun_out/r5/local_kernel_stats_$tag.csv | cut -d, -f1-5
