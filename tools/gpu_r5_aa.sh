# Round 5, batch AA: kernel stats of one full-size C5 shard (eigen, release, predict)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-aa1}
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_shard_$tag -o run -- python3 -u tools/c5_shard.py 0 > gpurun_out/r5/prof_shard_$tag.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5/prof_shard_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/prof_shard_$tag.log | grep shard | tail -2 | cut -c1-300
f=$(find gpurun_out/r5/prof_shard_$tag -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5/shard_kernel_stats_$tag.csv
find gpurun_out/r5/prof_shard_$tag -name "*kernel_trace.csv" -delete
head -14 gpurun_out/r5/shard_kernel_stats_$tag.csv | cut -d, -f1-5
