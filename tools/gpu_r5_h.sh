# Round 5, batch H: the default bench line, then rocprofv3 kernel stats of two C4 steps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-h1}
timeout -k 10 1000 python -u bench.py > gpurun_out/r5/bench_$tag.json 2> gpurun_out/r5/bench_$tag.err
echo bench_rc=$?
tail -c 600 gpurun_out/r5/bench_$tag.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_$tag -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pmc off --io off --c2 off --knn2 off --prep off --c5 off > gpurun_out/r5/prof_$tag.log 2>&1
echo prof_rc=$?
f=$(find gpurun_out/r5/prof_$tag -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/r5/kernel_stats_$tag.csv && head -14 "$f" | cut -d, -f1-8
find gpurun_out/r5/prof_$tag -name "*kernel_trace.csv" -delete
