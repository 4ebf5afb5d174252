# Round 5, batch W: kernel stats of the C5 10k one-call eigen (budget 0.75, one wave)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-w1}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_onecall_$tag -o run -- python3 -u tools/probe_c5_onecall.py 10000 big > gpurun_out/r5/prof_onecall_$tag.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5/prof_onecall_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/prof_onecall_$tag.log | grep -E "^all|^big|^mid|eigen" | tail -5
f=$(find gpurun_out/r5/prof_onecall_$tag -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5/onecall_kernel_stats_$tag.csv
find gpurun_out/r5/prof_onecall_$tag -name "*kernel_trace.csv" -delete
head -14 gpurun_out/r5/onecall_kernel_stats_$tag.csv | cut -d, -f1-6
