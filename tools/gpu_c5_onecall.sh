# C5 one-call breakdown (tools/probe_c5_onecall.py) with a rocprofv3 kernel-stats pass
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 400 python -u tools/probe_c5_onecall.py 10000 all,big,mid > gpurun_out/c5oc_$tag.log 2>&1 && cat gpurun_out/c5oc_$tag.log | grep -v graph &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c5oc_prof_$tag -o run -- python -u tools/probe_c5_onecall.py 10000 all > gpurun_out/c5oc_prof_$tag.log 2>&1
echo "prof rc=$?"
f=$(find gpurun_out/c5oc_prof_$tag -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-4 $f | head -14
