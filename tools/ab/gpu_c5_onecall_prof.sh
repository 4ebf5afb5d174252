# Kernel trace of the config-5 one-call eigen leg (10k users): which kernels set its time.
# usage: bash tools/ab/gpu_c5_onecall_prof.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/${1:-c5prof}
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python3 -u bench.py --c5 only --c5-users 100 > $out/c5.json 2> $out/c5.err || { echo rc=$?; tail -5 $out/c5.err; exit 1; }
grep -v amdgpu $out/c5.err | tail -12
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
head -15 "$f"
