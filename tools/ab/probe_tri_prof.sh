# tridiagonal-path probe under rocprofv3 kernel stats (20k C2 users, both methods)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tri3 -o run -- python3 tools/probe_tri.py 20000 > gpurun_out/tri3.log 2>&1 || { tail -5 gpurun_out/tri3.log; exit 1; }
grep -E "tridiag:|jacobi:|rotations" gpurun_out/tri3.log
sed "s/(anonymous namespace):://g" gpurun_out/prof_tri3/run_kernel_stats.csv | cut -d, -f1-4 | head -6
