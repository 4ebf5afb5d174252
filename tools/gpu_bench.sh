# Default bench run (N=1), JSON line + stderr progress into gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
name=${1:-r3_bench}
shift
timeout -k 10 1100 python -u bench.py "$@" > gpurun_out/$name.json 2> gpurun_out/$name.err
echo bench_rc=$?
tail -c 6000 gpurun_out/$name.json
