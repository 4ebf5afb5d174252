# Round 6: the default bench line (all legs), stderr kept apart.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-b1}
timeout -k 10 1100 python3 -u bench.py ${BENCH_ARGS:-} > gpurun_out/r6_bench_$tag.json 2> gpurun_out/r6_bench_$tag.err
rc=$?; echo bench_rc=$rc; tail -c 600 gpurun_out/r6_bench_$tag.json; tail -3 gpurun_out/r6_bench_$tag.err
