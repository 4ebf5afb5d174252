# Round-4 final: GPU suite + smoke, then the default bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
bash tools/gpu_suite.sh r4_suite_$tag
timeout -k 10 1000 python -u bench.py > gpurun_out/r04_bench_$tag.json 2> gpurun_out/r04_bench_$tag.err
echo bench_rc=$?
tail -c 400 gpurun_out/r04_bench_$tag.json
