# Round check on one GPU: the -m gpu suite, smoke(), then tools/profile_round.sh <tag>.
# usage: bash tools/round_check.sh <tag>
set -o pipefail
tag=${1:-v5}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/profile_round.sh $tag
# config-4 per-GPU shard (125k users x 50k items, the metric's 1M-user config split over 8)
timeout -k 10 600 python3 -u bench.py --users 125000 --items 50000 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --knn2 off --c5 off > gpurun_out/scale_c4_$tag.log 2>&1 || { echo C4_FAILED; tail -5 gpurun_out/scale_c4_$tag.log; exit 1; }
tail -1 gpurun_out/scale_c4_$tag.log | cut -c1-200
echo ROUND_OK
