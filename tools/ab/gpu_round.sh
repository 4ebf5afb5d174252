# One round checkpoint on the GPU box: every -m gpu test, the default bench line, and the
# rocprofv3 kernel stats of a short C4 run.  usage: bash tools/gpu_round.sh <tag> [tests|bench|prof]...
set -o pipefail
tag=${1:-v0}; shift
steps=${*:-tests bench prof}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in $steps; do
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread \
      > gpurun_out/gpu_tests_$tag.log 2>&1 || { echo TESTS_FAILED; tail -n 40 gpurun_out/gpu_tests_$tag.log; exit 1; }
    tail -n 2 gpurun_out/gpu_tests_$tag.log ;;
  bench)
    timeout -k 10 800 python -u bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo BENCH_FAILED; tail -n 20 gpurun_out/bench_$tag.log; exit 1; }
    tail -n 1 gpurun_out/bench_$tag.log | cut -c1-400 ;;
  prof)
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
      python3 bench.py --steps 3 --warmup 1 --profile-steps-only > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_FAILED; tail -n 20 gpurun_out/prof_$tag.log; exit 1; }
    tail -n 1 gpurun_out/prof_$tag.log | cut -c1-300 ;;
  dist)
    # N = 2 rehearsal on one GPU: two ranks share the device over gloo (the driver's 8-GPU runs use RCCL)
    CF_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --users 200000 \
      --no-cpu-baseline --pmc off > gpurun_out/dist2_$tag.log 2>&1 || { echo DIST_FAILED; tail -n 30 gpurun_out/dist2_$tag.log; exit 1; }
    grep '"metric"' gpurun_out/dist2_$tag.log | cut -c1-400 ;;
  esac
done
echo ROUND_OK
