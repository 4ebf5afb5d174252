# fused-step correctness + A/B: tools/ab/gpu_fused_ab.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -x -v --timeout 240 --timeout-method thread > gpurun_out/step_test_$tag.log 2>&1 || { echo STEP_TEST_FAILED; tail -30 gpurun_out/step_test_$tag.log; exit 1; }
tail -n 3 gpurun_out/step_test_$tag.log
for f in on off; do
  timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --profile-steps-only --fused $f > gpurun_out/fab_${tag}_$f.log 2>&1 || { echo BENCH_$f FAILED; tail -20 gpurun_out/fab_${tag}_$f.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/fab_${tag}_$f.log').read().strip().splitlines()[-1]);print('$f', round(d['value']), round(d['ms_per_step'],1), json.dumps(d['stages'].get('fused')))"
done
