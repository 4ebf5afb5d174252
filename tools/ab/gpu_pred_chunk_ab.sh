# Predictor users per launch pair (CF_PRED_CHUNK) on the C4 step, plus the fused-path bitwise test
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/step_tests.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|FAILED" gpurun_out/step_tests.log | tail -3
[ $rc -eq 0 ] || exit 1
for c in 8192 2048 4096 16384 32768; do
  CF_PRED_CHUNK=$c timeout -k 10 300 python -u bench.py --profile-steps-only --steps 3 --warmup 1 > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/chunk_$c.json'));print('chunk $c',round(d['value']),round(d['ms_per_step'],1),{k:round(v,1) for k,v in d.get('stages',{}).items() if 'ms' in k})"
done
