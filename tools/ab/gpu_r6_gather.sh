# Round 6: batched graph gather in the split kernel + pipelined B load in the RESUME kernel: parity
# tests, then the C4 step with this build and with the previous one (CF_MI355X_LIB) on the same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-g1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_eigen.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gather_tests_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "passed|failed|Error" gpurun_out/r6_gather_tests_$tag.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in new prev new prev; do
  if [ $v = prev ]; then export CF_MI355X_LIB=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_prev.so; else unset CF_MI355X_LIB; fi
  timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_gather_steps_${v}_$tag.json 2> gpurun_out/r6_gather_steps_${v}_$tag.err
  rc=$?; [ $rc -eq 0 ] || { echo steps_${v}_rc=$rc; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r6_gather_steps_${v}_$tag.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), round(d['ms_per_step'],1), round(d['stages']['eigen_ms'],1), round(d['stages']['predict_ms'],1))" | tee -a gpurun_out/r6_gather_summary_$tag.txt
done
