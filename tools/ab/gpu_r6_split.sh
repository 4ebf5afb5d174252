# Round 6: split-storage Jacobi -- parity tests, the per-bucket A/B probe (split on / off), then the
# C4 step (bench --profile-steps-only) with the split layout on and off on the same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-a1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_eigen.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_split_tests_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r6_split_tests_$tag.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_eigen_buckets.py 20000 ${KS:-136,144,160,176,180} 1,0 > gpurun_out/r6_split_probe_$tag.log 2>&1
rc=$?; echo probe_rc=$rc; grep "k=" gpurun_out/r6_split_probe_$tag.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$STEPS" ]; then
  timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_split_steps_on_$tag.json 2> gpurun_out/r6_split_steps_on_$tag.err
  rc=$?; echo steps_on_rc=$rc; tail -c 400 gpurun_out/r6_split_steps_on_$tag.json
  [ $rc -eq 0 ] || exit $rc
  CF_EIGEN_SPLIT=0 timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_split_steps_off_$tag.json 2> gpurun_out/r6_split_steps_off_$tag.err
  echo steps_off_rc=$?; tail -c 400 gpurun_out/r6_split_steps_off_$tag.json
fi
