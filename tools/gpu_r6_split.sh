# Round 6: split-storage Jacobi -- parity tests, then the per-bucket A/B probe (split on / off).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-a1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_eigen.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_split_tests_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r6_split_tests_$tag.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_eigen_buckets.py 20000 ${KS:-128,136,144,160,176,180} 1,0 > gpurun_out/r6_split_probe_$tag.log 2>&1
echo probe_rc=$?; cat gpurun_out/r6_split_probe_$tag.log | grep "k="
