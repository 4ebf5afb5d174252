# Round 6: the split kernel with the refinement + epilogue folded in (CF_EIGEN_SPLIT_FINISH=1):
# parity tests, then the per-bucket probe with it off / on, then the C4 step with it on.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-f1}
CF_EIGEN_SPLIT_FINISH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_eigen.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_finish_tests_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "passed|failed|Error" gpurun_out/r6_finish_tests_$tag.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_eigen_buckets.py 20000 ${KS:-144,176,180} 1 > gpurun_out/r6_finish_probe0_$tag.log 2>&1
rc=$?; echo probe0_rc=$rc; grep "k=" gpurun_out/r6_finish_probe0_$tag.log
[ $rc -eq 0 ] || exit $rc
CF_EIGEN_SPLIT_FINISH=1 timeout -k 10 300 python -u tools/probe_eigen_buckets.py 20000 ${KS:-144,176,180} 1 > gpurun_out/r6_finish_probe1_$tag.log 2>&1
rc=$?; echo probe1_rc=$rc; grep "k=" gpurun_out/r6_finish_probe1_$tag.log
[ $rc -eq 0 ] || exit $rc
CF_EIGEN_SPLIT_FINISH=1 timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_finish_steps_$tag.json 2> gpurun_out/r6_finish_steps_$tag.err
echo steps_rc=$?; tail -c 300 gpurun_out/r6_finish_steps_$tag.json
