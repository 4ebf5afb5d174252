# Spill-path check: GPU parity tests of the k > 192 path, then the throughput probe.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eigen.py -k spill -x -v --timeout 200 --timeout-method thread > gpurun_out/spill_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/spill_tests.log; exit 1; }
tail -3 gpurun_out/spill_tests.log
timeout -k 10 300 python -u tools/probe_spill.py ${PROBE:-256:256 600:256 1500:256} > gpurun_out/spill_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/spill_probe.log; exit 1; }
cat gpurun_out/spill_probe.log
