# predictor iteration: GPU predict/config/pipeline tests, then the C4 probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_pipeline.py -m gpu > gpurun_out/pred_tests_$tag.log 2>&1 || { echo TESTS_FAILED; grep -E "PASSED|FAILED|Error|error" gpurun_out/pred_tests_$tag.log | tail -30; tail -60 gpurun_out/pred_tests_$tag.log; exit 1; }
grep -E "PASSED|FAILED|compared|rows" gpurun_out/pred_tests_$tag.log | tail -40
timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/probe_c4_$tag.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/probe_c4_$tag.log; exit 1; }
cat gpurun_out/probe_c4_$tag.log
