# Staged spill waves pipelined on two side streams: spill / C5 / local GPU tests, then the C5
# one-call breakdown with CF_SPILL_PIPE=1 (default) and 0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py tests/test_gpu_local.py -k "spill or c5 or local" -x -v --timeout 300 --timeout-method thread > gpurun_out/pipe_tests_$tag.log 2>&1
echo "tests rc=$?"; grep -E "passed|failed" gpurun_out/pipe_tests_$tag.log | tail -3
timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 all > gpurun_out/pipe1_$tag.log 2>&1 && grep "^all" gpurun_out/pipe1_$tag.log &&
CF_SPILL_PIPE=0 timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 all > gpurun_out/pipe0_$tag.log 2>&1 && grep "^all" gpurun_out/pipe0_$tag.log
