# GPU test subset: tools/gpu_tests.sh <log name> <pytest args...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
name=$1; shift
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread "$@" > gpurun_out/$name.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/$name.log; exit 1; }
grep -E "PASSED|FAILED|compared|rows|passed|failed" gpurun_out/$name.log | tail -40
