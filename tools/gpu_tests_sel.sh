# usage: bash tools/gpu_tests_sel.sh <pytest selection...>   (one pytest process, per-test timeout)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1
rc=$?
tail -30 gpurun_out/sel_tests.log
exit $rc
