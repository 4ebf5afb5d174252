# Round 6: the full GPU suite + smoke, then the default bench line (all legs).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-s1}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r6_suite_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "FAILED|passed|failed|Error" gpurun_out/r6_suite_$tag.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_suite_${tag}_smoke.log 2>&1
echo smoke_rc=$?; tail -2 gpurun_out/r6_suite_${tag}_smoke.log
