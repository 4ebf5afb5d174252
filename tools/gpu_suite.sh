# Full GPU test suite + smoke, output straight into gpurun_out/ (no pipes: progress stays visible)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
name=${1:-r3_suite}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/$name.log 2>&1
echo pytest_rc=$?
grep -E "FAILED|passed|failed|Error" gpurun_out/$name.log | tail -15
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${name}_smoke.log 2>&1
echo smoke_rc=$?
tail -3 gpurun_out/${name}_smoke.log
