# Round 5: full GPU test suite + smoke (output under gpurun_out/r5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
name=${1:-suite}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r5/$name.log 2>&1
echo pytest_rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5/$name.log | tail -15
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/${name}_smoke.log 2>&1
echo smoke_rc=$?
tail -3 gpurun_out/r5/${name}_smoke.log
