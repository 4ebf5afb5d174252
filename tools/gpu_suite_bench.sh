cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/r3s2_suite_v9.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "FAILED|passed|failed" gpurun_out/r3s2_suite_v9.log | tail -8
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s2_smoke_v9.log 2>&1 || exit 1
tail -2 gpurun_out/r3s2_smoke_v9.log
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_c4_v5.json 2> gpurun_out/bench_c4_v5.err
echo bench_rc=$?
python -c "import json;d=json.load(open('gpurun_out/bench_c4_v5.json'));print(d['value'],d['ms_per_step'],d['stages'] if 'stages' in d else '')"
