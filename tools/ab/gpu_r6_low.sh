# Round 6: buckets 5-8 in the split layout (refinement + epilogue in the split kernel): parity, the
# per-bucket probe (split from bucket 5 vs off), and the C4 step with the split layout from bucket 5
# against the default (from bucket 9) on the same box.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-l1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_low_tests_$tag.log 2>&1
rc=$?; echo pytest_rc=$rc; grep -E "passed|failed|Error" gpurun_out/r6_low_tests_$tag.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_eigen_buckets.py 20000 ${KS:-72,96,112,128} 5,0 > gpurun_out/r6_low_probe_$tag.log 2>&1
rc=$?; echo probe_rc=$rc; grep "k=" gpurun_out/r6_low_probe_$tag.log
[ $rc -eq 0 ] || exit $rc
CF_EIGEN_SPLIT=${MIN:-5} timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_low_steps_on_$tag.json 2> gpurun_out/r6_low_steps_on_$tag.err
rc=$?; echo steps_on_rc=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --profile-steps-only --steps 5 --warmup 2 > gpurun_out/r6_low_steps_def_$tag.json 2> gpurun_out/r6_low_steps_def_$tag.err
echo steps_def_rc=$?
python3 - <<PY
import json
for f in ("on", "def"):
    d = json.loads(open(f"gpurun_out/r6_low_steps_{f}_$tag.json").read().strip().splitlines()[-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 1), round(d["stages"]["eigen_ms"], 1), round(d["stages"]["predict_ms"], 1))
PY
