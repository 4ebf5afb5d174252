# Round 5, batch Q: no k cap for compute_eigens users (k > CF_SPILL_MAX_K: the eigen HUGE layout,
# the spill predictor's per-row arrays in HBM) -- the new k = 5400 test, the spill / C5 / HUGE
# tests around it, then the C5 legs to check the spill predictor's timing is unchanged
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-q1}
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_configs.py::test_uncapped_user_above_5000" \
  "tests/test_gpu_configs.py::test_c5_tail_k_up_to_5000" \
  "tests/test_gpu_local.py::test_spill_huge_layout_bit_identical" \
  "tests/test_gpu_local.py::test_local_calc_large_unit_predictions" \
  tests/test_gpu_eigen.py -k "spill or uncapped or c5 or huge or large_unit" -s > gpurun_out/r5/uncap_tests_$tag.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r5/uncap_tests_$tag.log; exit 1; }
tail -5 gpurun_out/r5/uncap_tests_$tag.log
timeout -k 10 400 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/uncap_c5_$tag.json 2> gpurun_out/r5/uncap_c5_$tag.err || { echo "c5 failed"; tail -3 gpurun_out/r5/uncap_c5_$tag.err; exit 1; }
python - $tag <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r5/uncap_c5_{sys.argv[1]}.json").read().strip().splitlines()[-1])
c = d.get("config5", d)
for k in ("spill", "spill_big"):
    print(k, {x: c[k][x] for x in c[k] if isinstance(c[k][x], (int, float))})
print("one_call", c["one_call"])
PY
