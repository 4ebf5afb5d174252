# Round 5, batch V: eigen spill budget 0.75 by default -- spill / C5 / HUGE tests, the C5 legs,
# and one full-size C5 shard (eigen, release, predict)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-v1}
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_eigen.py tests/test_gpu_configs.py tests/test_gpu_local.py -k "spill or uncapped or c5 or huge or large_unit or release" -s > gpurun_out/r5/budget_tests_$tag.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r5/budget_tests_$tag.log; exit 1; }
tail -2 gpurun_out/r5/budget_tests_$tag.log
timeout -k 10 400 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/budget_c5_$tag.json 2> gpurun_out/r5/budget_c5_$tag.err || { echo "c5 failed"; tail -3 gpurun_out/r5/budget_c5_$tag.err; exit 1; }
python - gpurun_out/r5/budget_c5_$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config5", d)
for k in ("spill", "spill_big"):
    print(k, "eigen", round(c[k]["ms"], 1), "predict", round(c[k]["predict_ms"], 1), "ratings/s", round(c[k]["ratings_per_s"]))
print("one_call eigen ms", round(c["one_call"]["eigen_ms"], 1))
PY
timeout -k 10 400 python -u tools/c5_shard.py 0 > gpurun_out/r5/c5_shard0_$tag.log 2>&1 || { echo "shard failed"; tail -5 gpurun_out/r5/c5_shard0_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/c5_shard0_$tag.log | tail -3
