# Round 5, batch AG: multi-workgroup basis above k = 768 (up to one user per CU) -- the spill / C5 / uncapped
# tests, then the C5 legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-s1}
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_configs.py tests/test_gpu_predict.py -k "spill or uncapped or c5" -s > gpurun_out/r5/bmin_tests_$tag.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r5/bmin_tests_$tag.log; exit 1; }
tail -3 gpurun_out/r5/bmin_tests_$tag.log
timeout -k 10 400 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/bmin_c5_$tag.json 2> gpurun_out/r5/bmin_c5_$tag.err || { echo "c5 failed"; tail -3 gpurun_out/r5/bmin_c5_$tag.err; exit 1; }
python - $tag <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r5/bmin_c5_{sys.argv[1]}.json").read().strip().splitlines()[-1])
c = d.get("config5", d)
for k in ("spill", "spill_big"):
    print(k, {x: c[k][x] for x in c[k] if isinstance(c[k][x], (int, float))})
print("one_call", c["one_call"])
PY
timeout -k 10 400 python -u tools/c5_shard.py 0 > gpurun_out/r5/c5_shard0_$tag.log 2>&1 || { echo "shard failed"; tail -5 gpurun_out/r5/c5_shard0_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/c5_shard0_$tag.log | tail -2
