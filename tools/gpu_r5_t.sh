# Round 5, batch T: cf_release_workspaces before the C5 one-call eigen (the predictor legs'
# spill workspace no longer shrinks its budget); the release test; the C5 legs twice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-t1}
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_eigen.py -k "release or spill_path_mixed" > gpurun_out/r5/release_tests_$tag.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r5/release_tests_$tag.log; exit 1; }
tail -2 gpurun_out/r5/release_tests_$tag.log
for i in 1 2; do
timeout -k 10 400 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/rel_c5_${tag}_$i.json 2> gpurun_out/r5/rel_c5_${tag}_$i.err || { echo "c5 failed"; tail -3 gpurun_out/r5/rel_c5_${tag}_$i.err; exit 1; }
python - gpurun_out/r5/rel_c5_${tag}_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config5", d)
for k in ("spill", "spill_big"):
    print(k, "eigen", round(c[k]["ms"], 1), "predict", round(c[k]["predict_ms"], 1), "ratings/s", round(c[k]["ratings_per_s"]))
print("one_call eigen ms", round(c["one_call"]["eigen_ms"], 1))
PY
done
