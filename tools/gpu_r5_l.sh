# Round 5, batch L: the C4 out_eigen_ round trip at full size in text (all 1M records) beside
# the binary form, through bench.py's I/O leg (secondary legs off)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-l1}
df -h /tmp | tail -1
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pmc off --c2 off --knn2 off --prep off --c5 off --io-text-users 1000000 > gpurun_out/r5/io_full_$tag.json 2> gpurun_out/r5/io_full_$tag.err
echo bench_rc=$?
python - <<PY
import json
d = json.loads(open("gpurun_out/r5/io_full_$tag.json").read().strip().splitlines()[-1])
print(json.dumps(d.get("config4_eigen_io"), indent=1))
print("value", d["value"], "eigen_ms", d["stages"]["eigen_ms"], "predict_ms", d["stages"]["predict_ms"])
PY
