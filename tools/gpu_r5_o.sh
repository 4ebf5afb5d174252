# Round 5, batch O: the C2 leg with its local_calc CPU baseline (truncated units beside the
# device on the same units), other secondary legs off
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-o1}
timeout -k 10 1000 python -u bench.py --steps 1 --warmup 1 --pmc off --io off --knn2 off --prep off --c5 off > gpurun_out/r5/lcbase_$tag.json 2> gpurun_out/r5/lcbase_$tag.err
echo bench_rc=$?
python - <<PY
import json
d = json.loads(open("gpurun_out/r5/lcbase_$tag.json").read().strip().splitlines()[-1])
print(json.dumps(d["config2"]["local_calc"], indent=1))
PY
