# Round 5, batch P: the multi-CU cut of the spill eigen path (CF_SPILL_MC_MIN: users above it run
# the staged multi-CU solver, below it one workgroup each) on the C5 legs (sample groups + the
# 10k one call)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-p1}
for v in ${CUTS:-1536 1024 768}; do
  CF_SPILL_MC_MIN=$v timeout -k 10 400 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/mccut_${v}_$tag.json 2> gpurun_out/r5/mccut_${v}_$tag.err || { echo "cut $v failed"; tail -3 gpurun_out/r5/mccut_${v}_$tag.err; exit 1; }
  python - $v $tag <<'PY'
import json, sys
v, tag = sys.argv[1], sys.argv[2]
d = json.loads(open(f"gpurun_out/r5/mccut_{v}_{tag}.json").read().strip().splitlines()[-1])
c = d.get("config5", d)
print("cut", v, "spill eigen ms", round(c["spill"]["ms"], 1), "spill_big eigen ms", round(c["spill_big"]["ms"], 1),
      "one_call ms", round(c["one_call"]["eigen_ms"], 1))
PY
done
