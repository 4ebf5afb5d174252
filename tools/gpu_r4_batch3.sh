# eigen: Householder + QL (tri) vs Jacobi + refinement on the C4 shard (time, projector escapes);
# C5 leg (spill predictor column filter over the smaller set)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 400 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 tri > gpurun_out/r4_tri_$tag.log 2>&1; echo rc=$?
grep -E "^(on|tri|off)" gpurun_out/r4_tri_$tag.log | cut -c1-330
timeout -k 10 500 python -u bench.py --c5 only > gpurun_out/r4_c5_$tag.log 2>&1 || { echo c5 failed; tail -5 gpurun_out/r4_c5_$tag.log; exit 1; }
python - "$tag" <<'PY'
import json, sys
txt = open(f"gpurun_out/r4_c5_{sys.argv[1]}.log").read()
d = json.loads([l for l in txt.splitlines() if l.startswith("{")][-1])
c5 = d.get("config5", d)
for g in ("lds", "spill", "spill_big", "one_call"):
    print(g, {k: v for k, v in c5.get(g, {}).items() if isinstance(v, (int, float))})
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -v -s --timeout 500 --timeout-method thread > gpurun_out/r4_local_$tag.log 2>&1
echo local_rc=$?; grep -E "PASSED|FAILED|bisection:|spill units:|Error|assert" gpurun_out/r4_local_$tag.log | head -20
