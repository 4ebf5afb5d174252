# C5 leg A/B of the staged multi-CU cut (CF_SPILL_MC_MIN): bench.py --c5 only per setting
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
shift
for c in "$@"; do
  CF_SPILL_MC_MIN=$c timeout -k 10 400 python -u bench.py --c5 only > gpurun_out/r4_c5mc${c}_$tag.log 2>&1 || { echo "mc_min=$c failed"; exit 1; }
  echo "mc_min=$c"; python - "$c" "$tag" <<'PY'
import json, sys
c, tag = sys.argv[1], sys.argv[2]
txt = open(f"gpurun_out/r4_c5mc{c}_{tag}.log").read()
d = json.loads([l for l in txt.splitlines() if l.startswith("{")][-1])
c5 = d.get("config5", d)
def walk(o, pre=""):
    if isinstance(o, dict):
        for k, v in o.items():
            walk(v, pre + k + ".")
    elif isinstance(o, (int, float)) and any(s in pre for s in ("_s.", "_ms.", "per_s.", "users.", "ratings")):
        print(f"  {pre[:-1]} = {o:.4g}")
walk(c5)
PY
done
