# C4-shard predictor A/B of the in-tree build against every variants/libcf_*.so (tools/build_variant.sh):
# tools/probe_c4.py timing + phases per build, outputs compared with the in-tree build's, then the
# predictor / step GPU tests on the in-tree build.  usage: gpu_probe_variants.sh <tag> [users]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}; users=${2:-125000}
run() {   # name, env...
  local name=$1; shift
  env "$@" PROBE_SAVE=gpurun_out/pv_$name.npz timeout -k 10 300 python -u tools/probe_c4.py $users > gpurun_out/pv_${name}_$tag.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/pv_${name}_$tag.log; exit 1; }
  echo "== $name"; grep -E "^(eigen|predict|phase|fast)" gpurun_out/pv_${name}_$tag.log | cut -c1-250
}
run intree CF_NOTHING=1
for f in collaborative_filtering_amd/variants/libcf_*.so; do
  [ -e "$f" ] || continue
  v=$(basename $f .so); run ${v#libcf_} CF_MI355X_LIB=$GRAFT_REPO_ROOT/$f
done
run intree2 CF_NOTHING=1
python - <<'PY'
import glob, numpy as np
a = np.load("gpurun_out/pv_intree.npz")
for f in sorted(glob.glob("gpurun_out/pv_*.npz")):
    if f.endswith("pv_intree.npz"):
        continue
    b = np.load(f)
    d = np.abs(a["mse"].astype(np.float64) - b["mse"])
    print(f, "kk equal", bool((a["kk"] == b["kk"]).all()), "mse bits differ", int((a["mse"].view(np.uint32) != b["mse"].view(np.uint32)).sum()),
          "max |d|", float(np.nanmax(d)), "rows |d| > 1e-4", int((d > 1e-4).sum()))
PY
rm -f gpurun_out/pv_*.npz
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_step.py -k "predict or step or mask" -x -q --timeout 300 --timeout-method thread > gpurun_out/pv_tests_$tag.log 2>&1
echo tests_rc=$?; tail -3 gpurun_out/pv_tests_$tag.log
