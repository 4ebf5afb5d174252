# Predictor A/B on the C4 125k-user shard (tools/probe_c4.py): in-tree build (eigen->predictor
# masks, tail-only last basis step, DPP wave sums) vs CF_PRED_TAIL=0 vs the ds_bpermute wave-sum
# variant (variants/libcf_shfl.so); outputs compared; then the predictor / step GPU tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
run() {   # name, env...
  local name=$1; shift
  env "$@" PROBE_SAVE=gpurun_out/pab_$name.npz timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/pab_${name}_$tag.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/pab_${name}_$tag.log; exit 1; }
  echo "== $name"; grep -E "^(eigen|predict|phase|fast)" gpurun_out/pab_${name}_$tag.log | cut -c1-250
}
run intree CF_NOTHING=1
run tail0 CF_PRED_TAIL=0
run shfl CF_MI355X_LIB=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_shfl.so
run nomask CF_STEP_MASKS=0
[ -e collaborative_filtering_amd/variants/libcf_ieee.so ] && run ieee CF_MI355X_LIB=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_ieee.so
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/pab_intree.npz")
import os
for nm in [x for x in ("tail0", "shfl", "nomask", "ieee") if os.path.exists(f"gpurun_out/pab_{x}.npz")]:
    b = np.load(f"gpurun_out/pab_{nm}.npz")
    d = np.abs(a["mse"].astype(np.float64) - b["mse"])
    print(nm, "kk equal", bool((a["kk"] == b["kk"]).all()), "mse bits differ", int((a["mse"].view(np.uint32) != b["mse"].view(np.uint32)).sum()),
          "of", a["mse"].size, "max |d|", float(np.nanmax(d)), "rows |d| > 1e-4", int((d > 1e-4).sum()))
PY
rm -f gpurun_out/pab_*.npz
timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/pab_refine_$tag.log 2>&1 && tail -1 gpurun_out/pab_refine_$tag.log | cut -c1-330 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_step.py -k "predict or step or mask" -x -q --timeout 300 --timeout-method thread > gpurun_out/pab_tests_$tag.log 2>&1
echo tests_rc=$?; tail -3 gpurun_out/pab_tests_$tag.log
