# Predictor A/B: eigen->predictor complement masks (CF_STEP_MASKS) and the tail-only last basis
# step (CF_PRED_TAIL): C4 shard predict time + phases, outputs bit-equal, predictor tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
for mt in 00 10 11; do
  CF_STEP_MASKS=${mt:0:1} CF_PRED_TAIL=${mt:1:1} PROBE_SAVE=gpurun_out/mt$mt.npz timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/mt${mt}_$tag.log 2>&1 || exit 1
  echo "masks,tail=$mt"; grep -E "^(eigen|predict|phase|fast)" gpurun_out/mt${mt}_$tag.log | cut -c1-250
done
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/mt00.npz")
for mt in ("10", "11"):
    b = np.load(f"gpurun_out/mt{mt}.npz")
    print(mt, "kk equal", bool((a["kk"] == b["kk"]).all()), "mse bits differ", int((a["mse"].view(np.uint32) != b["mse"].view(np.uint32)).sum()),
          "of", a["mse"].size, "max |d|", float(np.nanmax(np.abs(a["mse"] - b["mse"]))))
PY
rm -f gpurun_out/mt*.npz   # ~100 MB each: gpurun_out comes back only under 64 MiB
timeout -k 10 500 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_step.py -k "predict or step" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_tail_tests_$tag.log 2>&1
echo tests_rc=$?; tail -3 gpurun_out/r4_tail_tests_$tag.log
