# Round 5, batch R: the k > kSmallCap spill predictor users on <T, 0, 2> (per-row arrays in HBM,
# two workgroups per CU) vs <T, CF_SPILL_MAX_K, 1> (LDS rows, one per CU): C5 sample big group
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-r1}
for v in 0 1; do
  CF_PSPILL_BIG2=$v timeout -k 10 300 python -u tools/probe_pspill_ab.py 1000 2816 5000 gpurun_out/r5/big2_${v}_$tag.npz > gpurun_out/r5/big2_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/big2_${v}_$tag.log; exit 1; }
  cat gpurun_out/r5/big2_${v}_$tag.log
done
python - $tag <<'PY'
import sys, numpy as np
t = sys.argv[1]
a, b = np.load(f"gpurun_out/r5/big2_0_{t}.npz"), np.load(f"gpurun_out/r5/big2_1_{t}.npz")
print("kk equal", np.array_equal(a["kk"], b["kk"]), "mse bit-identical", np.array_equal(a["mse"], b["mse"], equal_nan=True),
      "max |d mse|", float(np.nanmax(np.abs(a["mse"] - b["mse"]))))
PY
