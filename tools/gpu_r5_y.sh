# Round 5, batch Y: multi-workgroup spill basis (spill_basis_mc) vs one workgroup per user
# (CF_PSPILL_BASIS_MC=0): timing and bit-identity of mse / kk on the C5 sample's k > 2816 users
# and on its 192 < k <= 3072 users (a chunk mixing both basis kernels)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-y1}
for set in "2816 5000" "192 3072"; do
  lo=${set% *}; hi=${set#* }
  for v in 0 1; do
    CF_PSPILL_BASIS_MC=$v timeout -k 10 300 python -u tools/probe_pspill_ab.py 1000 $lo $hi gpurun_out/r5/bmc_${lo}_${v}_$tag.npz > gpurun_out/r5/bmc_${lo}_${v}_$tag.log 2>&1 || { echo "variant $v ($set) failed"; tail -5 gpurun_out/r5/bmc_${lo}_${v}_$tag.log; exit 1; }
    echo "== k in ($lo, $hi], basis_mc=$v"; grep -v amdgpu.ids gpurun_out/r5/bmc_${lo}_${v}_$tag.log
  done
  python - $lo $tag <<'PY'
import sys, numpy as np
lo, t = sys.argv[1], sys.argv[2]
a, b = np.load(f"gpurun_out/r5/bmc_{lo}_0_{t}.npz"), np.load(f"gpurun_out/r5/bmc_{lo}_1_{t}.npz")
print("kk equal", np.array_equal(a["kk"], b["kk"]), "mse bit-identical", np.array_equal(a["mse"], b["mse"], equal_nan=True),
      "max |d mse|", float(np.nanmax(np.abs(a["mse"] - b["mse"]))), "nan", int(np.isnan(b["mse"]).sum()))
PY
done
