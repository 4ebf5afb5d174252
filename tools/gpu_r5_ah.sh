# Round 5, batch AH: workgroups per CU of the multi-workgroup spill basis (CF_PSPILL_BASIS_MC_W,
# default 2) on the C5 sample's k > 2816 and 192 < k <= 3072 users; bit-identity against 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-ah1}
for set in "2816 5000" "192 3072"; do
  lo=${set% *}; hi=${set#* }
  for v in ${WS:-2 4 1}; do
    CF_PSPILL_BASIS_MC_W=$v timeout -k 10 300 python -u tools/probe_pspill_ab.py 1000 $lo $hi gpurun_out/r5/bw_${lo}_${v}_$tag.npz > gpurun_out/r5/bw_${lo}_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/bw_${lo}_${v}_$tag.log; exit 1; }
    echo "== k in ($lo, $hi], w=$v"; grep -v amdgpu.ids gpurun_out/r5/bw_${lo}_${v}_$tag.log | grep pass
  done
  python - $lo $tag <<'PY'
import sys, numpy as np
lo, t = sys.argv[1], sys.argv[2]
a = np.load(f"gpurun_out/r5/bw_{lo}_4_{t}.npz")
for v in (8,):
    b = np.load(f"gpurun_out/r5/bw_{lo}_{v}_{t}.npz")
    print(v, "identical", np.array_equal(a["kk"], b["kk"]) and np.array_equal(a["mse"], b["mse"], equal_nan=True))
PY
done
