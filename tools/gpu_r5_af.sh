# Round 5, batch AF: the multi-workgroup basis threshold (CF_PSPILL_BASIS_MC_MIN; default 2816) on
# the C5 sample's 192 < k <= 3072 users; bit-identity against the default
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-af1}
for v in 2816 1536 768 384; do
  CF_PSPILL_BASIS_MC_MIN=$v timeout -k 10 300 python -u tools/probe_pspill_ab.py 1000 192 3072 gpurun_out/r5/bmin_${v}_$tag.npz > gpurun_out/r5/bmin_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/bmin_${v}_$tag.log; exit 1; }
  echo "== min $v"; grep -v amdgpu.ids gpurun_out/r5/bmin_${v}_$tag.log | grep pass
done
python - $tag <<'PY'
import sys, numpy as np
t = sys.argv[1]
a = np.load(f"gpurun_out/r5/bmin_2816_{t}.npz")
for v in (1536, 768, 384):
    b = np.load(f"gpurun_out/r5/bmin_{v}_{t}.npz")
    print(v, "kk equal", np.array_equal(a["kk"], b["kk"]), "mse bit-identical", np.array_equal(a["mse"], b["mse"], equal_nan=True))
PY
