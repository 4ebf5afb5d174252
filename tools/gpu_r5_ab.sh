# Round 5, batch AB: the G-mode Gram's row list staged in LDS (default build) vs read from the
# HBM row arrays (variants/libcf_rows0.so), C5 sample k > 2816 users; bit-identity of mse / kk
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-ab1}
for v in rows0 default; do
  if [ $v = default ]; then lib=""; else lib=$PWD/collaborative_filtering_amd/variants/libcf_$v.so; fi
  CF_MI355X_LIB=$lib timeout -k 10 300 python -u tools/probe_pspill_ab.py 1000 2816 5000 gpurun_out/r5/rows_${v}_$tag.npz > gpurun_out/r5/rows_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/rows_${v}_$tag.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r5/rows_${v}_$tag.log
done
python - $tag <<'PY'
import sys, numpy as np
t = sys.argv[1]
a, b = np.load(f"gpurun_out/r5/rows_rows0_{t}.npz"), np.load(f"gpurun_out/r5/rows_default_{t}.npz")
print("kk equal", np.array_equal(a["kk"], b["kk"]), "mse bit-identical", np.array_equal(a["mse"], b["mse"], equal_nan=True))
PY
