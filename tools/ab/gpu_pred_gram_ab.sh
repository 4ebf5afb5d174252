# Round 5, batch M: predictor variant A/B on the C4 125k-user shard (tools/probe_c4.py): time,
# output equality and WRITE_SIZE per predictor kernel.  usage: gpu_r5_m.sh TAG VARIANT...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-m1}; shift
vars="intree $*"
for v in $vars; do
  lib=""; [ $v != intree ] && lib=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_$v.so
  CF_MI355X_LIB=$lib PROBE_SAVE=gpurun_out/r5/pv_$v.npz timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/r5/pv_${v}_$tag.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r5/pv_${v}_$tag.log; exit 1; }
  echo "== $v"; grep -E "^(eigen|predict)" gpurun_out/r5/pv_${v}_$tag.log
done
python - $vars <<'PY'
import sys, numpy as np
a = np.load("gpurun_out/r5/pv_intree.npz")
for v in sys.argv[2:]:
    b = np.load(f"gpurun_out/r5/pv_{v}.npz")
    print(v, "kk equal", bool((a["kk"] == b["kk"]).all()), "mse bits differ", int((a["mse"].view(np.uint32) != b["mse"].view(np.uint32)).sum()), "of", a["mse"].size)
PY
rm -f gpurun_out/r5/pv_*.npz
for v in $vars; do
  lib=""; [ $v != intree ] && lib=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_$v.so
  CF_MI355X_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5/pvw_$v -o run -- python3 tools/probe_c4.py 125000 > gpurun_out/r5/pvw_$v.log 2>&1 || { echo "pmc $v failed rc=$?"; exit 1; }
  python - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f"gpurun_out/r5/pvw_{v}/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.Counter(); n = collections.Counter()
for r in csv.DictReader(open(f)):
    nm = r["Kernel_Name"]
    for key in ("pred_basis_kernel", "pred_rating_kernel", "pred_dense_kernel"):
        if key in nm:
            acc[key] += float(r["Counter_Value"]) * 1024; n[key] += 1
print(v, "WRITE_SIZE", {k: f"{acc[k]/1e9:.2f} GB / {n[k]} launches" for k in acc})
PY
  rm -rf gpurun_out/r5/pvw_$v
done
