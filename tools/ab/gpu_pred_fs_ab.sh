# Round 5, batch D: predictor basis-kernel spills: in-tree (16-column
# forward-substitution panels) vs variants/libcf_fs8.so (8-column), C4 125k-user shard: time,
# outputs, and WRITE_SIZE / FETCH_SIZE per predictor kernel (rocprofv3 --pmc, one pass each)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-d1}
run() {   # name, env...
  local name=$1; shift
  env "$@" PROBE_SAVE=gpurun_out/r5/pab_$name.npz timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/r5/pab_${name}_$tag.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/r5/pab_${name}_$tag.log; exit 1; }
  echo "== $name"; grep -E "^(eigen|predict|phase|fast)" gpurun_out/r5/pab_${name}_$tag.log | cut -c1-250
}
run intree CF_NOTHING=1
run fs8 CF_MI355X_LIB=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_fs8.so
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/r5/pab_intree.npz"); b = np.load("gpurun_out/r5/pab_fs8.npz")
print("fs8 kk equal", bool((a["kk"] == b["kk"]).all()), "mse bits differ", int((a["mse"].view(np.uint32) != b["mse"].view(np.uint32)).sum()), "of", a["mse"].size)
PY
rm -f gpurun_out/r5/pab_*.npz
for v in intree fs8; do
  for c in WRITE_SIZE FETCH_SIZE; do
    lib=""; [ $v = fs8 ] && lib=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_fs8.so
    CF_MI355X_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r5/pmc_${v}_$c -o run -- python3 tools/probe_c4.py 125000 > gpurun_out/r5/pmc_${v}_$c.log 2>&1 || { echo "pmc $v $c failed rc=$?"; exit 1; }
    python - "$v" "$c" <<'PY'
import csv, glob, sys, collections
v, c = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/r5/pmc_{v}_{c}/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.Counter(); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if r["Counter_Name"] != c: continue
    nm = r["Kernel_Name"]
    for key in ("pred_basis_kernel", "pred_rating_kernel", "pred_dense_kernel", "eigen_kernel"):
        if key in nm:
            acc[key] += float(r["Counter_Value"]) * 1024; n[key] += 1
print(v, c, {k: f"{acc[k]/1e9:.2f} GB over {n[k]} launches" for k in acc})
PY
    rm -rf gpurun_out/r5/pmc_${v}_$c
  done
done
