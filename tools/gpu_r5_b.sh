# Round 5, batch B: the C2 predictor per sort direction (orthogonality of the stored blocks)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
for s in 2 1; do
  CF_EIGEN_SORT=$s timeout -k 10 300 python -u tools/probe_c2_orth.py > gpurun_out/r5/c2_orth_sort$s.log 2>&1 || { echo "orth probe sort $s rc=$?"; tail -5 gpurun_out/r5/c2_orth_sort$s.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5/c2_orth_sort$s.log
done
