# Sorted sweeps: C4 125k-user eigen probe at close-pair thresholds 4 / 6 / 8 tol
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
for c in 4 6 8; do
  CF_EIGEN_CLOSE=$c timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/sortclose${c}_$tag.log 2>&1 || exit 1
  echo "close=$c"; tail -1 gpurun_out/sortclose${c}_$tag.log | cut -c1-400
done
