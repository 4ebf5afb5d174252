# Eigen refinement A/B: C4 eigen parity tests at several close-pair thresholds, then timing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v6}
for c in 16 8 4; do
  CF_EIGEN_CLOSE=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "c4_eigen or c2_eigen" -v -s --timeout 200 --timeout-method thread > gpurun_out/r4_close${c}_$tag.log 2>&1
  echo "close=$c rc=$?"; grep -E "passed|failed|AssertionError: \[" gpurun_out/r4_close${c}_$tag.log | tail -4
done
for c in 16 8 4; do
  CF_EIGEN_CLOSE=$c timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/refine_close${c}_$tag.log 2>&1 || exit 1
  echo "close=$c"; tail -1 gpurun_out/refine_close${c}_$tag.log | cut -c1-330
done
timeout -k 10 300 python -u tools/probe_refine.py 125000 off > gpurun_out/refine_off_$tag.log 2>&1 && tail -1 gpurun_out/refine_off_$tag.log | cut -c1-330
