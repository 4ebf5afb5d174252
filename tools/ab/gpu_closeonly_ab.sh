# Eigen close-only sweeps A/B: probe timing + parity on C4 users, then the C2/C4 eigen tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
for co in 0 1; do
  CF_EIGEN_CLOSEONLY=$co timeout -k 10 300 python -u tools/probe_refine.py 125000 on:1e-3:1e-2 > gpurun_out/refine_co${co}_$tag.log 2>&1 || exit 1
  echo "closeonly=$co"; tail -1 gpurun_out/refine_co${co}_$tag.log | cut -c1-330
done
timeout -k 10 300 python -u tools/probe_refine.py 125000 off > gpurun_out/refine_off_$tag.log 2>&1 && tail -1 gpurun_out/refine_off_$tag.log | cut -c1-330
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -k "c4_eigen or c2_eigen or c5_mix" -v -s --timeout 300 --timeout-method thread > gpurun_out/r4_co_tests_$tag.log 2>&1
echo tests_rc=$?; grep -E "passed|failed|AssertionError: \[" gpurun_out/r4_co_tests_$tag.log | tail -4
