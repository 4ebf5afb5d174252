# Round 5, batch G: systolic Jacobi levels (cf_eigen.hip) -- DPP semantics probe, eigen / step /
# config parity tests, then C4 125k-shard eigen time systolic vs LDS levels (CF_EIGEN_SYSTOLIC=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-g1}
timeout -k 10 60 ./bin/dpp_probe > gpurun_out/r5/dpp_probe_$tag.log 2>&1; rc=$?
cat gpurun_out/r5/dpp_probe_$tag.log
[ $rc = 0 ] || { echo "dpp probe rc=$rc"; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_step.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r5/sys_tests_$tag.log 2>&1
echo tests_rc=$?
grep -E "PASSED|FAILED|passed|failed|C5 k=|C4:|C2:" gpurun_out/r5/sys_tests_$tag.log | cut -c1-220 | tail -40
for v in 0 1; do
  CF_EIGEN_SYSTOLIC=$v timeout -k 10 300 python -u tools/probe_c4.py 125000 > gpurun_out/r5/sys_c4_${v}_$tag.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/r5/sys_c4_${v}_$tag.log; exit 1; }
  echo "== systolic=$v"; grep -E "^(eigen|predict)" gpurun_out/r5/sys_c4_${v}_$tag.log
done
