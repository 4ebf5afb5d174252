# Register-block Jacobi bring-up: lane-permutation probe, eigen parity tests with RB, RB vs
# column-path timing (C2 mix and k = 180) -- logs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 5 60 ./tools/perm_probe > gpurun_out/perm_probe.txt 2>&1; echo perm_rc=$?
head -40 gpurun_out/perm_probe.txt | tail -24
CF_EIGEN_RB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_eigen.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/rb_eigen_tests.log 2>&1
echo tests_rc=$?
grep -E "FAILED|passed|failed|Error|assert" gpurun_out/rb_eigen_tests.log | head -12
for rb in 0 1; do
  CF_EIGEN_RB=$rb timeout -k 10 200 python -u tools/probe_eigen_ab.py 100000 180 > gpurun_out/rb_ab_k180_$rb.log 2>&1; echo k180_rb$rb rc=$?; tail -n 1 gpurun_out/rb_ab_k180_$rb.log | cut -c1-400
  CF_EIGEN_RB=$rb timeout -k 10 200 python -u tools/probe_eigen_ab.py 100000 0 > gpurun_out/rb_ab_c2_$rb.log 2>&1; echo c2_rb$rb rc=$?; tail -n 1 gpurun_out/rb_ab_c2_$rb.log | cut -c1-400
done
