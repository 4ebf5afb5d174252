set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/ab/gpu_eigen_ab.sh 100000 0 main k8 k16 && bash tools/ab/gpu_eigen_ab.sh 30000 180 main k8 k16 && \
for v in k8 k16; do
  CF_MI355X_LIB=$PWD/collaborative_filtering_amd/variants/libcf_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "eigen or c4 or c2" > gpurun_out/kt_$v.log 2>&1 || { echo "TESTS $v FAILED"; tail -20 gpurun_out/kt_$v.log; exit 1; }
  echo "$v: $(tail -n 1 gpurun_out/kt_$v.log)"
done && bash tools/gpu_tests_sel.sh tests/test_gpu_predict.py tests/test_gpu_configs.py tests/test_gpu_step.py tests/test_pipeline.py -m gpu
