# A/B of the eigen stopping threshold (kSigRot = 16 main, 32, 64 variants), then every -m gpu
# test under each variant: tools/ab/gpu_sigrot_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab/gpu_eigen_ab.sh 100000 0 main k32 k64 && bash tools/ab/gpu_eigen_ab.sh 100000 180 main k32 k64 || exit 1
for v in k32 k64; do
  CF_MI355X_LIB=$PWD/collaborative_filtering_amd/variants/libcf_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$v.log 2>&1
  rc=$?
  echo "$v tests rc=$rc: $(tail -n 1 gpurun_out/gpu_tests_$v.log)"
  [ $rc -le 1 ] || exit 1
done
