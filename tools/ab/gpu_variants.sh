# A/B timing of predictor variant libraries: tools/gpu_variants.sh tag v1 v2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; shift
for v in "$@"; do
  CF_MI355X_LIB=$PWD/collaborative_filtering_amd/variants/libcf_$v.so timeout -k 10 200 python -u tools/probe_c4.py 125000 > gpurun_out/var_${tag}_$v.log 2>&1 || { echo "VARIANT $v FAILED"; tail -5 gpurun_out/var_${tag}_$v.log; exit 1; }
  echo "== $v"; grep -E "^predict|phase share|fast path wave|fast ratings|block cycles" gpurun_out/var_${tag}_$v.log
done
