# A/B of eigen variants: tools/ab/gpu_eigen_ab.sh <users> <kfix> <variant names...> (main = the in-tree lib)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
users=$1; kfix=$2; shift 2
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/collaborative_filtering_amd/libcf_mi355x.so; else lib=$PWD/collaborative_filtering_amd/variants/libcf_$v.so; fi
  CF_MI355X_LIB=$lib timeout -k 10 200 python -u tools/probe_eigen_ab.py $users $kfix > gpurun_out/eab_$v.log 2>&1 || { echo "VARIANT $v FAILED"; tail -5 gpurun_out/eab_$v.log; exit 1; }
  tail -n 1 gpurun_out/eab_$v.log
done
