# Spill eigen A/B: spill GPU tests on the in-tree build, then the throughput probe on
# variants/lib_base.so (CF_MI355X_LIB) and the in-tree build.  usage: bash tools/gpu_spill_ab.sh <tag> [probe args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-spill_ab}
shift
out=gpurun_out/$tag
mkdir -p $out
args=${*:-1500:64 4000:24}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_eigen.py -k spill -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; tail -20 $out/tests.log; exit 1; }
tail -1 $out/tests.log
CF_MI355X_LIB=$GRAFT_REPO_ROOT/variants/lib_base.so timeout -k 10 400 python3 -u tools/probe_spill.py $args > $out/base.log 2>&1 || { echo base_rc=$?; tail -5 $out/base.log; exit 1; }
echo base; grep -v amdgpu.ids $out/base.log
timeout -k 10 400 python3 -u tools/probe_spill.py $args > $out/new.log 2>&1 || { echo new_rc=$?; tail -5 $out/new.log; exit 1; }
echo new; grep -v amdgpu.ids $out/new.log
