# Round 5, batch J: QL with 32 iterations per pass over Z in the staged path (QL-only kernel) vs
# 16 (variants/libcf_qb16.so): the C5 10k-user one-call eigen stage and its k > 3072 users alone,
# output digests (bit-identity), then the spill parity tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-j1}
for v in qb32 qb16; do
  lib=""; [ $v = qb16 ] && lib=$GRAFT_REPO_ROOT/collaborative_filtering_amd/variants/libcf_qb16.so
  CF_MI355X_LIB=$lib PROBE_HASH=1 timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 all,big > gpurun_out/r5/ql_${v}_$tag.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r5/ql_${v}_$tag.log; exit 1; }
  echo "== $v"; grep -E "^(all|big)" gpurun_out/r5/ql_${v}_$tag.log | cut -c1-300
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_local.py tests/test_gpu_configs.py -m gpu -k "spill or c5 or huge or local" -v -s --timeout 600 --timeout-method thread > gpurun_out/r5/ql_tests_$tag.log 2>&1
echo tests_rc=$?
grep -E "PASSED|FAILED|passed|failed|C5 k=" gpurun_out/r5/ql_tests_$tag.log | cut -c1-200 | tail -40
