# Round 5, batch AD: staged QL with the idle CUs' extra parts for the largest users (default) vs
# the uniform split (CF_SPILL_QL_EXTRA=0): C5 10k one-call sample, digests of every output
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-ad1}
for v in 0 1; do
  PROBE_HASH=1 CF_SPILL_QL_EXTRA=$v timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 big,all > gpurun_out/r5/qlx_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/qlx_${v}_$tag.log; exit 1; }
  echo "== ql_extra $v"; grep -v amdgpu.ids gpurun_out/r5/qlx_${v}_$tag.log
done
