# Round 5, batch N: the staged tridiagonalisation's symv reading v from the slot (4 workgroups
# per CU) vs its LDS copy (CF_SPILL_SYMV_LDS=1, 2 per CU): C5 one-call + k > 3072 alone, digests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-n1}
for v in slot lds; do
  env_v=0; [ $v = lds ] && env_v=1
  CF_SPILL_SYMV_LDS=$env_v PROBE_HASH=1 timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 all,big > gpurun_out/r5/symv_${v}_$tag.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r5/symv_${v}_$tag.log; exit 1; }
  echo "== $v"; grep -E "^(all|big)" gpurun_out/r5/symv_${v}_$tag.log | cut -c1-300
done
