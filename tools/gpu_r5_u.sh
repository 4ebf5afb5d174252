# Round 5, batch U: the spill eigen workspace budget (CF_SPILL_BUDGET, fraction of the context's
# share of free HBM; 0.5 default) on the C5 10k-user one-call sample, waves per staged range
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-u1}
for b in ${BUDGETS:-0.5 0.75}; do
  CF_SPILL_VERBOSE=1 CF_SPILL_BUDGET=$b timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 all > gpurun_out/r5/budget_${b}_$tag.log 2>&1 || { echo "budget $b failed"; tail -5 gpurun_out/r5/budget_${b}_$tag.log; exit 1; }
  echo "== budget $b"; grep -v amdgpu.ids gpurun_out/r5/budget_${b}_$tag.log | tail -8
done
