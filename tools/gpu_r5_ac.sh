# Round 5, batch AC: spill_mc_symv with z's old value loaded with the slab (default) vs at the +=
# (variants/libcf_zpre0.so): the C5 10k one-call sample's k > 3072 users, digests of every output
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-ac1}
for v in zpre0 default; do
  if [ $v = default ]; then lib=""; else lib=$PWD/collaborative_filtering_amd/variants/libcf_$v.so; fi
  PROBE_HASH=1 CF_MI355X_LIB=$lib timeout -k 10 300 python -u tools/probe_c5_onecall.py 10000 big,all > gpurun_out/r5/zpre_${v}_$tag.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/r5/zpre_${v}_$tag.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/r5/zpre_${v}_$tag.log
done
