# Round-4 batch 8: per-bucket eigen cost on C4 (tools/probe_eigen_buckets.py), then the C5 one-call
# breakdown (tools/gpu_c5_onecall.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 300 python -u tools/probe_eigen_buckets.py 20000 > gpurun_out/eigbk_$tag.log 2>&1; echo "buckets rc=$?"; grep "^k=" gpurun_out/eigbk_$tag.log
bash tools/gpu_c5_onecall.sh $tag
