# Round 5, batch K: BASELINE config 5 at its own size, one GPU's share (tools/c5_shard.py: the
# 100k-user set split over 8 by sum k^3; shards 0 and 4 here), with a heartbeat file
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-k1}
timeout -k 10 1000 python -u tools/c5_shard.py ${SHARDS:-0 4} > gpurun_out/r5/c5shard_$tag.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; date +%T >> gpurun_out/r5/c5shard_hb_$tag.log; done
wait $pid; rc=$?
echo shard_rc=$rc
grep -v amdgpu.ids gpurun_out/r5/c5shard_$tag.log | cut -c1-400
