# Round-4 pending GPU checks: knn2 graph out-degrees (local_calc unit sizes), the top-k and C5
# tail tests, then the C5 multi-CU cut A/B (tools/gpu_c5_mc_ab.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 240 python -u tools/graph_degrees.py c2 c4 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4_degrees_$tag.log || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_configs.py -k "topk or c5_tail" -v -s --timeout 500 --timeout-method thread > gpurun_out/r4_topk_c5tail_$tag.log 2>&1
echo tests_rc=$?; grep -E "PASSED|FAILED|passed|failed|eigvalsh" gpurun_out/r4_topk_c5tail_$tag.log | tail -12
bash tools/gpu_c5_mc_ab.sh $tag 3072 1536 1024
