# Round 5: the C4 / C5 config tests after the pinning changes (progress printed per test)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-f1}
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 600 --timeout-method thread -k "c4_predict or c5_tail or spill_rank or c5_mix" > gpurun_out/r5/cfg_$tag.log 2>&1
echo rc=$?; grep -E "PASSED|FAILED|C5 k=|spill rank|C4:|C4 rank|Error|assert" gpurun_out/r5/cfg_$tag.log | tail -30
