# multi-CU local units parity, then the round-4 profile (rocprof C4 steps, spill tests, big probe)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-v1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_local.py -k "mc_cut or bisection" -v -s --timeout 500 --timeout-method thread > gpurun_out/r4_localmc_$tag.log 2>&1
rc=$?; echo localmc_rc=$rc; grep -E "PASSED|FAILED|multi-CU cut|bisection:|Error|assert" gpurun_out/r4_localmc_$tag.log | head -12
[ $rc -le 1 ] || exit 1
bash tools/gpu_prof_r4.sh $tag
