# Round 5, batch I: C5 tail value checks, the k > 3072 spill predictor's phase split, and the
# C5 10k-user one-call eigen stage under rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-i1}
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -k "c5_tail" -v -s --timeout 500 --timeout-method thread > gpurun_out/r5/c5tail_$tag.log 2>&1
echo tests_rc=$?
grep -E "PASSED|FAILED|C5 k=|user [0-9]|Error|assert" gpurun_out/r5/c5tail_$tag.log | cut -c1-300 | tail -30
timeout -k 10 400 python -u tools/probe_pspill_c5.py 1000 3072 5000 > gpurun_out/r5/pspill_big_$tag.log 2>&1
echo pspill_rc=$?
grep -v amdgpu.ids gpurun_out/r5/pspill_big_$tag.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/c5oc_prof_$tag -o run -- python3 -u tools/probe_c5_onecall.py 10000 all > gpurun_out/r5/c5oc_prof_$tag.log 2>&1
echo prof_rc=$?
grep -v amdgpu.ids gpurun_out/r5/c5oc_prof_$tag.log | tail -5 | cut -c1-300
f=$(find gpurun_out/r5/c5oc_prof_$tag -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp $f gpurun_out/r5/c5oc_kernel_stats_$tag.csv && cut -d, -f1-4 $f | head -24
find gpurun_out/r5/c5oc_prof_$tag -name '*kernel_trace.csv' -delete
