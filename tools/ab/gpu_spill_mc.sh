# Staged multi-CU spill path for k > 3072: spill / C5 GPU tests, then the bench C5 leg with it
# (default) and without (CF_SPILL_MC=0).  usage: bash tools/ab/gpu_spill_mc.sh <tag> [notests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-spill_mc}
out=gpurun_out/$tag
mkdir -p $out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 700 python3 -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -k "spill or c5" -x -v --timeout 500 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -5 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
timeout -k 10 500 python3 -u bench.py --c5 only > $out/c5_mc.json 2> $out/c5_mc.err || { echo rc=$?; tail -5 $out/c5_mc.err; exit 1; }
grep -v amdgpu $out/c5_mc.err
# per-phase cycles (cf_debug_spill) at k = 4000 / 5000
timeout -k 10 300 python3 -u tools/probe_spill.py 4000:24 5000:8 > $out/probe.log 2>&1 || { echo probe_rc=$?; tail -5 $out/probe.log; exit 1; }
grep -v amdgpu $out/probe.log
