# Spill predictor C-mode (underdetermined rows) + the min-norm LS pin of rank-deficient rows:
# config and predictor GPU tests, then the C5 leg with the k > 3072 users predicted.
# usage: bash tools/ab/gpu_cmode.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/${1:-cmode}
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_predict.py -x -v -s --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -5 $out/tests.log; exit 1; }
grep -E "rank-deficient|passed" $out/tests.log | tail -8
timeout -k 10 600 python3 -u bench.py --c5 only --c5-predict-kmax 5000 --c5-onecall-users 100 > $out/c5.json 2> $out/c5.err || { echo c5_rc=$?; grep -v amdgpu $out/c5.err | tail -5; exit 1; }
grep -v amdgpu $out/c5.err
