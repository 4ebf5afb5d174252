# Round 6: bucket-12-on-Householder+QL hybrid vs all-Jacobi eigen (CF_EIGEN_HYBRID), C4 step
# (profile-steps-only, same box, back to back) and the eigen parity tests under the hybrid.
# usage: tools/ab/gpu_r6_hybrid.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-a}
for h in 0 1; do
  CF_EIGEN_HYBRID=$h timeout -k 10 420 python3 -u bench.py --profile-steps-only --steps 4 --warmup 1 > gpurun_out/r6_hyb${h}_$tag.log 2>&1 || { echo "bench h=$h failed"; tail -5 gpurun_out/r6_hyb${h}_$tag.log; exit 1; }
  python3 - "$h" gpurun_out/r6_hyb${h}_$tag.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
st = d["stages"]
print(f"hybrid={sys.argv[1]}: value {d['value']:.0f} users/s, ms/step {d['ms_per_step']:.1f}, eigen {st['eigen_ms']:.1f} ms, predict {st['predict_ms']:.1f} ms")
PY
done
CF_EIGEN_HYBRID=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "c2_ or c4_ or eigen" > gpurun_out/r6_hyb_tests_$tag.log 2>&1
echo hybrid_tests_rc=$?; tail -3 gpurun_out/r6_hyb_tests_$tag.log
