# CF_EIGEN_HYBRID (Householder + QL for bucket 12, Jacobi below) vs Jacobi: eigen GPU tests over
# all three methods, then C4 steps per method (bench --eigen-method), interleaved.
# usage: bash tools/ab/gpu_hybrid_ab.sh <tag> [notests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-hybrid_ab}
out=gpurun_out/$tag
mkdir -p $out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_eigen.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -5 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
run() {
  env "$@" timeout -k 10 400 python3 -u bench.py --profile-steps-only --steps 3 --warmup 1 > $out/$name.json 2> $out/$name.err || { echo rc=$?; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); st=d['stages']; print('$name', round(d['ms_per_step'],1), round(st['eigen_ms'],1), round(st['predict_ms'],1))"
}
name=hybrid_a run CF_EIGEN_METHOD=hybrid
name=jacobi_a run CF_EIGEN_METHOD=jacobi
name=hybrid_b run CF_EIGEN_METHOD=hybrid
name=jacobi_b run CF_EIGEN_METHOD=jacobi
