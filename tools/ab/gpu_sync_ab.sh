# Eigen step synchronisation A/B: GPU eigen/config tests on the default (per-wave progress
# counters), then C4 steps with CF_EIGEN_SYNC=barrier vs default, and the single-stream
# bucket launch (CF_EIGEN_STREAMS=1).  usage: bash tools/gpu_sync_ab.sh <tag> [tests]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-sync_ab}
out=gpurun_out/$tag
mkdir -p $out
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest tests/test_gpu_eigen.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; grep -E "FAILED|Error|assert" $out/tests.log | head -20; tail -5 $out/tests.log; exit 1; }
  tail -2 $out/tests.log
fi
run() {
  env "$@" timeout -k 10 400 python3 -u bench.py --profile-steps-only --steps 3 --warmup 1 > $out/$name.json 2> $out/$name.err || { echo rc=$?; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); st=d['stages']; print('$name', round(d['ms_per_step'],1), {k: (round(v,1) if isinstance(v,float) else v) for k, v in st.items() if 'ms' in k or 'sweep' in k})"
}
name=p2p run CF_EIGEN_SYNC=p2p
name=barrier run CF_EIGEN_SYNC=barrier
name=p2p_1stream run CF_EIGEN_SYNC=p2p CF_EIGEN_STREAMS=1
name=p2p_b run CF_EIGEN_SYNC=p2p
