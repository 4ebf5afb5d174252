# knn2 kernel A/B: GPU knn tests on the default kernel, then the config-3 leg per kernel
# (CF_KNN2_KERNEL=tile: one 512-thread workgroup per tile).  usage: bash tools/gpu_knn2ab.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-knn2ab}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_knn.py -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { echo tests_rc=$?; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for k in halves tile halves; do
  CF_KNN2_KERNEL=$k timeout -k 10 300 python3 -u bench.py --knn2 only --no-cpu-baseline --pmc off --knn2-reps 3 > $out/leg_$k.json 2> $out/leg_$k.err || { echo leg_rc=$?; tail -5 $out/leg_$k.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/leg_$k.json')); print('$k', d['kernel_ms'], d['roofline']['frac'], d['k_chunked'])"
done
