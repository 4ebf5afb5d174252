# Eigen bucket launches on two aux streams (default) vs the caller's stream only
# (CF_EIGEN_STREAMS=1): C4 steps only, alternating.  usage: bash tools/gpu_streams_ab.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-streams_ab}
out=gpurun_out/$tag
mkdir -p $out
for v in 2 1 2 1; do
  CF_EIGEN_STREAMS=$v timeout -k 10 400 python3 -u bench.py --profile-steps-only --steps 4 --warmup 1 > $out/s$v.json 2> $out/s$v.err || { echo rc=$?; tail -5 $out/s$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/s$v.json')); st=d.get('stages',{}); print('streams=$v', d['ms_per_step'], {k: v for k, v in st.items() if 'ms' in k})"
done
