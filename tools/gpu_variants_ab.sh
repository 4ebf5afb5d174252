# Library variants A/B on one box: C4 steps (--profile-steps-only) for every variants/lib_*.so
# (CF_MI355X_LIB; builds of other commits, git-ignored) and the in-tree build, twice each,
# interleaved.  usage: bash tools/gpu_variants_ab.sh <tag> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-variants_ab}
shift
out=gpurun_out/$tag
mkdir -p $out
run() {
  env "$@" timeout -k 10 400 python3 -u bench.py --profile-steps-only --steps 3 --warmup 1 $extra > $out/$name.json 2> $out/$name.err || { echo rc=$?; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); st=d['stages']; print('$name', round(d['ms_per_step'],1), round(st['eigen_ms'],1), round(st['predict_ms'],1))"
}
extra="$*"
for rep in 1 2; do
  for f in variants/lib_*.so; do
    [ -e "$f" ] || continue
    v=$(basename $f .so); name=${v}_$rep run CF_MI355X_LIB=$GRAFT_REPO_ROOT/$f
  done
  name=intree_$rep run CF_NOTHING=1
done
