# Library variants A/B on one box: C4 steps with CF_MI355X_LIB pointing at builds of earlier
# commits (variants/, git-ignored) against the in-tree build.  usage: bash tools/gpu_variants_ab.sh <tag> [env...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-variants_ab}
shift
out=gpurun_out/$tag
mkdir -p $out
run() {
  env "$@" timeout -k 10 400 python3 -u bench.py --profile-steps-only --steps 3 --warmup 1 > $out/$name.json 2> $out/$name.err || { echo rc=$?; tail -5 $out/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$name.json')); st=d['stages']; print('$name', round(d['ms_per_step'],1), round(st['eigen_ms'],1), round(st['predict_ms'],1))"
}
for v in pre_csr head; do name=$v run CF_MI355X_LIB=$GRAFT_REPO_ROOT/variants/lib_$v.so; done
name=cur_barrier run CF_EIGEN_SYNC=barrier
name=cur_p2p run CF_EIGEN_SYNC=p2p
for v in pre_csr head; do name=${v}_2 run CF_MI355X_LIB=$GRAFT_REPO_ROOT/variants/lib_$v.so; done
name=cur_barrier_2 run CF_EIGEN_SYNC=barrier
