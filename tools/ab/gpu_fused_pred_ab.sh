# Fused predictor A/B: C4 steps, fused (noinline halves), fused (inlined, variant lib), two-kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() { timeout -k 10 400 python -u bench.py --profile-steps-only --steps 3 --warmup 1 > gpurun_out/fab_$1.json 2> gpurun_out/fab_$1.err; }
CF_PRED_FUSED=1 run call || exit 1
CF_PRED_FUSED=1 CF_MI355X_LIB=$PWD/collaborative_filtering_amd/variants/libcf_finl.so run inl || exit 1
CF_PRED_FUSED=0 run off || exit 1
for f in call inl off; do python -c "import json;d=json.load(open('gpurun_out/fab_$f.json'));print('$f',round(d['value']),round(d['ms_per_step'],1),{k:round(v,1) for k,v in d.get('stages',{}).items() if 'ms' in k})"; done
