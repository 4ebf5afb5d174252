# Round 5, batch E: per-user staged slots (one wave where HBM allows): the C5 leg (1000-user
# sample + the 10k-user one call) and the uncapped C2 local_calc leg; then batch D (predictor
# spills A/B)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-e1}
timeout -k 10 600 python -u bench.py --c5 only --no-cpu-baseline > gpurun_out/r5/c5_$tag.json 2> gpurun_out/r5/c5_$tag.err
echo c5_rc=$?; tail -c 1500 gpurun_out/r5/c5_$tag.json
timeout -k 10 600 python -u tools/local_leg.py c2 1 > gpurun_out/r5/local_leg_$tag.log 2>&1
echo local_rc=$?; grep -v amdgpu.ids gpurun_out/r5/local_leg_$tag.log | tail -1 | cut -c1-600
bash tools/gpu_r5_d.sh $tag
