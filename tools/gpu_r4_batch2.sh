# predictor variant A/B (closed form, tile skip), then the k > 3072 spill predictor kernel split
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_probe_variants.sh v1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pspill_big -o run -- python3 -u tools/probe_pspill_c5.py 1000 3072 5000 > gpurun_out/pspill_big_v1.log 2>&1
echo rc=$?; grep -v amdgpu.ids gpurun_out/pspill_big_v1.log | tail -12 | cut -c1-300
f=$(find gpurun_out/pspill_big -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" | cut -d, -f1-8
