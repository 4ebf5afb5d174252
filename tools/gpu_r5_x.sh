# Round 5, batch X: kernel stats of the spill predictor on the C5 sample's k > 2816 users
# (basis kernel: one workgroup per user; predict kernel: persistent, two per CU)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
tag=${1:-x2}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_pbig_$tag -o run -- python3 -u tools/probe_pspill_ab.py 1000 2816 5000 /tmp/pbig.npz > gpurun_out/r5/prof_pbig_$tag.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r5/prof_pbig_$tag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5/prof_pbig_$tag.log | tail -3
f=$(find gpurun_out/r5/prof_pbig_$tag -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/r5/pbig_kernel_stats_$tag.csv
find gpurun_out/r5/prof_pbig_$tag -name "*kernel_trace.csv" -delete
head -8 gpurun_out/r5/pbig_kernel_stats_$tag.csv | cut -d, -f1-6
