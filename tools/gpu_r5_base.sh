# Round-5 baselines: C2 predictor per sort direction, and the kernel
# statistics of the C2 local_calc leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
for s in 2 1 0; do
  CF_EIGEN_SORT=$s PROBE_CFG=c2 PROBE_SAVE=gpurun_out/r5/c2_sort$s.npz timeout -k 10 300 python -u tools/probe_c4.py 100000 > gpurun_out/r5/c2_sort$s.log 2>&1 || { echo "probe sort $s failed rc=$?"; exit 1; }
  grep -E "eigen:|predict:|phase share|fast ratings|block cycles" gpurun_out/r5/c2_sort$s.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_local -o run -- python3 -u tools/local_leg.py c2 1 > gpurun_out/r5/local_leg_prof.log 2>&1
echo local_rc=$?
tail -2 gpurun_out/r5/local_leg_prof.log | cut -c1-600
f=$(find gpurun_out/r5/prof_local -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -16 "$f" | cut -d, -f1-8
