# Larger shapes on one GPU: config-4 per-GPU shard (125k users x 50k items) and knn2 at 50k x 1M.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py --users 125000 --items 50000 --steps 3 --warmup 1 --no-cpu-baseline --pmc off --knn2 off --c5 off > gpurun_out/scale_c4.log 2>&1 || { echo C4_FAILED; tail -5 gpurun_out/scale_c4.log; exit 1; }
tail -1 gpurun_out/scale_c4.log | cut -c1-900
timeout -k 10 600 python3 -u bench.py --knn2 only --knn2-items 50000 --knn2-users 1000000 --no-cpu-baseline --knn2-reps 1 > gpurun_out/scale_knn2.log 2>&1 || { echo KNN2_FAILED; tail -5 gpurun_out/scale_knn2.log; exit 1; }
tail -1 gpurun_out/scale_knn2.log | cut -c1-700
