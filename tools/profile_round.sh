# Round profile: default bench line, rocprofv3 kernel stats of a short run, and knn2 PMC passes.
# usage: bash tools/profile_round.sh <tag>
set -o pipefail
tag=${1:-v4}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_$tag.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -1 gpurun_out/bench_$tag.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pmc off > gpurun_out/prof_$tag.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof_$tag.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  name=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_knn2_${tag}_$name -o run -- python3 bench.py --knn2 only --no-cpu-baseline --knn2-reps 1 > gpurun_out/pmc_knn2_${tag}_$name.log 2>&1 || { echo PMC_FAILED $name; tail -5 gpurun_out/pmc_knn2_${tag}_$name.log; exit 1; }
done
echo PROFILE_OK
