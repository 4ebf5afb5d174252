# knn2 (config 3) leg: HIP-event timing, rocprofv3 kernel stats and two SQ counter passes.
# usage: bash tools/gpu_knn2.sh <tag> [extra bench args]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${1:-knn2}
shift
out=gpurun_out/$tag
mkdir -p $out
run="python3 -u bench.py --knn2 only --no-cpu-baseline --pmc off $*"
timeout -k 10 300 $run --knn2-reps 3 > $out/leg.json 2> $out/leg.err || { echo leg_rc=$?; exit 1; }
tail -c 3000 $out/leg.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- $run --knn2-reps 1 > $out/trace.log 2>&1 || { echo trace_rc=$?; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $out/pmc1 -o run -- $run --knn2-reps 0 > $out/pmc1.log 2>&1 || { echo pmc1_rc=$?; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC -d $out/pmc2 -o run -- $run --knn2-reps 0 > $out/pmc2.log 2>&1 || { echo pmc2_rc=$?; exit 1; }
echo done
