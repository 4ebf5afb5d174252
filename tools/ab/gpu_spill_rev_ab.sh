# Spill predictor claim order within a user: ascending rows (default) vs reversed (CF_PSPILL_REV=1)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_fwd.log 2>&1 || exit 1
echo "== forward"; grep -E "ratings in" gpurun_out/pspill_fwd.log
CF_PSPILL_REV=1 timeout -k 10 300 python -u tools/probe_pspill_c5.py 1000 > gpurun_out/pspill_rev.log 2>&1 || exit 1
echo "== reversed"; grep -E "ratings in" gpurun_out/pspill_rev.log
