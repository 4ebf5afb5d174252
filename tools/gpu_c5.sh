# C5 probe: spill-path GPU tests, then the bench C5 leg (progress on stderr into the log)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
users=${1:-2000}
timeout -k 10 600 python -u bench.py --c5 only --c5-users $users > gpurun_out/r3_c5_$users.log 2>&1
echo rc=$?
tail -c 4000 gpurun_out/r3_c5_$users.log
