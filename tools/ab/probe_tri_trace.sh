# per-launch durations of both eigen methods (20k C2 users): rocprofv3 kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_trace -o run -- python3 tools/probe_tri.py 20000 > gpurun_out/trace.log 2>&1 || { tail -5 gpurun_out/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_trace/*kernel_trace.csv")[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r["Kernel_Name"]
    if "tri_" in n or "eigen_kernel" in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(n.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", ""), g, round(d, 3))
PY
