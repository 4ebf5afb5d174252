"""Per-kernel register / spill / occupancy table of one .hip file (hipcc -Rpass-analysis).
usage: python tools/kres.py <file.hip> [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Iinclude",
                      "-Icollaborative_filtering_amd/csrc", "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} vspill={r.get('VGPRs Spill')} "
              f"sspill={r.get('SGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')} scratch={r.get('ScratchSize [bytes/lane]')}")
