"""A/B timing of the eigen stage (cf_eigen_run) on the config-2 user mix: run under
CF_MI355X_LIB=<variant .so>.  Prints the median stage time over 5 passes, the mean sweep
count and checksums of the outputs (m, evals) for a quick cross-variant comparison.
usage: python tools/probe_eigen_ab.py [users] [kfix]"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
kfix = int(sys.argv[2]) if len(sys.argv) > 2 else 0
seed = 2026101502
k = synth.degrees(seed, users) if not kfix else np.full(users, kfix, np.uint32)
off, items, rat = synth.user_items(seed, k, 10000, threads=16)
W = synth.graph_model(seed, 10000, threads=16)
ctx = Context(0)
ctx.upload_graph_dense(W)
plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev))
run = lambda: plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
ctx.debug_stats(True)
run()
torch.cuda.synchronize()
st = ctx.debug_stats(True, read=True)
ctx.debug_stats(False)
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    run()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t)
m = d["m"].cpu().numpy()
ev = d["evals"].cpu().numpy()
print(f"lib {os.path.basename(os.environ.get('CF_MI355X_LIB', 'libcf_mi355x.so'))} users {users} kfix {kfix}: "
      f"eigen {np.median(ts) * 1e3:.1f} ms ({users / np.median(ts):.0f} users/s) stats {st} "
      f"m_sum {int(m.sum())} evals_sum {float(ev.astype(np.float64).sum()):.6f}", flush=True)
