"""Diagnostics: Jacobi sweep counts and eigen-stage time vs tolerance on the bench workload."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
k = synth.degrees(2026101502, users)
off, items, rat = synth.user_items(2026101502, k, 10000, threads=16)
W = synth.graph_model(2026101502, 10000, threads=16)
ctx = Context(0); ctx.upload_graph_dense(W); plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off); n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev))
def run():
    plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
for tol in [1.0, 2.0, 4.0, 8.0]:
    ctx.set_jacobi(tol, 30)
    ctx.debug_stats(True)
    run(); torch.cuda.synchronize()
    st = ctx.debug_stats(True, read=True)
    ctx.debug_stats(False)
    t = time.perf_counter(); run(); torch.cuda.synchronize(); dt = time.perf_counter() - t
    print(f"tol_scale={tol} {st} time={dt*1e3:.1f} ms users/s={users/dt:.0f}", flush=True)
