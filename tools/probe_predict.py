"""Diagnostics: predictor phase cycles on the bench workload."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
k = synth.degrees(2026101502, users)
off, items, rat = synth.user_items(2026101502, k, 10000, threads=16)
W = synth.graph_model(2026101502, 10000, threads=16)
ctx = Context(0); ctx.upload_graph_dense(W); plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off); n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)), rat=T(rat),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
         mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
torch.cuda.synchronize()
def pred():
    plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                     CF_SIGS_COMPAT, d["mse"], d["kk"])
pred(); torch.cuda.synchronize()
t = time.perf_counter(); pred(); torch.cuda.synchronize(); dt = time.perf_counter() - t
print(f"predict {n} ratings in {dt*1e3:.1f} ms -> {n/dt:.0f}/s", flush=True)
ctx.debug_phases(True); pred(); torch.cuda.synchronize()
ph = ctx.debug_phases(True, read=True)
tot = sum(ph.values())
print({k_: f"{v/tot*100:.1f}%" for k_, v in ph.items()}, "cycles/prediction:", tot / n * 1.0)
m = d["m"].cpu().numpy(); kk = d["kk"].cpu().numpy()
print("m mean", m.mean(), "kk mean", kk.mean(), "k mean", k.mean())
