"""why the C2 predictor is slower with ascending norm-sorted sweeps.  Runs the
C2 eigen stage under the CF_EIGEN_SORT of the environment, then per user: max |U^T U - I| over
its m stored columns (the predictor takes no basis above kOrthoMax = 1e-2 and sends every rating
of the user down the block-wide path), and the predictor's path counts (cf_debug_phases).
usage: CF_EIGEN_SORT=2 probe_c2_orth.py [users=100000]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
cfg = wlm.CONFIGS["c2"]
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c2", Context, 0, dev, torch)
k = wlm.user_degrees(cfg)[:users]
off, items, rat = synth.user_items(cfg["seed"], k, cfg["items"], threads=16)
ctx = Context(0)
ctx.upload_graph_dense(d_W.view(cfg["items"], -1))
plan = ctx.plan(off)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n = int(off[-1])
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)), rat=T(rat),
         m=torch.zeros(users, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
         mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
ctx.debug_phases(True)
plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                 CF_SIGS_COMPAT, d["mse"], d["kk"])
torch.cuda.synchronize()
ph = ctx.debug_phases(True, read=True)
ctx.debug_phases(False)
print("sort", os.environ.get("CF_EIGEN_SORT", "default"), "fast", ph["n_fast"], "block-wide", ph["n_dense"], flush=True)
m = d["m"].cpu().numpy()
dev_u = np.zeros(users)
ev_all = d["evals"].cpu().numpy()
for kk in np.unique(k):
    us = np.nonzero(k == kk)[0]
    for c0 in range(0, len(us), 4096):
        sel = us[c0:c0 + 4096]
        idx = torch.from_numpy((eoff[sel][:, None] + np.arange(kk * kk)[None, :]).astype(np.int64)).to(dev)
        mm = torch.from_numpy(m[sel].astype(np.int64)).to(dev)
        blk = d["evecs"][idx].view(len(sel), kk, kk).double()   # k x k slot, row-major k x m (m <= k)
        # row-major k x m stored in the first k*m entries: re-view per user by m
        out = np.zeros(len(sel))
        for mv in torch.unique(mm).tolist():
            s2 = (mm == mv).nonzero().flatten()
            U = blk[s2].reshape(len(s2), -1)[:, :kk * mv].view(len(s2), kk, mv)
            G = U.transpose(1, 2) @ U - torch.eye(mv, dtype=torch.float64, device=dev)
            out[s2.cpu().numpy()] = G.abs().amax(dim=(1, 2)).cpu().numpy()
        dev_u[sel] = out
bad = np.argsort(-dev_u)[:12]
print("users with max|U^T U - I| > 1e-2:", int(np.sum(dev_u > 1e-2)), "> 1e-4:", int(np.sum(dev_u > 1e-4)),
      "max", float(dev_u.max()), flush=True)
for u in bad:
    b = int(off[u])
    ev = ev_all[b:b + min(int(m[u]), int(k[u]))]
    print(f"  user {u}: k {k[u]} m {m[u]} dev {dev_u[u]:.3e} evals[:4] {ev[:4]} min gap "
          f"{float(np.min(np.diff(ev))) if len(ev) > 1 else 0:.2e}", flush=True)
