"""Dump real C4 user subgraphs (W_u of the knn2 graph, 50k items) plus this build's eigen
records of them, for CPU modelling of the eigen kernel (tools/jacobi_gram_model.py).
usage: dump_c4_users.py [out=gpurun_out/c4_users.npz] [per_band=24]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import Context

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c4_users.npz"
per = int(sys.argv[2]) if len(sys.argv) > 2 else 24
cfg = wlm.CONFIGS["c4"]
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
print("graph", gs, flush=True)
n = 20000
k = wlm.user_degrees(cfg, n)
off, items, _ = synth.user_items(cfg["seed"], k, cfg["items"], threads=16)
rng = np.random.default_rng(7)
sel = []
for lo, hi in ((177, 180), (150, 176), (90, 110), (40, 60)):
    ids = np.nonzero((k >= lo) & (k <= hi))[0]
    sel.extend(rng.choice(ids, size=min(per, len(ids)), replace=False).tolist())
sel = np.array(sorted(sel))
W2 = d_W.view(cfg["items"], cfg["items"])
blobs = {}
for u in sel:
    it = torch.from_numpy(items[off[u]:off[u + 1]].astype(np.int64)).to(dev)
    blobs[f"W_{u}"] = W2[it][:, it].cpu().numpy()
so, si, _ = wlm.sub_csr(off, items, np.zeros(len(items), np.float32), sel)
with Context(0) as ctx:
    ctx.upload_graph_dense(W2)
    ctx.debug_stats(True)
    res = ctx.eigen_batch(so, si)
    st = ctx.debug_stats(True, read=True)
print("stats", st, flush=True)
for j, u in enumerate(sel):
    sigs, evals, U = res.block(j)
    blobs[f"m_{u}"] = np.int32(res.m[j])
    blobs[f"sigs_{u}"] = sigs
    blobs[f"ev_{u}"] = evals
    blobs[f"U_{u}"] = U
np.savez_compressed(out, users=sel, **blobs)
print("wrote", out, len(sel), "users", flush=True)
