"""Diagnose cf_step_run vs sequential differences: run the sequential pair twice and the fused
step once, report which outputs differ and where (bucket k, nc class)."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, CF_SIGS_OWN, Context, evec_offsets

seed, n_items = 2026101502, 2000
k = synth.degrees(seed, 6000, k_median=90.0, sigma=0.6, kmin=2, kmax=180)
k[[5, 777, 4000]] = [260, 201, 230]
off, items, rats = synth.user_items(seed, k, n_items, threads=8)
W = synth.graph_model(seed, n_items, threads=8)
ctx = Context(0)
ctx.upload_graph_dense(W)
plan = ctx.plan(off)
dev = torch.device("cuda")
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off)
n, U = int(off[-1]), len(k)
d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))
uid = np.repeat(np.arange(U), k.astype(np.int64))
for mode in (CF_SIGS_COMPAT, CF_SIGS_OWN):
    outs = []
    for how in ("seq", "seq", "fused", "fused"):
        o = dict(m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
                 evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
                 mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev),
                 pred=torch.zeros(n, dtype=torch.float64, device=dev))
        if how == "seq":
            plan.eigen_run(d_off, d_items, d_eoff, o["m"], o["sigs"], o["evals"], o["evecs"])
            plan.predict_run(d_off, d_items, d_rat, o["m"], o["evals"], d_eoff, o["evecs"], o["sigs"], mode,
                             o["mse"], o["kk"], o["pred"])
        else:
            plan.step_run(d_off, d_items, d_rat, d_eoff, o["m"], o["sigs"], o["evals"], o["evecs"], mode,
                          o["mse"], o["kk"], o["pred"])
        torch.cuda.synchronize()
        outs.append({kk: v.cpu().numpy() for kk, v in o.items()})
    for a, b, name in ((0, 1, "seq vs seq"), (2, 3, "fused vs fused"), (0, 2, "seq vs fused")):
        for key in outs[a]:
            x, y = outs[a][key], outs[b][key]
            diff = np.nonzero(x.view(np.uint8).reshape(len(x), -1).any(1) != False) if False else None
            ne_ = ~((x == y) | (np.isnan(x.astype(np.float64)) & np.isnan(y.astype(np.float64)))) if x.dtype.kind == "f" else x != y
            if ne_.any():
                idx = np.nonzero(ne_)[0]
                ks = k[uid[idx]] if key in ("mse", "kk", "pred", "sigs", "evals") and len(x) == n else None
                print(f"mode {mode} {name}: {key} differs at {len(idx)} entries; k of those users "
                      f"{np.unique(ks)[:20] if ks is not None else '-'}; e.g. {x[idx[:3]]} vs {y[idx[:3]]}")
    print(f"mode {mode} done", flush=True)
