"""Diagnostics on the C4 workload (knn2 graph, 50k items): predictor phase cycles, the nc /
c / lim distribution of the ratings, and stage times of a user range.
usage: probe_c4.py [users=125000] [first=0]   (PROBE_CFG=c2 for the C2 workload)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cname = os.environ.get("PROBE_CFG", "c4")
cfg = wlm.CONFIGS[cname]
dev = torch.device("cuda")
t0 = time.time()
d_W, _, gs = wlm.config_graph(cname, Context, 0, dev, torch)
print("graph", gs, f"{time.time() - t0:.1f}s", flush=True)
k_all = wlm.user_degrees(cfg)
k = k_all[first:first + users]
off, items, rat = synth.user_items(cfg["seed"], k, cfg["items"], threads=16, u_base=first)
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


def eig():
    plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])


def pred():
    plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                     CF_SIGS_COMPAT, d["mse"], d["kk"])


for f, name in ((eig, "eigen"), (pred, "predict")):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    e1.synchronize()
    print(f"{name}: {e0.elapsed_time(e1):.1f} ms for {users} users / {n} ratings", flush=True)

if os.environ.get("PROBE_SAVE"):   # outputs of the timed configuration, for A/B equality checks
    np.savez(os.environ["PROBE_SAVE"], mse=d["mse"].cpu().numpy(), kk=d["kk"].cpu().numpy())
ctx.debug_phases(True)
pred()
torch.cuda.synchronize()
ph = ctx.debug_phases(True, read=True)
ctx.debug_phases(False)
cyc = {k_: ph[k_] for k_ in ("setup", "basis", "fast", "dense")}
tot = sum(cyc.values())
print("phase share of block cycles:", {k_: f"{v / tot * 100:.1f}%" for k_, v in cyc.items()},
      "| fast ratings", ph["n_fast"], "block-wide ratings", ph["n_dense"],
      "| wide-K share of block-wide cycles", f"{ph['wide'] / max(ph['dense'], 1) * 100:.1f}%",
      "| gram share of setup+basis", f"{ph['gram'] / max(ph['setup'] + ph['basis'], 1) * 100:.1f}%")
wf = max(ph["w_fast"], 1)
print("fast path wave-cycles: gathers+border", f"{ph['w_gather'] / wf * 100:.1f}%", "LDL^T",
      f"{ph['w_ldlt'] / wf * 100:.1f}%", "per fast rating", wf / max(ph["n_fast"], 1))
nbig = max(ph["n_fast"] - ph["n_nc4"] - ph["n_nc16"], 1)
print("fast ratings: nc<=4", ph["n_nc4"], "cyc", ph["cyc_nc4"] / max(ph["n_nc4"], 1), "| 5..16", ph["n_nc16"],
      ph["cyc_nc16"] / max(ph["n_nc16"], 1), "| >16", nbig, ph["cyc_ncbig"] / nbig)
print("block cycles per user", tot / users, "per rating", tot / n)

m = d["m"].cpu().numpy()
kk = d["kk"].cpu().numpy()
ev = d["evals"].cpu().numpy()
sg = d["sigs"].cpu().numpy()
kr = np.repeat(k.astype(np.int64), k)
nc = kr - kk
print("k mean", k.mean(), "m mean", m.mean(), "m/k", (m / k).mean(), "kk mean", kk.mean())
print("nc: mean", nc.mean(), "p50", np.median(nc), "p90", np.percentile(nc, 90), "p99", np.percentile(nc, 99),
      "frac >62", (nc > 62).mean(), "frac 0", (nc == 0).mean(), "frac <=4", (nc <= 4).mean())
uid = np.repeat(np.arange(users), k)
row = np.arange(n) - off[:-1].astype(np.int64)[uid]
lim = np.zeros(n, np.int64)
for u in range(min(users, 20000)):
    b, e = int(off[u]), int(off[u + 1])
    mu = min(int(m[u]), e - b)
    lim[b:e] = np.minimum(np.maximum(np.searchsorted(ev[b:b + mu], sg[:e - b], side="right"), 2), m[u])
sel = uid < min(users, 20000)
ls, cs, ns = lim[sel], kk[sel], nc[sel]
print("lim mean", ls.mean(), "| c < lim (rank-deficient)", (cs < ls).mean(), "| wide & c<lim", ((ns > 62) & (cs < ls)).mean(),
      "| wide & c>=lim", ((ns > 62) & (cs >= ls)).mean())
print("wide ratings: c mean", cs[ns > 62].mean() if (ns > 62).any() else 0, "lim mean", ls[ns > 62].mean() if (ns > 62).any() else 0,
      "nc mean", ns[ns > 62].mean() if (ns > 62).any() else 0)
h = np.histogram(nc, bins=[0, 1, 5, 9, 17, 33, 63, 96, 128, 200])[0]
print("nc histogram [0,1,5,9,17,33,63,96,128,200):", h.tolist())
