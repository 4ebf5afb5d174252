"""Diagnostics: predictor phase cycles on the bench workload."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
n_items = int(os.environ.get("ITEMS", "10000"))
k = synth.degrees(2026101502, users) if not os.environ.get("KFIX") else np.full(users, int(os.environ["KFIX"]), dtype=np.uint32)
off, items, rat = synth.user_items(2026101502, k, n_items, threads=16)
W = synth.graph_model(2026101502, n_items, threads=16)
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
cyc = {k_: ph[k_] for k_ in ("setup", "basis", "fast", "dense")}
print("per user: gram", ph["gram"] / users, "setup", ph["setup"] / users, "basis", ph["basis"] / users,
      "| block-wide ratings", ph["n_dense"], "wide-K share of block-wide cycles", ph["wide"] / max(ph["dense"], 1))
tot = sum(cyc.values())
print({k_: f"{v/tot*100:.1f}%" for k_, v in cyc.items()}, "cycles/prediction:", tot / n,
      "fast", ph["n_fast"], "dense", ph["n_dense"])
m = d["m"].cpu().numpy(); kk = d["kk"].cpu().numpy()
wf = max(ph["w_fast"], 1)
print("fast path, summed over waves: gathers+border", f"{ph['w_gather']/wf*100:.1f}%", "LDL^T", f"{ph['w_ldlt']/wf*100:.1f}%",
      "rest", f"{(wf-ph['w_gather']-ph['w_ldlt'])/wf*100:.1f}%", "wave-cycles per fast rating", wf / max(ph["n_fast"], 1))
nbig = max(ph["n_fast"] - ph["n_nc4"] - ph["n_nc16"], 1)
print("completed fast ratings: nc<=4", ph["n_nc4"], "cyc/rating", ph["cyc_nc4"] / max(ph["n_nc4"], 1),
      "| 5..16", ph["n_nc16"], ph["cyc_nc16"] / max(ph["n_nc16"], 1), "| >16", nbig, ph["cyc_ncbig"] / nbig)
print("m mean", m.mean(), "kk mean", kk.mean(), "k mean", k.mean())
# lim distribution (compat sig table: w_lim of row r is sigs[r] of the global table)
ev = d["evals"].cpu().numpy(); sg = d["sigs"].cpu().numpy()
lims = []; cs = []
for u in range(min(users, 3000)):
    b, e = int(off[u]), int(off[u + 1]); mu = int(m[u])
    for r in range(e - b):
        above = np.nonzero(ev[b:b + mu] > sg[r])[0]
        lim = int(above[0]) if len(above) else mu
        lims.append(min(max(lim, 2), mu)); cs.append(kk[b + r])
lims = np.array(lims); cs = np.array(cs)
print("lim mean", lims.mean(), "p50", np.median(lims), "p90", np.percentile(lims, 90), "max", lims.max())
print("c mean", cs.mean(), "lim^3 mean", (lims.astype(float) ** 3).mean())
# complement size and zero-column filter statistics
ev_off = eoff
ncs = []; drops = []; drop0 = 0; nrat = 0; prefix = 0
for u in range(min(users, 1500)):
    b, e = int(off[u]), int(off[u + 1]); mu = int(m[u]); ku = e - b
    if mu <= 0: continue
    Uu = d["evecs"][int(ev_off[u]):int(ev_off[u]) + ku * mu].cpu().numpy().reshape(ku, mu)
    it = items[b:e]
    for r in range(ku):
        conn = W[it[r], it] > 0.1
        above = np.nonzero(ev[b:b + mu] > sg[r])[0]
        lim = min(max(int(above[0]) if len(above) else mu, 2), mu)
        keep = (Uu[conn][:, :lim] >= 1e-4).any(axis=0) if conn.any() else np.zeros(lim, bool)
        ncs.append(ku - conn.sum()); nd = lim - keep.sum(); drops.append(nd)
        drop0 += (not keep[0]); nrat += 1; prefix += keep.all()
ncs = np.array(ncs); drops = np.array(drops)
print("nc mean", ncs.mean(), "p50", np.median(ncs), "p90", np.percentile(ncs, 90), "frac nc<=8", (ncs <= 8).mean(), "frac nc<=16", (ncs <= 16).mean())
print("dropped cols mean", drops.mean(), "frac prefix", prefix / nrat, "frac col0 dropped", drop0 / nrat, "max drop", drops.max())
# why ratings leave the fast path (sample)
reasons = dict(c0=0, nc_big=0, drop=0, singular=0, ill=0, fast=0, nc_big_singular=0)
for u in range(min(users, 600)):
    b, e = int(off[u]), int(off[u + 1]); mu = int(m[u]); ku = e - b
    if mu < 2: continue
    Uu = d["evecs"][int(ev_off[u]):int(ev_off[u]) + ku * mu].cpu().numpy().reshape(ku, mu).astype(np.float64)
    it = items[b:e]
    for r in range(ku):
        conn = W[it[r], it] > 0.1
        above = np.nonzero(ev[b:b + mu] > sg[r])[0]
        lim = min(max(int(above[0]) if len(above) else mu, 2), mu)
        c = int(conn.sum()); nc = ku - c
        if c == 0: reasons["c0"] += 1; continue
        keep = (Uu[conn][:, :lim] >= 1e-4).any(axis=0)
        if not keep.all(): reasons["drop"] += 1; continue
        if nc > 62:
            reasons["nc_big"] += 1
            if c < lim: reasons["nc_big_singular"] += 1
            continue
        if c < lim: reasons["singular"] += 1; continue
        Q, _ = np.linalg.qr(Uu[:, :lim])
        B = Q[~conn]
        K = np.eye(nc) - B @ B.T
        if nc and np.linalg.eigvalsh(K).min() < 1e-6: reasons["ill"] += 1
        else: reasons["fast"] += 1
print("reasons", reasons)
# entry-work distribution and tail length (all users)
tot_e = 0.0; tot_tail = 0.0; tot_lim = 0.0; nr = 0; e_by = np.zeros(8)
bins = [0, 4, 8, 16, 24, 32, 48, 63, 10**9]
for u in range(users):
    b, e = int(off[u]), int(off[u + 1]); mu = int(m[u]); ku = e - b
    if mu < 2: continue
    lim = np.minimum(np.maximum(np.searchsorted(ev[b:b + mu], sg[:ku], side="right"), 2), mu)
    nc_u = ku - kk[b:e]
    w = (nc_u + 1) * (nc_u + 2) / 2 * lim
    tot_e += w.sum(); tot_tail += (lim.max() - lim).sum(); tot_lim += lim.sum(); nr += ku
    e_by += np.histogram(nc_u, bins=bins, weights=w)[0]
print("entry FMA per rating", tot_e / nr, "mean lim", tot_lim / nr, "mean tail Lu-lim", tot_tail / nr)
print("entry-work share by nc bins", dict(zip([f"<{b}" for b in bins[1:]], np.round(e_by / e_by.sum(), 3))))
mse_h = d["mse"].cpu().numpy()
print("NaN mse: total", int(np.isnan(mse_h).sum()), "with c=0", int((np.isnan(mse_h) & (kk == 0)).sum()),
      "with c>0", int((np.isnan(mse_h) & (kk > 0)).sum()))
