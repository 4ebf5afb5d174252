"""Diagnostics: spill predictor (192 < k <= 3072) phase cycles on the bench's config-5 sample
(lognormal k, median 100, sigma ln(15)/1.645, C4 knn2 graph of 50k items), as bench.py's c5 leg
builds it.

usage: python tools/probe_pspill_c5.py [users=1000] [kmin=192] [kmax=3072]   (users with kmin < k <= kmax)
"""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import CF_SIGS_OWN, Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
kmin = int(sys.argv[2]) if len(sys.argv) > 2 else 192
kmax = int(sys.argv[3]) if len(sys.argv) > 3 else 3072
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
n_items = wlm.CONFIGS["c4"]["items"]
seed = 2026101505
k0 = synth.degrees(seed, users, k_median=100.0, sigma=float(np.log(15.0) / 1.6449), kmin=20, kmax=5000)
off0, items0, rat0 = synth.user_items(seed, k0, n_items, threads=16)
sel = np.nonzero((k0 > kmin) & (k0 <= kmax))[0]
ks = k0[sel]
off = np.zeros(len(ks) + 1, np.uint64); off[1:] = np.cumsum(ks.astype(np.uint64))
items = np.concatenate([items0[int(off0[u]):int(off0[u + 1])] for u in sel])
rat = np.concatenate([rat0[int(off0[u]):int(off0[u + 1])] for u in sel])
ctx = Context(0); ctx.upload_graph_dense(d_W.view(n_items, -1)); plan = ctx.plan(off)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eoff, ne = evec_offsets(off); n = int(off[-1]); nu = len(ks)
d = dict(off=T(off.view(np.int64)), items=T(items.view(np.int32)), eoff=T(eoff.view(np.int64)), rat=T(rat),
         m=torch.zeros(nu, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
         evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
         mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
t = time.perf_counter()
plan.eigen_run(d["off"], d["items"], d["eoff"], d["m"], d["sigs"], d["evals"], d["evecs"])
torch.cuda.synchronize()
print(f"eigen {nu} users {time.perf_counter() - t:.2f}s", flush=True)
def pred():
    plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                     CF_SIGS_OWN, d["mse"], d["kk"])
t = time.perf_counter(); pred(); torch.cuda.synchronize(); dt = time.perf_counter() - t
print(f"spill users {nu} (k mean {ks.mean():.0f}, max {ks.max()}), {n} ratings in {dt*1e3:.1f} ms -> {n/dt:.0f}/s",
      flush=True)
out = np.zeros(16, np.uint64)
lib = ctx.lib
lib.cf_debug_phases(ctx.h, 1, ctypes.c_void_p(0))
t = time.perf_counter(); pred(); torch.cuda.synchronize(); dt2 = time.perf_counter() - t
lib.cf_debug_phases(ctx.h, 1, ctypes.c_void_p(out.ctypes.data))
names = ["sets+mean", "col filter", "P entries", "b and K", "LDLt", "dense"]
tot = float(out[:6].sum())
print(f"(debug pass {dt2*1e3:.1f} ms)", {nm: f"{out[i] / tot * 100:.1f}%" for i, nm in enumerate(names)},
      "block-cycles/rating", tot / n)
print("raw", [int(x) for x in out])
kk = d["kk"].cpu().numpy().astype(np.int64)
nc = np.concatenate([ks[u] - kk[int(off[u]):int(off[u + 1])] for u in range(nu)])
print("nc percentiles 50/90/99/max", np.percentile(nc, [50, 90, 99]), nc.max(),
      "sum nc^3/3 (GF)", (nc.astype(float) ** 3).sum() / 3e9, "sum kk^3/3 (GF)", (kk.astype(float) ** 3).sum() / 3e9)
m = d["m"].cpu().numpy()
print("k, m per user (largest 10):", sorted(zip(ks.tolist(), m.tolist()))[-10:])
print("sum k^3 (G)", (ks.astype(float) ** 3).sum() / 1e9)
print("nan", int(torch.isnan(d["mse"]).sum().item()))
