"""A/B timing of the spill predictor on the bench's config-5 sample (users with kmin < k <= kmax),
two timed passes, outputs saved for a bit-identity check between variants (env-selected).

usage: python tools/probe_pspill_ab.py users kmin kmax out.npz
"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import CF_SIGS_OWN, Context, evec_offsets

users, kmin, kmax, out_path = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
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
for rep in range(2):
    d["mse"].zero_()
    t = time.perf_counter()
    plan.predict_run(d["off"], d["items"], d["rat"], d["m"], d["evals"], d["eoff"], d["evecs"], d["sigs"],
                     CF_SIGS_OWN, d["mse"], d["kk"])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"pass {rep}: {nu} users (k mean {ks.mean():.0f}, max {ks.max()}), {n} ratings in {dt*1e3:.1f} ms "
          f"-> {n/dt:.0f}/s", flush=True)
np.savez(out_path, mse=d["mse"].cpu().numpy(), kk=d["kk"].cpu().numpy())
