"""C5 one-call breakdown: the bench's 10k-user config-5 sample (seed 2026101506) in one
cf_eigen_run, then its k > 3072 users alone and its 192 < k <= 3072 users alone (HIP-synchronised
wall time each).  Run under rocprofv3 --kernel-trace --stats for the per-kernel split.
usage: python tools/probe_c5_onecall.py [users=10000] [parts=all,big,mid]
"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
parts = (sys.argv[2] if len(sys.argv) > 2 else "all,big,mid").split(",")
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
n_items = wlm.CONFIGS["c4"]["items"]
seed = 2026101506
k0 = synth.degrees(seed, users, k_median=100.0, sigma=float(np.log(15.0) / 1.6449), kmin=20, kmax=5000)
off0, items0, _ = synth.user_items(seed, k0, n_items, threads=16)
ctx = Context(0)
ctx.upload_graph_dense(d_W.view(n_items, -1))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
sels = {"all": np.arange(users), "big": np.nonzero(k0 > 3072)[0], "mid": np.nonzero((k0 > 192) & (k0 <= 3072))[0]}
for name in parts:
    sel = sels[name]
    ks = k0[sel]
    off = np.zeros(len(ks) + 1, np.uint64)
    off[1:] = np.cumsum(ks.astype(np.uint64))
    items = np.concatenate([items0[int(off0[u]):int(off0[u + 1])] for u in sel])
    eoff, ne = evec_offsets(off)
    n = int(off[-1])
    plan = ctx.plan(off)
    d_o, d_i, d_e = T(off.view(np.int64)), T(items.view(np.int32)), T(eoff.view(np.int64))
    d_m = torch.zeros(len(ks), dtype=torch.int32, device=dev)
    d_s = torch.zeros(n, device=dev)
    d_v = torch.zeros(n, device=dev)
    d_x = torch.zeros(ne, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    plan.eigen_run(d_o, d_i, d_e, d_m, d_s, d_v, d_x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    kf = ks.astype(np.float64)
    print(f"{name}: {len(ks)} users (k {ks.min()}..{ks.max()}, >3072: {(ks > 3072).sum()}) eigen {dt:.2f} s "
          f"({np.sum(9 * kf ** 3) / dt / 1e12:.2f} TFLOP/s of 9k^3)", flush=True)
    if os.environ.get("PROBE_HASH"):   # bit-identity across builds: digests of every output
        import hashlib
        dig = {nm: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:16]
               for nm, t in (("m", d_m), ("sigs", d_s), ("evals", d_v), ("evecs", d_x))}
        print(f"{name} digests {dig}", flush=True)
    plan.close()
    del d_x
    torch.cuda.empty_cache()
