"""Per-bucket eigen cost on the C4 graph: N users of one fixed k each (items drawn like the C4
workload's), one eigen call per k on one stream (debug stats on), ms and us per user, sweeps.
usage: probe_eigen_buckets.py [users=20000] [ks=112,120,128,136,144,152,160,168,176,180] [split=1,0]
(split: cf_set_eigen_split modes to run each k with; buckets 9-12 take the split layout at 1)"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from collaborative_filtering_amd import synth, workloads as wlm
from collaborative_filtering_amd.api import Context, evec_offsets

users = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
ks = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "112,120,128,136,144,152,160,168,176,180").split(",")]
cfg = wlm.CONFIGS["c4"]
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
splits = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,0").split(",")]
ctx = Context(0)
ctx.upload_graph_dense(d_W.view(cfg["items"], -1))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
for kk in ks:
    k = np.full(users, kk, np.int32)
    off, items, _ = synth.user_items(cfg["seed"] + kk, k, cfg["items"], threads=16)
    plan = ctx.plan(off)
    eoff, ne = evec_offsets(off)
    n = int(off[-1])
    d = [T(off.view(np.int64)), T(items.view(np.int32)), T(eoff.view(np.int64)),
         torch.zeros(users, dtype=torch.int32, device=dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev),
         torch.zeros(ne, device=dev)]
    for sp in splits:
        ctx.set_eigen_split(sp)
        plan.eigen_run(*d)
        torch.cuda.synchronize()
        t = time.perf_counter()
        plan.eigen_run(*d)
        torch.cuda.synchronize()
        dt_fast = time.perf_counter() - t
        ctx.debug_stats(True)
        t = time.perf_counter()
        plan.eigen_run(*d)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = ctx.debug_stats(True, read=True)
        ev = d[5].cpu().numpy()
        print(f"k={kk} bucket {(kk + 15) // 16} split={sp}: {dt_fast * 1e3:.1f} ms ({dt_fast / users * 1e6:.2f} us/user; "
              f"stats run {dt * 1e3:.1f} ms), sweeps {st['sweeps_mean']:.2f}, "
              f"assembly cyc/user {st.get('assembly_cyc_per_user', float('nan')):.0f}, jacobi cyc/user {st['jacobi_cyc_per_user']:.0f}, "
              f"cyc/step {st['jacobi_cyc_per_step']:.0f}, epi cyc/user {st['epilogue_cyc_per_user']:.0f}, "
              f"m sum {int(d[3].sum())}, ev sum {float(np.float64(ev).sum()):.6f}", flush=True)
        ctx.debug_stats(False)
    ctx.set_eigen_split(True)
    plan.close()
    del d
    torch.cuda.empty_cache()
