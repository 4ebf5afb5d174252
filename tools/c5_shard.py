"""BASELINE config 5 at its own size, one GPU's share: the 100k-user power-law set (lognormal k,
median 100, p95 / median 15, clipped to [20, 5000], 50k items, the config-4 knn2 graph) split over
8 GPUs by sum(k^3) (multi.cost_split, as bench.py --gpus 8 splits C4), and shard R run here as
that rank would: ONE cf_eigen_run over its users, then ONE cf_predict_run_f32 over every rating
(own sigs: a rank without the global compat prefix).  HIP-event times, one JSON line per shard.

usage: python tools/c5_shard.py R [R ...]      (shards of 8)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from collaborative_filtering_amd import multi, synth, workloads as wlm  # noqa: E402
from collaborative_filtering_amd._native import CF_MAX_K  # noqa: E402
from collaborative_filtering_amd.api import CF_SIGS_OWN, Context, evec_offsets  # noqa: E402

WORLD = 8
cfg = wlm.CONFIGS["c5"]
dev = torch.device("cuda")
d_W, _, gs = wlm.config_graph("c4", Context, 0, dev, torch)
n_items = wlm.CONFIGS["c4"]["items"]
k_all = wlm.c5_degrees(cfg["users"], cfg["kmax"])
cuts = multi.cost_split(k_all, WORLD)
print(f"c5: {len(k_all)} users, k p50 {int(np.median(k_all))} p95 {int(np.percentile(k_all, 95))} max "
      f"{int(k_all.max())}, sum k^3 {float(np.sum(k_all.astype(np.float64) ** 3)):.3e}; shard users "
      f"{np.diff(cuts).tolist()}", flush=True)
ctx = Context(0)
ctx.upload_graph_dense(d_W.view(n_items, -1))
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
stream = torch.cuda.current_stream(dev)
for r in [int(x) for x in sys.argv[1:]] or [0]:
    lo, hi = int(cuts[r]), int(cuts[r + 1])
    # the shard's users: the global generator's, so every shard reads the same data a rank would
    off_all, items_all, rat_all = synth.user_items(cfg["seed"], k_all[:hi], n_items, threads=16)
    k = k_all[lo:hi]
    b0 = int(off_all[lo])
    off = (off_all[lo:hi + 1] - off_all[lo]).astype(np.uint64)
    items, rat = items_all[b0:], rat_all[b0:]
    del off_all, items_all, rat_all
    eo, ne = evec_offsets(off)
    n = int(off[-1])
    print(f"shard {r}: users {lo}..{hi} ({len(k)}), ratings {n}, spill {int(np.sum(k > CF_MAX_K))}, "
          f"k > 3072 {int(np.sum(k > 3072))}, evec floats {ne / 1e9:.2f} G", flush=True)
    d_o, d_i, d_e = T(off.view(np.int64)), T(items.view(np.int32)), T(eo.view(np.int64))
    d_m = torch.zeros(len(k), dtype=torch.int32, device=dev)
    d_s = torch.zeros(n, dtype=torch.float32, device=dev)
    d_v = torch.zeros(n, dtype=torch.float32, device=dev)
    d_x = torch.zeros(ne, dtype=torch.float32, device=dev)
    d_mse = torch.zeros(n, dtype=torch.float32, device=dev)
    d_kk = torch.zeros(n, dtype=torch.int32, device=dev)
    plan = ctx.plan(off)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t = time.perf_counter()
    e[0].record(stream)
    plan.eigen_run(d_o, d_i, d_e, d_m, d_s, d_v, d_x, stream=stream.cuda_stream)
    e[1].record(stream)
    e[1].synchronize()
    print(f"shard {r}: eigen {e[0].elapsed_time(e[1]) / 1e3:.1f} s", flush=True)
    ctx.release_workspaces()   # the eigen workspace would shrink the predictor's (both sized from free HBM)
    e[3].record(stream)
    plan.predict_run(d_o, d_i, T(rat), d_m, d_v, d_e, d_x, d_s, CF_SIGS_OWN, d_mse, d_kk, stream=stream.cuda_stream)
    e[2].record(stream)
    e[2].synchronize()
    wall = time.perf_counter() - t
    eig, pred = e[0].elapsed_time(e[1]) / 1e3, e[3].elapsed_time(e[2]) / 1e3
    mse = d_mse.cpu().numpy()
    kk = d_kk.cpu().numpy()
    print(json.dumps({"shard": r, "of": WORLD, "users": int(len(k)), "ratings": n,
                      "spill_users": int(np.sum(k > CF_MAX_K)), "big_users": int(np.sum(k > 3072)),
                      "eigen_s": eig, "predict_s": pred, "wall_s": wall,
                      "users_per_s": len(k) / eig, "ratings_per_s": n / pred,
                      "m_mean": float(d_m.float().mean().item()),
                      "nan_predictions": int(np.isnan(mse).sum()), "c0_rows": int(np.sum(kk == 0)),
                      "rmse": float(np.sqrt(np.nanmean(mse)))}), flush=True)
    plan.close()
    del d_x, d_mse, d_kk, d_s, d_v
    torch.cuda.empty_cache()
