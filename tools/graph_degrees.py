"""Out-degree (w > 0.1) distribution of the C2 / C4 knn2 item graphs: the local_calc unit sizes
n = 1 + out-degree (local_calc.cpp:268-272).  usage: graph_degrees.py [c2|c4 ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from collaborative_filtering_amd import workloads as wlm
from collaborative_filtering_amd.api import Context

dev = torch.device("cuda")
for name in sys.argv[1:] or ["c2", "c4"]:
    d_W, _, gs = wlm.config_graph(name, Context, 0, dev, torch)
    n = wlm.CONFIGS[name]["items"]
    deg = (d_W.view(n, n) > 0.1).sum(dim=1).cpu().numpy()
    q = np.percentile(deg, [50, 90, 99, 99.9, 100])
    print(f"{name}: items {n}, edges w>0.1 {int(deg.sum())}, out-degree p50/p90/p99/p99.9/max "
          f"{q.astype(int).tolist()}, units n >= 5000: {int(np.sum(deg + 1 >= 5000))} "
          f"({np.mean(deg + 1 >= 5000) * 100:.2f} %), n > 192: {int(np.sum(deg + 1 > 192))}", flush=True)
    del d_W
    torch.cuda.empty_cache()
