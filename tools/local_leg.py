"""bench.py's local_calc leg alone: `bin/local_calc --pct P` on a config's knn2 graph (default C2),
every (movie, test user) pair of the sampled movies' units through cf_local_calc.
usage: local_leg.py [config=c2] [pct=1]"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

import bench
from collaborative_filtering_amd.api import Context

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
pct = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
sys.argv = [sys.argv[0]]
args = bench.parse()
cfg = bench.CONFIGS[name]
args.users = cfg["users"]
dev = torch.device("cuda")
t0 = time.time()


def beat():   # a long cf_local_calc call prints nothing; gpurun takes 3 silent minutes for a hang
    while True:
        time.sleep(30)
        print(f"... {time.time() - t0:.0f}s", flush=True)


threading.Thread(target=beat, daemon=True).start()
d_W, _, gs = bench.train_graph(Context, 0, dev, torch, cfg["seed"], cfg["train_users"], cfg["items"])
ctx = Context(0)
wl = bench.Workload(args, cfg, 0, 1, dev, torch, ctx, d_W.view(cfg["items"], cfg["items"]))
print("setup", f"{time.time() - t0:.1f}s", flush=True)
out = bench.local_calc_leg(ctx, wl, d_W.view(cfg["items"], cfg["items"]), pct=pct,
                           cpu_seconds=float(os.environ.get("LOCAL_CPU_SECONDS", "0")))
print(json.dumps(out), flush=True)
