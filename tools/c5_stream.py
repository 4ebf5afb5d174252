"""BASELINE config 5 as a whole on ONE GPU in ONE call (VERDICT r5 missing 2 / next item 3).

The 100k-user power-law set (lognormal k, median 100, p95 ~1500, cap 5000; the config-4 knn2
graph) runs through cf_eigen_batch_stream -- the entry point bin/precompute_local drives -- in
memory-bounded chunks, every chunk's records digested (xxh3 per user over m, sigs, the m
evals and the k x m block) in the sink as they arrive.  Then the same users run as the 8
k^3-balanced shards of tools/c5_shard.py (one cf_eigen_run + cf_pack_eigen_run per shard, the
multi-GPU path's ranges), digested the same way: every user's record must be equal.  (The
records themselves, ~120 GB binary / ~1.2 TB text, do not fit the box's 79 GB disk, hence the
digests.)  Progress lines go to stdout; the last line is the JSON summary.

usage: python tools/c5_stream.py [--chunk-gb G] [--users N] [--no-ref]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import xxhash

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from collaborative_filtering_amd import _native, multi, synth, workloads as wlm  # noqa: E402
from collaborative_filtering_amd.api import Context, evec_offsets  # noqa: E402
from collaborative_filtering_amd._native import ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chunk-gb", type=float, default=0.0)
ap.add_argument("--users", type=int, default=0)
ap.add_argument("--no-ref", action="store_true")
args = ap.parse_args()

t0 = time.perf_counter()
cfg = wlm.CONFIGS["c5"]
dev = torch.device("cuda")
n_items = wlm.CONFIGS["c4"]["items"]
d_W, _, _ = wlm.config_graph("c4", Context, 0, dev, torch)
k_all = wlm.c5_degrees(cfg["users"], cfg["kmax"])
if args.users:
    k_all = k_all[:args.users]
n_users = len(k_all)
off, items, _ = synth.user_items(cfg["seed"], k_all, n_items, threads=16)
off = off.astype(np.uint64)
_, n_slots = evec_offsets(off)
print(f"c5: {n_users} users, k p50 {int(np.median(k_all))} p95 {int(np.percentile(k_all, 95))} max {int(k_all.max())}, "
      f"ratings {int(off[-1])}, eigenvector slots {4 * n_slots / 1e9:.1f} GB; setup {time.perf_counter() - t0:.0f} s",
      flush=True)
ctx = Context(0)
ctx.upload_graph_dense(d_W.view(n_items, -1))
del d_W
torch.cuda.empty_cache()


def digest(m, sg, ev, blk):
    h = xxhash.xxh3_64()
    h.update(np.int32(m).tobytes())
    h.update(sg.tobytes())
    h.update(ev.tobytes())
    h.update(blk.tobytes())
    return h.intdigest()


# ---- (1) one cf_eigen_batch_stream call over every user ----------------------------------
dig_s = np.zeros(n_users, dtype=np.uint64)
ms = np.zeros(n_users, dtype=np.int32)
seen = [0, 0.0]
t_call = time.perf_counter()


def sink(_user, cp):
    c = cp.contents
    n = int(c.count)
    off_c = np.ctypeslib.as_array(c.item_off, shape=(n + 1,))
    po = np.ctypeslib.as_array(c.packed_off, shape=(n + 1,))
    ne, npk = int(off_c[-1]), int(po[-1])
    m = np.ctypeslib.as_array(c.m, shape=(n,))
    sg = np.ctypeslib.as_array(c.sigs, shape=(max(ne, 1),))
    ev = np.ctypeslib.as_array(c.evals, shape=(max(ne, 1),))
    vv = np.ctypeslib.as_array(c.evecs, shape=(max(npk, 1),))
    for u in range(n):
        b, e = int(off_c[u]), int(off_c[u + 1])
        q = min(int(m[u]), e - b)
        dig_s[c.first + u] = digest(m[u], sg[b:e], ev[b:b + q], vv[int(po[u]):int(po[u + 1])])
    ms[c.first:c.first + n] = m
    seen[0] += 1
    seen[1] += 4.0 * npk
    print(f"  chunk {seen[0]}: users {c.first}..{c.first + n}, {4 * npk / 1e9:.2f} GB of records, "
          f"t = {time.perf_counter() - t_call:.1f} s", flush=True)
    return 0


lib = _native.load()
cb = _native.EIGEN_SINK(sink)
st = _native.EigenStreamStats()
arr = (ctypes.c_void_p * 1)(ctx.h)
rc = lib.cf_eigen_batch_stream(arr, 1, n_users, ptr(off), ptr(items), int(args.chunk_gb * 1e9), cb, None,
                               ctypes.byref(st))
stream_s = time.perf_counter() - t_call
if rc != 0:
    print(f"cf_eigen_batch_stream failed ({rc}): {lib.cf_last_error(ctx.h).decode()}", flush=True)
    sys.exit(1)
print(f"stream: {st.chunks} chunks (budget {st.chunk_slot_bytes / 1e9:.1f} GB of slots, largest "
      f"{st.max_chunk_slot_bytes / 1e9:.1f} GB), {stream_s:.1f} s = {n_users / stream_s:.0f} users/s; peak device "
      f"memory {st.own_peak_bytes / 1e9:.1f} GB own / {st.device_peak_bytes / 1e9:.1f} GB in use", flush=True)
res = {"users": n_users, "ratings": int(off[-1]), "slot_bytes": 4 * n_slots, "record_bytes": seen[1],
       "chunks": st.chunks, "chunk_slot_budget_bytes": st.chunk_slot_bytes,
       "max_chunk_slot_bytes": st.max_chunk_slot_bytes, "own_peak_device_bytes": st.own_peak_bytes,
       "device_peak_bytes_in_use": st.device_peak_bytes, "stream_s": stream_s, "stream_users_per_s": n_users / stream_s,
       "m_mean": float(ms.mean())}

# ---- (2) the 8 k^3-balanced shards, one cf_eigen_run each (tools/c5_shard.py's ranges) ---------
if not args.no_ref:
    cuts = multi.cost_split(k_all, 8)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)   # noqa: E731
    stream = torch.cuda.current_stream(dev)
    dig_r = np.zeros(n_users, dtype=np.uint64)
    t_ref = time.perf_counter()
    for r in range(8):
        lo, hi = int(cuts[r]), int(cuts[r + 1])
        if hi <= lo:
            continue
        so = (off[lo:hi + 1] - off[lo]).astype(np.uint64)
        si = items[int(off[lo]):int(off[hi])]
        eo, ne = evec_offsets(so)
        n = int(so[-1])
        nu = hi - lo
        d_o, d_i, d_e = T(so.view(np.int64)), T(si.view(np.int32)), T(eo.view(np.int64))
        d_m = torch.zeros(nu, dtype=torch.int32, device=dev)
        d_s = torch.zeros(n, dtype=torch.float32, device=dev)
        d_v = torch.zeros(n, dtype=torch.float32, device=dev)
        d_x = torch.zeros(ne, dtype=torch.float32, device=dev)
        plan = ctx.plan(so)
        plan.eigen_run(d_o, d_i, d_e, d_m, d_s, d_v, d_x, stream=stream.cuda_stream)
        d_po = torch.zeros(nu + 1, dtype=torch.int64, device=dev)
        ctx.pack_eigen_run(nu, d_o, d_m, None, None, d_po, None, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        d_pk = torch.empty(max(int(d_po[-1].item()), 1), dtype=torch.float32, device=dev)
        ctx.pack_eigen_run(nu, d_o, d_m, d_e, d_x, d_po, d_pk, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        del d_x
        m, sg, ev = d_m.cpu().numpy(), d_s.cpu().numpy(), d_v.cpu().numpy()
        po, pk = d_po.cpu().numpy(), d_pk.cpu().numpy()
        for u in range(nu):
            b, e = int(so[u]), int(so[u + 1])
            q = min(int(m[u]), e - b)
            dig_r[lo + u] = digest(m[u], sg[b:e], ev[b:b + q], pk[int(po[u]):int(po[u + 1])])
        plan.close()
        del d_pk, d_o, d_i, d_e, d_m, d_s, d_v, d_po, pk
        torch.cuda.empty_cache()
        ctx.release_workspaces()
        print(f"  shard {r}: users {lo}..{hi}, t = {time.perf_counter() - t_ref:.1f} s, equal so far "
              f"{int(np.sum(dig_r[lo:hi] == dig_s[lo:hi]))} / {nu}", flush=True)
    res["ref_shards_s"] = time.perf_counter() - t_ref
    res["records_equal"] = int(np.sum(dig_r == dig_s))
    res["records_equal_all"] = bool(np.array_equal(dig_r, dig_s))
res["wall_s"] = time.perf_counter() - t0
print(json.dumps(res), flush=True)
