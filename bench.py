#!/usr/bin/env python3
"""Benchmark of the MI355X hot path: per-user Laplacian eigendecomposition
(precompute_local_threads) fused with the graph-signal predictor
(local_calc_precomp), on device-resident synthetic MovieLens-shaped data.

Workload (default): BASELINE config 4, the one the metric is quoted on -- ONE global set of
1,000,000 test users x 50,000 items, k lognormal (median 100, sigma 0.5) clipped to
[20, 180], Zipf(1) items, ratings 1..5, seed 2026101504.  The item graph is knn2's output
(cf_item_cosine_run, the int8 MFMA path) over a 500,000-user train population from the same
generator (seed + 1), built in untimed setup.

One step = one pass of the hot path over the rank's users with inputs resident in HBM:
    cf_eigen_run       compute_eigens for every user (precompute_local_threads.cpp:100-213)
 -> cf_pack_eigen_run  the records packed contiguously (the binary out_eigen_ payload)
 -> cf_predict_run_f32 neigh_program::apply for every test rating (local_calc_precomp.cpp:217-380)
 -> (N > 1) gather of the packed records to rank 0 over RCCL p2p
Users are range-split across ranks by cumulative k^3 (multi.cost_split) out of the ONE
global set: total work is fixed as N grows ("scaling": "strong").

Prints ONE JSON line (rank 0).  `value` = user-subgraph eigendecomps/sec of the whole job
through the step; predicted ratings/sec and per-stage rates are extra fields.  See DESIGN.md
sec. 6 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3   # MI355X fp32 vector peak (packed FMA), MI355X_MICROARCH.md
FP64_PEAK_TFLOPS = 78.6    # fp64 vector peak
HBM_PEAK_GBS = 8000.0
INT8_PEAK_TOPS = 5000.0    # int8 MFMA dense (2x bf16 2.5 PF), MI355X_MICROARCH.md

CONFIGS = {
    "c4": {"name": "BASELINE config 4", "users": 1_000_000, "items": 50_000, "seed": 2026101504,
           "train_users": 500_000},
    "c2": {"name": "BASELINE config 2", "users": 100_000, "items": 10_000, "seed": 2026101502,
           "train_users": 400_000},
}
K_MEDIAN, K_SIGMA, K_MIN, K_MAX = 100.0, 0.5, 20, 180


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c4")
    p.add_argument("--users", type=int, default=0, help="global test users (default: the config's)")
    p.add_argument("--fused", choices=["on", "off"], default="off",
                   help="on: cf_step_run (per-bucket eigen/predict overlap); off: cf_eigen_run then cf_predict_run_f32")
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--profile-steps-only", action="store_true", help="no legs, no PMC, no CPU baseline")
    p.add_argument("--pmc", choices=["auto", "off"], default="auto",
                   help="N=1: HBM traffic from two rocprofv3 --pmc child passes (FETCH_SIZE, WRITE_SIZE)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)   # one pass, no output
    p.add_argument("--io", choices=["auto", "off"], default="auto",
                   help="C4-size out_eigen_ write/parse leg (binary all records, text the first 100k)")
    p.add_argument("--io-text-users", type=int, default=100_000,
                   help="records of the C4 text out_eigen_ round trip (the binary form always takes all)")
    p.add_argument("--c2", choices=["auto", "off"], default="auto",
                   help="N=1 secondary leg: BASELINE config 2 (100k x 10k) steps and the out_eigen_ text phases")
    p.add_argument("--knn2", choices=["auto", "off", "only"], default="auto",
                   help="BASELINE config 3 knn2 leg (N=1, rank 0): int8 MFMA item cosine, 20k items x 500k users")
    p.add_argument("--prep", choices=["auto", "off", "only"], default="auto",
                   help="data-prep leg (N=1, rank 0): GPU knn regroup + k-fold order on the config-2 ratings")
    p.add_argument("--knn2-users", type=int, default=500_000)
    p.add_argument("--knn2-items", type=int, default=20_000)
    p.add_argument("--knn2-reps", type=int, default=3)
    p.add_argument("--c5", choices=["auto", "off", "only"], default="auto",
                   help="BASELINE config 5 sample (N=1, rank 0): power-law k mix through the LDS + spill paths")
    p.add_argument("--c5-users", type=int, default=1000, help="config-5 sample of the per-path legs (eigen + predict)")
    p.add_argument("--c5-onecall-users", type=int, default=10000,
                   help="config-5 sample of the one-call eigen leg (every user in one cf_eigen_run)")
    p.add_argument("--c5-kmax", type=int, default=5000, help="cap of the config-5 degrees (SURVEY 8d: 5000)")
    p.add_argument("--c5-predict-kmax", type=int, default=5000,
                   help="predict the C5 sample's groups up to this k (the per-rating systems grow as k^3)")
    p.add_argument("--eigen-method", choices=["jacobi", "tridiag"],
                   default=os.environ.get("CF_EIGEN_METHOD", "jacobi"),
                   help="k <= 192 eigensolver of the timed step (cf_set_eigen_method)")
    return p.parse_args()


def host_threads():
    """Host threads this process can use: the affinity mask, capped by the cgroup CPU quota
    (on the GPU box the mask lists all 256 CPUs of the machine but the quota is 16), plus the
    machine's counts for the record."""
    import shutil
    import subprocess

    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:   # cgroup v2 CPU quota, if any ("max 100000" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    nproc = None
    if shutil.which("nproc"):
        try:
            nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
        except (subprocess.SubprocessError, ValueError):
            pass
    threads = max(1, min(aff, int(np.ceil(quota)))) if quota else aff
    return threads, {"nproc": nproc, "affinity_cpus": aff, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota}


def train_graph(ctx_cls, dev_index, dev, torch, seed, n_train, n_items, keep_host=False):
    """The item graph of a config: knn2 (cf_item_cosine_run, int8 MFMA, cnt > 5, w > 0.01)
    over a train population from the same generator (seed + 1).  Runs on its own context
    (closed afterwards, releasing the code plane).  Returns (device dense W, host copy or
    None, knn2 stats)."""
    from collaborative_filtering_amd import synth

    tseed = seed + 1
    tk = synth.degrees(tseed, n_train, k_median=K_MEDIAN, sigma=K_SIGMA, kmin=K_MIN, kmax=K_MAX)
    toff, titems, trat = synth.user_items(tseed, tk, n_items, threads=16)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_W = torch.empty(n_items * n_items, dtype=torch.float32, device=dev)
    with ctx_cls(dev_index) as kctx:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(dev)
        e0.record(stream)
        kctx.item_cosine_run(n_train, n_items, T(toff.view(np.int64)), T(titems.view(np.int32)), T(trat), 1, d_W,
                             stream=stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        _, gemm_ms, path = kctx.knn2_timing()
    W2 = d_W.view(n_items, n_items)
    stats = {"train_users": n_train, "train_seed": tseed, "knn2_ms": e0.elapsed_time(e1), "knn2_kernel_ms": gemm_ms,
             "knn2_path": path, "edges_w_gt_0.01": int((W2 > 0).sum().item()),
             "edges_w_gt_0.1": int((W2 > 0.1).sum().item())}
    W_host = d_W.cpu().numpy().reshape(n_items, n_items) if keep_host else None
    return d_W, W_host, stats


class Workload:
    """One rank's share of a config: its users (range of the global set), device buffers."""

    def __init__(self, args, cfg, rank, world, dev, torch, ctx, W_dev):
        from collaborative_filtering_amd import synth
        from collaborative_filtering_amd.api import evec_offsets
        from collaborative_filtering_amd.multi import compat_prefix_users, cost_split

        self.torch = torch
        self.U = args.users or cfg["users"]
        self.seed = cfg["seed"]
        self.n_items = cfg["items"]
        k_all = synth.degrees(self.seed, self.U, k_median=K_MEDIAN, sigma=K_SIGMA, kmin=K_MIN, kmax=K_MAX)
        self.split = cost_split(k_all, world)
        lo, hi = int(self.split[rank]), int(self.split[rank + 1])
        self.lo, self.hi = lo, hi
        self.k = k_all[lo:hi]
        self.k_all = k_all
        self.off, self.items, self.ratings = synth.user_items(self.seed, self.k, self.n_items, threads=16, u_base=lo)
        self.evec_off, n_evec = evec_offsets(self.off)
        self.n_users = hi - lo
        self.n_entries = int(self.off[-1])
        ctx.upload_graph_dense(W_dev)
        self.plan = ctx.plan(self.off)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.d_off = T(self.off.view(np.int64))
        self.d_items = T(self.items.view(np.int32))
        self.d_rat = T(self.ratings)
        self.d_eoff = T(self.evec_off.view(np.int64))
        nu = max(self.n_users, 1)
        self.d_m = torch.zeros(nu, dtype=torch.int32, device=dev)
        self.d_sigs = torch.zeros(max(self.n_entries, 1), dtype=torch.float32, device=dev)
        self.d_evals = torch.zeros(max(self.n_entries, 1), dtype=torch.float32, device=dev)
        self.d_evecs = torch.zeros(max(n_evec, 1), dtype=torch.float32, device=dev)
        self.d_mse = torch.zeros(max(self.n_entries, 1), dtype=torch.float32, device=dev)
        self.d_kk = torch.zeros(max(self.n_entries, 1), dtype=torch.int32, device=dev)
        self.d_poff = torch.zeros(self.n_users + 1, dtype=torch.int64, device=dev)
        self.d_packed = None
        self.ctx = ctx
        # compat w_lim reads the GLOBAL concatenated sig table (local_calc_precomp.cpp:414,437,440):
        # its rows [0, kmax) are the sigs of the first j users of the global set.  Rank 0 owns them
        # (its d_sigs); every other rank recomputes those users in its step (multi.compat_prefix_users)
        self.pre = None
        j = compat_prefix_users(k_all)
        if (lo > 0 or hi < j) and j > 0:
            poff, pitems, _ = synth.user_items(self.seed, k_all[:j], self.n_items, threads=16, u_base=0)
            peoff, pn = evec_offsets(poff)
            self.pre = {"plan": ctx.plan(poff), "off": T(poff.view(np.int64)), "items": T(pitems.view(np.int32)),
                        "eoff": T(peoff.view(np.int64)), "m": torch.zeros(j, dtype=torch.int32, device=dev),
                        "sigs": torch.zeros(int(poff[-1]), dtype=torch.float32, device=dev),
                        "evals": torch.zeros(int(poff[-1]), dtype=torch.float32, device=dev),
                        "evecs": torch.zeros(max(pn, 1), dtype=torch.float32, device=dev), "users": j}
        self.prefix_users = j

    def eigen(self, sp):
        self.plan.eigen_run(self.d_off, self.d_items, self.d_eoff, self.d_m, self.d_sigs, self.d_evals, self.d_evecs,
                            stream=sp)

    def pack(self, sp):
        """The records packed contiguously (cf_pack_eigen_run); the buffer is sized once."""
        if self.d_packed is None:
            self.ctx.pack_eigen_run(self.n_users, self.d_off, self.d_m, None, None, self.d_poff, None, stream=sp)
            self.torch.cuda.synchronize()
            self.d_packed = self.torch.empty(max(int(self.d_poff[-1].item()), 1), dtype=self.torch.float32,
                                             device=self.d_m.device)
        self.ctx.pack_eigen_run(self.n_users, self.d_off, self.d_m, self.d_eoff, self.d_evecs, self.d_poff,
                                self.d_packed, stream=sp)

    def step(self, sp):
        """cf_step_run: both stages with per-bucket overlap (identical outputs)."""
        from collaborative_filtering_amd.api import CF_SIGS_COMPAT

        self.plan.step_run(self.d_off, self.d_items, self.d_rat, self.d_eoff, self.d_m, self.d_sigs, self.d_evals,
                           self.d_evecs, CF_SIGS_COMPAT, self.d_mse, self.d_kk, stream=sp)

    def sig_table(self, sp):
        """The compat sig table of this rank: its own d_sigs on rank 0 (the global set's first
        users are its first users); elsewhere the prefix users' sigs, recomputed on this GPU."""
        if self.pre is None:
            return self.d_sigs
        p = self.pre
        p["plan"].eigen_run(p["off"], p["items"], p["eoff"], p["m"], p["sigs"], p["evals"], p["evecs"], stream=sp)
        return p["sigs"]

    def predict(self, sp):
        from collaborative_filtering_amd.api import CF_SIGS_COMPAT

        tab = self.sig_table(sp)
        self.plan.predict_run(self.d_off, self.d_items, self.d_rat, self.d_m, self.d_evals, self.d_eoff, self.d_evecs,
                              tab, CF_SIGS_COMPAT, self.d_mse, self.d_kk, stream=sp)


_PHASE = ["start"]


def phase(name):
    """Name the bench phase for the stderr heartbeat (and print it there)."""
    _PHASE[0] = name
    print(f"[bench] {name}", file=sys.stderr, flush=True)


def _heartbeat(t0):
    # one stderr line every 30 s: long silent phases (graph build, PMC passes, the I/O and
    # local_calc legs) stay visible to a supervisor that takes a silent process for a hung one
    import threading

    def beat():
        while True:
            time.sleep(30)
            print(f"[bench] {time.time() - t0:.0f} s: {_PHASE[0]}", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    args = parse()
    if not args.pmc_child:
        _heartbeat(time.time())
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("CF_DIST_BACKEND", "nccl")   # "gloo" only to rehearse N>1 on one GPU
    n_vis = max(1, torch.cuda.device_count())
    dev_index = local_rank % n_vis
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", dev_index)

    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd.api import Context

    if args.c5 == "only":
        with Context(dev_index) as cctx:
            W, _, _ = train_graph(Context, dev_index, dev, torch, CONFIGS["c4"]["seed"], CONFIGS["c4"]["train_users"],
                                  CONFIGS["c4"]["items"])
            print(json.dumps(c5_leg(args, cctx, dev, torch, W.view(CONFIGS["c4"]["items"], -1))), flush=True)
        return
    if args.knn2 == "only":
        with Context(dev_index) as kctx:
            if args.pmc_child:   # one knn2 call for the PMC collector, then exit
                knn2_workload_call(args, kctx, dev, torch)
                return
            print(json.dumps(knn2_leg(args, kctx, dev, torch)), flush=True)
        return
    if args.prep == "only":
        with Context(dev_index) as pctx:
            res = prep_leg(args, pctx, dev, torch)
            if not args.pmc_child:
                print(json.dumps(res), flush=True)
        return

    if args.fused == "on" and world > 1:
        # cf_step_run builds its compat table from the rank's own first users; ranks > 0 need the
        # global set's (Workload.sig_table), which only the two-call step provides
        raise SystemExit("--fused on is single-rank only")
    cfg = CONFIGS[args.config]
    solo = rank == 0 and world == 1 and not args.profile_steps_only and not args.pmc_child
    want_cpu = solo and not args.no_cpu_baseline

    # ---- workload (untimed setup) -------------------------------------------------
    phase("setup: item graph and workload")
    t_setup = time.time()
    d_W, W_host, gstats = train_graph(Context, dev_index, dev, torch, cfg["seed"], cfg["train_users"], cfg["items"],
                                      keep_host=want_cpu)
    ctx = Context(dev_index)
    ctx.set_eigen_method(args.eigen_method)
    wl = Workload(args, cfg, rank, world, dev, torch, ctx, d_W.view(cfg["items"], cfg["items"]))
    del d_W
    torch.cuda.empty_cache()
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    setup_s = time.time() - t_setup

    gather_state = {}

    def gather(kind):
        """Both record kinds of every rank to rank 0 (per-peer RCCL p2p): kind "eigen" = the
        packed eigen records (out_eigen_), started right after the pack so the transfer runs
        beside the predictor; kind "pred" = the prediction rows (out_res_: mse, kk), as the
        reference saves out_res_ from every rank (local_calc_precomp.cpp:576).  Rank 0 receives
        into preallocated outputs (no concatenation).  Returns the outstanding works."""
        from collaborative_filtering_amd.multi import exchange_counts, gather_to_rank0

        if "counts" not in gather_state:   # sizes are fixed for the workload: exchanged once
            coll_dev = dev if backend == "nccl" else torch.device("cpu")
            gather_state["n_packed"] = int(wl.d_poff[-1].item())
            cnt = exchange_counts([wl.n_users, wl.n_entries, wl.n_entries, gather_state["n_packed"], wl.n_entries,
                                   wl.n_entries], device=coll_dev)
            gather_state["counts"] = {"eigen": cnt[:, :4], "pred": cnt[:, 4:]}
        if kind == "eigen":
            parts = [wl.d_m[:wl.n_users], wl.d_sigs[:wl.n_entries], wl.d_evals[:wl.n_entries],
                     wl.d_packed[:gather_state["n_packed"]]]
        else:
            parts = [wl.d_mse[:wl.n_entries], wl.d_kk[:wl.n_entries]]
        if backend != "nccl":
            parts = [p_.cpu() for p_ in parts]
        res, works = gather_to_rank0(parts, gather_state["counts"][kind], out=gather_state.get(kind), async_op=True)
        if res is not None:
            gather_state[kind] = res   # rank 0 reuses its receive buffers every step
        return works

    n_ev = 4
    evs = []

    fused_eig = []

    def step(record):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(n_ev)] if record else None
        if record:
            e[0].record(stream)
        if args.fused == "on":
            # cf_step_run: the predictor of each k-bucket overlaps the later eigen buckets
            wl.step(sp)
            if record:
                e[1].record(stream)
            wl.pack(sp)
            if record:
                e[2].record(stream)
        else:
            wl.eigen(sp)
            wl.pack(sp)
            if record:
                e[1].record(stream)
            works = gather("eigen") if world > 1 else []   # beside the predictor
            wl.predict(sp)
            if record:
                e[2].record(stream)
            if world > 1:
                works += gather("pred")
                for w in works:
                    w.wait()
        if record:
            e[3].record(stream)
            evs.append(e)
            if args.fused == "on":
                fused_eig.append(wl.plan.step_timing()[0])

    if args.pmc_child:   # one step for the PMC collector, then exit
        step(False)
        torch.cuda.synchronize(dev)
        return

    phase("warmup and timed steps")
    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)

    # ---- timed region: exactly K steps between barrier+sync pairs --------------------
    # (per-bucket HIP event pairs on the eigen launch streams, read after the region: the
    # dominant kernel's in-step duration for the roofline)
    ctx.eigen_bucket_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    bucket_ms, bucket_sw_ms = ctx.eigen_bucket_timing(False, read=True, sweeps=True)
    if world > 1:
        coll_dev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-stage durations: HIP events on the launch streams, recorded inside the timed steps
    gat_ms = [e[2].elapsed_time(e[3]) for e in evs]
    gat_s = float(np.median(gat_ms)) / 1e3
    overlap = None
    if args.fused == "on":
        # eigen = step start -> last eigen bucket (cf_step_timing; the predictor runs beside it);
        # the predictor's own duration is measured in isolation below (cf_predict_run_f32 alone)
        fused_ms = [e[0].elapsed_time(e[1]) for e in evs]
        eig_s = float(np.median(fused_eig)) / 1e3
        torch.cuda.synchronize(dev)
        iso = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        iso[0].record(stream)
        wl.eigen(sp)
        iso[1].record(stream)
        wl.predict(sp)
        iso[2].record(stream)
        iso[2].synchronize()
        eig_iso_s, pred_s = iso[0].elapsed_time(iso[1]) / 1e3, iso[1].elapsed_time(iso[2]) / 1e3
        overlap = {"fused_step_ms": float(np.median(fused_ms)), "eigen_span_ms": eig_s * 1e3,
                   "eigen_isolated_ms": eig_iso_s * 1e3, "predict_isolated_ms": pred_s * 1e3,
                   "sequential_sum_ms": (eig_iso_s + pred_s) * 1e3,
                   "note": "cf_step_run overlaps each k-bucket's predictor with the later eigen buckets; "
                           "eigen_span = step start to the last eigen bucket inside the timed steps; the "
                           "isolated times come from one untimed sequential pass (cf_eigen_run, then "
                           "cf_predict_run_f32) and are what the predictor roofline uses"}
    else:
        eig_ms = [e[0].elapsed_time(e[1]) for e in evs]
        pred_ms = [e[1].elapsed_time(e[2]) for e in evs]
        eig_s = float(np.median(eig_ms)) / 1e3
        pred_s = float(np.median(pred_ms)) / 1e3
    # Jacobi sweep counts of one more (untimed) eigen pass, for the executed-flop estimate
    # (one stream: every k-bucket alone on the GPU, timed too -- the dominant kernel's
    # stand-alone duration, which a rocprofv3 average over the run's launches mixes in)
    ctx.debug_stats(True)
    ctx.eigen_bucket_timing(True)
    wl.eigen(sp)
    torch.cuda.synchronize(dev)
    bucket_alone_ms, bucket_sw_alone_ms = ctx.eigen_bucket_timing(False, read=True, sweeps=True)
    jstats = ctx.debug_stats(False, read=True)

    # ---- accounting -------------------------------------------------------------------
    m_h = wl.d_m.cpu().numpy()[:wl.n_users]
    kk_h = wl.d_kk.cpu().numpy()[:wl.n_entries]
    mse_h = wl.d_mse.cpu().numpy()[:wl.n_entries]
    evals_h = wl.d_evals.cpu().numpy()
    sigs_h = wl.d_sigs.cpu().numpy()
    step_s = elapsed / args.steps
    n_pred_local = wl.n_entries
    if world > 1:
        coll_dev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(n_pred_local)], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t)
        n_pred_total = int(t.item())
    else:
        n_pred_total = n_pred_local
    value = wl.U / step_s
    roof_eigen = eigen_roofline(wl.k, m_h, eig_s, jstats, bucket_ms, bucket_alone_ms, bucket_sw_ms, bucket_sw_alone_ms)
    pred_acc = predictor_flops(wl.off, wl.k, m_h, kk_h, evals_h, sigs_h)
    roof_pred = predict_roofline(pred_acc, pred_s)
    dominant_is_pred = pred_s >= eig_s
    # the contract's roofline is the DOMINANT KERNEL's (the stage-level figure did
    # not follow for it): eigen_kernel<12, true>'s algorithmic flops per launch over its mean
    # in-step HIP-event duration at the top level; the stage-level numbers move to "stage"
    dom = roof_eigen.get("dominant")
    if dom and dom.get("achieved") is not None:
        stage = {kk: roof_eigen.pop(kk) for kk in ("kernel", "achieved", "frac", "algorithmic_flops_per_stage",
                                                   "algorithmic_bytes_per_stage", "algorithmic_GBps",
                                                   "executed_flops_per_stage", "executed_TFLOPs", "executed_frac")
                 if kk in roof_eigen}
        stage["note"] = "the eigen stage as a whole: every k-bucket launch and the record pack over the stage span"
        roof_eigen["stage"] = stage
        roof_eigen.update({"kernel": dom["kernel"], "achieved": dom["achieved"], "frac": dom["frac"],
                           "algorithmic_flops_per_launch": dom["flops_per_launch"],
                           "ms_per_launch": dom["ms_per_launch"],
                           "per_unit": "9k^3 + 4k^2 flops per user (SURVEY 8d) x the launch's users"})
    devices = None
    if world > 1:
        coll_dev = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([dev_index], dtype=torch.int64, device=coll_dev)
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        devices = sorted(set(int(x.item()) for x in allv))
    n_gpus = len(devices) if devices else 1

    kf_all = wl.k_all.astype(np.float64)
    result = {
        "metric": "user-subgraph eigendecomps/sec + predicted ratings/sec, 1M users avg deg 100",
        "value": value,
        "unit": "user-subgraph eigendecomps/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 (eigen) / f64 (predict)",
        "data": "synthetic (splitmix64 MovieLens-shaped: Zipf(1) items, lognormal k, ratings 1..5); item graph = "
                "this repo's knn2 (int8 MFMA) over a train population of the same generator",
        "config": {
            "workload": f"{cfg['name']}: {wl.U} users x {wl.n_items} items, one global set range-split by k^3; "
                        "batched per-user Laplacian + eigensolve fused with the local_calc_precomp predictor",
            "users_global": wl.U,
            "users_per_gpu": wl.U // max(world, 1),
            "items": wl.n_items,
            "seed": wl.seed,
            "k_mean": float(kf_all.mean()),
            "k_range": [int(wl.k_all.min()), int(wl.k_all.max())],
            "predictions": n_pred_total,
            "parallelism": f"user range split x{world} (cost_split on sum k^3)" + (
                f", ranks on devices {devices}" if devices else ""),
            "graph": gstats,
            "eigen_method": args.eigen_method,
        },
        "predicted_ratings_per_s": n_pred_total / step_s,
        "stages": {
            "eigen_ms": eig_s * 1e3,
            "predict_ms": pred_s * 1e3,
            "gather_ms": gat_s * 1e3 if world > 1 else 0.0,
            "eigen_users_per_s": wl.n_users / eig_s,
            "predict_ratings_per_s": n_pred_local / pred_s,
            "rank0_users": wl.n_users,
            "fused": overlap,
            "note": "per-stage times are rank 0's (HIP events, median over the timed steps); with --fused on "
                    "eigen_ms is the eigen span of the overlapped step and predict_ms the predictor alone "
                    "(see fused); with --fused off eigen_ms includes the record pack",
        },
        "roofline": roof_pred if dominant_is_pred else roof_eigen,
        "roofline_other": roof_eigen if dominant_is_pred else roof_pred,
        "setup_s": setup_s,
        "m_mean": float(m_h.mean()),
        "kk_mean": float(kk_h.mean()),
        "nan_predictions": int(np.isnan(mse_h).sum()),
        "nc_gt_62_frac": float(np.mean((np.repeat(wl.k, wl.k) - kk_h) > 62)),
        "rank_deficient_predictions": {
            "rows": pred_acc["rank_deficient_rows"], "frac": pred_acc["rank_deficient_frac"],
            "c0_rows": pred_acc["c0_rows"],
            "clamp_bounds": at_bound_stats(wl.off, wl.k, m_h, kk_h, evals_h, sigs_h, wl.ratings, mse_h),
            "note": "rank 0's rows with 0 < c < lim (U_CS^T U_CS singular): the reference's explicit inverse "
                    "returns rounding noise clamped to [1, 5] there, this kernel the minimum-norm least-squares "
                    "prediction (tests pin every fast-path row to numpy's min-norm solution and count the "
                    "block-wide ones); clamp_bounds: the share of them at pred 1 or 5 (cpu_baseline.clamp_bounds "
                    "has the oracle's share on its sample)"},
    }

    # ---- HBM traffic (rank 0, N=1): two rocprofv3 --pmc passes over one child step ------
    if solo and args.pmc == "auto":
        phase("PMC traffic passes (rocprofv3 children)")
        tr = pmc_traffic(args)
        if tr is not None:
            dom = roof_eigen.get("dominant")
            if dom and dom.get("emax", 12) == 12 and "12" in (dom.get("kernel") or ""):
                f12, w12 = tr["eigen12"]
                dom["traffic"] = 2.0 * f12 + w12
                dom["traffic_note"] = f"2 x FETCH_SIZE + WRITE_SIZE of the one {dom['kernel']} launch of a child step"
                if "stage" in roof_eigen:   # the top level is the dominant kernel's: its own traffic
                    roof_eigen["traffic"] = dom["traffic"]
                    roof_eigen["traffic_note"] = dom["traffic_note"] + " (MI355X_MICROARCH.md's gfx950 correction)"
            if "predict_by_kernel" in tr:
                roof_pred["traffic_by_kernel"] = {kname: {"fetch_raw": f, "write": w_, "traffic": 2.0 * f + w_}
                                                  for kname, (f, w_) in tr["predict_by_kernel"].items()}
            for key, roof in (("predict", roof_pred), ("eigen", roof_eigen.get("stage", roof_eigen))):
                fetch, write = tr[key]
                roof["traffic"] = 2.0 * fetch + write
                roof["traffic_fetch_bytes_raw"] = fetch
                roof["traffic_write_bytes"] = write
                roof["traffic_note"] = ("HBM bytes per stage pass from rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE "
                                        "(separate passes over one child step of the same workload); "
                                        "traffic = 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of "
                                        "MI355X_MICROARCH.md (calibrated for 16 B/lane streaming reads; these "
                                        "kernels' narrower gathers are uncalibrated); Infinity-Cache hits count")
                stage_s = pred_s if key == "predict" else eig_s
                roof["traffic_GBps"] = roof["traffic"] / stage_s / 1e9
        else:
            result["pmc"] = "unavailable (rocprofv3 missing or the collector failed)"

    # ---- CPU baseline (rank 0, N=1): the oracle in precompute_local_threads form ---------
    if want_cpu:
        phase("CPU baseline sample")
        result["cpu_baseline"] = cpu_baseline(args, wl, W_host,
                                              dev={"m": m_h, "kk": kk_h, "evals": evals_h, "sigs": sigs_h,
                                                   "mse": mse_h} if world == 1 else None, ctx=ctx)
    del W_host

    # ---- secondary legs (rank 0, N=1; not part of `value`) -----------------------------
    if solo and args.io == "auto" and args.config == "c4":
        phase("C4 out_eigen_ I/O leg")
        # the C4-size out_eigen_ round trip: binary form of all 1M records,
        # text form of the first 100k (the full text file would be ~128 GB)
        try:
            result["config4_eigen_io"] = text_phases(wl, text_users=args.io_text_users, label="C4 record set")
        except OSError as exc:
            result["config4_eigen_io"] = f"skipped: {exc}"
    if solo and args.c2 == "auto" and args.config != "c2":
        wl.plan.close()
        del wl
        torch.cuda.empty_cache()
        phase("C2 leg (steps, out_eigen_ text, local_calc --pct 1)")
        result["config2"] = c2_leg(args, ctx, dev_index, dev, torch)
    if solo and args.knn2 == "auto":
        torch.cuda.empty_cache()
        phase("C3 knn2 leg")
        result["knn2"] = knn2_leg(args, ctx, dev, torch)
    if solo and args.prep == "auto":
        torch.cuda.empty_cache()
        phase("data-prep leg")
        result["prep"] = prep_leg(args, ctx, dev, torch)
    if solo and args.c5 == "auto":
        phase("C5 leg")
        torch.cuda.empty_cache()
        W, _, _ = train_graph(Context, dev_index, dev, torch, CONFIGS["c4"]["seed"], CONFIGS["c4"]["train_users"],
                              CONFIGS["c4"]["items"])
        result["config5"] = c5_leg(args, ctx, dev, torch, W.view(CONFIGS["c4"]["items"], -1))
        del W

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def eigen_roofline(k, m_h, eig_s, jstats, bucket_ms=None, bucket_alone_ms=None, sw_ms=None, sw_alone_ms=None):
    kf = k.astype(np.float64)
    flops = float(np.sum(9.0 * kf ** 3 + 4.0 * kf ** 2))
    # algorithmic bytes: item ids in, W_u entries (index+weight), sigs/evals/evecs out
    byt = float(np.sum(4 * kf) + 8 * np.sum(kf * kf) + np.sum(4 * (2 * kf + m_h + kf * m_h)))
    achieved = flops / eig_s / 1e12
    exe = float(np.sum(6.0 * kf ** 3)) * jstats["sweeps_mean"]
    return {
        "bound": "valu",
        "roof_note": "fp32 vector roof 157.3 TF/s (the Jacobi kernel is VALU + LDS, no MFMA); algorithmic flops = "
                     "9k^3 + 4k^2 per user (Golub-Van Loan symmetric QR with vectors, SURVEY 8d)",
        "kernel": "eigen_kernel<EMAX> (all k-bucket launches of one eigen stage, + the record pack)",
        "achieved": achieved,
        "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": achieved / FP32_PEAK_TFLOPS,
        "traffic": None,
        "algorithmic_flops_per_stage": flops,
        "algorithmic_bytes_per_stage": byt,
        "algorithmic_GBps": byt / eig_s / 1e9,
        # one-sided Jacobi executes ~3k^3 FMA (6k^3 flops) per sweep: a dot and a two-column
        # rotation per pair; sweeps from cf_debug_stats, mean over users
        "sweeps_mean": jstats["sweeps_mean"],
        "executed_flops_per_stage": exe,
        "executed_TFLOPs": exe / eig_s / 1e12,
        "executed_frac": exe / eig_s / 1e12 / FP32_PEAK_TFLOPS,
        **({"dominant": eigen_dominant(k, bucket_ms, bucket_alone_ms, sw_ms, sw_alone_ms)} if bucket_ms is not None else {}),
    }


def eigen_dominant(k, bucket_ms, bucket_alone_ms=None, sw_ms=None, sw_alone_ms=None):
    """The dominant launch of the eigen stage (bucket 12: 176 < k <= 192, one per step) and every
    other LDS bucket: algorithmic flops per launch (9k^3 + 4k^2 per user) over the
    launch's duration from cf_eigen_bucket_timing_split (HIP events on the aux stream it runs on, mean
    over the timed steps; it co-runs with the other buckets on the second stream, as in a rocprofv3
    kernel trace of the step).  A bucket in the split layout is two kernels back to
    back, split_sweep_kernel<e> (gather, assembly, sweeps) and eigen_kernel<e, .., RESUME>
    (refinement, epilogue): the launch is the pair, its flops the whole eigensolve, and the sweep
    kernel's own share is reported beside it (sweeps_ms)."""
    kf = k.astype(np.float64)
    emax = np.ceil(kf / 16.0).astype(np.int64)
    rows = []
    for e in range(1, 13):
        sel = (emax == e) & (kf <= 192)
        ms = float(bucket_ms[e])
        if not sel.any() or ms <= 0:
            continue
        fl = float(np.sum(9.0 * kf[sel] ** 3 + 4.0 * kf[sel] ** 2))
        row = {"emax": e, "users": int(sel.sum()), "flops_per_launch": fl, "ms_per_launch": ms,
               "achieved_TFLOPs": fl / ms / 1e9, "frac": fl / ms / 1e9 / FP32_PEAK_TFLOPS}
        if sw_ms is not None and float(sw_ms[e]) > 0:
            row["sweeps_ms"] = float(sw_ms[e])
        rows.append(row)
    dom = max(rows, key=lambda r: r["ms_per_launch"]) if rows else None

    def name(r):
        base = "eigen_kernel<12, true>" if r["emax"] == 12 else f"eigen_kernel<{r['emax']}>"
        if "sweeps_ms" in r:
            return f"split_sweep_kernel<{r['emax']}> + " + base[:-1] + ", RESUME>"
        return base
    out = {"kernel": name(dom) if dom else None,
           "unit": "TFLOP/s", "peak": FP32_PEAK_TFLOPS, "buckets": rows,
           "note": "per-launch algorithmic flops / the launch's HIP-event duration in the timed steps "
                   "(mean); the stage-level achieved/frac above divides the whole stage's flops by the "
                   "stage span (all buckets + the record pack, two streams)"}
    if dom:
        out.update({"users": dom["users"], "flops_per_launch": dom["flops_per_launch"],
                    "ms_per_launch": dom["ms_per_launch"], "achieved": dom["achieved_TFLOPs"],
                    "frac": dom["frac"]})
        if "sweeps_ms" in dom:
            out["sweeps_ms"] = dom["sweeps_ms"]
        if bucket_alone_ms is not None and float(bucket_alone_ms[dom["emax"]]) > 0:
            ms_a = float(bucket_alone_ms[dom["emax"]])
            out.update({"alone_ms": ms_a, "alone_frac": dom["flops_per_launch"] / ms_a / 1e9 / FP32_PEAK_TFLOPS,
                        "alone_note": "the same launch alone on the GPU (one stream, the untimed sweep-count "
                                      "pass); a rocprofv3 average over a run's launches mixes this one with the "
                                      "co-running in-step ones"})
            if sw_alone_ms is not None and float(sw_alone_ms[dom["emax"]]) > 0:
                out["alone_sweeps_ms"] = float(sw_alone_ms[dom["emax"]])
    return out


def predict_roofline(acc, pred_s):
    tf = acc["algorithmic_flops"] / pred_s / 1e12
    exe = acc["executed_flops"] / pred_s / 1e12
    return {
        "bound": "valu",
        "roof_note": "fp64 roof 78.6 TF/s (VALU = MFMA dense fp64 peak).  algorithmic = a LOWER BOUND of the "
                     "algorithm these kernels run (DESIGN 3.2): per user the Gram U^T U (k Lu^2, symmetric) and "
                     "one k x k Gram of the basis X (k^3); per rating the Gram of its min(nc, d)-row system "
                     "(ns^2 max(nc, d)) and its LDL^T (ns^3/3).  ref_* fields give SURVEY 8d's count of "
                     "the reference's explicit-inverse work per pair for comparison",
        "kernel": "pred_basis_kernel<float> + pred_rating_kernel<float> (all chunk launches of one predict stage)",
        "achieved": tf,
        "peak": FP64_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": tf / FP64_PEAK_TFLOPS,
        "traffic": None,
        "algorithmic_flops_per_stage": acc["algorithmic_flops"],
        "executed_flops_per_stage": acc["executed_flops"],
        "executed_TFLOPs": exe,
        "executed_frac": exe / FP64_PEAK_TFLOPS,
        "ref_flops_per_stage": acc["ref_flops"],
        "ref_equivalent_TFLOPs": acc["ref_flops"] / pred_s / 1e12,
        "algorithmic_bytes_per_stage": acc["algorithmic_bytes"],
        "algorithmic_GBps": acc["algorithmic_bytes"] / pred_s / 1e9,
        "lim_mean": acc["lim_mean"],
    }


def c2_leg(args, ctx, dev_index, dev, torch):
    """BASELINE config 2 (100k users x 10k items, graph = knn2 over 400k train users) through
    the same step, plus the out_eigen_ text phases (compute and text-write timed
    separately): the parallel %g writer (cfh_write_eigen) and the parallel parser
    (cfh_load_eigen, load_precomputed_data) on the whole C2 record set, on the host's threads."""
    from collaborative_filtering_amd.api import Context

    cfg = CONFIGS["c2"]
    a = argparse.Namespace(**vars(args))
    a.users = cfg["users"]
    d_W, _, gstats = train_graph(Context, dev_index, dev, torch, cfg["seed"], cfg["train_users"], cfg["items"])
    wl = Workload(a, cfg, 0, 1, dev, torch, ctx, d_W.view(cfg["items"], cfg["items"]))
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    for _ in range(2):
        wl.eigen(sp)
        wl.pack(sp)
        wl.predict(sp)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 5
    eig, pred = [], []
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        e[0].record(stream)
        wl.eigen(sp)
        wl.pack(sp)
        e[1].record(stream)
        wl.predict(sp)
        e[2].record(stream)
        e[2].synchronize()
        eig.append(e[0].elapsed_time(e[1]))
        pred.append(e[1].elapsed_time(e[2]))
    step_s = (time.perf_counter() - t0) / reps
    out = {"workload": f"{cfg['name']}: {wl.U} users x {wl.n_items} items, seed {wl.seed}", "graph": gstats,
           "users_per_s": wl.U / step_s, "ms_per_step": step_s * 1e3, "predicted_ratings_per_s": wl.n_entries / step_s,
           "eigen_ms": float(np.median(eig)), "predict_ms": float(np.median(pred)),
           "eigen_users_per_s": wl.U / float(np.median(eig)) * 1e3,
           "predict_ratings_per_s": wl.n_entries / float(np.median(pred)) * 1e3,
           "nc_gt_62_frac": float(np.mean((np.repeat(wl.k, wl.k) - wl.d_kk.cpu().numpy()[:wl.n_entries]) > 62))}
    # ---- out_eigen_ text phases (host) -----------------------------------------------
    try:
        out["text_io"] = text_phases(wl)
    except OSError as exc:
        out["text_io"] = f"skipped: {exc}"
    # ---- local_calc (a8) on the same graph: `local_calc --pct 1` ------------------------
    try:
        out["local_calc"] = local_calc_leg(ctx, wl, d_W.view(cfg["items"], cfg["items"]), pct=1,
                                           cpu_seconds=0.0 if args.no_cpu_baseline else 40.0)
    except Exception as exc:   # reported, never fatal for the headline
        out["local_calc"] = f"failed: {exc}"
    del d_W
    wl.plan.close()
    return out


def local_calc_leg(ctx, wl, W, pct=1, seed=2026, nmax=None, cpu_seconds=40.0):
    """local_calc's engine 2 (local_calc.cpp:262-526, cf_local_calc) as `bin/local_calc --pct P`
    runs it: movies sampled with probability P %, each movie's unit = [m, out-neighbours with
    w > 0.1] of the resident knn2 graph, test ratings = the config's user ratings grouped by
    movie (users ascending).  Host-pointer call (PCIe included)."""
    n_items = wl.n_items
    rng = np.random.default_rng(seed)
    movies = np.nonzero(rng.random(n_items) * 100.0 < pct)[0]
    # test ratings CSR over movies, users ascending
    uid = np.repeat(np.arange(wl.n_users, dtype=np.int64), wl.k)
    mv = wl.items[:wl.n_entries].astype(np.int64)
    order = np.lexsort((uid, mv))
    toff = np.zeros(n_items + 1, np.uint64)
    np.add.at(toff, mv + 1, 1)
    toff = np.cumsum(toff).astype(np.uint64)
    tuser = uid[order].astype(np.uint32)
    trat = wl.ratings[:wl.n_entries][order].astype(np.float32)
    # units of the sampled movies that have test ratings (the rest write no rows, :269-272)
    moff, mitems, ns, over = [0], [], [], []
    for m in movies:
        if toff[m + 1] == toff[m]:
            continue
        row = W[int(m)].cpu().numpy()
        nb = np.nonzero(row.astype(np.float64) > 0.1)[0]
        nb = nb[nb != m]
        if nmax is not None and 1 + len(nb) > nmax:   # an optional cap (none by default): left out, counted
            over.append(1 + len(nb))
            continue
        mitems.append(np.concatenate([[m], nb]).astype(np.uint32))
        moff.append(moff[-1] + 1 + len(nb))
        ns.append(1 + len(nb))
    ns = np.array(ns)
    moff = np.array(moff, np.uint64)
    mitems = np.concatenate(mitems) if mitems else np.zeros(0, np.uint32)
    t = time.perf_counter()
    mse, kk, pred, wlim, lim = ctx.local_calc(moff, mitems, toff, tuser, trat)
    dt = time.perf_counter() - t
    pairs = int(np.sum(kk >= 0))
    sel = kk > 0
    cpu = None
    if cpu_seconds > 0 and len(ns):
        try:
            cpu = local_calc_cpu_baseline(ctx, W, moff, mitems, ns, toff, tuser, trat, cpu_seconds)
        except Exception as exc:   # reported, never fatal
            cpu = f"failed: {exc}"
    return {"movies_sampled": int(len(movies)), "units": int(len(ns)),
            "unit_n": {"mean": float(ns.mean()) if len(ns) else 0.0, "max": int(ns.max()) if len(ns) else 0,
                       "gt_192": int(np.sum(ns > 192)), "gt_5000": int(np.sum(ns > 5000))},
            "units_over_cap": {"count": len(over), "n_min": int(min(over)) if over else 0,
                               "n_max": int(max(over)) if over else 0,
                               "note": "no cap: every sampled unit is in the call" if nmax is None else
                               f"units with n > {nmax} left out of the call"},
            "predictions": pairs, "seconds": dt, "predictions_per_s": pairs / dt if dt > 0 else 0.0,
            "rank_deficient_frac": float(np.mean(kk[sel] < lim[sel])) if sel.any() else 0.0,
            "cpu_baseline": cpu,
            "note": f"bin/local_calc --pct {pct} on this config's knn2 graph: {len(ns)} movie units, every (movie, "
                    "test user) pair of them; host-pointer cf_local_calc (PCIe included)"}


def local_calc_cpu_baseline(ctx, W, moff, mitems, ns, toff, tuser, trat, budget_s):
    """The oracle's local_calc (cfo_local_calc: fp64 tridiagonal QL for es(ll2) once per movie,
    then per pair L2_h L2_h^T and its eigensolve, local_calc.cpp:262-526) beside the device on
    the same bounded sample, one host thread per movie as GraphLab's engine schedules vertex
    programs.  The C2 graph's units are large (n p50 ~4.7k: one fp64 eigensolve of the smallest
    sampled unit alone is ~90 s on a core), so the sample is the `threads` smallest sampled
    units truncated to their first n_fit items ([movie, its first out-neighbours]), n_fit sized
    by the cost model (5.8e-9 n^3 s per movie + 3.5e-9 n^3 s per pair, fp64 on one core) for at
    least 8 pairs per movie in the budget; the device runs the same truncated units (all their
    pairs) in its own call, and the oracle's kk and w_lim are checked against that call."""
    import concurrent.futures as cf

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as orc

    threads, _ = host_threads()
    n_fit = int((budget_s / (5.8e-9 + 8 * 3.5e-9)) ** (1.0 / 3.0))
    order = np.argsort(ns)[:threads]
    Wh = W.cpu().numpy()
    toff = np.asarray(toff, dtype=np.uint64)
    # the truncated units, and the device on them
    t_moff, t_items, t_ns = [0], [], []
    for v in order:
        n = min(int(ns[v]), n_fit)
        b = int(moff[v])
        t_items.append(np.asarray(mitems[b:b + n], dtype=np.uint32))
        t_moff.append(t_moff[-1] + n)
        t_ns.append(n)
    t_moff = np.array(t_moff, np.uint64)
    t_items = np.concatenate(t_items)
    ctx.local_calc(t_moff, t_items, toff, tuser, trat)   # warm-up (plans, workspaces)
    t = time.perf_counter()
    _, kk_g, _, wlim_g, _ = ctx.local_calc(t_moff, t_items, toff, tuser, trat)
    dt_gpu = time.perf_counter() - t
    gpu_pairs = int(np.sum(kk_g >= 0))
    jobs = []
    for i in range(len(t_ns)):
        n = t_ns[i]
        t_movie, t_pair = 5.8e-9 * n ** 3, 3.5e-9 * n ** 3
        npairs = int((budget_s - t_movie) // t_pair)
        if npairs < 1:
            continue
        b, e = int(t_moff[i]), int(t_moff[i + 1])
        m = int(t_items[b])
        nbrs = [int(x) for x in t_items[b + 1:e]]
        t0, t1 = int(toff[m]), int(toff[m + 1])
        users = tuser[t0:t1][:npairs]
        jobs.append((i, m, nbrs, t0, users))
    if not jobs:
        return {"skipped": f"no truncated unit fits the {budget_s:.0f} s budget"}
    test = {}
    for it in set([j[1] for j in jobs] + [x for j in jobs for x in j[2]]):
        us, rs = tuser[int(toff[it]):int(toff[it + 1])], trat[int(toff[it]):int(toff[it + 1])]
        test[it] = dict(zip(us.tolist(), rs.tolist()))

    def one(job):
        v, m, nbrs, t0, users = job
        Wl = orc.local_graph(m, nbrs, Wh)
        sub = {m: {u: test[m][u] for u in users.tolist()}}
        for it in nbrs:
            sub[it] = test.get(it, {})
        _, R = orc.local_ratings(m, nbrs, sub)
        return v, t0, orc.local_calc(Wl, R)

    t = time.perf_counter()
    with cf.ThreadPoolExecutor(len(jobs)) as ex:
        res = list(ex.map(one, jobs))
    dt = time.perf_counter() - t
    n_pred = sum(len(j[4]) for j in jobs)
    kk_eq, wl_err = 0, 0.0
    for v, t0, (mse_o, kk_o, pred_o, wl_o, lim_o) in res:
        for i in range(len(kk_o)):
            kk_eq += int(kk_g[t0 + i] == kk_o[i])
            if kk_o[i] > 0:
                wl_err = max(wl_err, abs(float(wlim_g[t0 + i]) - wl_o[i]) / max(1e-3, wl_o[i]))
    return {"value": n_pred / dt, "unit": "predictions/s", "cores": len(jobs), "kind": "port",
            "sample": f"{len(jobs)} smallest sampled units truncated to n = {sorted(set(t_ns))} items ([movie, first "
                      f"out-neighbours]), {n_pred} (movie, test user) pairs, oracle cfo_local_calc, one thread per movie",
            "seconds": dt, "device_same_units": {"predictions": gpu_pairs, "seconds": dt_gpu,
                                                  "predictions_per_s": gpu_pairs / dt_gpu if dt_gpu > 0 else 0.0},
            "kk_equal_device": f"{kk_eq}/{n_pred}", "wlim_max_rel_diff_device": wl_err}


def text_phases(wl, text_users=None, label="whole C2 record set"):
    """out_eigen_ write + parse phases on the host (compute and text-write timed
    separately): the text form (cfh_write_eigen = bin/precompute_local's %g writer) on the first
    `text_users` records (all when None) and the binary form on all of them; cfh_load_eigen =
    load_precomputed_data of bin/local_calc_precomp.  Download from HBM excluded."""
    import ctypes
    import shutil

    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd._native import ptr

    L = synth.host_lib()
    L.cfh_write_eigen.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32] + \
        [ctypes.c_void_p] * 8
    L.cfh_write_eigen.restype = ctypes.c_int
    L.cfh_load_eigen.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]
    L.cfh_load_eigen.restype = ctypes.c_int64
    threads, _ = host_threads()
    m = wl.d_m.cpu().numpy()[:wl.n_users]
    sigs = wl.d_sigs.cpu().numpy()
    evals = wl.d_evals.cpu().numpy()
    poff = wl.d_poff.cpu().numpy().astype(np.uint64)
    packed = wl.d_packed.cpu().numpy()
    uid = np.arange(wl.n_users, dtype=np.uint32)
    tmpdir = os.environ.get("CF_BENCH_TMP", "/tmp")
    path = os.path.join(tmpdir, f"cf_bench_out_eigen_{os.getpid()}").encode()
    res = {"threads": threads, "dir": tmpdir}
    try:
        n_text = wl.n_users if text_users is None else min(wl.n_users, int(text_users))
        passes = [("text", 0, n_text), ("binary", 1, wl.n_users)]
        if n_text < wl.n_users:   # the binary form on the text sample too: bytes/s on the same records
            passes.append(("binary_text_sample", 1, n_text))
        for fmt, binary, n_rec in passes:
            k = np.diff(wl.off[:n_rec + 1].astype(np.int64))
            mm = m[:n_rec].astype(np.int64)
            rec_est = (12 + 8 * k + 4 * mm + 4 * k * mm) * (3 if not binary else 1)
            est = int(np.sum(rec_est))
            free = shutil.disk_usage(tmpdir).free
            if est > 0.8 * free and not binary and n_rec == wl.n_users:
                # the whole text form does not fit the disk: write and parse it in consecutive
                # record ranges (each a complete out_eigen_ file of its users, deleted after its
                # parse), so every record still goes through the text writer and parser
                cum = np.cumsum(rec_est)
                cuts, start = [0], 0
                while start < n_rec:
                    end = int(np.searchsorted(cum, (cum[start - 1] if start else 0) + 0.6 * free, side="right"))
                    end = max(end, start + 1)
                    cuts.append(min(end, n_rec))
                    start = cuts[-1]
                w_s = r_s = 0.0
                size = 0
                ok = True
                for r0, r1 in zip(cuts[:-1], cuts[1:]):
                    t = time.perf_counter()
                    rc = L.cfh_write_eigen(path, 0, threads, 0, r1 - r0, ptr(uid[r0:]), ptr(wl.off[r0:]), ptr(m[r0:]),
                                           ptr(wl.items), ptr(sigs), ptr(evals), ptr(poff[r0:]), ptr(packed))
                    w_s += time.perf_counter() - t
                    size += os.path.getsize(path.decode())
                    t = time.perf_counter()
                    n = L.cfh_load_eigen(path, threads, None, 0)
                    r_s += time.perf_counter() - t
                    ok = ok and rc == 0 and n == r1 - r0
                    os.remove(path.decode())
                res[fmt] = {"records": n_rec, "files": len(cuts) - 1, "write_s": w_s, "parse_s": r_s, "bytes": size,
                            "write_GBps": size / w_s / 1e9, "parse_GBps": size / r_s / 1e9, "ok": bool(ok),
                            "note": f"{len(cuts) - 1} consecutive record ranges (the {est / 1e9:.0f} GB estimate exceeds "
                                    f"{free / 1e9:.0f} GB free in {tmpdir})"}
                continue
            if est > 0.8 * free:
                res[fmt] = f"skipped: ~{est / 1e9:.1f} GB would not fit the {free / 1e9:.1f} GB free in {tmpdir}"
                continue
            t = time.perf_counter()
            rc = L.cfh_write_eigen(path, 0, threads, binary, n_rec, ptr(uid), ptr(wl.off), ptr(m),
                                   ptr(wl.items), ptr(sigs), ptr(evals), ptr(poff), ptr(packed))
            w_s = time.perf_counter() - t
            size = os.path.getsize(path.decode())
            t = time.perf_counter()
            n = L.cfh_load_eigen(path, threads, None, 0)
            r_s = time.perf_counter() - t
            res[fmt] = {"records": n_rec, "write_s": w_s, "parse_s": r_s, "bytes": size,
                        "write_GBps": size / w_s / 1e9, "parse_GBps": size / r_s / 1e9,
                        "ok": bool(rc == 0 and n == n_rec)}
            os.remove(path.decode())
    finally:
        try:
            os.remove(path.decode())
        except OSError:
            pass
    res["note"] = (f"{label} (download excluded): cfh_write_eigen = the out_eigen_ writer of bin/precompute_local "
                   "(text: %g via to_chars, records formatted on `threads` threads; binary CFEIGEN1: fp32 blocks, "
                   "pieces pwrite()n in place), cfh_load_eigen = load_precomputed_data of bin/local_calc_precomp "
                   "(records parsed in parallel); file in `dir`")
    return res


def c5_leg(args, ctx, dev, torch, W):
    """BASELINE config 5, bounded sample: a power-law degree mix (lognormal k, median 100,
    p95 ~1.5k, clipped to [20, --c5-kmax = 5000]) through cf_eigen_run -- k <= 192 on the LDS
    Jacobi path, larger k on the fp64 spill path -- on the config-4 (50k-item) graph, then the
    predictor (cf_predict_run_f32, own sigs) over every rating of those users: k <= 192 on
    predict_kernel, larger k on the spill predictor.  Reports users/s and ratings/s of the
    mix and the per-path split (HIP events around each plan)."""
    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd._native import CF_MAX_K, CF_SPILL_MAX_K
    from collaborative_filtering_amd.api import CF_SIGS_OWN, evec_offsets

    seed = 2026101505
    n_items = int(W.shape[0])
    sigma = float(np.log(15.0) / 1.6449)            # p95 / median = 15
    k = synth.degrees(seed, args.c5_users, k_median=100.0, sigma=sigma, kmin=20,
                      kmax=min(args.c5_kmax, CF_SPILL_MAX_K))
    off, items, ratings = synth.user_items(seed, k, n_items, threads=16)
    ctx.upload_graph_dense(W)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {"workload": f"BASELINE config 5 sample: {args.c5_users} users, lognormal k (median 100, "
                       f"sigma {sigma:.3f}, p95 {int(np.percentile(k, 95))}, max {int(k.max())}), "
                       f"{n_items} items (config-4 knn2 graph), seed {seed}"}
    stream = torch.cuda.current_stream(dev)
    total_ms = total_pms = 0.0
    n_pred = 0
    groups = (("lds", k <= CF_MAX_K), ("spill", (k > CF_MAX_K) & (k <= 3072)), ("spill_big", k > 3072))
    for name, sel in groups:
        ks = k[sel]
        if len(ks) == 0:
            continue
        print(f"[c5] {name}: {len(ks)} users, k {int(ks.min())}..{int(ks.max())}", file=sys.stderr, flush=True)
        o = np.zeros(len(ks) + 1, dtype=np.uint64)
        o[1:] = np.cumsum(ks.astype(np.uint64))
        it = np.concatenate([items[int(off[u]):int(off[u + 1])] for u in np.nonzero(sel)[0]])
        rt = np.concatenate([ratings[int(off[u]):int(off[u + 1])] for u in np.nonzero(sel)[0]])
        eo, ne = evec_offsets(o)
        d_o, d_i, d_e = T(o.view(np.int64)), T(it.view(np.int32)), T(eo.view(np.int64))
        d_m = torch.zeros(len(ks), dtype=torch.int32, device=dev)
        d_s = torch.zeros(len(it), dtype=torch.float32, device=dev)
        d_v = torch.zeros(len(it), dtype=torch.float32, device=dev)
        d_x = torch.zeros(ne, dtype=torch.float32, device=dev)
        plan = ctx.plan(o)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        plan.eigen_run(d_o, d_i, d_e, d_m, d_s, d_v, d_x, stream=stream.cuda_stream)
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        total_ms += ms
        print(f"[c5] {name}: eigen {ms:.1f} ms", file=sys.stderr, flush=True)
        if int(ks.max()) > args.c5_predict_kmax:   # the per-rating systems grow as k^3
            kf = ks.astype(np.float64)
            out[name] = {"users": int(len(ks)), "k_mean": float(kf.mean()), "ms": ms, "users_per_s": len(ks) / ms * 1e3,
                         "GFLOPs_9k3": float(np.sum(9 * kf ** 3)) / ms / 1e6, "m_mean": float(d_m.float().mean().item()),
                         "predict": f"skipped (k > --c5-predict-kmax {args.c5_predict_kmax})"}
            plan.close()
            del d_x
            torch.cuda.empty_cache()
            continue
        d_mse = torch.zeros(len(it), dtype=torch.float32, device=dev)
        d_kk = torch.zeros(len(it), dtype=torch.int32, device=dev)
        p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p0.record(stream)
        plan.predict_run(d_o, d_i, T(rt), d_m, d_v, d_e, d_x, d_s, CF_SIGS_OWN, d_mse, d_kk,
                         stream=stream.cuda_stream)
        p1.record(stream)
        p1.synchronize()
        pms = p0.elapsed_time(p1)
        total_pms += pms
        n_pred += len(it)
        print(f"[c5] {name}: predict {pms:.1f} ms ({len(it)} ratings)", file=sys.stderr, flush=True)
        kf = ks.astype(np.float64)
        out[name] = {"users": int(len(ks)), "k_mean": float(kf.mean()), "ms": ms,
                     "users_per_s": len(ks) / ms * 1e3,
                     "GFLOPs_9k3": float(np.sum(9 * kf ** 3)) / ms / 1e6,
                     "m_mean": float(d_m.float().mean().item()),
                     "predict_ms": pms, "ratings": int(len(it)), "ratings_per_s": len(it) / pms * 1e3,
                     "kk_mean": float(d_kk.float().mean().item()),
                     "nan_predictions": int(torch.isnan(d_mse).sum().item())}
        plan.close()
        del d_x
        torch.cuda.empty_cache()
    # a larger sample of the same generator in ONE eigen call, as bin/precompute_local runs it:
    # the spill bucket's k ranges launch with slots sized per range, the k > 3072 range on its
    # own stream (staged multi-CU solver) beside the smaller ranges and the LDS buckets
    n1 = max(args.c5_onecall_users, 1)
    if n1 != args.c5_users:
        del off, items, ratings
        k = synth.degrees(seed + 1, n1, k_median=100.0, sigma=sigma, kmin=20, kmax=min(args.c5_kmax, CF_SPILL_MAX_K))
        off, items, _ = synth.user_items(seed + 1, k, n_items, threads=16)
    # the predictor legs' spill workspace would shrink the eigen call's (both sized from free HBM);
    # a drop-in precompute_local process has neither
    ctx.release_workspaces()
    print(f"[c5] all: one eigen call over {len(k)} users ({int(np.sum(k > CF_MAX_K))} spill, "
          f"{int(np.sum(k > 3072))} with k > 3072)", file=sys.stderr, flush=True)
    eo, ne = evec_offsets(off)
    d_o, d_i, d_e = T(off.view(np.int64)), T(items.view(np.int32)), T(eo.view(np.int64))
    d_m = torch.zeros(len(k), dtype=torch.int32, device=dev)
    d_s = torch.zeros(len(items), dtype=torch.float32, device=dev)
    d_v = torch.zeros(len(items), dtype=torch.float32, device=dev)
    d_x = torch.zeros(ne, dtype=torch.float32, device=dev)
    plan = ctx.plan(off)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    plan.eigen_run(d_o, d_i, d_e, d_m, d_s, d_v, d_x, stream=stream.cuda_stream)
    e1.record(stream)
    e1.synchronize()
    all_ms = e0.elapsed_time(e1)
    print(f"[c5] all: eigen {all_ms:.1f} ms", file=sys.stderr, flush=True)
    kf = k.astype(np.float64)
    out["one_call"] = {"users": int(len(k)), "seed": seed + 1 if n1 != args.c5_users else seed,
                       "spill_users": int(np.sum(k > CF_MAX_K)), "big_users": int(np.sum(k > 3072)),
                       "k_p95": int(np.percentile(k, 95)), "k_max": int(k.max()),
                       "eigen_ms": all_ms, "users_per_s": len(k) / all_ms * 1e3,
                       "GFLOPs_9k3": float(np.sum(9 * kf ** 3)) / all_ms / 1e6,
                       "m_mean": float(d_m.float().mean().item()),
                       "note": "every user in one cf_eigen_run (the drop-in precompute_local's batch); the "
                               "per-group legs above run each group of the smaller sample alone"}
    plan.close()
    del d_x
    torch.cuda.empty_cache()
    out["users_per_s"] = out["one_call"]["users_per_s"]
    out["users_per_s_note"] = "eigen stage, one_call sample"
    out["groups_users_per_s"] = args.c5_users / total_ms * 1e3
    out["ms"] = total_ms
    out["predict_ms"] = total_pms
    out["ratings_per_s"] = n_pred / total_pms * 1e3 if total_pms else None
    out["predicted_ratings"] = n_pred
    return out


def prep_leg(args, ctx, dev, torch):
    """SURVEY 8f item 3, data prep on the GPU: the knn regroup (cf_knn_regroup_run: per-movie
    train / test lists with last-read-wins, sorted unique co-rated lists) and the k-fold order
    (cf_fold_order_run, 5 folds) over the config-2 ratings (100k users x 10k items, ~10.7M
    ratings, 20% of each user's ratings in the validate role).  HBM-bound: SURVEY 8d's 24 B
    per rating (12 read + 12 written) plus 4 B per co-rated entry written.  Inputs resident,
    HIP events around each call; the CPU baseline is the oracle restatement on a sample."""
    from collaborative_filtering_amd import synth
    from collaborative_filtering_amd._native import ptr

    cfg = CONFIGS["c2"]
    seed, n_users, n_items = cfg["seed"], cfg["users"], cfg["items"]
    k = synth.degrees(seed, n_users, k_median=100.0, sigma=0.5, kmin=20, kmax=180)
    off, items, rats = synth.user_items(seed, k, n_items, threads=16)
    n = int(off[-1])
    user = np.repeat(np.arange(n_users, dtype=np.uint32), k.astype(np.int64))
    validate = (np.random.default_rng(seed).random(n) < 0.2).astype(np.uint8)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    reps = 1 if args.pmc_child else 3   # the PMC collector's child: one regroup, nothing else
    d_user, d_movie, d_rat, d_val = T(user.view(np.int32)), T(items.view(np.int32)), T(rats), T(validate)
    U32 = lambda m: torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    OFF = lambda: torch.empty(n_items + 1, dtype=torch.int64, device=dev)
    F32 = lambda m: torch.empty(max(m, 1), dtype=torch.float32, device=dev)
    tro, teo, eo = OFF(), OFF(), OFF()
    tru, teu, trr, ter = U32(n), U32(n), F32(n), F32(n)
    cap = n_items * (n_items - 1)
    edg = U32(cap)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    L = ctx.lib
    reg_ms, fold_ms = [], []
    rank = np.random.default_rng(5).permutation(n_users).astype(np.uint32)
    d_rank, d_order = T(rank.view(np.int32)), U32(n)
    for rep in range(reps):
        rc = L.cf_knn_regroup_run(ctx.h, n, n_users, n_items, ptr(d_user), ptr(d_movie), ptr(d_rat), ptr(d_val),
                                  ptr(tro), ptr(tru), ptr(trr), ptr(teo), ptr(teu), ptr(ter), ptr(eo), ptr(edg),
                                  cap, ctypes_void(sp))
        ctx._chk(rc, "cf_knn_regroup_run")
        reg_ms.append(ctx.prep_timing())
        if args.pmc_child:
            torch.cuda.synchronize(dev)
            return None
        rc = L.cf_fold_order_run(ctx.h, n, n_users, ptr(d_user), ptr(d_rank), ptr(d_order), ctypes_void(sp))
        ctx._chk(rc, "cf_fold_order_run")
        fold_ms.append(ctx.prep_timing())
    n_tr, n_te, n_edg = int(tro[-1].item()), int(teo[-1].item()), int(eo[-1].item())
    reg_s, fold_s = float(np.median(reg_ms[1:])) / 1e3, float(np.median(fold_ms[1:])) / 1e3
    byt = 24.0 * n + 4.0 * n_edg
    # full-size properties: every rating kept once (no duplicates in this set), the fold order
    # is a permutation grouped by rank
    order = d_order[:n].cpu().numpy().view(np.uint32)
    ok_fold = bool(np.array_equal(np.sort(order), np.arange(n, dtype=np.uint32)) and
                   np.all(np.diff(rank[user[order]].astype(np.int64)) >= 0))
    out = {
        "workload": f"config-2 ratings: {n_users} users x {n_items} items, {n} ratings (20% validate), seed {seed}",
        "regroup_ms": reg_s * 1e3, "fold_order_ms": fold_s * 1e3,
        "ratings_per_s": n / reg_s, "train": n_tr, "test": n_te, "corated_entries": n_edg,
        "kept_all": n_tr + n_te == n, "fold_order_grouped": ok_fold,
        "roofline": {"bound": "hbm", "kernel": "cf_knn_regroup_run (radix sorts, co-rated bitmap, row writes)",
                     "achieved": byt / reg_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": byt / reg_s / 1e9 / HBM_PEAK_GBS, "traffic": None,
                     "algorithmic_bytes": byt,
                     "note": "24 B per rating (SURVEY 8d: 12 read + 12 written) + 4 B per co-rated entry; the "
                             "two sorts and the bitmap are several passes over that"},
    }
    if args.pmc == "auto" and not args.pmc_child:
        tr = pmc_traffic(args, prep=True)
        if tr is not None:
            fetch, write = tr["prep"]
            out["roofline"].update({
                "traffic": 2.0 * fetch + write, "traffic_fetch_bytes_raw": fetch, "traffic_write_bytes": write,
                "traffic_note": "HBM bytes of every kernel of ONE cf_knn_regroup_run in a child call (the "
                                "regroup kernels and rocprim's radix sorts and scans), rocprofv3 --pmc FETCH_SIZE "
                                "and WRITE_SIZE in separate passes; traffic = 2 x FETCH_SIZE + WRITE_SIZE"})
    if not args.no_cpu_baseline:
        # the oracle's C++ restatement with the reference's containers (a std::map per movie and
        # role, sorted unique co-rated lists) on every host thread, over the WHOLE rating set, so
        # its entry counts must equal the GPU's
        import ctypes

        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "libcf_oracle.so"))
        lib.cfo_knn_regroup_mt.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
        threads, _ = host_threads()
        cnt = np.zeros(3, np.uint64)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        t = time.perf_counter()
        lib.cfo_knn_regroup_mt(n, P(user), P(items), P(rats), P(validate), n_items, n_users, threads, P(cnt))
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": n / dt, "unit": "ratings/s", "cores": threads, "kind": "port",
                               "sample": f"all {n} ratings, oracle cfo_knn_regroup_mt (C++: std::map per movie and "
                                         f"role, last assignment wins; sorted unique co-rated lists), {threads} threads",
                               "seconds": dt,
                               "counts_equal_gpu": bool(int(cnt[0]) == n_tr and int(cnt[1]) == n_te and
                                                        int(cnt[2]) == n_edg)}
    return out


def ctypes_void(p):
    import ctypes

    return ctypes.c_void_p(p or 0)


def knn2_workload_call(args, ctx, dev, torch):
    """The knn2 leg's workload and one cf_item_cosine_run on it (the PMC child's pass)."""
    from collaborative_filtering_amd import synth

    seed = 2026101503
    n_items, n_users = args.knn2_items, args.knn2_users
    kd = synth.degrees(seed, n_users, k_median=89.0, sigma=0.5, kmin=20, kmax=2000)
    off, items, rats = synth.user_items(seed, kd, n_items, threads=16)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_off, d_items, d_rat = T(off.view(np.int64)), T(items.view(np.int32)), T(rats)
    d_W = torch.empty(n_items * n_items, dtype=torch.float32, device=dev)
    ctx.item_cosine_run(n_users, n_items, d_off, d_items, d_rat, 1, d_W,
                        stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)


def knn2_leg(args, ctx, dev, torch):
    """BASELINE config 3: knn2 weights_calc (knn2.cpp:127-164) over I items x U train users,
    integer ratings 1..5, on the int8 MFMA path; the dense item-weight matrix stays in HBM.
    Timed with HIP events on the launch stream: the whole call (rating scan, plane build,
    similarity kernel) and, from cf_knn2_timing, the similarity kernel alone.  Parity at
    full size: rows sampled for the CPU baseline are compared bit-exactly with the oracle."""
    from collaborative_filtering_amd import synth

    seed = 2026101503
    n_items, n_users = args.knn2_items, args.knn2_users
    kd = synth.degrees(seed, n_users, k_median=89.0, sigma=0.5, kmin=20, kmax=2000)   # mean ~100
    off, items, rats = synth.user_items(seed, kd, n_items, threads=16)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_off, d_items, d_rat = T(off.view(np.int64)), T(items.view(np.int32)), T(rats)
    d_W = torch.empty(n_items * n_items, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    call_ms, plane_ms, gemm_ms = [], [], []
    path = 0
    for rep in range(1 + args.knn2_reps):
        e0.record(stream)
        ctx.item_cosine_run(n_users, n_items, d_off, d_items, d_rat, 1, d_W, stream=sp)
        e1.record(stream)
        e1.synchronize()
        pm, gm, path = ctx.knn2_timing()
        if rep:
            call_ms.append(e0.elapsed_time(e1))
            plane_ms.append(pm)
            gemm_ms.append(gm)
    call_s, gemm_s = float(np.median(call_ms)) / 1e3, float(np.median(gemm_ms)) / 1e3
    I, U = float(n_items), float(n_users)
    ops = 2.0 * 4.0 * U * I * (I + 1) / 2                      # 4 products, MAC = 2 ops, upper triangle
    nt = -(-n_items // 128)
    ldu = -(-n_users // 128) * 128
    ops_exec = 2.0 * 4.0 * ldu * (nt * (nt + 1) / 2) * 128.0 * 128.0
    bytes_alg = float(n_items) * ldu + 4.0 * I * I              # code plane read once + weights written
    W_s = d_W.view(n_items, n_items)
    sym = bool(torch.equal(W_s, W_s.t()))
    nnz = int((W_s > 0).sum().item())
    # K-chunk streaming: the same launch in 4 user chunks with the int32 tile
    # partials carried in HBM; the weights must be the same bits
    chunk = -(-n_users // 4 // 128) * 128
    d_W2 = torch.empty_like(d_W)
    ctx.set_knn2_chunk(chunk)
    try:
        e0.record(stream)
        ctx.item_cosine_run(n_users, n_items, d_off, d_items, d_rat, 1, d_W2, stream=sp)
        e1.record(stream)
        e1.synchronize()
        chunked = {"users_per_chunk": chunk, "chunks": ctx.knn2_chunks(), "call_ms": e0.elapsed_time(e1),
                   "bit_identical": bool(torch.equal(d_W, d_W2))}
    finally:
        ctx.set_knn2_chunk(0)
    del d_W2
    acc, exact = ctx.knn2_exactness()
    out = {
        "workload": f"BASELINE config 3: knn2 item cosine, {n_items} items x {n_users} train users, "
                    f"mean deg {float(kd.mean()):.1f}, integer ratings 1..5 (Zipf(1) items, seed {seed})",
        "path": {1: "int8 MFMA, one code plane", 2: "int8 MFMA, three planes", 3: "fp32 MFMA"}.get(path, path),
        "call_ms": call_s * 1e3,
        "plane_build_ms": float(np.median(plane_ms)),
        "kernel_ms": gemm_s * 1e3,
        "item_pairs_per_s": I * (I - 1) / 2 / call_s,
        "useful_pair_updates": float(np.sum(kd.astype(np.float64) ** 2)),
        "edges_w_gt_0.01": nnz,
        "symmetric": sym,
        "k_chunked": chunked,
        "max_float_accumulator": acc,
        "reference_floats_exact": exact,
        "roofline": {
            "bound": "mfma",
            "kernel": "knn2_code_kernel (v_mfma_i32_32x32x32_i8)",
            "achieved": ops / gemm_s / 1e12,
            "peak": INT8_PEAK_TOPS,
            "unit": "TOPS",
            "frac": ops / gemm_s / 1e12 / INT8_PEAK_TOPS,
            "traffic": None,
            "algorithmic_ops": ops,
            "executed_ops": ops_exec,
            "executed_frac": ops_exec / gemm_s / 1e12 / INT8_PEAK_TOPS,
            "algorithmic_bytes": bytes_alg,
            "algorithmic_GBps": bytes_alg / gemm_s / 1e9,
            "note": "ops = 2 x 4 products x U x I(I+1)/2 (SURVEY 8d: num=R^T R, den1=S^T B, den2=B^T S, "
                    "cnt=B^T B on the upper triangle); executed counts the 128-item tile and 128-user padding",
        },
    }
    if args.pmc == "auto" and not args.pmc_child:
        tr = pmc_traffic(args, knn2=True)
        if tr is not None:
            fetch, write = tr["knn2"]
            out["roofline"].update({
                "traffic": 2.0 * fetch + write, "traffic_fetch_bytes_raw": fetch, "traffic_write_bytes": write,
                "traffic_note": "HBM bytes of the one knn2_code_kernel launch of a child call, rocprofv3 --pmc "
                                "FETCH_SIZE and WRITE_SIZE in separate passes; traffic = 2 x FETCH_SIZE + "
                                "WRITE_SIZE (MI355X_MICROARCH.md's gfx950 correction)"})
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref as orc

        threads, _ = host_threads()
        rng = np.random.default_rng(3)
        cal = rng.choice(n_items, size=2, replace=False).astype(np.int32)
        t = time.perf_counter()
        orc.knn2_rows(off.astype(np.int64), items.astype(np.int32), rats.astype(np.float64), n_items, cal)
        per = (time.perf_counter() - t) / 2
        n_rows = int(max(2, min(200 * threads, threads * args.cpu_seconds * 0.5 / max(per, 1e-3))))
        rows = np.sort(rng.choice(n_items, size=n_rows, replace=False)).astype(np.int32)
        t = time.perf_counter()
        Wr = orc.knn2_rows(off.astype(np.int64), items.astype(np.int32), rats.astype(np.float64), n_items, rows,
                           threads=threads)
        cpu_s = time.perf_counter() - t
        Wg = W_s[torch.from_numpy(rows.astype(np.int64)).to(dev)].cpu().numpy()
        out["parity_rows_bit_exact"] = bool(np.array_equal(Wg, Wr))
        out["parity_rows"] = n_rows
        out["cpu_baseline"] = {
            "value": n_rows * (I - 1) / cpu_s,
            "unit": "item-pair similarities/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{n_rows} random rows x {n_items} items of the same workload, oracle weights_calc "
                      f"(sorted-list intersection per pair, float accumulators as knn2.cpp:127-146), rows over "
                      f"{threads} threads (the item maps are built once, serially, inside the timed call)",
        }
    del d_W
    torch.cuda.empty_cache()
    return out


def pmc_traffic(args, knn2=False, prep=False):
    """FETCH_SIZE and WRITE_SIZE (bytes) summed over the predict_kernel and eigen_kernel
    launches of one child step, each counter in its own rocprofv3 run (MI355X_MICROARCH.md:
    FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2, so they cannot share a pass).  knn2: the
    knn2_code_kernel launch of one child knn2 call instead."""
    import csv
    import re
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    out = {"predict": [0.0, 0.0], "eigen": [0.0, 0.0], "eigen12": [0.0, 0.0], "knn2": [0.0, 0.0], "prep": [0.0, 0.0]}
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", args.config,
             "--users", str(args.users)]
    if knn2:
        child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--knn2", "only", "--knn2-users",
                 str(args.knn2_users), "--knn2-items", str(args.knn2_items)]
    if prep:
        child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--prep", "only", "--no-cpu-baseline"]
    env = dict(os.environ, TMPDIR="/tmp")
    for slot, counter in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        d = tempfile.mkdtemp(prefix="cf_pmc_", dir="/tmp")
        cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--", *child]
        try:
            subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           timeout=300, check=True)
            path = os.path.join(d, "run_counter_collection.csv")
            for r in csv.DictReader(open(path)):
                name = r["Kernel_Name"]
                if prep:   # every kernel of the one regroup call but torch's own
                    if not re.search(r"at::native", name) and r["Counter_Name"] == counter:
                        out["prep"][slot] += float(r["Counter_Value"]) * 1024.0
                    continue
                if knn2:
                    if re.search(r"knn2_(code|i8|f32)_kernel", name) and r["Counter_Name"] == counter:
                        out["knn2"][slot] += float(r["Counter_Value"]) * 1024.0
                    continue
                key = "predict" if re.search(r"pred_(basis|rating|dense)_kernel<|spill_(basis|predict)_kernel<", name) \
                    else "eigen" if re.search(r"eigen_kernel<|split_sweep_kernel<", name) else None
                if key and r["Counter_Name"] == counter:
                    out[key][slot] += float(r["Counter_Value"]) * 1024.0   # the counter is in KiB
                    kn = re.search(r"(pred_basis|pred_rating|pred_dense|spill_basis|spill_predict)_kernel", name)
                    if kn:   # the predictor's split per kernel
                        out.setdefault("predict_by_kernel", {}).setdefault(kn.group(1), [0.0, 0.0])[slot] += \
                            float(r["Counter_Value"]) * 1024.0
                    # the dominant launch alone: bucket 12's kernel (narrow layout), or its split pair
                    if re.search(r"eigen_kernel<12, ?true|split_sweep_kernel<12[,>]", name):
                        out["eigen12"][slot] += float(r["Counter_Value"]) * 1024.0
        except (subprocess.SubprocessError, OSError, KeyError, ValueError):
            return None
        finally:
            shutil.rmtree(d, ignore_errors=True)
    return out


def row_lim(off, k, m, evals, sigtab):
    """lim of every row (local_calc_precomp.cpp:271-279): #(stored eigenvalues of the user <=
    w_lim), at least 2, at most m, with the compat w_lim of row r = sigtab[r]; one global
    searchsorted over keys offset by 16 x user (eigenvalues lie in [0, 2], w_lim < 16)."""
    off = np.asarray(off, dtype=np.int64)
    k = np.asarray(k, dtype=np.int64)
    n = int(off[-1])
    uid = np.repeat(np.arange(len(k)), k)
    row = np.arange(n) - off[:-1][uid]
    mu = np.asarray(m, dtype=np.int64)[uid]
    mu_k = np.minimum(np.asarray(m, dtype=np.int64), k)          # stored eigenvalues per user
    valid = row < mu_k[uid]
    ekeys = (uid * 16.0 + np.asarray(evals[:n], dtype=np.float64))[valid]
    start = np.concatenate([[0], np.cumsum(mu_k)])[:-1]
    w = np.asarray(sigtab, dtype=np.float64)[row]
    lim = np.searchsorted(ekeys, uid * 16.0 + w, side="right") - start[uid]
    return np.minimum(np.maximum(lim, 2), mu).astype(np.float64)


def at_bound_stats(off, k, m, kk, evals, sigtab, ratings, mse):
    """Rank-deficient rows (0 < c < lim) and the share of them whose prediction sits at a clamp
    bound (pred in {1, 5}: with integer ratings r that is mse == (r-1)^2 or (r-5)^2, bit for
    bit), next to the same share over the full-rank rows (c >= lim)."""
    lim = row_lim(off, k, m, evals, sigtab)
    c = np.asarray(kk, dtype=np.float64)
    r = np.asarray(ratings, dtype=np.float64)
    e = np.asarray(mse, dtype=np.float32)
    bound = (e == np.float32((r - 1.0) ** 2)) | (e == np.float32((r - 5.0) ** 2))
    rd = (c > 0) & (c < lim)
    fr = c >= lim
    return {"rows": int(len(c)), "rank_deficient_rows": int(rd.sum()),
            "rank_deficient_at_bound_frac": float(bound[rd].mean()) if rd.any() else 0.0,
            "full_rank_at_bound_frac": float(bound[fr].mean()) if fr.any() else 0.0}


def predictor_flops(off, k, m, kk, evals, sigtab):
    """Flop and byte counts of the predict stage (outside the timed region), vectorised.

    algorithmic (lower bound of this kernel's algorithm): per user k Lu^2 (Gram,
    symmetric) + k^3 (one Gram of the k x k basis X); per pair ns^2 max(nc, d) + ns^3 / 3 (the
    Gram of its system and the LDL^T), nc = k - c, d = k - lim, ns = min(nc, d).
    ref (the reference's explicit-inverse work per pair): 2cL^2 + 2L^3 + 2cL + 2L^2 +
    2L with c = kk and L = lim (compat w_lim = sigtab[r]); bytes = 4cL + 4c + 12 per pair.
    executed (this kernel, pred_basis_kernel + pred_rating_kernel): see the comments below.
    """
    off = np.asarray(off, dtype=np.int64)
    k = np.asarray(k, dtype=np.int64)
    n = int(off[-1])
    uid = np.repeat(np.arange(len(k)), k)
    lim = row_lim(off, k, m, evals, sigtab)
    c = np.asarray(kk, dtype=np.float64)
    kr = k[uid].astype(np.float64)
    nc = kr - c
    ref = float(np.sum(2 * c * lim ** 2 + 2 * lim ** 3 + 2 * c * lim + 2 * lim ** 2 + 2 * lim))
    byt = float(np.sum(4 * c * lim + 4 * c + 12))
    lu = np.zeros(len(k))
    np.maximum.at(lu, uid, lim)
    kf = k.astype(np.float64)
    du = kf - lu                                   # complement columns of the basis X = [Q | W]
    d = kr - lim                                   # complement width of the rating's prefix
    ns = np.minimum(nc, d)                         # rows of the rating's system (K or G form)
    # lower bound: per user the Gram U^T U (k Lu^2) and one k x k Gram of the basis (k^3, the
    # orthogonality check every basis needs); per rating the Gram of its gathered system
    # (ns^2 max(nc, d), symmetric) and its LDL^T (ns^3 / 3)
    alg = float(np.sum(kf * lu * lu + kf ** 3)) + float(np.sum(ns * ns * np.maximum(nc, d) + ns ** 3 / 3))
    # executed (block_gemm computes whole 64 x 64 blocks; lower-triangle products ~half):
    # Gram k Lu^2, Q = U T1 k Lu^2, Q^T Omega and Y 4 k Lu du, Y^T Y k du^2 + du^3 / 3, W k du^2,
    # one joint T step 2 k^3, X^T r and X^T 1 4 k^2; per rating the bordered Gram and LDL^T
    exe = float(np.sum(2 * kf * lu * lu + 4 * kf * lu * du + 2 * kf * du * du + du ** 3 / 3 + 2 * kf ** 3
                       + 4 * kf * kf))
    exe += float(np.sum((ns + 1) * (ns + 2) * np.maximum(nc, d) + ns ** 3 / 3 + 4 * ns ** 2))
    # structurally rank-deficient rows: 0 < c < lim, so U_CS^T U_CS (lim' x lim', rank <= c) is
    # singular before the column filter -- the reference returns rounding noise there, this
    # kernel the minimum-norm least-squares prediction
    rdef = int(np.sum((c > 0) & (c < lim)))
    return {"algorithmic_flops": alg, "executed_flops": exe, "ref_flops": ref, "algorithmic_bytes": byt,
            "lim_mean": float(lim.mean()) if n else 0.0, "rank_deficient_rows": rdef,
            "rank_deficient_frac": rdef / max(n, 1), "c0_rows": int(np.sum(c == 0))}


def end_to_end_agreement(ctx, wl, W, users, so, si, sr, m_o, sigs_o, evals_o, evecs_o, eoff_o, threads,
                         max_users=300):
    """how far the drop-in's predictions are from the reference's, end to end.

    For the first users of the CPU sample: device eigens (the timed run's fp32 records) -> device
    predictor (cf_predict_precomp_sel_f32) against oracle eigens (fp64 restatement of
    compute_eigens) -> oracle neigh_program::apply (explicit inverse), both with each user's OWN
    sigs as w_lim (the compat table differs between the full run and the sample by construction).
    Every row is put in exactly one class, in this order:
      c0             no connected item (kk = 0): NaN on both sides;
      lim_differs    the two sides' lim differ (an eigenvalue within fp32 noise of w_lim);
      filter_differs the signed zero-column filter keeps different columns (:284-304);
      rank_deficient |S| > c: U_CS^T U_CS singular (reference: rounding noise, device: min-norm);
      cluster_cut    lim cuts a cluster (oracle gap at the cut < 1e-3): span(U_S) undetermined;
      ill_conditioned cond(U_CS^T U_CS) > 1e8;
      comparable     everything else: |d pred| is reported and checked against tolerances."""
    from collaborative_filtering_amd.api import CF_SIGS_OWN

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as orc

    torch = wl.torch
    nu = int(min(len(users), max_users))
    su = users[:nu]
    so, si, sr = so[:nu + 1], si[:int(so[nu])], sr[:int(so[nu])]
    ks = np.diff(so).astype(np.int64)
    # device records of these users (own evals/sigs/blocks), copied out of the resident run
    m_d = wl.d_m.cpu().numpy()[su]
    rows = np.concatenate([np.arange(int(wl.off[u]), int(wl.off[u + 1])) for u in su])
    sig_d = wl.d_sigs[torch.from_numpy(rows).to(wl.d_sigs.device)].cpu().numpy()
    ev_d = wl.d_evals[torch.from_numpy(rows).to(wl.d_sigs.device)].cpu().numpy()
    blocks = [wl.d_evecs[int(wl.evec_off[u]):int(wl.evec_off[u]) + int(wl.k[u]) * int(m_d[i])]
              for i, u in enumerate(su)]
    peoff = np.zeros(nu, dtype=np.uint64)
    peoff[1:] = np.cumsum([b.numel() for b in blocks])[:-1]
    evec_d = torch.cat(blocks).cpu().numpy() if blocks else np.zeros(1, np.float32)
    sel = np.ones(len(rows), dtype=np.uint8)
    mse_d, kk_d, pred_d = ctx.predict_precomp(so.astype(np.uint64), si.astype(np.uint32), sr.astype(np.float32), m_d,
                                              ev_d.astype(np.float64), peoff, evec_d, sig_d.astype(np.float64),
                                              sig_mode=CF_SIGS_OWN, want_pred=True)
    mse_o, kk_o, pred_o = orc.predict_batch(so, si, sr, m_o[:nu], evals_o, eoff_o[:nu], evecs_o, sigs_o, W,
                                            compat=False, n_threads=threads, want_pred=True)
    del sel
    counts = {c: 0 for c in ("c0", "lim_differs", "filter_differs", "rank_deficient", "cluster_cut",
                             "ill_conditioned", "comparable")}
    kk_equal = int(np.sum(kk_d == kk_o))
    dpred = []
    for i in range(nu):
        b, e = int(so[i]), int(so[i + 1])
        k = e - b
        it = si[b:e].astype(np.int64)
        Cm = np.asarray(W[np.ix_(it, it)], dtype=np.float64) > 0.1
        mo, md = int(m_o[i]), int(m_d[i])
        Uo = evecs_o[int(eoff_o[i]):int(eoff_o[i]) + k * mo].reshape(k, mo)
        Ud = evec_d[int(peoff[i]):int(peoff[i]) + k * md].reshape(k, md).astype(np.float64)
        evo = np.zeros(mo)
        evo[:min(mo, k)] = evals_o[b:b + min(mo, k)]
        evd = np.zeros(md)
        evd[:min(md, k)] = ev_d[b:b + min(md, k)]
        Ko = Cm.astype(np.int32) @ (Uo >= 1e-4).astype(np.int32) > 0
        Kd = Cm.astype(np.int32) @ (Ud >= 1e-4).astype(np.int32) > 0
        for r in range(k):
            c = int(Cm[r].sum())
            if c == 0:
                counts["c0"] += 1
                continue
            lo = int(np.clip(np.sum(evo <= sigs_o[b + r]), 2, mo))
            ld = int(np.clip(np.sum(evd <= sig_d[b + r]), 2, md))
            if lo != ld:
                counts["lim_differs"] += 1
                continue
            S = np.nonzero(Ko[r, :lo])[0]
            if not np.array_equal(S, np.nonzero(Kd[r, :lo])[0]):
                counts["filter_differs"] += 1
                continue
            if len(S) > c or len(S) == 0:
                counts["rank_deficient"] += 1
                continue
            if lo < mo and lo < len(evo) and abs(evo[lo] - evo[lo - 1]) < 1e-3:
                counts["cluster_cut"] += 1
                continue
            G = Uo[np.nonzero(Cm[r])[0]][:, S]
            sv = np.linalg.svd(G, compute_uv=False)
            if sv[-1] <= 0 or (sv[0] / sv[-1]) ** 2 > 1e8:
                counts["ill_conditioned"] += 1
                continue
            counts["comparable"] += 1
            dpred.append(abs(float(pred_d[b + r]) - float(pred_o[b + r])))
    dp = np.asarray(dpred) if dpred else np.zeros(1)
    n_rows = int(so[-1])
    comp = counts["comparable"]
    return {
        "users": nu, "rows": n_rows, "kk_equal_frac": kk_equal / max(n_rows, 1),
        "classes": counts, "comparable_frac": comp / max(n_rows, 1),
        "comparable_agree_frac": {f"{t:g}": float(np.mean(dp <= t)) if comp else None for t in (1e-6, 1e-4, 1e-3, 1e-2)},
        "comparable_dpred_median": float(np.median(dp)) if comp else None,
        "comparable_dpred_max": float(dp.max()) if comp else None,
        "note": "device fp32 eigens -> device predictor vs oracle fp64 eigens -> oracle explicit-inverse predictor "
                "on the same users, own sigs as w_lim on both sides; rows classed in the order listed in "
                "bench.end_to_end_agreement (c0, lim_differs, filter_differs, rank_deficient, cluster_cut, "
                "ill_conditioned, comparable); agree_frac = share of comparable rows with |d pred| <= tolerance"}


def cpu_baseline(args, wl, W, dev=None, ctx=None):
    """The oracle in precompute_local_threads / local_calc_precomp form (fp64, the reference's
    dense LU inverse + 2 GEMMs + Householder/QL eigensolver; neigh_program::apply per rating
    with the explicit-inverse Gram) on a std::thread pool of all the host threads this
    process may use, over a bounded random sample of the same users."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref as orc

    threads, hinfo = host_threads()
    rng = np.random.default_rng(1)
    order = rng.permutation(wl.n_users)
    off, items, ratings, k = wl.off, wl.items, wl.ratings, wl.k

    def sample_arrays(users):
        ks = k[users].astype(np.int64)
        so = np.zeros(len(users) + 1, dtype=np.int64)
        so[1:] = np.cumsum(ks)
        si = np.concatenate([items[int(off[u]):int(off[u + 1])] for u in users]).astype(np.int32)
        sr = np.concatenate([ratings[int(off[u]):int(off[u + 1])] for u in users]).astype(np.float64)
        return so, si, sr

    # calibrate on a small sample, then size the sample to ~cpu_seconds * 0.6 of wall time
    cal = order[:max(threads * 4, 64)]
    so, si, _ = sample_arrays(cal)
    t = time.perf_counter()
    orc.precompute_batch(so, si, W, n_threads=threads, faithful=True)
    rate = len(cal) / (time.perf_counter() - t)
    n = int(min(wl.n_users, max(len(cal), rate * args.cpu_seconds * 0.6)))
    users = order[:n]
    so, si, sr = sample_arrays(users)
    t = time.perf_counter()
    m, sigs, evals, evecs, eoff = orc.precompute_batch(so, si, W, n_threads=threads, faithful=True)
    eig_s = time.perf_counter() - t
    # predictor over the first users of the sample (compat w_lim over the sample's records),
    # sized to ~cpu_seconds * 0.4
    npu = max(1, min(n, threads * 2))
    t = time.perf_counter()
    orc.predict_batch(so[:npu + 1], si[:int(so[npu])], sr[:int(so[npu])], m[:npu], evals, eoff[:npu], evecs,
                      sigs, W, compat=True, n_threads=threads)
    per_user = (time.perf_counter() - t) / npu
    npu = int(min(n, max(npu, args.cpu_seconds * 0.4 / max(per_user, 1e-9))))
    t = time.perf_counter()
    mse_o, kk_o, _ = orc.predict_batch(so[:npu + 1], si[:int(so[npu])], sr[:int(so[npu])], m[:npu], evals,
                                       eoff[:npu], evecs, sigs, W, compat=True, n_threads=threads)
    pred_s = time.perf_counter() - t
    n_pred = int(so[npu])
    ks = np.diff(so[:npu + 1])
    bound_o = at_bound_stats(so[:npu + 1], ks, m[:npu], kk_o, evals, sigs, sr[:n_pred], mse_o)
    # the device's rows of the same users (its own eigen records, compat table of the full run)
    su = users[:npu]
    rows_d = np.concatenate([np.arange(int(off[u]), int(off[u + 1])) for u in su])
    bound_d = at_bound_stats(so[:npu + 1], ks, dev["m"][su], dev["kk"][rows_d], dev["evals"][rows_d],
                             dev["sigs"], ratings[rows_d], dev["mse"][rows_d]) if dev else None
    e2e = None
    if dev is not None and ctx is not None:
        try:
            t = time.perf_counter()
            e2e = end_to_end_agreement(ctx, wl, W, users, so, si, sr, m, sigs, evals, evecs, eoff, threads)
            e2e["seconds"] = time.perf_counter() - t
        except Exception as exc:   # noqa: BLE001 -- a diagnostic, never the bench line's failure
            e2e = f"failed: {exc!r}"
    return {
        "end_to_end": e2e,
        "value": n / eig_s,
        "unit": "user-subgraph eigendecomps/s",
        "cores": threads,
        "host": hinfo,
        "kind": "port",
        "sample": f"{n} random users of the same workload, oracle compute_eigens with the reference's dense LU "
                  f"inverse + 2 GEMMs + Householder/QL eigensolver (fp64), {threads}-thread pool",
        "predicted_ratings_per_s": n_pred / pred_s,
        "predict_sample": f"{n_pred} predictions ({npu} users), oracle neigh_program::apply (fp64, explicit "
                          f"PartialPivLU-class inverse per rating, compat w_lim), {threads}-thread pool",
        "clamp_bounds": {
            "oracle": bound_o, "device_same_users": bound_d,
            "note": "rows at a clamp bound (pred 1 or 5) among the rank-deficient rows (0 < c < lim) of the "
                    "predict sample: the oracle restates the reference's explicit inverse of the singular "
                    "U_CS^T U_CS (rounding noise, mostly clamped), the device returns the minimum-norm "
                    "least-squares prediction (DESIGN 3.2, INTEGRATION.md)"},
    }


if __name__ == "__main__":
    main()
