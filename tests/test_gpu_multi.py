"""Multi-GPU product path on the GPU box: cf_eigen_batch_multi over several
contexts (on a one-GPU box they share device 0, the peer copies degenerate to local copies,
the code path is the same), cf_pack_eigen_run, and bin/precompute_local --devices N (the
chunks of cf_eigen_batch_stream dealt to the devices), whose out_eigen_ must be byte-identical
to the one-device, one-chunk file (precompute_local_threads.cpp:300-314
thread pool -> one range per GPU; :196-211 one out_eigen_)."""
import os
import subprocess

import numpy as np
import pytest

import cases
import pipeline_util as pu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_eigen_batch_multi_matches_single(gpu_ctx):
    import torch

    from collaborative_filtering_amd.api import Context, cost_split_native, eigen_batch_multi, evec_offsets

    W = cases.item_graph(300, 0.5, seed=21)
    ks = list(np.random.default_rng(4).integers(2, 200, size=180)) + [1, 193, 240]
    off, items = cases.user_items(300, ks, seed=5)
    gpu_ctx.upload_graph_dense(W)
    ref = gpu_ctx.eigen_batch(off, items)
    k = np.diff(off.astype(np.int64))
    for n_dev in (2, 3):
        ctxs = [Context(0) for _ in range(n_dev)]
        try:
            for c in ctxs:
                c.upload_graph_dense(W)
            res, split = eigen_batch_multi(ctxs, off, items)
        finally:
            for c in ctxs:
                c.close()
        assert np.array_equal(split, cost_split_native(off, n_dev))
        assert split[0] == 0 and split[-1] == len(ks) and np.all(np.diff(split) > 0)
        assert np.array_equal(res.m, ref.m)
        assert np.array_equal(res.sigs, ref.sigs)
        n = int(off[-1])
        for u in range(len(ks)):   # evals: first min(m, k) of each user
            b = int(off[u])
            q = min(int(ref.m[u]), int(k[u]))
            assert np.array_equal(res.evals[b:b + q], ref.evals[b:b + q])
        assert n == len(res.sigs)
        for u in range(len(ks)):
            _, _, U_ref = ref.block(u)
            _, _, U_got = res.block(u)
            assert np.array_equal(U_got, U_ref), u
    # the device pack alone, on the single context's slot layout
    eoff, n_evec = evec_offsets(off)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
    d_off, d_m = T(off.view(np.int64)), T(ref.m)
    d_eoff, d_ev = T(eoff.view(np.int64)), T(ref.evecs)
    d_poff = torch.zeros(len(ks) + 1, dtype=torch.int64, device="cuda:0")
    gpu_ctx.pack_eigen_run(len(ks), d_off, d_m, None, None, d_poff)
    torch.cuda.synchronize()
    total = int(d_poff[-1].item())
    assert total == int(np.sum(k * ref.m))
    d_pk = torch.zeros(total, dtype=torch.float32, device="cuda:0")
    gpu_ctx.pack_eigen_run(len(ks), d_off, d_m, d_eoff, d_ev, d_poff, d_pk)
    torch.cuda.synchronize()
    poff = d_poff.cpu().numpy()
    pk = d_pk.cpu().numpy()
    for u in range(len(ks)):
        _, _, U_ref = ref.block(u)
        assert np.array_equal(pk[poff[u]:poff[u + 1]], U_ref.ravel()), u


def _run(wd, *args, env=None):
    p = subprocess.run([os.path.join(ROOT, "bin", args[0]), *args[1:]], cwd=wd, capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    return p.stdout


@pytest.mark.parametrize("fmt", ["text", "binary"])
def test_precompute_local_devices_byte_identical(tmp_path, fmt):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    wd = str(tmp_path)
    pu.write_movielens(wd, n_users=400, n_items=150, test_frac=0.5, seed=17)
    _run(wd, "knn")
    _run(wd, "knn2")
    outs = {}
    for n_dev, chunk in ((1, 0), (2, 0), (4, 0), (1, 60000), (3, 60000)):
        out = f"out_eigen_d{n_dev}_c{chunk}"
        log = _run(wd, "precompute_local", "8", "--devices", str(n_dev), "--output", out, "--format", fmt,
                   "--chunk-bytes", str(chunk))
        assert f"on {n_dev} device(s)" in log, log
        n_chunks = int(log.split("eigen stream: ")[1].split()[0])
        assert (n_chunks == 1) if chunk == 0 else (n_chunks >= 3), log
        outs[(n_dev, chunk)] = open(os.path.join(wd, out), "rb").read()
    ref = outs[(1, 0)]
    assert len(ref) > 1000
    for key, v in outs.items():
        assert v == ref, key


def _c2_subsample(n_users, seed):
    from collaborative_filtering_amd import synth, workloads as wlm
    from collaborative_filtering_amd.api import Context

    import torch

    cfg = wlm.CONFIGS["c2"]
    d_W, _, _ = wlm.config_graph("c2", Context, 0, torch.device("cuda", 0), torch)
    k_all = wlm.user_degrees(cfg)
    users = np.sort(np.random.default_rng(seed).choice(len(k_all), size=n_users, replace=False))
    off_all, items_all, rat_all = synth.user_items(cfg["seed"], k_all, cfg["items"], threads=16)
    off, items, rat = wlm.sub_csr(off_all, items_all, rat_all, users)
    return d_W.view(cfg["items"], cfg["items"]), off, items, rat


def test_predict_precomp_multi_bit_identical(gpu_ctx):
    """cf_predict_precomp_multi over 2 and 3 contexts (sharing GPU 0) equals the one-context
    cf_predict_precomp_sel bit for bit on a C2 subsample in compat mode (every range reads the
    global concatenated sig table, local_calc_precomp.cpp:414,437,440)."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, cost_split_native, predict_precomp_multi

    d_W, off, items, rat = _c2_subsample(1500, seed=11)
    gpu_ctx.upload_graph_dense(d_W)
    res = gpu_ctx.eigen_batch(off, items)
    k = np.diff(off.astype(np.int64))
    evals = res.evals.astype(np.float64)
    evecs = res.evecs.astype(np.float64)
    sig = res.sigs.astype(np.float64)
    ref = gpu_ctx.predict_precomp(off, items, rat, res.m, evals, res.evec_off, evecs, sig, sig_mode=CF_SIGS_COMPAT)
    assert np.sum(ref[1] > 0) > 1000
    for n_dev in (2, 3):
        ctxs = [Context(0) for _ in range(n_dev)]
        try:
            for c in ctxs:
                c.upload_graph_dense(d_W)
            mse, kk, split = predict_precomp_multi(ctxs, off, items, rat, res.m, evals, res.evec_off, evecs, sig,
                                                   sig_mode=CF_SIGS_COMPAT)
        finally:
            for c in ctxs:
                c.close()
        assert np.array_equal(split, cost_split_native(off, n_dev)) and np.all(np.diff(split) > 0)
        assert int(off[split[1]]) > int(k.max())        # ranges past the first hold no prefix user
        assert np.array_equal(kk, ref[1])
        assert np.array_equal(mse, ref[0], equal_nan=True)


def test_predict_precomp_f32_blocks_bit_identical(gpu_ctx):
    """The binary out_eigen_ keeps its fp32 blocks (cf_predict_precomp_sel_f32 /
    cf_predict_precomp_multi_f32): predictions equal the fp64 entry points' on the widened
    blocks bit for bit, one context and two (compat mode, C2 subsample)."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT, Context, predict_precomp_multi

    d_W, off, items, rat = _c2_subsample(1200, seed=23)
    gpu_ctx.upload_graph_dense(d_W)
    res = gpu_ctx.eigen_batch(off, items)
    evals = res.evals.astype(np.float64)
    sig = res.sigs.astype(np.float64)
    ref = gpu_ctx.predict_precomp(off, items, rat, res.m, evals, res.evec_off, res.evecs.astype(np.float64), sig,
                                  sig_mode=CF_SIGS_COMPAT)
    assert np.sum(ref[1] > 0) > 800
    e32 = np.ascontiguousarray(res.evecs, dtype=np.float32)
    one = gpu_ctx.predict_precomp(off, items, rat, res.m, evals, res.evec_off, e32, sig, sig_mode=CF_SIGS_COMPAT)
    assert np.array_equal(one[1], ref[1])
    assert np.array_equal(one[0], ref[0], equal_nan=True)
    ctxs = [Context(0) for _ in range(2)]
    try:
        for c in ctxs:
            c.upload_graph_dense(d_W)
        mse, kk, _ = predict_precomp_multi(ctxs, off, items, rat, res.m, evals, res.evec_off, e32, sig,
                                           sig_mode=CF_SIGS_COMPAT)
    finally:
        for c in ctxs:
            c.close()
    assert np.array_equal(kk, ref[1])
    assert np.array_equal(mse, ref[0], equal_nan=True)


def test_bench_ranks_equal_single_rank(gpu_ctx):
    """bench.py's N>1 step on world = 2 and 3 ranks emulated by contexts on GPU 0: each rank's
    Workload (its cost_split range of the global set, the compat table rebuilt from the global
    prefix users on ranks > 0) predicts exactly the rows of the one-rank run, bit for bit."""
    import argparse

    import torch

    import bench

    from collaborative_filtering_amd import workloads as wlm
    from collaborative_filtering_amd.api import Context as _Ctx

    cfg = dict(bench.CONFIGS["c2"])
    d_W, _, _ = wlm.config_graph("c2", _Ctx, 0, torch.device("cuda", 0), torch)
    d_W = d_W.view(cfg["items"], cfg["items"])
    args = argparse.Namespace(users=6000)
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream

    def run(world):
        from collaborative_filtering_amd.api import Context

        mse, kk, ms, pre = [], [], [], []
        for rank in range(world):
            with Context(0) as ctx:
                wl = bench.Workload(args, cfg, rank, world, dev, torch, ctx, d_W)
                wl.eigen(sp)
                wl.predict(sp)
                torch.cuda.synchronize(dev)
                mse.append(wl.d_mse[:wl.n_entries].cpu().numpy())
                kk.append(wl.d_kk[:wl.n_entries].cpu().numpy())
                ms.append(wl.d_m[:wl.n_users].cpu().numpy())
                pre.append(wl.pre is not None)
                wl.plan.close()
                if wl.pre:
                    wl.pre["plan"].close()
        return np.concatenate(mse), np.concatenate(kk), np.concatenate(ms), pre

    mse1, kk1, m1, pre1 = run(1)
    assert pre1 == [False]
    assert np.sum(kk1 > 0) > 100000
    for world in (2, 3):
        mse, kk, m, pre = run(world)
        assert pre == [False] + [True] * (world - 1)
        assert np.array_equal(m, m1)
        assert np.array_equal(kk, kk1)
        assert np.array_equal(mse, mse1, equal_nan=True)


def test_local_calc_precomp_devices_byte_identical(tmp_path):
    """bin/local_calc_precomp --devices 1/2/3 (cf_predict_precomp_multi): one out_res_ set,
    byte-identical to the one-device run (the reference: every rank reads the whole out_eigen_,
    local_calc_precomp.cpp:485-486,509, and saves its rows of out_res_, :576)."""
    import glob

    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    wd = str(tmp_path)
    pu.write_movielens(wd, n_users=400, n_items=150, test_frac=0.5, seed=19)
    _run(wd, "knn")
    _run(wd, "knn2")
    _run(wd, "precompute_local", "8")
    outs = {}
    for n_dev in (1, 2, 3):
        log = _run(wd, "local_calc_precomp", "--pct", "100", "--seed", "1", "--devices", str(n_dev))
        if n_dev > 1:
            assert log.count("device part") == n_dev
        files = sorted(glob.glob(os.path.join(wd, "out_res_*")))
        outs[n_dev] = b"".join(open(f, "rb").read() for f in files)
    assert outs[1].count(b"\n") > 1000
    assert outs[2] == outs[1] and outs[3] == outs[1]
