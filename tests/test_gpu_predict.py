"""GPU parity: cf_predict_precomp (HIP fp64 predictor) vs the oracle's neigh_program::apply.

Stage-wise parity (hard part 2): both sides get the SAME eigen
blocks (the oracle's fp64 compute_eigens output, standing in for a parsed
out_eigen_), so the sign-dependent zero-column filter sees identical inputs.
kk must match exactly everywhere; c = 0 must give NaN on both sides; wherever the
Gram matrix U_CS^T U_CS has cond <= 1e8 both sides must be finite with
|d mse| <= 1e-6 * max(1, mse).  Rank-deficient Gram matrices (c < L) are counted,
not compared: there the reference's own output is decided by rounding noise of its
Eigen build (an exactly-zero LU pivot gives NaN, a tiny one gives a clamped 1 or 5).
"""
import numpy as np
import pytest

import cases
import oracle_ref as orc
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, CF_SIGS_OWN

pytestmark = pytest.mark.gpu


def gram_cond(items, evals, U, sigtab_row, W, r):
    """cond(U_CS^T U_CS) of row r as neigh_program::apply forms it (local_calc_precomp.cpp:
    254-309): C = connected items (w > 0.1), lim = first eigenvalue > w_lim (>= 2, <= m),
    S = the columns kept by the signed zero-column filter."""
    k, m = U.shape
    items = np.asarray(items, dtype=np.int64)
    C = np.nonzero(np.asarray(W[items[r], items], dtype=np.float64) > 0.1)[0]
    ev = np.asarray(evals[:m], dtype=np.float64)
    above = np.nonzero(ev > sigtab_row)[0]
    lim = int(above[0]) if len(above) else m
    lim = min(max(lim, 2), m)
    if len(C) == 0:
        return np.inf
    keep = np.nonzero((U[C, :lim] >= 1e-4).any(axis=0))[0]
    if len(keep) == 0:
        return np.inf
    G = U[np.ix_(C, keep)]
    return np.linalg.cond(G.T @ G)


def build_case(density, ks, seed, n_items=220):
    W = cases.item_graph(n_items, density, seed=seed, isolated_frac=0.02)
    off, items = cases.user_items(n_items, ks, seed=seed + 1)
    rat = cases.ratings_for(len(items), seed + 2)
    n_users = len(ks)
    m = np.zeros(n_users, np.int32)
    sigs = np.zeros(len(items))
    evals = np.zeros(len(items))
    blocks = []
    for u in range(n_users):
        b, e = int(off[u]), int(off[u + 1])
        it = items[b:e].astype(np.int64)
        mu, sg, ev, U, _ = orc.compute_eigens(W[np.ix_(it, it)].astype(np.float64))
        m[u] = mu
        sigs[b:e] = sg
        evals[b:b + min(mu, e - b)] = ev[: min(mu, e - b)]
        blocks.append((ev, U))
    k = np.diff(off.astype(np.int64))
    evec_off = np.zeros(n_users, np.uint64)
    evec_off[1:] = np.cumsum(k * np.maximum(k, 2))[:-1]
    evecs = np.zeros(int((k * np.maximum(k, 2)).sum()))
    for u, (ev, U) in enumerate(blocks):
        evecs[int(evec_off[u]): int(evec_off[u]) + U.size] = U.ravel()
    return W, off, items, rat, m, sigs, evals, evec_off, evecs, blocks


@pytest.mark.parametrize("density,mode", [(0.6, CF_SIGS_COMPAT), (0.6, CF_SIGS_OWN), (0.05, CF_SIGS_COMPAT),
                                          (0.9, CF_SIGS_OWN)])
def test_predict_matches_oracle(gpu_ctx, density, mode):
    ks = [1, 2, 3, 7, 20, 33, 50, 64, 65, 90, 128, 129, 150]
    W, off, items, rat, m, sigs, evals, evec_off, evecs, blocks = build_case(density, ks, seed=40)
    sigtab = sigs.copy()  # compat table = concatenation of every record's sigs in file order
    gpu_ctx.upload_graph_dense(W)
    mse_g, kk_g, pred_g = gpu_ctx.predict_precomp(off, items, rat, m, evals, evec_off, evecs, sigtab,
                                                  sig_mode=mode, want_pred=True)
    n_good = n_ill = 0
    bad = []
    for u in range(len(ks)):
        b, e = int(off[u]), int(off[u + 1])
        it = items[b:e].astype(np.int64)
        ev, U = blocks[u]
        ev_full = np.zeros(m[u])
        ev_full[: min(m[u], e - b)] = ev[: min(m[u], e - b)]
        tab = sigtab[: e - b] if mode == CF_SIGS_COMPAT else sigs[b:e]
        mse_o, kk_o, pred_o = orc.predict_user(it, rat[b:e], ev_full, U, tab, W)
        for r in range(e - b):
            g = b + r
            if kk_g[g] != kk_o[r]:
                bad.append((u, r, "kk", kk_g[g], kk_o[r]))
                continue
            cond = gram_cond(it, ev_full, U, tab[r], W, r)
            if kk_o[r] == 0:
                # no connected items: 0/0 mean -> NaN on both sides (:311)
                if not (np.isnan(mse_g[g]) and np.isnan(mse_o[r])):
                    bad.append((u, r, "c=0 not NaN", mse_g[g], mse_o[r]))
                continue
            if cond <= 1e8:
                if np.isnan(mse_g[g]) or np.isnan(mse_o[r]):
                    bad.append((u, r, "nan", mse_g[g], mse_o[r], cond))
                    continue
                n_good += 1
                if abs(float(mse_g[g]) - float(mse_o[r])) > 1e-6 * max(1.0, float(mse_o[r])):
                    bad.append((u, r, "mse", float(mse_g[g]), float(mse_o[r]), cond))
            else:
                n_ill += 1
    assert not bad, bad[:10]
    if density >= 0.6 and mode == CF_SIGS_OWN and density < 0.9:
        assert n_good > 100, (n_good, n_ill)
    print(f"density={density} mode={mode} well-conditioned={n_good} ill-conditioned={n_ill}")


def test_predict_device_f32_path_matches_f64(gpu_ctx):
    """The fused device path (fp32 eigen blocks, cf_predict_run_f32) on blocks that are
    exactly representable in fp32 gives the same kk and mse as the fp64 path."""
    import torch

    ks = [5, 20, 40, 64, 100]
    W, off, items, rat, m, sigs, evals, evec_off, evecs, _ = build_case(0.6, ks, seed=50)
    evals32, evecs32, sigs32 = evals.astype(np.float32), evecs.astype(np.float32), sigs.astype(np.float32)
    gpu_ctx.upload_graph_dense(W)
    mse64, kk64 = gpu_ctx.predict_precomp(off, items, rat, m, evals32.astype(np.float64), evec_off,
                                          evecs32.astype(np.float64), sigs32.astype(np.float64),
                                          sig_mode=CF_SIGS_OWN)
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    plan = gpu_ctx.plan(off)
    n = int(off[-1])
    d_mse = torch.zeros(n, dtype=torch.float32, device=dev)
    d_kk = torch.zeros(n, dtype=torch.int32, device=dev)
    plan.predict_run(T(off), T(items), T(rat), T(m), T(evals32), T(evec_off), T(evecs32), T(sigs32),
                     CF_SIGS_OWN, d_mse, d_kk)
    torch.cuda.synchronize()
    assert np.array_equal(d_kk.cpu().numpy(), kk64)
    a, b = d_mse.cpu().numpy(), mse64
    assert np.array_equal(np.isnan(a), np.isnan(b))
    ok = ~np.isnan(b)
    assert np.allclose(a[ok], b[ok], rtol=1e-6, atol=1e-6)


def test_predict_wide_complement_full_rank(gpu_ctx):
    """Ratings whose complement Cbar exceeds one wave's K system (nc > 62) while the
    Gram matrix keeps full rank (c >= lim): the block-wide K path must match the
    oracle like the per-wave one.  A low w_lim (0.3) keeps lim small."""
    ks = [150, 140, 130]
    W, off, items, rat, m, sigs, evals, evec_off, evecs, blocks = build_case(0.5, ks, seed=70)
    sigtab = np.full_like(sigs, 0.3)
    gpu_ctx.upload_graph_dense(W)
    mse_g, kk_g, _ = gpu_ctx.predict_precomp(off, items, rat, m, evals, evec_off, evecs, sigtab,
                                             sig_mode=CF_SIGS_OWN, want_pred=True)
    n_wide = 0
    bad = []
    for u in range(len(ks)):
        b, e = int(off[u]), int(off[u + 1])
        it = items[b:e].astype(np.int64)
        ev, U = blocks[u]
        ev_full = np.zeros(m[u])
        ev_full[: min(m[u], e - b)] = ev[: min(m[u], e - b)]
        tab = sigtab[b:e]
        mse_o, kk_o, _ = orc.predict_user(it, rat[b:e], ev_full, U, tab, W)
        for r in range(e - b):
            g = b + r
            assert kk_g[g] == kk_o[r]
            if (e - b) - kk_o[r] <= 62 or kk_o[r] == 0:
                continue
            if gram_cond(it, ev_full, U, tab[r], W, r) > 1e8:
                continue
            n_wide += 1
            if abs(float(mse_g[g]) - float(mse_o[r])) > 1e-6 * max(1.0, float(mse_o[r])):
                bad.append((u, r, float(mse_g[g]), float(mse_o[r])))
    assert not bad, bad[:10]
    assert n_wide > 20, n_wide


def _compare_users(off, items, rat, m, blocks, sigs, sigtab, mode, W, mse_g, kk_g, users):
    """kk exact; c = 0 NaN on both sides; |d mse| <= 1e-6 max(1, mse) where cond <= 1e8."""
    n_good = n_ill = 0
    bad = []
    for u in users:
        b, e = int(off[u]), int(off[u + 1])
        it = items[b:e].astype(np.int64)
        ev, U = blocks[u]
        ev_full = np.zeros(m[u])
        ev_full[: min(m[u], e - b)] = ev[: min(m[u], e - b)]
        tab = sigtab[: e - b] if mode == CF_SIGS_COMPAT else sigtab[b:e]
        mse_o, kk_o, _ = orc.predict_user(it, rat[b:e], ev_full, U, tab, W)
        for r in range(e - b):
            g = b + r
            if kk_g[g] != kk_o[r]:
                bad.append((u, r, "kk", kk_g[g], kk_o[r]))
                continue
            if kk_o[r] == 0:
                if not (np.isnan(mse_g[g]) and np.isnan(mse_o[r])):
                    bad.append((u, r, "c=0 not NaN", mse_g[g], mse_o[r]))
                continue
            cond = gram_cond(it, ev_full, U, tab[r], W, r)
            if cond <= 1e8:
                if np.isnan(mse_g[g]) or np.isnan(mse_o[r]):
                    bad.append((u, r, "nan", mse_g[g], mse_o[r], cond))
                    continue
                n_good += 1
                if abs(float(mse_g[g]) - float(mse_o[r])) > 1e-6 * max(1.0, float(mse_o[r])):
                    bad.append((u, r, "mse", float(mse_g[g]), float(mse_o[r]), cond))
            else:
                n_ill += 1
    return n_good, n_ill, bad


@pytest.mark.parametrize("density,mode,wlim,min_good", [(0.6, CF_SIGS_COMPAT, None, 200),
                                                        (0.05, CF_SIGS_OWN, None, 0),
                                                        (0.05, CF_SIGS_OWN, 0.3, 200),
                                                        (0.1, CF_SIGS_OWN, 0.2, 200),
                                                        (0.5, CF_SIGS_OWN, 0.3, 200)])
def test_predict_spill_users_match_oracle(gpu_ctx, density, mode, wlim, min_good):
    """Users above CF_MAX_K (the eigen spill bucket) take the HBM-workspace predictor
    (cf_predict_spill.hip) in the same call as LDS-path users.  Dense graphs exercise its
    Woodbury form (small complements, tiled P for large ones), the sparse graph its
    dense path (columns dropped by the zero-column filter, rank-deficient Gram
    matrices: almost all rank-deficient at the reference's own w_lim, hence min_good = 0;
    a low w_lim keeps them full rank), w_lim = 0.3 on a dense graph wide complements."""
    ks = [300, 193, 150, 257, 64, 210]
    W, off, items, rat, m, sigs, evals, evec_off, evecs, blocks = build_case(density, ks, seed=80, n_items=400)
    sigtab = sigs.copy() if wlim is None else np.full_like(sigs, wlim)
    gpu_ctx.upload_graph_dense(W)
    mse_g, kk_g, _ = gpu_ctx.predict_precomp(off, items, rat, m, evals, evec_off, evecs, sigtab,
                                             sig_mode=mode, want_pred=True)
    n_good, n_ill, bad = _compare_users(off, items, rat, m, blocks, sigs, sigtab, mode, W, mse_g, kk_g,
                                        range(len(ks)))
    assert not bad, bad[:10]
    assert n_good >= min_good, (n_good, n_ill)
    print(f"spill density={density} mode={mode} wlim={wlim} well-conditioned={n_good} ill-conditioned={n_ill}")



def test_spill_basis_mc_bit_identical(gpu_ctx, tmp_path):
    """spill_basis_mc (the basis of users with k > 2816 on several workgroups per user, one
    launch per phase) produces the tables of the one-workgroup spill_basis_kernel bit for bit:
    a child process with CF_PSPILL_BASIS_MC=0 runs the same case (k = 3300 and 2950 beside 900
    and 300 in one chunk), and every prediction, mse and kk must equal this process's."""
    import os
    import subprocess
    import sys

    from basis_mc_child import run_case

    ref = run_case(gpu_ctx)
    assert int(np.sum(ref["kk"] > 0)) > 1000
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "basis_mc_child.py")
    out = tmp_path / "basis_one_wg.npz"
    env = dict(os.environ, CF_PSPILL_BASIS_MC="0")
    r = subprocess.run([sys.executable, child, str(out)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    got = np.load(out)
    for k, v in ref.items():
        g = got[k]
        same = np.array_equal(g, v, equal_nan=True) if g.dtype.kind == "f" else np.array_equal(g, v)
        assert same, (k, int(np.sum(g != v)))
    print(f"spill_basis_mc == spill_basis_kernel on {len(ref['mse'])} ratings "
          f"({int(np.sum(np.isnan(ref['mse'])))} NaN)")


def test_dense_buffers_after_debug_phases_toggle():
    """the block-wide rating queue and factorisation regions were sized for
    one stream while the phase diagnostics were on, then indexed by the second stream of an
    overlapped call.  On a fresh context: diagnostics on, predict, diagnostics off, predict
    again -- the block-wide (nc > 62) ratings of both calls give the same kk and mse bits."""
    from collaborative_filtering_amd.api import Context

    ks = [150, 140, 130, 150, 140, 130]
    W, off, items, rat, m, sigs, evals, evec_off, evecs, blocks = build_case(0.5, ks, seed=70)
    sigtab = np.full_like(sigs, 0.3)
    with Context(0) as ctx:
        ctx.upload_graph_dense(W)
        ctx.debug_phases(True)
        mse1, kk1 = ctx.predict_precomp(off, items, rat, m, evals, evec_off, evecs, sigtab, sig_mode=CF_SIGS_OWN)
        ctx.debug_phases(False)
        mse2, kk2 = ctx.predict_precomp(off, items, rat, m, evals, evec_off, evecs, sigtab, sig_mode=CF_SIGS_OWN)
    assert np.array_equal(kk1, kk2)
    assert np.array_equal(mse1.view(np.uint32), mse2.view(np.uint32))
    nc = np.concatenate([np.full(int(off[u + 1] - off[u]), int(off[u + 1] - off[u])) for u in range(len(ks))]) - kk1
    assert int(np.sum(nc > 62)) > 20
