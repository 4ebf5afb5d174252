"""GPU parity on every BASELINE configuration's own generator and seed.

Each config's workload is built exactly as bench.py builds it (collaborative_filtering_amd/
workloads.py): the item graph is knn2's output (cf_item_cosine_run, int8 MFMA) over the
config's train population, the test users come from the same splitmix64 generator.  The
device path is the TIMED one -- cf_eigen_run -> cf_predict_run_f32 on fp32 eigen blocks in
HBM, compat w_lim, every k bucket in one call (bucket launches alternating between the two
aux streams, > 8192 workgroups per bucket at C2/C4) -- and it is checked stage-wise:

* eigen: a deterministic stratified sample (users from every k bucket of the eigen kernels)
  against the oracle's compute_eigens (SURVEY 8a tolerances: sigs rel 1e-5, m exact unless an
  eigenvalue sits within 1e-5 of the cut, eigenvalues abs 1e-5, clustered projectors 1e-3,
  residual / orthonormality 1e-4); size-independent properties (residual, orthonormality,
  sigs, m vs the cut, sign convention) on ~1000 more users against an L2 built in numpy;
* predict: the device's OWN fp32 blocks, downloaded and widened to fp64, are fed to the
  oracle's neigh_program::apply (compat table = the device's concatenated sigs); kk exact,
  NaN-ness exact, |d mse| <= 1e-6 max(1, mse) where cond(U_CS^T U_CS) <= 1e8; rank-deficient
  Gram matrices (cond > 1e8) are counted and reported, not compared (their value is rounding
  noise in the reference too);
* C3: knn2 rows of the full 20k x 500k problem bit-exact against the oracle's weights_calc;
* C5: the power-law mix through the LDS and fp64 spill paths in one call;
* C1: make_synthetic_als_data's algorithm (real-valued ratings, ids 1000..1999) through the
  drop-in binaries (tests/test_pipeline.py, parametrized "c1").

Parity is pinned to the oracle (tests/oracle_ref.py); the oracle is "parity unpinned"
against the reference binaries themselves.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_ref as orc
from test_gpu_predict import gram_cond

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch


class FusedRun:
    """One pass of bench.py's step (eigen -> predict, device-resident) over a user set."""

    def __init__(self, ctx, d_W, n_items, off, items, ratings, sig_mode=None):
        from collaborative_filtering_amd.api import CF_SIGS_COMPAT, evec_offsets

        torch = _torch()
        dev = torch.device("cuda", 0)
        self.torch, self.dev = torch, dev
        self.n_items = n_items
        self.off, self.items, self.ratings = off, items, ratings
        self.k = np.diff(off.astype(np.int64))
        self.d_W = d_W.view(n_items, n_items)
        ctx.upload_graph_dense(self.d_W)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.evec_off, n_evec = evec_offsets(off)
        n, nu = int(off[-1]), len(off) - 1
        self.d_off, self.d_items, self.d_rat = T(off.view(np.int64)), T(items.view(np.int32)), T(ratings)
        self.d_eoff = T(self.evec_off.view(np.int64))
        self.d_m = torch.zeros(nu, dtype=torch.int32, device=dev)
        self.d_sigs = torch.zeros(n, dtype=torch.float32, device=dev)
        self.d_evals = torch.zeros(n, dtype=torch.float32, device=dev)
        self.d_evecs = torch.zeros(max(n_evec, 1), dtype=torch.float32, device=dev)
        self.d_mse = torch.zeros(n, dtype=torch.float32, device=dev)
        self.d_kk = torch.zeros(n, dtype=torch.int32, device=dev)
        self.d_pred = torch.zeros(n, dtype=torch.float64, device=dev)
        self.sig_mode = CF_SIGS_COMPAT if sig_mode is None else sig_mode
        plan = ctx.plan(off)
        sp = torch.cuda.current_stream(dev).cuda_stream
        plan.eigen_run(self.d_off, self.d_items, self.d_eoff, self.d_m, self.d_sigs, self.d_evals, self.d_evecs,
                       stream=sp)
        plan.predict_run(self.d_off, self.d_items, self.d_rat, self.d_m, self.d_evals, self.d_eoff, self.d_evecs,
                         self.d_sigs, self.sig_mode, self.d_mse, self.d_kk, self.d_pred, stream=sp)
        torch.cuda.synchronize(dev)
        plan.close()
        self.m = self.d_m.cpu().numpy()
        self.sigs = self.d_sigs.cpu().numpy()
        self.mse = self.d_mse.cpu().numpy()
        self.kk = self.d_kk.cpu().numpy()
        self.pred = self.d_pred.cpu().numpy()
        del self.d_pred

    def free(self):
        del self.d_evecs, self.d_mse, self.d_kk, self.d_sigs, self.d_evals
        self.torch.cuda.empty_cache()

    def user(self, u):
        """(items, ratings, W_u float32 k x k, m, sigs, evals[m], U k x m) of user u, from HBM."""
        b, e = int(self.off[u]), int(self.off[u + 1])
        k, m = e - b, int(self.m[u])
        it = self.items[b:e].astype(np.int64)
        idx = self.torch.from_numpy(it).to(self.dev)
        Wu = self.d_W.index_select(0, idx).index_select(1, idx).cpu().numpy()
        ev = np.zeros(m, dtype=np.float32)
        ev[: min(m, k)] = self.d_evals[b:b + min(m, k)].cpu().numpy()
        o = int(self.evec_off[u])
        U = self.d_evecs[o:o + k * m].cpu().numpy().reshape(k, m)
        return it, self.ratings[b:e], Wu, m, self.sigs[b:e], ev, U


# ------------------------------------------------------------------------------------------
# stage checks shared by the configs
# ------------------------------------------------------------------------------------------
def eigen_check(run: FusedRun, users, label="eigen"):
    """Oracle compute_eigens vs the device block of each user (thread pool: ctypes drops the GIL).
    Returns the failures; the projector escapes (oracle_ref.compare_eigen_block) are counted
    over the whole sample, reported, and capped (a failure entry when over the cap)."""

    def one(u):
        esc = []
        it, _, Wu, m_g, sig_g, ev_g, U_g = run.user(u)
        k = len(it)
        m_ref, sig_ref, _, _, L2 = orc.compute_eigens(Wu.astype(np.float64))
        ev_full, V_full = orc.eigh(orc.sym_lower(L2))
        if np.max(np.abs(sig_g - sig_ref) / np.abs(sig_ref)) > 1e-5:
            return (u, k, "sigs"), esc
        if m_g != m_ref:
            smm = np.float32(np.float32(np.max(sig_ref - 0.01)) + 0.01)
            return (None if np.any(np.abs(ev_full - smm) <= 1e-5) else (u, k, f"m {m_g} != {m_ref}")), esc
        f = orc.compare_eigen_block(L2, m_ref, ev_full, V_full[:, :m_ref], m_g, ev_g, U_g, escapes=esc)
        return ((u, k, f) if f else None), esc

    with ThreadPoolExecutor(THREADS) as ex:
        res = list(ex.map(one, users))
    bad = [r[0] for r in res if r[0]]
    esc = [e for r in res for e in r[1]]
    if not orc.escapes_ok(esc, label):
        bad.append(("escapes over cap", orc.escape_summary(esc)))
    return bad


def eigen_properties(run: FusedRun, users, res_tol=1e-4):
    """Size-independent checks against an L2 assembled in numpy (precompute_local_threads.cpp:
    114-194): sigs, m vs the cut, ascending kept eigenvalues, residual, orthonormality, and
    the sign convention (column sums >= 0)."""

    def one(u):
        it, _, Wu, m, sig_g, ev_g, U_g = run.user(u)
        k = len(it)
        W = Wu.astype(np.float64)
        d = W.sum(axis=1)
        d[d == 0] = 1.0
        s = np.sqrt(1.0 / d)
        L2 = (s[:, None] * (np.diag(d) - W)) * s[None, :]
        A = np.tril(L2) + np.tril(L2, -1).T
        sig_ref = np.sqrt(np.sum(L2 * L2, axis=1)) + 0.01
        if np.max(np.abs(sig_g - sig_ref) / sig_ref) > 1e-5:
            return (u, "sigs")
        smm = np.float32(np.float32(np.max(sig_ref - 0.01)) + 0.01)
        kv = min(m, k)
        if kv > 2 and not np.all(ev_g[:kv - 1] <= smm + 1e-5):
            return (u, "m vs cut")
        if kv < k and m > 2 and not ev_g[kv - 1] <= smm + 1e-5:
            return (u, "m vs cut (last)")
        if np.any(np.diff(ev_g[:kv]) < -1e-6):
            return (u, "order")
        Ub = U_g[:, :kv].astype(np.float64)
        R = A @ Ub - Ub * ev_g[None, :kv]
        res = float(np.max(np.linalg.norm(R, axis=0))) if kv else 0.0
        orth = float(np.max(np.abs(Ub.T @ Ub - np.eye(kv)))) if kv else 0.0
        if res > res_tol or orth > res_tol:
            return (u, f"residual {res:.3g} orth {orth:.3g}")
        if np.any(Ub.sum(axis=0) < -1e-6):
            return (u, "sign")
        return None

    with ThreadPoolExecutor(THREADS) as ex:
        return [r for r in ex.map(one, users) if r]


PINV_COND_MAX = 1e7   # pinned to 1e-9 cond relative: at most 1e-2 (cond beyond: counted, not pinned)
LS_COND_MAX = 1e13    # full-rank rows pinned to lstsq within 1e-13 cond relative (< 1), beyond: counted


def pin_tol(why, cond, want):
    """Tolerance of a pinned row (pinv_prediction's `why`): the projector / G-mode systems are
    well-conditioned in their own coordinates (1e-9 cond(P_CC)); the full-rank LS rows carry
    ~eps cond(U_CS^T U_CS) on either side (1e-13 cond, 450 eps)."""
    scale = 1e-13 if why == "pinned, full rank (LS)" else 1e-9
    return max(1e-9, scale * max(1.0, cond)) * max(1.0, abs(want))


def _predict_nmax(k):
    """The fast-path system bound of k's predictor bucket (cf_debug_predict_nmax, lmax = 16 ceil(k/16))."""
    from collaborative_filtering_amd import _native
    return int(_native.load().cf_debug_predict_nmax(16 * ((k + 15) // 16)))


def pinv_prediction(U, ev, w_lim, Wu, rat, r, k):
    """The minimum-norm least-squares prediction of an underdetermined row (c < lim), which
    the fast paths return (cf_predict.hip's G-mode for k <= 192, the spill predictor's
    projector block for k > 192): clamp(mean + P_rC P_CC^-1 y_C), P the
    orthogonal projector on U[:, :lim] (basis-free).  Returns (prediction, cond(P_CC), why):
    prediction None when the row is not pinnable, `why` naming the reason -- it takes the
    block-wide path (a column dropped by the zero-column filter, r connected to itself, or for
    k <= 192 a system of d = k - lim rows above the bucket's nmax), where the device factors
    the singular U_CS^T U_CS itself like the reference, or P_CC is worse than PINV_COND_MAX."""
    m = len(ev)
    lim = m
    for j in range(m):
        if ev[j] > w_lim:
            lim = j
            break
    lim = min(max(lim, 2), m)
    C = np.nonzero(Wu[r].astype(np.float64) > 0.1)[0]
    c = len(C)
    if c == 0:
        return None, 0.0, "c = 0"
    if Wu[r, r] > 0.1:
        return None, 0.0, "block-wide: r connected to itself"
    if c >= lim:
        # full rank but ill-conditioned (cond(U_CS^T U_CS) > 1e8): the reference's formula,
        # v_S^T (U_CS^T U_CS)^-1 U_CS^T (r_C - mean) + mean, is the least-squares fit on the
        # rated rows; numpy's SVD-based lstsq is its stable evaluation.  Both sides solve the
        # same system to ~eps cond, so the pin is cond-scaled (LS_COND_MAX bounds it)
        if not np.all(np.any(U[C, :lim] >= 1e-4, axis=0)):
            return None, 0.0, "block-wide: dropped column"
        G = U[np.ix_(C, np.arange(lim))]
        cond = float(np.linalg.cond(G.T @ G))
        if not cond <= LS_COND_MAX:
            return None, cond, "full rank, cond(U_CS^T U_CS) > 1e13"
        mu = float(np.mean(rat[C]))
        x = np.linalg.lstsq(G, rat[C] - mu, rcond=None)[0]
        return min(max(mu + float(U[r, :lim] @ x), 1.0), 5.0), cond, "pinned, full rank (LS)"
    if k <= 192 and k - lim > _predict_nmax(k):
        return None, 0.0, "block-wide: system above nmax"
    if not np.all(np.any(U[C, :lim] >= 1e-4, axis=0)):
        return None, 0.0, "block-wide: dropped column"
    Qn, _ = np.linalg.qr(U[:, :lim])
    P = Qn @ Qn.T
    Pcc = P[np.ix_(C, C)]
    cond = float(np.linalg.cond(Pcc))
    if not cond <= PINV_COND_MAX:
        return None, cond, "cond(P_CC) > 1e7"
    mu = float(np.mean(rat[C]))
    pred = mu + float(P[r, C] @ np.linalg.solve(Pcc, rat[C] - mu))
    return min(max(pred, 1.0), 5.0), cond, "pinned"


def well_conditioned_rows(run: FusedRun, u, want, max_try=160, seed=0, scan=None):
    """Up to `want` rows of user u that the oracle comparison can use: U_CS^T U_CS full rank
    (|S| <= |C|: no more kept columns than connected items) and cond <= 1e8, chosen deliberately
    -- candidates with the fewest kept columns first (the oracle's explicit inverse is O(|S|^3)
    per row) -- instead of sampled at random, where at large k most rows are rank-deficient.
    (S can be far smaller than lim: the zero-column filter drops every column whose entries on
    C are all below 1e-4, and the large users' eigenvectors are localised.)  Returns (rows,
    candidates)."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT

    it, rat, Wu, m, sig_g, ev_g, U_g = run.user(u)
    k = len(it)
    tab = run.sigs[:k] if run.sig_mode == CF_SIGS_COMPAT else sig_g
    ev = ev_g.astype(np.float64)
    lim = np.array([min(max(int(np.searchsorted(ev, float(tab[r]), side="right")), 2), m) for r in range(k)])
    W = np.asarray(Wu, dtype=np.float64)
    U = U_g.astype(np.float64)
    nkeep = np.zeros(k, np.int64)
    nconn = np.zeros(k, np.int64)
    # (scan: a random subset of the rows examined, for the largest users)
    rows_scan = range(k) if scan is None or scan >= k else np.sort(np.random.default_rng(seed).choice(k, scan, replace=False))
    for r in rows_scan:   # the same C and S as gram_cond (local_calc_precomp.cpp:254-304)
        C = np.nonzero(W[r] > 0.1)[0]
        nconn[r] = len(C)
        if len(C):
            nkeep[r] = int((U[C, :lim[r]] >= 1e-4).any(axis=0).sum())
    cand = np.nonzero((nkeep > 0) & (nkeep <= nconn))[0]
    rng = np.random.default_rng(seed)
    cand = cand[np.lexsort((rng.random(len(cand)), nkeep[cand]))]
    n_cand = len(cand)
    cand = cand[:max_try]
    print(f"  user {u}: {n_cand} full-rank candidates of {k} rows, |S| {int(nkeep[cand].min()) if len(cand) else 0}.."
          f"{int(nkeep[cand].max()) if len(cand) else 0}", flush=True)
    loc = np.arange(k, dtype=np.int32)
    rows = []
    for i, r in enumerate(cand):
        if gram_cond(loc, ev, U, float(tab[r]), Wu, int(r)) <= 1e8:
            rows.append(int(r))
            if len(rows) >= want:
                break
        if i % 20 == 19:
            print(f"  user {u}: {i + 1} candidates examined, {len(rows)} well-conditioned", flush=True)
    return np.array(sorted(rows), dtype=np.int64), n_cand


def predict_check_chunked(run: FusedRun, u, rows, st, chunk=4):
    """predict_check on user u's rows a few at a time, printing progress (the oracle's explicit
    inverse per row takes seconds at k > 2000)."""
    good = ill = 0
    bad = []
    for c0 in range(0, len(rows), chunk):
        g, i, b = predict_check(run, [u], rows_of={u: rows[c0:c0 + chunk]}, ill_stats=st)
        good, ill, bad = good + g, ill + i, bad + b
        print(f"  user {u}: rows {c0 + min(chunk, len(rows) - c0)}/{len(rows)} checked", flush=True)
    return good, ill, bad


def lstsq_value_check(run: FusedRun, u, rows):
    """Rows of user u against numpy: kk = |C| exactly, the prediction equal to pinv_prediction's
    least-squares (full rank) or minimum-norm (rank-deficient) evaluation within pin_tol.
    Returns (rows compared by value, mismatches)."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT

    it, rat, Wu, m, sig_g, ev_g, U_g = run.user(u)
    k = len(it)
    b = int(run.off[u])
    tab = run.sigs[:k] if run.sig_mode == CF_SIGS_COMPAT else sig_g
    U = U_g.astype(np.float64)
    ev = ev_g.astype(np.float64)
    compared, bad = 0, []
    for t, r in enumerate(rows):
        g = b + int(r)
        c = int(np.sum(Wu[int(r)].astype(np.float64) > 0.1))
        if int(run.kk[g]) != c:
            bad.append((u, int(r), "kk", int(run.kk[g]), c))
            continue
        want, cond, why = pinv_prediction(U, ev, float(tab[r]), Wu, rat.astype(np.float64), int(r), k)
        if want is None:
            continue
        pg = float(run.pred[g])
        if abs(pg - want) > pin_tol(why, cond, want):
            bad.append((u, int(r), why, pg, want, cond))
        compared += 1
        print(f"  user {u}: row {t + 1}/{len(rows)} ({why}, cond {cond:.2g}) |diff| {abs(pg - want):.2g}", flush=True)
    return compared, bad


def value_rows(run: FusedRun, u, want, seed=0, scan=None):
    """`want` rows of user u for value comparisons: its well-conditioned rows first (the oracle
    comparison), then rows with c > 0 drawn at random (the rank-deficient ones are pinned to
    numpy's minimum-norm least-squares prediction by predict_check)."""
    rows, n_cand = well_conditioned_rows(run, u, want, seed=seed, scan=scan)
    b, k = int(run.off[u]), int(run.k[u])
    rest = np.setdiff1d(np.nonzero(run.kk[b:b + k] > 0)[0], rows)
    rng = np.random.default_rng(seed)
    extra = rng.choice(rest, size=min(len(rest), want - len(rows)), replace=False) if len(rows) < want else []
    print(f"  user {u}: {len(rows)} well-conditioned rows (of {n_cand} full-rank candidates) + {len(extra)} sampled",
          flush=True)
    return np.sort(np.concatenate([rows, np.asarray(extra, dtype=np.int64)])).astype(np.int64)


def predict_check(run: FusedRun, users, max_rows=None, seed=0, ill_stats=None, rows_of=None):
    """Stage-wise a7 parity on the device's own fp32 blocks.  Returns (good, ill, bad).

    Rank-deficient rows (cond(U_CS^T U_CS) > 1e8) are not compared by value -- the reference's
    explicit inverse of a singular Gram returns rounding noise there, this kernel the
    minimum-norm least-squares prediction -- but what is pinnable is: kk exact,
    the device's value finite (c > 0) and clamped into [1, 5]; `ill_stats` (a dict) receives
    the counts of the oracle's NaN rows and of the rows at a clamp bound on either side."""
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT

    compat = run.sig_mode == CF_SIGS_COMPAT
    rng = np.random.default_rng(seed)

    def one(u):
        it, rat, Wu, m, sig_g, ev_g, U_g = run.user(u)
        k = len(it)
        b = int(run.off[u])
        if rows_of is not None:
            rows = rows_of[u]
        else:
            rows = np.arange(k) if max_rows is None or k <= max_rows else \
                np.sort(rng.choice(k, size=max_rows, replace=False))
        tab = run.sigs[:k] if compat else sig_g
        loc = np.arange(k, dtype=np.int32)
        U = U_g.astype(np.float64)
        ev = ev_g.astype(np.float64)
        mse_o, kk_o, pred_o = orc.predict_user(loc, rat.astype(np.float64), ev, U, tab.astype(np.float64), Wu,
                                               rows=rows)
        good = ill = 0
        bad = []
        st = {"ill": 0, "oracle_nan": 0, "oracle_at_bound": 0, "device_at_bound": 0, "both_at_same_bound": 0,
              "pinv_pinned": 0, "pinv_max_err": 0.0}
        for t, r in enumerate(rows):
            g = b + int(r)
            if run.kk[g] != kk_o[t]:
                bad.append((u, int(r), "kk", int(run.kk[g]), int(kk_o[t])))
                continue
            if kk_o[t] == 0:
                if not (np.isnan(run.mse[g]) and np.isnan(mse_o[t])):
                    bad.append((u, int(r), "c=0 not NaN", float(run.mse[g]), float(mse_o[t])))
                continue
            cond = gram_cond(loc, ev, U, float(tab[r]), Wu, int(r))
            if cond <= 1e8:
                if np.isnan(run.mse[g]) or np.isnan(mse_o[t]):
                    bad.append((u, int(r), "nan", float(run.mse[g]), float(mse_o[t]), cond))
                    continue
                good += 1
                if abs(float(run.mse[g]) - float(mse_o[t])) > 1e-6 * max(1.0, float(mse_o[t])):
                    bad.append((u, int(r), "mse", float(run.mse[g]), float(mse_o[t]), cond))
            else:
                ill += 1
                pg, po = float(run.pred[g]), float(pred_o[t])
                if not (np.isfinite(run.mse[g]) and 1.0 <= pg <= 5.0):
                    bad.append((u, int(r), "rank-deficient row not finite / not clamped", float(run.mse[g]), pg))
                want, pcond, why = pinv_prediction(U, ev, float(tab[r]), Wu, rat.astype(np.float64), int(r), k)
                st["why: " + why] = st.get("why: " + why, 0) + 1
                if want is not None:
                    err = abs(pg - want)
                    st["pinv_pinned"] += 1
                    st["pinv_max_err"] = max(st["pinv_max_err"], err)
                    if err > pin_tol(why, pcond, want):
                        bad.append((u, int(r), "rank-deficient row != min-norm LS prediction", pg, want, pcond))
                st["ill"] += 1
                st["oracle_nan"] += int(np.isnan(mse_o[t]))
                ob, gb = po in (1.0, 5.0), pg in (1.0, 5.0)
                st["oracle_at_bound"] += int(ob)
                st["device_at_bound"] += int(gb)
                st["both_at_same_bound"] += int(ob and gb and po == pg)
        return good, ill, bad, st

    with ThreadPoolExecutor(THREADS) as ex:
        res = list(ex.map(one, users))
    if ill_stats is not None:
        for r in res:
            for key, v in r[3].items():
                ill_stats[key] = max(ill_stats.get(key, 0.0), v) if key == "pinv_max_err" else ill_stats.get(key, 0) + v
    return sum(r[0] for r in res), sum(r[1] for r in res), [b for r in res for b in r[2]]


# ------------------------------------------------------------------------------------------
# fixtures: one fused run per config (module scope: built once, shared by its tests)
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def c2_run(gpu_ctx):
    from collaborative_filtering_amd import synth, workloads as wlm
    from collaborative_filtering_amd.api import Context

    torch = _torch()
    cfg = wlm.CONFIGS["c2"]
    d_W, _, _ = wlm.config_graph("c2", Context, 0, torch.device("cuda", 0), torch)
    k = wlm.user_degrees(cfg)
    off, items, rat = synth.user_items(cfg["seed"], k, cfg["items"], threads=THREADS)
    run = FusedRun(gpu_ctx, d_W, cfg["items"], off, items, rat)
    yield run
    run.free()
    del d_W


@pytest.fixture(scope="module")
def c4_graph():
    from collaborative_filtering_amd import workloads as wlm
    from collaborative_filtering_amd.api import Context

    torch = _torch()
    d_W, _, stats = wlm.config_graph("c4", Context, 0, torch.device("cuda", 0), torch)
    yield d_W, stats
    del d_W
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c4_run(gpu_ctx, c4_graph):
    """The whole 1M-user C4 set, as bench.py's default N=1 step."""
    from collaborative_filtering_amd import synth, workloads as wlm

    cfg = wlm.CONFIGS["c4"]
    k = wlm.user_degrees(cfg)
    off, items, rat = synth.user_items(cfg["seed"], k, cfg["items"], threads=THREADS)
    run = FusedRun(gpu_ctx, c4_graph[0], cfg["items"], off, items, rat)
    yield run
    run.free()


def _report(name, good, ill, n_rows, ill_stats=None):
    print(f"{name}: {n_rows} predictions compared, {good} well-conditioned equal, {ill} with cond > 1e8 "
          f"(kk exact, device value finite and clamped; rank-deficient fast-path rows pinned to the "
          f"min-norm prediction, the rest counted by reason)")
    if ill_stats:
        print(f"{name} rank-deficient rows: {ill_stats}")


# ------------------------------------------------------------------------------------------
# C2: 100k users x 10k items
# ------------------------------------------------------------------------------------------
def test_c2_eigen_stratified(c2_run):
    from collaborative_filtering_amd import workloads as wlm

    users = wlm.stratified_users(c2_run.k, 24, seed=2)
    assert len(np.unique((c2_run.k[users] + 15) // 16)) == len(np.unique((c2_run.k + 15) // 16))
    bad = eigen_check(c2_run, users, "C2")
    assert not bad, bad[:10]


def test_c2_eigen_properties(c2_run):
    users = np.random.default_rng(3).choice(len(c2_run.k), size=1000, replace=False)
    bad = eigen_properties(c2_run, users)
    assert not bad, bad[:10]


def test_c2_predict_stagewise(c2_run):
    from collaborative_filtering_amd import workloads as wlm

    users = wlm.stratified_users(c2_run.k, 12, seed=4)
    ist = {}
    good, ill, bad = predict_check(c2_run, users, ill_stats=ist)
    n = int(c2_run.k[users].sum())
    _report("C2", good, ill, n, ist)
    assert not bad, bad[:10]
    assert good >= 0.5 * n, (good, ill, n)
    # whole-set invariants of the timed path: NaN only where c = 0, kk <= k - 1
    kk = c2_run.kk
    kr = np.repeat(c2_run.k, c2_run.k)
    assert np.all((kk >= 0) & (kk <= kr - 1))
    assert np.array_equal(np.isnan(c2_run.mse), kk == 0)


# ------------------------------------------------------------------------------------------
# C4: 1M users x 50k items (the metric's own workload)
# ------------------------------------------------------------------------------------------
def test_c4_graph_is_knn2_output(c4_graph):
    _, stats = c4_graph
    assert stats["knn2_path"] == 1 and stats["edges_w_gt_0.01"] > 10_000_000


def test_c4_eigen_stratified(c4_run):
    from collaborative_filtering_amd import workloads as wlm

    users = wlm.stratified_users(c4_run.k, 24, seed=5)
    bad = eigen_check(c4_run, users, "C4")
    assert not bad, bad[:10]


def test_c4_eigen_properties(c4_run):
    users = np.random.default_rng(6).choice(len(c4_run.k), size=1000, replace=False)
    bad = eigen_properties(c4_run, users)
    assert not bad, bad[:10]


def test_c4_predict_stagewise(c4_run):
    from collaborative_filtering_amd import workloads as wlm

    users = wlm.stratified_users(c4_run.k, 12, seed=7)
    ist = {}
    good, ill, bad = predict_check(c4_run, users, ill_stats=ist)
    n = int(c4_run.k[users].sum())
    _report("C4", good, ill, n, ist)
    assert not bad, bad[:10]
    assert good >= 0.3 * n, (good, ill, n)
    # every rank-deficient / ill-conditioned row is accounted for: pinned to numpy's min-norm
    # prediction, or counted under the reason it is not (block-wide path, cond, full rank)
    whys = {key: v for key, v in ist.items() if key.startswith("why: ")}
    assert sum(whys.values()) == ill, (whys, ill)
    assert ist.get("why: pinned", 0) + ist.get("why: pinned, full rank (LS)", 0) == ist["pinv_pinned"]
    assert ist["pinv_pinned"] >= 0.6 * ill, ist
    kk = c4_run.kk
    kr = np.repeat(c4_run.k, c4_run.k)
    assert np.all((kk >= 0) & (kk <= kr - 1))
    assert np.array_equal(np.isnan(c4_run.mse), kk == 0)
    # wide complements (nc > 62, the block-wide K path) are in the checked sample
    b = np.repeat(np.arange(len(c4_run.k)), c4_run.k)
    sel = np.isin(b, users)
    assert np.sum((kr - kk)[sel] > 62) > 50


# ------------------------------------------------------------------------------------------
# C5: power-law k through the LDS and spill paths, C4's 50k graph
# ------------------------------------------------------------------------------------------
def test_c5_mix_stagewise(gpu_ctx, c4_graph):
    from collaborative_filtering_amd import synth, workloads as wlm
    from collaborative_filtering_amd._native import CF_MAX_K

    k_all = wlm.c5_degrees(3000, kmax=1536)
    rng = np.random.default_rng(8)
    lds = rng.choice(np.nonzero(k_all <= CF_MAX_K)[0], size=40, replace=False)
    mid = np.nonzero((k_all > CF_MAX_K) & (k_all <= 420))[0][:14]
    big = np.nonzero(k_all > 1000)[0][:3]
    assert len(mid) >= 8 and len(big) == 3
    users = np.sort(np.concatenate([lds, mid, big]))
    off_all, items_all, rat_all = synth.user_items(wlm.CONFIGS["c5"]["seed"], k_all, 50_000, threads=THREADS)
    off, items, rat = wlm.sub_csr(off_all, items_all, rat_all, users)
    run = FusedRun(gpu_ctx, c4_graph[0], 50_000, off, items, rat)
    pos = {int(u): i for i, u in enumerate(users)}
    try:
        small = [pos[int(u)] for u in np.concatenate([lds, mid])]
        bad = eigen_check(run, small, "C5")
        assert not bad, bad[:10]
        bad = eigen_properties(run, [pos[int(u)] for u in big])
        assert not bad, bad
        good, ill, badp = predict_check(run, small, max_rows=40, seed=9)
        _report("C5", good, ill, len(small) * 40)
        assert not badp, badp[:10]
        assert good > 200, (good, ill)
    finally:
        run.free()


# ------------------------------------------------------------------------------------------
# C3: knn2 at full size, 20k items x 500k train users
# ------------------------------------------------------------------------------------------
def test_c3_knn2_rows_bit_exact(gpu_ctx):
    from collaborative_filtering_amd import workloads as wlm
    from collaborative_filtering_amd.api import Context

    torch = _torch()
    dev = torch.device("cuda", 0)
    kd, off, items, rats = wlm.c3_population(threads=THREADS)
    n_items = wlm.CONFIGS["c3"]["items"]
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_W = torch.empty(n_items * n_items, dtype=torch.float32, device=dev)
    with Context(0) as kctx:
        kctx.item_cosine_run(len(kd), n_items, T(off.view(np.int64)), T(items.view(np.int32)), T(rats), 1, d_W)
        torch.cuda.synchronize(dev)
        assert kctx.knn2_timing()[2] == 1          # the one-code-plane int8 path
    W = d_W.view(n_items, n_items)
    assert torch.equal(W, W.t())
    rows = np.array([0, 1, 2, 17, 999, 5000, 12345, 19999], dtype=np.int32)   # Zipf head to tail
    Wr = orc.knn2_rows(off.astype(np.int64), items.astype(np.int32), rats.astype(np.float64), n_items, rows)
    Wg = W[torch.from_numpy(rows.astype(np.int64)).to(dev)].cpu().numpy()
    assert np.array_equal(Wg, Wr)
    assert np.count_nonzero(Wg) > 1000
    del d_W, W
    torch.cuda.empty_cache()


def test_c3_knn2_topk_rows_bit_exact(gpu_ctx):
    """The optional top-K cap (cf_set_knn2_topk, `bin/knn2 --topk`; default off) at full C3 size
    (20k items x 500k users): the returned lists of Zipf head-to-tail rows equal a numpy argsort
    of the oracle's weights_calc rows (K largest, ties to the lower id), indices and weights
    bit-exact."""
    from collaborative_filtering_amd import workloads as wlm
    from collaborative_filtering_amd.api import Context

    K = 64
    kd, off, items, rats = wlm.c3_population(threads=THREADS)
    n_items = wlm.CONFIGS["c3"]["items"]
    with Context(0) as kctx:
        eo, col, w = kctx.item_cosine_edges(n_items, off, items, rats, topk=K)
    rows = np.array([0, 1, 2, 17, 999, 5000, 12345, 19999], dtype=np.int32)
    Wr = orc.knn2_rows(off.astype(np.int64), items.astype(np.int32), rats.astype(np.float64), n_items, rows,
                       threads=THREADS)
    capped = 0
    for t, a in enumerate(rows):
        nz = np.nonzero(Wr[t])[0]
        order = np.lexsort((nz, -Wr[t, nz].astype(np.float64)))
        want = np.sort(nz[order[:K]])
        b, e = int(eo[a]), int(eo[a + 1])
        assert np.array_equal(col[b:e], want.astype(np.uint32)), a
        assert np.array_equal(w[b:e], Wr[t, want]), a
        capped += len(nz) > K
    assert capped >= 4   # the cap binds on the head rows
    assert int(eo[-1]) <= K * n_items


def test_c5_tail_k_up_to_5000(gpu_ctx, c4_graph):
    """C5 as specified: its lognormal tail reaches the k = 5000 cap.  Users with k = 2000,
    3100, 4000 and 5000 (Zipf items of the 50k C4 graph) through the timed fused path: the
    fp64 spill solver (k > 3072 in its BIG layout: rc / rs / tau in the HBM slot) and the
    spill predictor (per-user slots).  Size-independent properties at full size on every
    user (residual, orthonormality, sigs, m vs the cut, order, sign); oracle parity at
    k = 2000 (m exact unless at the cut, eigenvalues 1e-5, clustered projectors, residual)
    and stage-wise predictor parity on rows of that user."""
    from collaborative_filtering_amd import synth, workloads as wlm

    ks = np.array([2000, 3100, 4000, 5000], dtype=np.uint32)
    off, items, rat = synth.user_items(wlm.CONFIGS["c5"]["seed"] + 7, ks, 50_000, threads=THREADS)
    run = FusedRun(gpu_ctx, c4_graph[0], 50_000, off, items, rat)
    try:
        assert np.all(run.m[:4] >= 2) and np.all(run.m[:4] <= ks)
        bad = eigen_properties(run, [0, 1, 2, 3])
        assert not bad, bad
        bad = eigen_check(run, [0], "C5 k=2000")
        assert not bad, bad
        kk = run.kk
        kr = np.repeat(run.k, run.k)
        assert np.all((kk >= 0) & (kk <= kr - 1))
        assert np.array_equal(np.isnan(run.mse), kk == 0)
        # Value comparisons on rows of the k = 2000 user: the well-conditioned
        # rows (|S| <= c, cond(U_CS^T U_CS) <= 1e8) against the oracle, found deliberately; on this
        # graph c (~60 connected items) is far below lim on almost every row, so the rest of the
        # sample is rank-deficient and is pinned by value to numpy's minimum-norm least-squares
        # prediction (pinv_prediction) -- the reference's explicit inverse of a singular Gram is
        # rounding noise there.
        r2000 = value_rows(run, 0, 30, seed=10)
        st = {}
        good, ill, badp = predict_check_chunked(run, 0, r2000, st)
        _report("C5 k=2000", good, ill, len(r2000), st)
        assert not badp, badp
        assert good + st.get("pinv_pinned", 0) >= 20, (good, st)
        # k > 3072 (staged multi-CU solver, BIG layout): the eigenvalues against LAPACK's
        # (numpy eigvalsh of the same fp64 sym_lower(L2), the oracle's own pin) to the spill
        # path's 1e-4, and predictor rows of the k = 3100 user against the
        # oracle's neigh_program::apply on the device's blocks
        for u in (1, 2, 3):
            it, _, Wu, m, _, ev_g, _ = run.user(u)
            W = Wu.astype(np.float64)
            d = W.sum(axis=1)
            d[d == 0] = 1.0
            sq = np.sqrt(1.0 / d)
            L2 = (sq[:, None] * (np.diag(d) - W)) * sq[None, :]
            ev_ref = np.linalg.eigvalsh(orc.sym_lower(L2))
            kv = min(m, len(it))
            err = float(np.max(np.abs(ev_g[:kv].astype(np.float64) - ev_ref[:kv])))
            print(f"C5 k={len(it)}: {kv} eigenvalues vs LAPACK eigvalsh, max err {err:.3g}", flush=True)
            assert err <= 1e-4, (len(it), err)
        # predictor rows of the k = 3100 user by value: its well-conditioned rows have |S| ~ 2700
        # (c covers most of the items), where the oracle's explicit inverse takes about a minute a
        # row, so the reference value is the reference's formula evaluated by numpy's lstsq on
        # U_CS (pinv_prediction: the same least-squares fit, cond-scaled tolerance) -- the oracle
        # itself is pinned to that evaluation on the k = 2000 rows above
        r3100 = value_rows(run, 1, 12, seed=11)
        compared, badp = lstsq_value_check(run, 1, r3100)
        print(f"C5 k=3100: {compared} of {len(r3100)} rows equal to numpy's least-squares evaluation", flush=True)
        assert not badp, badp
        assert compared >= 10, compared
    finally:
        run.free()


def test_uncapped_user_above_5000(gpu_ctx, c4_graph):
    """A user with k = 5400 > CF_SPILL_MAX_K, as the reference takes any k
    (precompute_local_threads.cpp:100-213 has no cap): the eigen path's HUGE layout on the
    staged multi-CU solver, and the spill predictor with its per-row arrays in HBM.  Eigen
    properties at full size, the eigenvalues against LAPACK's eigvalsh of the same fp64
    sym_lower(L2), kk of every row exact, NaN iff c = 0, and prediction rows by value against
    numpy's least-squares evaluation of the reference's formula."""
    from collaborative_filtering_amd import synth, workloads as wlm

    ks = np.array([5400], dtype=np.uint32)
    off, items, rat = synth.user_items(wlm.CONFIGS["c5"]["seed"] + 13, ks, 50_000, threads=THREADS)
    run = FusedRun(gpu_ctx, c4_graph[0], 50_000, off, items, rat)
    try:
        assert 2 <= run.m[0] <= ks[0]
        bad = eigen_properties(run, [0])
        assert not bad, bad
        it, _, Wu, m, _, ev_g, _ = run.user(0)
        W = Wu.astype(np.float64)
        d = W.sum(axis=1)
        d[d == 0] = 1.0
        sq = np.sqrt(1.0 / d)
        L2 = (sq[:, None] * (np.diag(d) - W)) * sq[None, :]
        ev_ref = np.linalg.eigvalsh(orc.sym_lower(L2))
        kv = min(m, len(it))
        err = float(np.max(np.abs(ev_g[:kv].astype(np.float64) - ev_ref[:kv])))
        print(f"k = {len(it)}: m = {m}, {kv} eigenvalues vs LAPACK eigvalsh, max err {err:.3g}", flush=True)
        assert err <= 1e-4, err
        kk = run.kk[:len(it)].astype(np.int64)
        c = (W > 0.1).sum(axis=1)
        assert np.array_equal(kk, c), int(np.sum(kk != c))
        assert np.array_equal(np.isnan(run.mse[:len(it)]), kk == 0)
        ok = ~np.isnan(run.mse[:len(it)])
        assert np.all((run.pred[:len(it)][ok] >= 1.0) & (run.pred[:len(it)][ok] <= 5.0))
        rows = value_rows(run, 0, 3, seed=13, scan=400)
        compared, badp = lstsq_value_check(run, 0, rows)
        print(f"k = {len(it)}: {compared} of {len(rows)} rows equal to numpy's least-squares evaluation", flush=True)
        assert not badp, badp
        assert compared >= 2, compared
    finally:
        run.free()


def test_spill_rank_deficient_rows_pinned(gpu_ctx, c4_graph):
    """Spill users (k > 192) on the C4 graph through the timed path: their rank-deficient rows
    (0 < c < lim) return the minimum-norm least-squares prediction -- from the complement basis
    X = [Q | W] as a d x d system when d = k - lim < c (G-mode), else from the c x c projector
    block -- pinned to numpy within 1e-9 max(1, cond(P_CC)) on 40 sampled rows per
    user; full-rank rows whose U_CS^T U_CS is worse than 1e8 (outside the oracle comparison)
    are pinned to numpy's lstsq within 1e-13 cond (pin_tol); the rows that are not pinnable
    are counted by reason."""
    from collaborative_filtering_amd import synth, workloads as wlm

    ks = np.array([260, 480, 900], dtype=np.uint32)
    off, items, rat = synth.user_items(wlm.CONFIGS["c5"]["seed"] + 9, ks, 50_000, threads=THREADS)
    run = FusedRun(gpu_ctx, c4_graph[0], 50_000, off, items, rat)
    rng = np.random.default_rng(3)
    counts, bad, worst = {}, [], 0.0
    try:
        for u in range(len(ks)):
            it, rat_u, Wu, m, sig_u, ev, U = run.user(u)
            k = len(it)
            b = int(off[u])
            tab = run.sigs[:k]   # compat: row i's w_lim is entry i of the concatenated table
            U64 = U.astype(np.float64)
            for r in rng.choice(k, size=40, replace=False):
                r = int(r)
                want, cond, why = pinv_prediction(U64, ev, float(tab[r]), Wu, rat_u.astype(np.float64), r, k)
                if want is None:
                    counts[why] = counts.get(why, 0) + 1
                    continue
                lim = min(max(int(np.argmax(ev > tab[r])) if np.any(ev > tab[r]) else m, 2), m)
                c = int(run.kk[b + r])
                key = why if why == "pinned, full rank (LS)" else \
                    ("pinned, g-mode" if k - lim < c else "pinned, projector block")
                counts[key] = counts.get(key, 0) + 1
                err = abs(float(run.pred[b + r]) - want)
                worst = max(worst, err / max(1.0, cond))
                if err > pin_tol(why, cond, want):
                    bad.append((u, r, float(run.pred[b + r]), want, cond, k - lim, c))
    finally:
        run.free()
    print(f"spill rank-deficient rows: {counts}, max err / cond {worst:.2e}", flush=True)
    assert not bad, bad[:10]
    assert sum(v for key, v in counts.items() if key.startswith("pinned")) >= 30, counts


def test_spill_big_single_workgroup(gpu_ctx, c4_graph):
    """The BIG layout (k > 3072) on one workgroup per user -- the path local_calc's units with
    n > 3072 take, and compute_eigens' with CF_SPILL_MC=0 -- next to the staged multi-CU solver
    the default run uses: the same size-independent properties at k = 3100 and 3400.  The
    switch is read once per process, so the test re-runs itself in a child with it set."""
    if os.environ.get("CF_SPILL_MC") != "0":
        env = dict(os.environ, CF_SPILL_MC="0")
        p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                            f"{os.path.abspath(__file__)}::test_spill_big_single_workgroup"],
                           env=env, capture_output=True, text=True, timeout=900)
        assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
        return
    from collaborative_filtering_amd import synth, workloads as wlm

    ks = np.array([3100, 3400], dtype=np.uint32)
    off, items, rat = synth.user_items(wlm.CONFIGS["c5"]["seed"] + 11, ks, 50_000, threads=THREADS)
    run = FusedRun(gpu_ctx, c4_graph[0], 50_000, off, items, rat)
    try:
        assert np.all(run.m >= 2) and np.all(run.m <= ks)
        bad = eigen_properties(run, [0, 1])
        assert not bad, bad
    finally:
        run.free()
