"""cf_step_run (eigen + predictor with per-bucket overlap on separate streams) writes exactly
what cf_eigen_run followed by cf_predict_run_f32 writes: same kernels, same inputs, only the
launch order across streams differs.  Both w_lim modes; users in every LDS bucket plus spill
users (k > 192) so the spill eigen / predictor run inside the fused schedule too."""
import numpy as np
import pytest

from collaborative_filtering_amd import synth
from collaborative_filtering_amd.api import CF_SIGS_COMPAT, CF_SIGS_OWN, evec_offsets

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sig_mode", [CF_SIGS_COMPAT, CF_SIGS_OWN])
def test_step_run_equals_sequential(gpu_ctx, sig_mode):
    torch = pytest.importorskip("torch")
    seed, n_items = 2026101502, 2000
    k = synth.degrees(seed, 6000, k_median=90.0, sigma=0.6, kmin=2, kmax=180)
    k[[5, 777, 4000]] = [260, 201, 230]          # spill users
    off, items, rats = synth.user_items(seed, k, n_items, threads=8)
    W = synth.graph_model(seed, n_items, threads=8)
    gpu_ctx.upload_graph_dense(W)
    plan = gpu_ctx.plan(off)
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eoff, ne = evec_offsets(off)
    n, U = int(off[-1]), len(k)

    def fresh():
        return dict(m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
                    evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
                    mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev),
                    pred=torch.zeros(n, dtype=torch.float64, device=dev))

    d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))
    a, b = fresh(), fresh()
    plan.eigen_run(d_off, d_items, d_eoff, a["m"], a["sigs"], a["evals"], a["evecs"])
    plan.predict_run(d_off, d_items, d_rat, a["m"], a["evals"], d_eoff, a["evecs"], a["sigs"], sig_mode,
                     a["mse"], a["kk"], a["pred"])
    plan.step_run(d_off, d_items, d_rat, d_eoff, b["m"], b["sigs"], b["evals"], b["evecs"], sig_mode,
                  b["mse"], b["kk"], b["pred"])
    eig_ms, tot_ms = plan.step_timing()
    torch.cuda.synchronize()
    assert 0 < eig_ms <= tot_ms
    for key in a:
        x, y = a[key].cpu().numpy(), b[key].cpu().numpy()
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), key   # bitwise, NaNs included
    plan.close()


def test_pipeline_is_deterministic(gpu_ctx):
    """Three runs of cf_eigen_run -> cf_predict_run_f32 on fresh buffers write the same bits.
    (A barrier race in the predictor's basis kernel once corrupted ~0.1% of the k >= 100 users
    differently from run to run; this would have caught it.)"""
    torch = pytest.importorskip("torch")
    seed, n_items = 2026101502, 2000
    k = synth.degrees(seed, 6000, k_median=90.0, sigma=0.6, kmin=2, kmax=180)
    k[[11, 1234, 5000]] = [240, 199, 310]          # spill users (persistent-workgroup kernels)
    off, items, rats = synth.user_items(seed, k, n_items, threads=8)
    gpu_ctx.upload_graph_dense(synth.graph_model(seed, n_items, threads=8))
    plan = gpu_ctx.plan(off)
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eoff, ne = evec_offsets(off)
    n, U = int(off[-1]), len(k)
    d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))
    runs = []
    for _ in range(3):
        o = dict(m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
                 evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev),
                 mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev))
        plan.eigen_run(d_off, d_items, d_eoff, o["m"], o["sigs"], o["evals"], o["evecs"])
        plan.predict_run(d_off, d_items, d_rat, o["m"], o["evals"], d_eoff, o["evecs"], o["sigs"], CF_SIGS_OWN,
                         o["mse"], o["kk"])
        torch.cuda.synchronize()
        runs.append({key: v.cpu().numpy() for key, v in o.items()})
    for r in runs[1:]:
        for key in r:
            assert np.array_equal(r[key].view(np.uint8), runs[0][key].view(np.uint8)), key
    plan.close()


def test_fused_predictor_equals_two_kernel_path():
    """pred_fused_kernel (CF_PRED_FUSED=1: basis and ratings of a user in one persistent
    workgroup, one slot per resident workgroup) writes the same bits as the default chunked
    two-kernel path: with the switch set, cf_predict_run takes the fused kernel while
    cf_step_run keeps the two kernels, so test_step_run_equals_sequential compares them
    bitwise.  The switch is read once per process, hence the child."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, CF_PRED_FUSED="1")
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu",
                        f"{os.path.abspath(__file__)}::test_step_run_equals_sequential"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert "2 passed" in p.stdout, p.stdout[-2000:]


def test_mask_handoff_bit_identical_and_invalidated(gpu_ctx):
    """The complement masks the eigen kernel hands to the predictor (cf_set_step_masks) give the
    same bits as the predictor's own graph gather; a graph reload or another item array makes the
    predictor gather again (a stale mask set would change the connected sets)."""
    torch = pytest.importorskip("torch")
    seed, n_items = 2026101503, 1500
    k = synth.degrees(seed, 3000, k_median=80.0, sigma=0.6, kmin=2, kmax=192)
    k[[3, 2000]] = [250, 205]          # spill users (no masks on their path)
    off, items, rats = synth.user_items(seed, k, n_items, threads=8)
    W = synth.graph_model(seed, n_items, threads=8)
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eoff, ne = evec_offsets(off)
    n, U = int(off[-1]), len(k)
    d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))
    plan = gpu_ctx.plan(off)

    def run(masks, eigen=True, rec=None):
        gpu_ctx.set_step_masks(masks)
        o = {key: rec[key] for key in ("m", "sigs", "evals", "evecs")} if rec else dict(
            m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
            evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev))
        if eigen:
            plan.eigen_run(d_off, d_items, d_eoff, o["m"], o["sigs"], o["evals"], o["evecs"])
        o["mse"] = torch.zeros(n, device=dev)
        o["kk"] = torch.zeros(n, dtype=torch.int32, device=dev)
        o["pred"] = torch.zeros(n, dtype=torch.float64, device=dev)
        plan.predict_run(d_off, d_items, d_rat, o["m"], o["evals"], d_eoff, o["evecs"], o["sigs"], CF_SIGS_COMPAT,
                         o["mse"], o["kk"], o["pred"])
        torch.cuda.synchronize()
        return o

    def same(x, y):
        for key in ("mse", "kk", "pred"):
            a, b = x[key].cpu().numpy(), y[key].cpu().numpy()
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), key

    try:
        for layout in ("dense", "csr"):
            gpu_ctx.set_graph_layout(layout)
            gpu_ctx.upload_graph_dense(W)
            with_masks = run(True)
            same(with_masks, run(False, eigen=False, rec=with_masks))
            # another graph: the masks of the eigen run above must not be used
            W2 = W.copy()
            W2[W2 > 0] = np.where(np.random.default_rng(1).random(int((W2 > 0).sum())) < 0.5, 0.05, 0.9)
            gpu_ctx.upload_graph_dense(W2)
            gpu_ctx.set_step_masks(True)
            stale = run(True, eigen=False, rec=with_masks)
            same(stale, run(False, eigen=False, rec=with_masks))
    finally:
        gpu_ctx.set_step_masks(True)
        gpu_ctx.set_graph_layout("dense")
        plan.close()


def test_mask_handoff_items_rewritten_in_place(gpu_ctx):
    """the mask handoff is keyed by plan, graph generation and the item-array
    pointers, so a caller that rewrites d_items IN PLACE between eigen_run and predict_run
    keeps every key.  The eigen kernel stores a fingerprint of each user's (offset, k, items)
    beside the masks and the basis kernel recomputes it from the arrays it is handed: rewritten
    users must gather the graph themselves, so the predictions equal a masks-off run on the
    new items bit for bit."""
    torch = pytest.importorskip("torch")
    seed, n_items = 2026101507, 1500
    k = synth.degrees(seed, 2000, k_median=80.0, sigma=0.6, kmin=2, kmax=192)
    off, items, rats = synth.user_items(seed, k, n_items, threads=8)
    W = synth.graph_model(seed, n_items, threads=8)
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    eoff, ne = evec_offsets(off)
    n, U = int(off[-1]), len(k)
    d_off, d_items, d_rat, d_eoff = T(off.view(np.int64)), T(items.view(np.int32)), T(rats), T(eoff.view(np.int64))
    plan = gpu_ctx.plan(off)
    rec = dict(m=torch.zeros(U, dtype=torch.int32, device=dev), sigs=torch.zeros(n, device=dev),
               evals=torch.zeros(n, device=dev), evecs=torch.zeros(ne, device=dev))

    def predict(masks):
        gpu_ctx.set_step_masks(masks)
        o = dict(mse=torch.zeros(n, device=dev), kk=torch.zeros(n, dtype=torch.int32, device=dev),
                 pred=torch.zeros(n, dtype=torch.float64, device=dev))
        plan.predict_run(d_off, d_items, d_rat, rec["m"], rec["evals"], d_eoff, rec["evecs"], rec["sigs"],
                         CF_SIGS_COMPAT, o["mse"], o["kk"], o["pred"])
        torch.cuda.synchronize()
        return {key: v.cpu().numpy() for key, v in o.items()}

    try:
        gpu_ctx.upload_graph_dense(W)
        gpu_ctx.set_step_masks(True)
        plan.eigen_run(d_off, d_items, d_eoff, rec["m"], rec["sigs"], rec["evals"], rec["evecs"])
        torch.cuda.synchronize()
        # rewrite every other user's items in place (new ascending sets, same k, same pointers)
        rng = np.random.default_rng(5)
        items2 = items.copy()
        for u in range(0, U, 2):
            b, e = int(off[u]), int(off[u + 1])
            items2[b:e] = np.sort(rng.choice(n_items, size=e - b, replace=False)).astype(np.uint32)
        d_items.copy_(T(items2.view(np.int32)))
        torch.cuda.synchronize()
        handed = predict(True)      # keys still match: the fingerprints must reject the rewritten users
        gathered = predict(False)   # the predictor's own graph gather on the new items
        for key in ("mse", "kk", "pred"):
            assert np.array_equal(handed[key].view(np.uint8), gathered[key].view(np.uint8)), key
        assert not np.array_equal(items, items2)
    finally:
        gpu_ctx.set_step_masks(True)
        plan.close()
