"""Multi-GPU product path on the GPU box: cf_eigen_batch_multi over several
contexts (on a one-GPU box they share device 0, the peer copies degenerate to local copies,
the code path is the same), cf_pack_eigen_run, and bin/precompute_local --devices N, whose
out_eigen_ must be byte-identical to the one-device file (precompute_local_threads.cpp:300-314
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
    for n_dev in (1, 2, 4):
        out = f"out_eigen_d{n_dev}"
        log = _run(wd, "precompute_local", "8", "--devices", str(n_dev), "--output", out, "--format", fmt)
        if n_dev > 1:
            assert log.count("device part") == n_dev
        outs[n_dev] = open(os.path.join(wd, out), "rb").read()
    assert len(outs[1]) > 1000
    assert outs[2] == outs[1] and outs[4] == outs[1]
