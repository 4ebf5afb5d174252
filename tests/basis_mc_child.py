"""Child process of test_gpu_predict.py::test_spill_basis_mc_bit_identical: eigen + prediction of
the case below under the environment it was started with (CF_PSPILL_BASIS_MC, read once per
process by libcf_mi355x) and every output saved to the .npz named on the command line.
usage: basis_mc_child.py OUT.npz"""
import os
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(TESTS))
sys.path.insert(0, TESTS)

import cases  # noqa: E402


def basis_mc_case():
    """Users with k > 2816 (spill_basis_mc) beside smaller spill users in the same chunk (the
    one-workgroup basis kernel), on a 3400-item graph dense enough for wide complements."""
    W = cases.item_graph(3400, 0.35, seed=61)
    off, items = cases.user_items(3400, [3300, 2950, 900, 300], seed=62)
    rat = (np.random.default_rng(63).integers(1, 6, size=int(off[-1]))).astype(np.float32)
    return W, off, items, rat


def run_case(ctx):
    from collaborative_filtering_amd.api import CF_SIGS_COMPAT

    W, off, items, rat = basis_mc_case()
    ctx.upload_graph_dense(W)
    res = ctx.eigen_batch(off, items)
    mse, kk, pred = ctx.predict_precomp(off, items, rat, res.m, res.evals.astype(np.float64), res.evec_off,
                                        res.evecs, res.sigs.astype(np.float64), sig_mode=CF_SIGS_COMPAT,
                                        want_pred=True)
    return dict(m=res.m, mse=mse, kk=kk, pred=pred)


if __name__ == "__main__":
    from collaborative_filtering_amd.api import Context

    ctx = Context(0)
    out = run_case(ctx)
    ctx.close()
    np.savez(sys.argv[1], **out)
    print("child done", {k: v.shape for k, v in out.items()}, flush=True)
