"""Child process of test_gpu_local.py::test_spill_huge_layout_bit_identical: runs the staged
spill cases under the environment it was started with (CF_SPILL_HUGE_MIN / CF_SPILL_HUGE_DE,
read once per process by libcf_mi355x) and saves every output to the .npz named on the
command line.  usage: spill_layout_child.py OUT.npz"""
import os
import sys

import numpy as np

TESTS = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(TESTS))
sys.path.insert(0, TESTS)

from test_gpu_local import mc_cut_case, staged_user_case  # noqa: E402


def run_cases(ctx):
    """Both staged cases on one context: local_calc's two n ~ 1650 units (modes 1 and 3 of the
    spill solver) and three compute_eigens users with k > 1536 (mode 0) on the same graph."""
    G, moff, mitems, toff, tuser, trat, _ = mc_cut_case()
    ctx.upload_graph_dense(G)
    mse, kk, pred, wlim, lim = ctx.local_calc(moff, mitems, toff, tuser, trat)
    off, items = staged_user_case(G)
    r = ctx.eigen_batch(off, items)
    return dict(mse=mse, kk=kk, pred=pred, wlim=wlim, lim=lim, m=r.m, sigs=r.sigs, evals=r.evals, evecs=r.evecs)


if __name__ == "__main__":
    from collaborative_filtering_amd.api import Context

    ctx = Context(0)
    out = run_cases(ctx)
    ctx.close()
    np.savez(sys.argv[1], **out)
    print("child done", {k: v.shape for k, v in out.items()}, flush=True)
