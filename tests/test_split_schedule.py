"""CPU: the split-storage Jacobi's sweep schedule (cf_eigen_split.hip) for every k it takes.

cf_debug_split_schedule builds the schedule the kernel reads and replays it on column labels:
every pair of columns meets exactly once per sweep, no traveling column is used twice in a step,
no two lane groups touch one LDS slot in a level change, and the end-of-sweep layout is the
recorded one.  The step count must equal the recursive-halving ordering's of cf_eigen.hip
(sum over levels of ceil(ceil(k / 2^L) / 2)), so a sweep costs the same number of barriers.
"""
import ctypes

import pytest

from collaborative_filtering_amd import _native

# bucket emax -> (lane groups, LDS slots, smallest k, largest k)
GEOM = {5: (40, 40, 65, 80), 6: (48, 48, 81, 96), 7: (56, 56, 97, 112), 8: (64, 64, 113, 128),
        9: (72, 72, 129, 144), 10: (80, 80, 145, 160), 11: (88, 88, 161, 176), 12: (96, 90, 177, 180)}


def _full_steps(k):
    steps, L = 0, 0
    while True:
        seg = (k + (1 << L) - 1) >> L
        if seg < 2:
            return steps
        steps += (seg + 1) >> 1
        L += 1


@pytest.mark.parametrize("emax", sorted(GEOM))
def test_split_schedule_every_k(emax):
    lib = _native.load()
    ng, ns, klo, khi = GEOM[emax]
    for k in range(klo, khi + 1):
        st, lv, mg, ms = (ctypes.c_int() for _ in range(4))
        rc = lib.cf_debug_split_schedule(emax, k, ctypes.byref(st), ctypes.byref(lv), ctypes.byref(mg), ctypes.byref(ms))
        assert rc == 0, (emax, k)
        assert st.value == _full_steps(k), (emax, k, st.value)
        assert mg.value <= ng and ms.value <= ns, (emax, k, mg.value, ms.value)
        assert lv.value <= 9


def test_split_schedule_out_of_range():
    lib = _native.load()
    z = ctypes.c_int()
    assert lib.cf_debug_split_schedule(12, 181, ctypes.byref(z), ctypes.byref(z), ctypes.byref(z), ctypes.byref(z)) != 0
    assert lib.cf_debug_split_schedule(4, 60, ctypes.byref(z), ctypes.byref(z), ctypes.byref(z), ctypes.byref(z)) != 0
