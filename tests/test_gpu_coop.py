"""Stress test of the learners' cross-workgroup exact sums (ag_coop.h: the combining-tree
all-reduce k_lrts_train, k_bidder_train, the pipe and the per-epoch kernels run every epoch).
The built form hands partial sums between workgroups through relaxed agent-scope atomics
ordered by s_waitcnt + workgroup barriers (no fences); ag_coop_selftest runs thousands of
generations of interleaved sums over workgroups on every XCD and counts the totals that differ
from their closed form. The fenced form is the A/B build (make variant VFLAGS=-DAG_COOP_FENCED=1).
No reference counterpart: the reference sums on one CPU thread (torch), src/Models.py."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("workgroups,generations,regions", [(0, 4000, 1), (0, 2000, 3), (1024, 1000, 4), (2, 5000, 2)])
def test_combining_tree_sums_exact_under_stress(gpu, workgroups, generations, regions):
    from auctiongym_amd import _lib
    L = _lib.load()
    bad = ctypes.c_int64(-1)
    _lib.check(L.ag_coop_selftest(0, workgroups, generations, regions, ctypes.byref(bad)), "ag_coop_selftest", L)
    assert bad.value == 0


def test_selftest_refuses_bad_arguments(gpu):
    from auctiongym_amd import _lib
    L = _lib.load()
    bad = ctypes.c_int64(-1)
    assert L.ag_coop_selftest(0, 0, 10, 5, ctypes.byref(bad)) != 0  # regions > 4
    assert L.ag_coop_selftest(0, 1 << 20, 10, 1, ctypes.byref(bad)) != 0  # not co-resident
    assert L.ag_coop_selftest(0, 0, 10, 1, None) != 0
