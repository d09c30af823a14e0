"""Stress test of the learners' cross-workgroup exact sums (ag_coop.h: the combining-tree
all-reduce k_lrts_train, k_bidder_train, the pipe and the per-epoch kernels run every epoch).
The built form hands partial sums between workgroups through relaxed agent-scope atomics
ordered by s_waitcnt + workgroup barriers (no fences); ag_coop_selftest runs thousands of
generations of interleaved sums over workgroups on every XCD and counts the totals that differ
from their closed form. The fenced form is the A/B build (make variant VFLAGS=-DAG_COOP_FENCED=1).
No reference counterpart: the reference sums on one CPU thread (torch), src/Models.py."""
import ctypes
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "auction-gym_amd")
# the stress run in a child process of its own, under a time limit: a lost hand-off in the
# fence-free tree shows up as a workgroup spinning forever, which must fail this test, not hang
# the suite
_CHILD = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from auctiongym_amd import _lib
L = _lib.load()
bad = ctypes.c_int64(-1)
_lib.check(L.ag_coop_selftest(0, int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), ctypes.byref(bad)),
           "ag_coop_selftest", L)
print("WRONG_TOTALS", bad.value, flush=True)
"""


@pytest.mark.parametrize("workgroups,generations,regions", [(0, 4000, 1), (0, 2000, 3), (1024, 1000, 4), (2, 5000, 2),
                                                            (0, 4000, 0), (1024, 2000, 0), (2, 5000, 0), (17, 5000, 0)])
def test_combining_tree_sums_exact_under_stress(gpu, workgroups, generations, regions):
    try:
        r = subprocess.run([sys.executable, "-c", _CHILD, PKG, str(workgroups), str(generations), str(regions)],
                           capture_output=True, text=True, timeout=90)
    except subprocess.TimeoutExpired:
        pytest.fail("ag_coop_selftest did not finish in 90 s: a combining-tree hand-off was lost (spin)")
    assert r.returncode == 0, r.stderr[-3000:]
    assert "WRONG_TOTALS 0" in r.stdout, r.stdout


def test_selftest_refuses_bad_arguments(gpu):
    from auctiongym_amd import _lib
    L = _lib.load()
    bad = ctypes.c_int64(-1)
    assert L.ag_coop_selftest(0, 0, 10, 5, ctypes.byref(bad)) != 0  # regions > 4
    assert L.ag_coop_selftest(0, 0, 10, -1, ctypes.byref(bad)) != 0
    assert L.ag_coop_selftest(0, 1 << 20, 10, 1, ctypes.byref(bad)) != 0  # not co-resident
    assert L.ag_coop_selftest(0, 0, 10, 1, None) != 0
