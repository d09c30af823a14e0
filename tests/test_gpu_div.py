"""The learners' split FP64 division (csrc/ag_div.h): the BCE rows and policy fits divide by
1 + e, sigma and the logged propensity through one shared reciprocal each, the compiler's IEEE
division sequence without its scaling and fixup steps. ag_div_selftest divides random operand
pairs in the split form's range both ways on the device and counts the results whose bits
differ from `a / b` (the trainers' bit-exactness against the oracle rests on it; the trainer
parity tests in test_gpu_parity.py check the fits themselves). No reference counterpart."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 12345])
def test_split_division_equals_ieee_division(gpu, seed):
    from auctiongym_amd import _lib
    L = _lib.load()
    tested, bad = ctypes.c_int64(-1), ctypes.c_int64(-1)
    _lib.check(L.ag_div_selftest(0, 1 << 30, seed, ctypes.byref(tested), ctypes.byref(bad)), "ag_div_selftest", L)
    assert tested.value > (1 << 29)  # most pairs fall in the range
    assert bad.value == 0


def test_div_selftest_refuses_bad_arguments(gpu):
    from auctiongym_amd import _lib
    L = _lib.load()
    t = ctypes.c_int64(0)
    assert L.ag_div_selftest(0, 10, 1, ctypes.byref(t), None) != 0
    assert L.ag_div_selftest(0, -1, 1, ctypes.byref(t), ctypes.byref(t)) != 0
