import ctypes, sys
sys.path.insert(0, "auction-gym_amd")
from auctiongym_amd import _lib
L = _lib.load()
t = ctypes.c_int64(0); bad = ctypes.c_int64(0)
for seed in (1, 2, 3):
    _lib.check(L.ag_div_selftest(0, 1 << 31, seed, ctypes.byref(t), ctypes.byref(bad)), "ag_div_selftest", L)
    print("seed", seed, "tested", t.value, "mismatches", bad.value, flush=True)
