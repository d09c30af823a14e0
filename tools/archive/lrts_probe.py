"""Run one LR-TS update on the KAT population (optionally spread over cooperating
workgroups) -- a small command for profiler checks."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "tests")]
import test_gpu_parity as T  # noqa: E402

chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 0
kat, m0, q0, pm0 = T._kat_population()
eng = T._lrts_engine()
eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
eng.set_lrts_block_samples(chunk)
st = T._fill_store(eng, {a: (kat[f"a{a}_X"], kat[f"a{a}_A"], kat[f"a{a}_y"]) for a in range(6)})
print("epochs", eng.lrts_update(st))
eng.close()
