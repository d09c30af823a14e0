#!/usr/bin/env python3
"""Exit-time crash probe: one LR-TS update launched cooperatively (chunk 64:
several workgroups per agent, hipLaunchCooperativeKernel) or as a plain launch (chunk 0: one
workgroup per agent), then a normal interpreter exit. /proc/self/maps is written at exit so
the PCs of a crash trace (rocprofv3's signal handler prints them unsymbolised) can be mapped
to their libraries.     python tools/archive/exit_probe.py coop|plain OUTDIR
"""
import atexit
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "tests")]
mode, outdir = sys.argv[1], sys.argv[2]
os.makedirs(outdir, exist_ok=True)
atexit.register(lambda: shutil.copyfile("/proc/self/maps", os.path.join(outdir, f"maps_{mode}.txt")))

import test_gpu_parity as T  # noqa: E402

kat, m0, q0, pm0 = T._kat_population()
eng = T._lrts_engine()
eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
eng.set_lrts_block_samples(64 if mode == "coop" else 0)
st = T._fill_store(eng, {a: (kat[f"a{a}_X"], kat[f"a{a}_A"], kat[f"a{a}_y"]) for a in range(6)})
print(mode, "epochs", eng.lrts_update(st), flush=True)
eng.close()
