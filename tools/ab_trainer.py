#!/usr/bin/env python3
"""A/B of the learning bidders' update (ag_bidder_update) between library builds, in ONE
process, interleaved: the same population line, the same records, the same synthetic noise;
the fitted models must be bit-identical across builds.

    python tools/ab_trainer.py configs_2 r02 [more variants...]   (build/variants/*.so)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "tools")]
from auctiongym_amd import _lib  # noqa: E402
import trainer_sweep  # noqa: E402


def main():
    key = sys.argv[1]
    vdir = os.path.join(ROOT, "auction-gym_amd", "build", "variants")
    paths = {"base": _lib.LIB_PATH}
    for n in sys.argv[2:]:
        paths[n] = os.path.join(vdir, f"libauctiongym_hip_{n}.so")
    base = _lib.LIB_PATH
    res = {n: [] for n in paths}
    ref = None
    for rep in range(2):
        for n, p in paths.items():
            _lib.LIB_PATH = p
            ms, ep, state = trainer_sweep.one(key, 0)
            _lib.LIB_PATH = base
            if ref is None:
                ref = state
            same = bool(np.array_equal(state.view(np.uint32), ref.view(np.uint32)))
            res[n].append(ms)
            print(f"{key} {n} rep {rep}: update_ms={ms:.1f} epochs={ep} same_as_base={same}", flush=True)
    for n, t in res.items():
        print(f"{key} {n}: min update_ms {min(t):.1f}", flush=True)


if __name__ == "__main__":
    main()
