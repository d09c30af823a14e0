#!/usr/bin/env python3
"""A/B of the LR-TS update's split (AG_OPT_LRTS_BLOCK_SAMPLES: samples per cooperating
workgroup) on configs[1]'s won samples (bench.build_sp_ts, one simulate step), in ONE process,
interleaved; the posteriors must be bit-identical across splits. Diagnostic.

    python tools/archive/ab_lrts.py [chunk ...]     (0 = the default split)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "auction-gym_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    chunks = [int(x) for x in sys.argv[1:]] or [0, 2048, 1024]
    eng, inp, out, cnt, dims = bench.build_sp_ts(1 << 20, 0)
    eng.simulate(inp, out, cnt)
    st = eng.new_lrts_samples(1 << 20)
    eng.lrts_collect(inp, out, st)
    torch.cuda.synchronize()
    m0, q0, pm0 = (np.array(x) for x in eng.lrts_state())
    res, ref = {c: [] for c in chunks}, None
    for rep in range(3):
        for c in chunks:
            eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
            eng.set_lrts_block_samples(c)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ep = eng.lrts_update(st)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            state = [np.array(x) for x in eng.lrts_state()]
            if ref is None:
                ref = state
            same = all(np.array_equal(a, b) for a, b in zip(state, ref))
            res[c].append(ms)
            print(f"chunk {c} rep {rep}: {ms:.1f} ms epochs {list(ep)} same={same}", flush=True)
    for c, t in res.items():
        print(f"chunk {c}: min {min(t):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
