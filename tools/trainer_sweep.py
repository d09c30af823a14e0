#!/usr/bin/env python3
"""Learning bidders' update (ag_bidder_update) at a BASELINE config's scale for several
records-per-workgroup settings: time, epochs, and whether the fitted models are bit-identical
to the first setting's (they must be: the win-rate / imitation / DR / DM fits use exact sums).

    python tools/trainer_sweep.py configs_2 8192 4096 2048
    python tools/trainer_sweep.py configs_2:65536 256 1073741824   (2^16 auctions per step)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "auction-gym_amd")]
import bench  # noqa: E402


def one(key, chunk, batch=0):
    eng, what, B, ak, bk, st16, dims = bench.build_population(key, 0)
    B = batch or B
    N, P = dims["N"], dims["P"]
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    eng.generate_noise(0, 0, inp)
    out = eng.alloc_outputs(B)
    eng.simulate(inp, out, eng.new_counters())
    sst = eng.new_shading_samples(B * P, learning=True)
    eng.shading_collect(inp, out, sst, first_auction=0)
    if chunk:
        eng.set_bidder_block_samples(chunk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ep, stat = eng.bidder_update(sst, None, np.zeros(N, np.int64), 0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    state, init = eng.dr_state()
    learners = np.nonzero(bk >= 2)[0]
    eng.close()
    return ms, [[int(x) for x in ep[a]] for a in learners[:4]], np.asarray(state)[learners].copy()


def main():
    args = sys.argv[1:]
    if args[0].startswith("--lib="):  # an A/B build: make variant NAME=x -> --lib=x
        from auctiongym_amd import _lib
        _lib.LIB_PATH = os.path.join(ROOT, "auction-gym_amd", "build", "variants",
                                     f"libauctiongym_hip_{args.pop(0)[6:]}.so")
    sys.argv[1:] = args
    key = sys.argv[1]
    batch = 0
    if key.count(":"):
        key, batch = key.split(":")[0], int(key.split(":")[1])
    chunks = [int(c) for c in sys.argv[2:]] or [0]
    ref = None
    for c in chunks:
        ms, ep, state = one(key, c, batch)
        same = None if ref is None else bool(np.array_equal(state.view(np.uint32), ref.view(np.uint32)))
        if ref is None:
            ref = state
        longest = max(sum(e) for e in ep)  # the agents train concurrently
        print(f"{key} chunk={c} update_ms={ms:.1f} epochs={ep} us_per_epoch={ms * 1e3 / max(1, longest):.1f}"
              f" same_as_first={same}", flush=True)


if __name__ == "__main__":
    main()
