#!/usr/bin/env python3
"""Fixed vs per-auction cost of the simulate path: ag_simulate of one population line
(configs_1..4, as tools/ab_pop.py builds them) at several batch sizes, HIP-event medians;
run under rocprofv3 --kernel-trace for the per-kernel split.
    python tools/archive/size_sweep.py configs_1 [fused|generic]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402


def build(key):
    if key == "configs_1":
        from auctiongym_amd.engine import AuctionEngine
        items, values = bench.catalogue(bench.SP_TS)
        N, K, D = items.shape
        OE = bench.SP_TS["obs_embedding_size"]
        eng = AuctionEngine(N, 2, K, D - 1, OE, _lib.SECOND_PRICE, 1.0, device=0)
        eng.set_agent_params(np.ones(N, np.int32), np.zeros(N, np.int32))
        eng.load_catalog(items, values)
        g = torch.Generator().manual_seed(0)
        m = torch.empty(N, K, OE + 1)
        for a in range(N):
            m[a].normal_(0.0, 1.0, generator=g)
        eng.load_lrts(m.numpy(), np.ones((N, K, OE + 1), np.float32), thompson_sampling=True)
        return eng, np.ones(N, np.int32)
    eng, what, B, ak, bk, st16, dims = bench.build_population(key, 0)
    eng.set_dr_state(st16, np.where(bk >= 2, 1, 0).astype(np.int32))
    return eng, ak


def main():
    key = sys.argv[1]
    mode = sys.argv[2] if len(sys.argv) > 2 else None
    eng, ak = build(key)
    if mode:
        eng.set_simulate_kernel(True if mode == "generic" else mode)
    compact = bool((ak == 1).any() and (ak != 1).any())
    for B in (1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 22):
        inp = eng.alloc_inputs(B)
        eng.generate(1, 0, inp)
        eng.generate_noise(1, 0, inp, compact=compact)
        out = eng.alloc_outputs(B)
        cnt = eng.new_counters()
        for _ in range(10):
            eng.simulate(inp, out, cnt)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.simulate(inp, out, cnt)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(f"{key} {mode or 'auto'} B={B}: median {np.median(ts) * 1e3:.1f} us  "
              f"({np.median(ts) * 1e6 / B:.3f} ns/auction)", flush=True)
        del inp, out


if __name__ == "__main__":
    main()
