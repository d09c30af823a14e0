#!/usr/bin/env python3
"""A/B of the two simulate kernels on the bench workload (SP_Oracle shape, 2^24 auctions):
the dedicated k_oracle (default) vs the general k_simulate, interleaved in ONE process after
the clock ramp (tools/warm_probe.py); HIP events on the launch stream. Diagnostic only.

    python tools/ab_oracle.py [B]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    items, values = bench.catalogue()
    eng = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    fields = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    out = {False: eng.alloc_outputs(B, fields), True: eng.alloc_outputs(B, fields)}
    cnt = {False: eng.new_counters(), True: eng.new_counters()}
    st = torch.cuda.current_stream()
    for _ in range(150):
        eng.simulate(inp, out[False], cnt[False])
    for g in (False, True):
        eng.set_simulate_kernel(g)
        cnt[g].zero_()
        eng.simulate(inp, out[g], cnt[g])
    torch.cuda.synchronize()
    same = all(torch.equal(out[False][k], out[True][k]) for k in fields) and torch.equal(cnt[False], cnt[True])
    print("outputs and counters identical:", same, flush=True)
    iso = {False: [], True: []}
    sus = {False: [], True: []}
    for r in range(12):
        for g in (False, True):
            eng.set_simulate_kernel(g)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            eng.simulate(inp, out[g], cnt[g])
            b.record(st)
            torch.cuda.synchronize()
            iso[g].append(a.elapsed_time(b))
            a.record(st)
            for _ in range(20):
                cnt[g].zero_()
                eng.simulate(inp, out[g], cnt[g])
            b.record(st)
            torch.cuda.synchronize()
            sus[g].append(a.elapsed_time(b) / 20)
    bpa = bench.algorithmic_bytes_per_auction(5, 2, False)
    for g, name in ((False, "k_oracle"), (True, "k_simulate (general)")):
        mi, ms = float(np.median(iso[g])), float(np.median(sus[g]))
        print(f"{name:22s} isolated {mi:.4f} ms ({bpa * B / mi / 1e6:6.0f} GB/s)  "
              f"back-to-back (+counter zeroing) {ms:.4f} ms ({bpa * B / ms / 1e6:6.0f} GB/s)")


if __name__ == "__main__":
    main()
