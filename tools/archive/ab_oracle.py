#!/usr/bin/env python3
"""A/B of the two simulate kernels on the bench workload (SP_Oracle shape, 2^24 auctions):
the dedicated k_oracle (default) vs the general k_simulate, interleaved in ONE process after
the clock ramp (tools/archive/warm_probe.py); HIP events on the launch stream. Diagnostic only.

    python tools/archive/ab_oracle.py [B]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    # variants: (generic kernel?, blocks per CU); AG_AB_BPC="4,5,6": only k_oracle at those
    bpc = os.environ.get("AG_AB_BPC")
    variants = ([(False, int(x)) for x in bpc.split(",")] if bpc else
                [(False, 0), (True, 0), (False, 1), (False, 2), (False, 3), (False, 4)])
    out = {v: eng.alloc_outputs(B, fields) for v in variants}
    cnt = {v: eng.new_counters() for v in variants}
    st = torch.cuda.current_stream()
    def use(v):
        eng.set_simulate_kernel(v[0])
        eng.set_blocks_per_cu(v[1])
    for _ in range(150):
        eng.simulate(inp, out[variants[0]], cnt[variants[0]])
    for g in variants:
        use(g)
        cnt[g].zero_()
        eng.simulate(inp, out[g], cnt[g])
    torch.cuda.synchronize()
    v0 = variants[0]
    same = all(all(torch.equal(out[v0][k], out[g][k]) for k in fields) and torch.equal(cnt[v0], cnt[g])
               for g in variants)
    print("outputs and counters identical:", same, flush=True)
    iso = {g: [] for g in variants}
    sus = {g: [] for g in variants}
    for r in range(12):
        for g in variants:
            use(g)
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
    for g in variants:
        name = ("k_simulate (general)" if g[0] else "k_oracle") + (f" {g[1]}/CU" if g[1] else "")
        mi, ms = float(np.median(iso[g])), float(np.median(sus[g]))
        print(f"{name:22s} isolated {mi:.4f} ms ({bpa * B / mi / 1e6:6.0f} GB/s)  "
              f"back-to-back (+counter zeroing) {ms:.4f} ms ({bpa * B / ms / 1e6:6.0f} GB/s)")


if __name__ == "__main__":
    main()
