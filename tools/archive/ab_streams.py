#!/usr/bin/env python3
"""Write-stream sensitivity of the headline kernel (k_oracle, SP_Oracle shape): the same
launch with output fields left out (NULL pointers: the kernel skips those stores), back to
back in ONE process, and the achieved GB/s on the bytes each variant actually moves. If
dropping the small streams (winner 4 B, outcome 1 B) raises GB/s, packing them pays; if
GB/s stays flat, the stream count is not what holds the kernel below the copy peak.
Diagnostic only.

    python tools/archive/ab_streams.py [B]
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

P, E = 2, 5
BYTES = {"winner": 4, "price": 8, "outcome": 1, "item": 4 * P, "bid": 8 * P, "est_ctr": 8 * P,
         "true_ctr": 8 * P, "best_ev": 8 * P}
ALL = tuple(BYTES)
VARIANTS = {
    "all 13 streams": ALL,
    "no outcome (12)": tuple(f for f in ALL if f != "outcome"),
    "no outcome, winner (11)": tuple(f for f in ALL if f not in ("outcome", "winner")),
    "no true_ctr (11)": tuple(f for f in ALL if f != "true_ctr"),
    "no item (11)": tuple(f for f in ALL if f != "item"),
    "no est/true_ctr (9)": tuple(f for f in ALL if f not in ("est_ctr", "true_ctr")),
}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
    items, values = bench.catalogue()
    eng = AuctionEngine(6, P, 12, E, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    reads = 8 * E + 4 * P + 8
    outs = {n: eng.alloc_outputs(B, f) for n, f in VARIANTS.items()}
    cnt = eng.new_counters()
    st = torch.cuda.current_stream()
    for _ in range(40):
        cnt.zero_()
        eng.simulate(inp, outs["all 13 streams"], cnt)
    torch.cuda.synchronize()
    t = {n: [] for n in VARIANTS}
    for r in range(8):
        for n in VARIANTS:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(10):
                cnt.zero_()
                eng.simulate(inp, outs[n], cnt)
            b.record(st)
            torch.cuda.synchronize()
            t[n].append(a.elapsed_time(b) / 10)
    for n, f in VARIANTS.items():
        bpa = reads + sum(BYTES[k] for k in f)
        ms = float(np.median(t[n]))
        print(f"{n:26s} {bpa:4d} B/auction  {ms:.4f} ms  {bpa * B / ms / 1e6:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
