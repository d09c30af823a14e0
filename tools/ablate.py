#!/usr/bin/env python3
"""Ablation timings of ag_simulate on the bench workload (interleaved rounds in ONE
process, HIP events on the launch stream; median over rounds). Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
    rounds = 15
    items, values = bench.catalogue()
    eng = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    full = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    out = eng.alloc_outputs(B, full)
    cnt = eng.new_counters()
    variants = {
        "bench (all outputs + counters)": (False, full, True, 2),
        "bench, 1 auction per lane": (False, full, True, 1),
        "no counters": (False, full, False, 2),
        "counters, winner/price only": (False, ("winner", "price"), True, 2),
        "no outputs, no counters": (False, (), False, 2),
        "exact item scan": (True, full, True, 1),
    }
    times = {k: [] for k in variants}
    st = torch.cuda.current_stream()
    for _ in range(150):  # past the clock ramp of a fresh process (tools/archive/warm_probe.py)
        eng.simulate(inp, out, cnt)
    for r in range(rounds):
        for name, (exact, fields, want_cnt, lanes) in variants.items():
            eng.set_item_search(exact)
            eng.set_lane_auctions(lanes)
            o = {k: out[k] for k in fields}
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            eng.simulate(inp, o, cnt if want_cnt else None)
            b.record(st)
            torch.cuda.synchronize()
            if r >= 2:
                times[name].append(a.elapsed_time(b))
    bpa = bench.algorithmic_bytes_per_auction(5, 2, False)
    for name, t in times.items():
        ms = float(np.median(t))
        print(f"{name:34s} {ms:8.4f} ms  {B / ms / 1e6:9.1f} G auctions/s  "
              f"{bpa * B / ms / 1e6:8.1f} GB/s(141B)")
    # back-to-back (sustained, as in bench.py) vs isolated launches
    for lanes in (2, 1):
        eng.set_item_search(False)
        eng.set_lane_auctions(lanes)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(20)]
        for a, b in evs:
            a.record(st)
            eng.simulate(inp, out, cnt)
            b.record(st)
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) for a, b in evs[3:]]
        print(f"back-to-back bench, {lanes} auct/lane     mean {np.mean(t):.4f} ms  median "
              f"{np.median(t):.4f} ms  {bpa * B / np.mean(t) / 1e6:8.1f} GB/s")
    # pure streaming reference: read 56 B + write 85 B per auction with a copy
    src = torch.empty(B * 56 // 8, dtype=torch.float64, device="cuda")
    dst = torch.empty(B * 85 // 8, dtype=torch.float64, device="cuda")
    ts = []
    for r in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        dst[: src.numel()].copy_(src)
        dst[src.numel():].fill_(1.0)
        b.record(st)
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    print(f"{'torch copy+fill same bytes':34s} {ms:8.4f} ms  {bpa * B / ms / 1e6:8.1f} GB/s")
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in evs:
        a.record(st)
        dst[: src.numel()].copy_(src)
        dst[src.numel():].fill_(1.0)
        b.record(st)
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in evs[3:]]
    print(f"{'torch copy+fill back-to-back':34s} {np.mean(t):8.4f} ms  {bpa * B / np.mean(t) / 1e6:8.1f} GB/s")


if __name__ == "__main__":
    main()
