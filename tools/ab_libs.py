#!/usr/bin/env python3
"""A/B timing of library builds of the same ABI (make variant NAME=... VFLAGS=...) on the
bench workload, interleaved in ONE process (cdna_hip_programming.md rule 24).

    python tools/ab_libs.py [variant names...]      (default: every build/variants/*.so)
    AB_LOG2B=27 AB_HEAD=1: 2^27 auctions with the bench headline's fields (the winner word)
"""
import glob
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
    names = sys.argv[1:]
    vdir = os.path.join(ROOT, "auction-gym_amd", "build", "variants")
    paths = {"base": _lib.LIB_PATH}
    if names:
        for n in names:
            paths[n] = os.path.join(vdir, f"libauctiongym_hip_{n}.so")
    else:
        for p in sorted(glob.glob(os.path.join(vdir, "*.so"))):
            paths[os.path.basename(p)[len("libauctiongym_hip_"):-3]] = p
    B = 1 << int(os.environ.get("AB_LOG2B", "24"))
    items, values = bench.catalogue()
    engs = {}
    for n, p in paths.items():
        e = AuctionEngine(6, 2, 12, 5, 4, _lib.SECOND_PRICE, 1.0, device=0, lib_path=p)
        e.load_catalog(items, values)
        e.set_blocks_per_cu(int(os.environ.get("AG_BPC", "0")))
        engs[n] = e
    base = engs["base"]
    inp = base.alloc_inputs(B)
    base.generate(0, 0, inp)
    full = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    if os.environ.get("AB_HEAD"):
        from auctiongym_amd.engine import HEADLINE_FIELDS
        full = HEADLINE_FIELDS
    ref = base.alloc_outputs(B, full)
    cref = base.new_counters()
    base.simulate(inp, ref, cref)
    out = base.alloc_outputs(B, full)
    cnt = base.new_counters()
    st = torch.cuda.current_stream()
    times = {n: [] for n in engs}
    for _ in range(max(10, (150 << 24) // B)):  # past the clock ramp of a fresh process (tools/archive/warm_probe.py)
        cnt.zero_()
        base.simulate(inp, out, cnt)
    for r in range(25):
        for n, e in engs.items():
            cnt.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            e.simulate(inp, out, cnt)
            b.record(st)
            torch.cuda.synchronize()
            if r >= 3:
                times[n].append(a.elapsed_time(b))
            if r == 0:
                same = all(torch.equal(out[k], ref[k]) for k in full) and torch.equal(cnt, cref)
                print(f"{n}: outputs identical to base: {same}")
    # sustained: 20 launches back to back per variant (as bench.py times them), interleaved
    sus = {n: [] for n in engs}
    for r in range(6):
        for n, e in engs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(20):
                cnt.zero_()
                e.simulate(inp, out, cnt)
            b.record(st)
            torch.cuda.synchronize()
            if r >= 1:
                sus[n].append(a.elapsed_time(b) / 20)
    bpa = bench.algorithmic_bytes_per_auction(5, 2, False, packed_winner="winner_outcome" in full)
    for n, t in times.items():
        ms, lo = float(np.median(t)), float(np.min(t))
        ss = float(np.median(sus[n]))
        print(f"{n:12s} isolated median {ms:.4f} ms  min {lo:.4f} ms  {bpa * B / ms / 1e6:7.1f} GB/s | "
              f"sustained {ss:.4f} ms  {bpa * B / ss / 1e6:7.1f} GB/s")


if __name__ == "__main__":
    main()
