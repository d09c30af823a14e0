#!/usr/bin/env python3
"""The ABI 17 winner | outcome word vs the per-field winner and outcome arrays on the headline kernel (k_oracle,
SP_Oracle shape, 2^27 auctions unless given): the same launch back to back in ONE process,
alternating, with the outputs checked equal bit for bit. Also the general kernel on
SP_Truthful_TS (configs_1) when --pop is given. Diagnostic only.

    python tools/archive/ab_packed.py [B] [--pop]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402
from auctiongym_amd.engine import AuctionEngine, HEADLINE_FIELDS, unpack_outputs  # noqa: E402


P, E = 2, 5
FIELDS = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")


def timeit(fn, reps=8, inner=10):
    st = torch.cuda.current_stream()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(inner):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / inner)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 27
    items, values = bench.catalogue()
    eng = AuctionEngine(6, P, 12, E, 4, _lib.SECOND_PRICE, 1.0, device=0)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    per_field = eng.alloc_outputs(B, FIELDS)
    packed = eng.alloc_outputs(B, HEADLINE_FIELDS)
    cnt = eng.new_counters()
    cnt2 = eng.new_counters()
    eng.simulate(inp, per_field, cnt)
    torch.cuda.synchronize()
    eng.simulate(inp, packed, cnt2)
    torch.cuda.synchronize()
    up = unpack_outputs(packed)
    for f in FIELDS:
        a, b = per_field[f], up[f].contiguous()
        if a.dtype == torch.float64:
            a, b = a.view(torch.int64), b.view(torch.int64)
        assert torch.equal(a, b), f
    assert torch.equal(cnt, cnt2)
    print("packed == per-field, bit for bit", flush=True)
    reads = 8 * E + 4 * P + 8
    writes = {"per-field (13 streams)": 4 + 8 + 1 + 36 * P}
    outs = {"per-field (13 streams)": (per_field, None)}
    writes["per-field, winner_outcome (12)"] = 4 + 8 + 36 * P
    outs["per-field, winner_outcome (12)"] = (eng.alloc_outputs(B, HEADLINE_FIELDS), None)
    writes["per-field, winner_outcome, 5/CU"] = 4 + 8 + 36 * P
    outs["per-field, winner_outcome, 5/CU"] = (packed, 5)
    engs = {n: eng for n in outs}
    for v in [a[len("--lib="):] for a in sys.argv[1:] if a.startswith("--lib=")]:  # make variant builds
        ev = AuctionEngine(6, P, 12, E, 4, _lib.SECOND_PRICE, 1.0, device=0,
                           lib_path=os.path.join(ROOT, "auction-gym_amd", "build", "variants", f"libauctiongym_hip_{v}.so"))
        ev.load_catalog(items, values)
        for n in ("per-field (13 streams)", "per-field, winner_outcome (12)"):
            writes[f"{v}: {n}"] = writes[n]
            outs[f"{v}: {n}"] = outs[n]
            engs[f"{v}: {n}"] = ev
    for _ in range(30):
        cnt.zero_()
        eng.simulate(inp, per_field, cnt)
    torch.cuda.synchronize()
    t = {n: [] for n in outs}
    for r in range(6):
        for n, (o, lay) in outs.items():
            e = engs[n]
            e.set_blocks_per_cu(lay or 0)

            def step(o=o, e=e):
                cnt.zero_()
                e.simulate(inp, o, cnt)
            t[n] += timeit(step, reps=2, inner=5)
    for n in outs:
        ms = float(np.median(t[n]))
        bpa = reads + writes[n]
        print(f"{n:34s} {bpa:4d} B/auction  {ms:.4f} ms  {bpa * B / ms / 1e6:6.0f} GB/s  "
              f"141-B figure {141 * B / ms / 1e6:6.0f} GB/s = {141 * B / ms / 1e6 / 8000:.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
