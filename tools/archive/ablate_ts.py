"""Ablation timings of the general (LR-TS) simulate kernel on the SP_Truthful_TS bench
workload. Diagnostic only."""
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
    B = 1 << 20
    items, values = bench.catalogue(bench.SP_TS)
    N, K, D = items.shape
    m = np.random.default_rng(0).normal(0, 1, (N, K, 5)).astype(np.float32)
    q = np.ones_like(m)
    engs = {}
    for name, ts, lrts in (("TS sampled", True, True), ("TS MAP only", False, True), ("Oracle kernel", False, False)):
        e = AuctionEngine(N, 2, K, 5, 4, _lib.SECOND_PRICE, 1.0, device=0)
        e.set_agent_params(np.full(N, 1 if lrts else 0, np.int32), np.zeros(N, np.int32))
        e.load_catalog(items, values)
        if lrts:
            e.load_lrts(m, q, thompson_sampling=ts)
        engs[name] = e
    e0 = engs["TS sampled"]
    inp = e0.alloc_inputs(B)
    e0.generate(0, 0, inp)
    e0.generate_noise(0, 0, inp)
    out = e0.alloc_outputs(B)
    cnt = e0.new_counters()
    st = torch.cuda.current_stream()
    variants = {"TS sampled, all outputs + counters": ("TS sampled", None, True),
                "TS sampled, no counters": ("TS sampled", None, False),
                "TS sampled, winner only": ("TS sampled", ("winner",), False),
                "TS MAP only (no noise reads)": ("TS MAP only", None, True),
                "Oracle kernel on same inputs": ("Oracle kernel", None, True)}
    for _ in range(30):
        e0.simulate(inp, out, cnt)
    times = {k: [] for k in variants}
    for r in range(12):
        for name, (en, fields, wc) in variants.items():
            o = out if fields is None else {k: out[k] for k in fields}
            i2 = inp if en != "Oracle kernel" else {k: inp[k] for k in ("ctx", "part", "u")}
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            engs[en].simulate(i2, o, cnt if wc else None)
            b.record(st)
            torch.cuda.synchronize()
            if r >= 2:
                times[name].append(a.elapsed_time(b))
    for name, t in times.items():
        print(f"{name:38s} {np.median(t):.4f} ms  {B / np.median(t) / 1e6:7.2f} G auctions/s")


if __name__ == "__main__":
    main()
