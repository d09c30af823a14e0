#!/usr/bin/env python3
"""Host issue cost of the record-parallel learner updates, measured in ONE
process: the FP_DR_TS population (configs_3, 3 DoublyRobustBidders + 3 LR-TS allocators) after its
iteration 0, its learners' update run record-parallel at world 1 with a same-size device copy of
each epoch's int64 totals standing in for the all-reduce (sharding.rp_epoch_blocks):

  - "from C": the launches back to back from one host call (4 x 64 per call, no exchange) --
    the per-epoch kernel time;
  - "eager": one ctypes launch + one torch copy per epoch from Python (the round-4 loop);
  - "graph": each block of 64 (launch + copy) captured once in a hipGraph and replayed.

Every mode must end in the same models and epochs (checked). Prints per-launch wall times.

    python tools/rp_issue.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import sharding  # noqa: E402


def main():
    eng, what, B, ak, bk, st16, dims, lo, inp, out, cnt = bench.population_first_iteration("configs_3", 0)
    P = eng.P
    lst = eng.new_lrts_samples(B)
    sst = eng.new_shading_samples(B * P, learning=True)
    eng.lrts_collect(inp, out, lst)
    eng.shading_collect(inp, out, sst, first_auction=lo)
    learners = [a for a in range(eng.N) if bk[a] >= 2]
    lrts = [a for a in range(eng.N) if ak[a] == 1]
    dr0 = eng.dr_state()
    m0, q0, pm0 = eng.lrts_state()
    torch.cuda.synchronize()

    calls = {"n": 0}
    orig_b, orig_l = eng.bidder_rp_epoch, eng.lrts_rp_epoch

    def count_b(launches=1, traces=None):
        calls["n"] += launches
        return orig_b(launches, traces)

    def count_l(launches=1):
        calls["n"] += launches
        return orig_l(launches)
    eng.bidder_rp_epoch, eng.lrts_rp_epoch = count_b, count_l
    # graph mode: the wrapped calls run once, at capture (no launch); each replay of a block runs
    # `poll` launches -- so launches = blocks replayed x poll (rp_epoch_blocks returns the blocks)
    blocks = {"n": 0}
    orig_blocks = sharding.rp_epoch_blocks

    def count_blocks(*a, **k):
        blocks["n"] = orig_blocks(*a, **k)
        return blocks["n"]
    sharding.rp_epoch_blocks = count_blocks

    res = {}
    for what_ in ("bidders", "lrts"):
        for mode in ("from C", "eager", "graph", "eager", "graph", "from C"):
            eng.set_dr_state(*dr0)
            eng.load_lrts(m0, q0, pm0)
            scratch = None

            def copy(t):
                nonlocal scratch
                if scratch is None or scratch.numel() != t.numel():
                    scratch = torch.empty_like(t)
                scratch.copy_(t)
            kw = {} if mode == "from C" else {"exchange": copy, "graph": mode == "graph"}
            calls["n"] = blocks["n"] = 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if what_ == "bidders":
                ep, stat = sharding.bidder_update_record_parallel(eng, sst, learners, **kw)
                result = (np.asarray(ep).copy(), eng.dr_state()[0].copy())
            else:
                ep = sharding.lrts_update_record_parallel(eng, lst, lrts, **kw)
                result = (np.asarray(ep).copy(), eng.lrts_state()[0].copy())
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if mode == "graph":
                calls["n"] = blocks["n"] * sharding.RP_POLL_LAUNCHES
            key = (what_, mode)
            if key in res:
                assert all(np.array_equal(a, b) for a, b in zip(res[key][2], result)), key
            res.setdefault(key, [[], calls["n"], result])[0].append(dt)
        ref = res[(what_, "from C")][2]
        for mode in ("eager", "graph"):
            assert all(np.array_equal(a, b) for a, b in zip(ref, res[(what_, mode)][2])), (what_, mode)
    print(f"{what}: B = {B}; every mode ends in the same models and epochs", flush=True)
    for (what_, mode), (ts, n, _) in res.items():
        t = min(ts)
        print(f"{what_:8s} {mode:7s} {n:6d} launches  {t * 1e3:9.1f} ms  {t / n * 1e6:7.2f} us per launch", flush=True)
    for what_ in ("bidders", "lrts"):
        c = min(res[(what_, "from C")][0]) / res[(what_, "from C")][1]
        for mode in ("eager", "graph"):
            ts, n, _ = res[(what_, mode)]
            print(f"{what_:8s} {mode:7s} issue + exchange cost per epoch {min(ts) / n * 1e6 - c * 1e6:7.2f} us "
                  f"(kernel {c * 1e6:.2f} us per epoch)", flush=True)


if __name__ == "__main__":
    main()
