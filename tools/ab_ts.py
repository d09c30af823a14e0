#!/usr/bin/env python3
"""A/B timing of library builds (make variant NAME=... VFLAGS=...) on the general simulate
kernel: SP_Truthful_TS (configs[1], 8 LR-TS agents, 1M auctions, Thompson noise resident)
and the mixed population (configs[4], 2M auctions, fitted policies), interleaved in one
process; outputs checked identical to the base build.

    python tools/ab_ts.py name1 name2 ...
    python tools/ab_ts.py bt256 bt1024     (base build, AG_OPT_SIM_BLOCK_THREADS forced)
    python tools/ab_ts.py gm1              (base build, AG_OPT_SIM_GENERAL_MODE = 1: the full
                                            general build for TruthfulBidder-only populations)
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

FULL = ("winner", "price", "second_price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")


def ts_engine(path):
    items, values = bench.catalogue(bench.SP_TS)
    N, K, D = items.shape
    e = AuctionEngine(N, 2, K, D - 1, 4, _lib.SECOND_PRICE, 1.0, device=0, lib_path=path)
    e.set_agent_params(np.ones(N, np.int32), np.zeros(N, np.int32))
    e.load_catalog(items, values)
    g = torch.Generator().manual_seed(0)
    m = torch.empty(N, K, 5)
    for a in range(N):
        m[a].normal_(0.0, 1.0, generator=g)
    e.load_lrts(m.numpy(), np.ones((N, K, 5), np.float32), thompson_sampling=True)
    return e


def time_all(engs, inp, fields, reps=25):
    base = engs["base"]
    ref = base.alloc_outputs(inp["u"].numel(), fields)
    cref = base.new_counters()
    base.simulate(inp, ref, cref)
    out = base.alloc_outputs(inp["u"].numel(), fields)
    cnt = base.new_counters()
    st = torch.cuda.current_stream()
    times = {n: [] for n in engs}
    for r in range(reps):
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
                same = all(torch.equal(out[k], ref[k]) or torch.equal(out[k].isnan(), ref[k].isnan()) and
                           torch.equal(out[k].nan_to_num(), ref[k].nan_to_num()) for k in fields)
                print(f"  {n}: outputs identical to base: {same and torch.equal(cnt, cref)}", flush=True)
    return {n: float(np.median(t)) for n, t in times.items()}


def main():
    vdir = os.path.join(ROOT, "auction-gym_amd", "build", "variants")
    paths = {"base": _lib.LIB_PATH}
    opts = {}
    for n in sys.argv[1:]:
        if n.startswith("bt") or n.startswith("gm"):
            paths[n] = _lib.LIB_PATH
            opts[n] = (_lib.OPT_SIM_BLOCK_THREADS if n.startswith("bt") else _lib.OPT_SIM_GENERAL_MODE, int(n[2:]))
        else:
            paths[n] = os.path.join(vdir, f"libauctiongym_hip_{n}.so")

    def apply(n, e):
        if n in opts:
            e._check(e.L.ag_set_option(e._h, opts[n][0], opts[n][1]), "ag_set_option")
        return e
    B = 1 << 20
    engs = {n: apply(n, ts_engine(p)) for n, p in paths.items()}
    inp = engs["base"].alloc_inputs(B)
    engs["base"].generate(0, 0, inp)
    engs["base"].generate_noise(0, 0, inp)
    print("configs_1 (SP_Truthful_TS, 1M auctions)")
    for n, ms in time_all(engs, inp, FULL).items():
        print(f"  {n:10s} {ms:.4f} ms  {B / ms / 1e6:.3f} G auctions/s", flush=True)
    for e in engs.values():
        e.close()
    # mixed population with fitted policies (bench configs_4 shapes; learners marked fitted)
    engs = {}
    for n, p in paths.items():
        _lib.LIB_PATH, keep = p, _lib.LIB_PATH
        e, what, B4, ak, bk, st16, dims = bench.build_population("configs_4", 0)
        _lib.LIB_PATH = keep
        e.set_dr_state(st16, np.where(bk >= 2, 1, 0).astype(np.int32))
        engs[n] = apply(n, e)
    inp = engs["base"].alloc_inputs(B4)
    engs["base"].generate(1, 0, inp)
    engs["base"].generate_noise(1, 0, inp)
    print("configs_4 (mixed 32 bidders, 2M auctions)")
    for n, ms in time_all(engs, inp, FULL + ("gamma", "propensity")).items():
        print(f"  {n:10s} {ms:.4f} ms  {B4 / ms / 1e6:.3f} G auctions/s", flush=True)


if __name__ == "__main__":
    main()
