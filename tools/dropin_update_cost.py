#!/usr/bin/env python3
"""Cost of the drop-in Agent.update for LR-TS allocators. SP_Truthful_TS (configs[1]:
8 LR-TS agents, the reference's rounds_per_iter), one iteration simulated through the drop-in
Auction, then the reference's main-loop updates (src/main.py:124-137: agent.update() for each
agent in order) three ways:

  - immediate: each agent's update trained at its call, alone (round 4's behaviour: a resumable
    session per agent, blocks of single-epoch launches; forced here by reading the posterior
    right after each update), with 256 and 64 launches per poll;
  - deferred (round 5, Auction._settle_lrts): the updates only mark the agents; the first read
    trains every pending agent in one persistent launch;
  - batched: the same logs, engine.lrts_update directly (what the bench's configs_1 update times).

The final posteriors and epochs must be identical (exact sums; checked). Prints wall times.

    python tools/dropin_update_cost.py [rounds]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import Auction as A  # noqa: E402
from auctiongym_amd import main as M  # noqa: E402


def build(rounds):
    torch.manual_seed(7)  # the Thompson draws come from torch's global generator: the same logs every build
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(bench.SP_TS, f)
        path = f.name
    try:
        rng, config, agent_configs, items, vals, _, max_slots, E, var, OE = M.parse_config(path)
    finally:
        os.unlink(path)
    agents = M.instantiate_agents(rng, agent_configs, vals, items)
    auction, _, rpi, _ = M.instantiate_auction(rng, config, items, vals, agents, max_slots, E, var, OE)
    auction.simulate_batch(rounds or rpi)
    torch.cuda.synchronize()
    return auction, agents


def per_agent(rounds, launches, immediate=True):
    auction, agents = build(rounds)
    orig = A._lrts_train
    A._lrts_train = lambda eng, st, mask, launches_=launches: orig(eng, st, mask, launches_)
    try:
        ts = []
        t_all = time.perf_counter()
        for ag in agents:
            t0 = time.perf_counter()
            ag.update(iteration=0, plot=False)
            if immediate:
                _ = ag.allocator.epochs  # settles this agent's update now
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ep = [int(a.allocator.epochs) for a in agents]  # (deferred: the settle runs here)
        torch.cuda.synchronize()
        total = time.perf_counter() - t_all
    finally:
        A._lrts_train = orig
    return total, ts, auction._engine.lrts_state(), ep


def batched(rounds):
    auction, agents = build(rounds)
    auction._flush()
    eng = auction._engine
    st = auction._stores["lrts"]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ep = eng.lrts_update(st)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, eng.lrts_state(), [int(x) for x in ep]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    per_agent(rounds, 256)  # warm (module loads, first launches)
    res = {}
    for rep in range(2):
        for key, launches, imm in (("immediate, 256 launches per poll", 256, True),
                                   ("immediate, 64 launches per poll", 64, True),
                                   ("deferred (one launch at the first read)", 256, False)):
            r = per_agent(rounds, launches, imm)
            if key not in res or r[0] < res[key][0]:
                res[key] = r
    b = [batched(rounds) for _ in range(2)]
    bt = min(x[0] for x in b)
    ref = b[0][1]
    for key, (total, ts, state, ep) in res.items():
        same = all(np.array_equal(x, y) for x, y in zip(state, ref)) and ep == b[0][2]
        print(f"{key}: {total * 1e3:8.1f} ms  (per update() call {', '.join(f'{t * 1e3:.1f}' for t in ts)} ms; "
              f"epochs {ep}; posteriors and epochs equal to batched: {same})", flush=True)
        assert same, key
    print(f"batched (engine.lrts_update, every LR-TS agent in one launch): {bt * 1e3:8.1f} ms (epochs {b[0][2]})",
          flush=True)
    print("posteriors identical across all modes: True", flush=True)


if __name__ == "__main__":
    main()
