#!/usr/bin/env python3
"""Drop-in replay rate: Auction.simulate_batch(B) on SP_Oracle.json as shipped
-- the reference's own numpy draws made in C (ag_replay_draw), copied to the GPU, resolved by
the kernel -- against the draws alone and the per-round Python loop they replace.

    python tools/replay_rate.py [B]
"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "auction-gym_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import auctiongym_amd.main as M  # noqa: E402
from auctiongym_amd.replay import draw_rounds, draw_rounds_native  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(bench.SP_ORACLE, f)
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(f.name)
    os.unlink(f.name)
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, *_ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    N, P = len(agents), config["num_participants_per_round"]
    auction.simulate_batch(1 << 14)  # warm: kernels, allocator
    torch.cuda.synchronize()
    res = {"rounds": B}
    t = time.perf_counter()
    draw_rounds_native(np.random.default_rng(1), B, N, P, E, var, max_slots)
    res["draw_native_ms"] = (time.perf_counter() - t) * 1e3
    n = min(B, 1 << 15)
    t = time.perf_counter()
    draw_rounds(np.random.default_rng(1), n, N, P, E, var, max_slots)
    res["draw_python_ms_per_2^20"] = (time.perf_counter() - t) * 1e3 * (1 << 20) / n
    t = time.perf_counter()
    auction.simulate_batch(B)
    _ = auction.revenue  # reads the counters back (synchronises)
    torch.cuda.synchronize()
    res["simulate_batch_ms"] = (time.perf_counter() - t) * 1e3
    res["simulate_batch_rounds_per_s"] = B / (res["simulate_batch_ms"] * 1e-3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
