#!/usr/bin/env python3
"""Drop-in Agent.update time on a learning config at the reference's 10k rounds per
iteration: the reference's own driver loop (src/main.py:112-152) through
auctiongym_amd -- simulate_batch of the iteration's rounds, then every agent's update() in
turn (LR-TS allocator on the GPU, the learning bidder's fits as the resumable per-epoch update
fed the reference's torch rsample draws window by window) -- timed per agent and iteration.
The config is the reference's FP_DR_TS.json / FP_DM_TS.json as captured in tests/golden
(*_driver_kat.npz "cfg"), rounds_per_iter set to 10000. One JSON line per iteration.

    python tools/archive/dropin_update_time.py [dr|dm] [iterations]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))

import torch  # noqa: E402

import auctiongym_amd.main as M  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "dr"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    k = np.load(os.path.join(ROOT, "tests", "golden", f"{tag}_driver_kat.npz"))
    cfg = json.loads(str(k["cfg"]))
    cfg["rounds_per_iter"] = 10000
    cfg["num_iter"] = iters
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(cfg, f)
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(f.name)
    os.unlink(f.name)
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, num_iter, rounds, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for it in range(num_iter):
        t0 = time.perf_counter()
        auction.simulate_batch(rounds)
        rev = auction.revenue
        t_sim = time.perf_counter() - t0
        per = []
        for a in agents:
            t1 = time.perf_counter()
            a.update(iteration=it)
            torch.cuda.synchronize()
            per.append({"agent": a.name, "s": time.perf_counter() - t1,
                        "epochs": [int(e) for e in getattr(a.bidder, "epochs", [])],
                        "records": a.num_logs()})
            a.clear_utility()
            a.clear_logs()
        auction.clear_revenue()
        print(json.dumps({"config": f"{tag.upper()} ({'FP_DR_TS' if tag == 'dr' else 'FP_DM_TS'}.json), "
                                    f"{rounds} rounds per iteration", "iteration": it,
                          "simulate_s": t_sim, "update_s": sum(p["s"] for p in per), "agents": per,
                          "revenue": rev,
                          "reference_update_s": 137.5 if tag == "dr" else 49.8,
                          "reference_what": "the reference's Agent.update of every agent per 10k-round iteration, "
                                            "one core of the survey container (SURVEY.md section 6)"}),
              flush=True)


if __name__ == "__main__":
    main()
