"""Diagnostics: the drop-in driver vs a reference driver capture (tests/golden/<tag>_driver_kat.npz).
Prints per iteration / agent how the revenue, utilities, fit epochs, parameters and the
torch / numpy generator states compare. Usage: python tools/archive/driver_compare.py dr|dm|ips"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
import auctiongym_amd.main as M  # noqa: E402

tag = sys.argv[1]
k = np.load(os.path.join(ROOT, "tests", "golden", f"{tag}_driver_kat.npz"))
cfg = json.loads(str(k["cfg"]))
fd, path = tempfile.mkstemp(suffix=".json")
with os.fdopen(fd, "w") as f:
    json.dump(cfg, f)
rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(path)
torch.manual_seed(0)
agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
auction, num_iter, rounds, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
for it in range(num_iter):
    auction.simulate_batch(rounds)
    rev = auction.revenue
    print(f"it{it} revenue {rev:.10g} ref {float(k[f'it{it}_revenue']):.10g} rel {abs(rev / float(k[f'it{it}_revenue']) - 1):.2e}"
          f" np_state_equal {json.dumps(rng.bit_generator.state) == str(k[f'it{it}_np_state'])}", flush=True)
    net = np.array([a.net_utility for a in agents])
    print("   net maxrel", np.max(np.abs(net - k[f"it{it}_net"]) / np.abs(k[f"it{it}_net"])))
    for i, a in enumerate(agents):
        a.update(iteration=it)
        b = a.bidder
        ep = getattr(b, "epochs", None)
        ts = torch.get_rng_state().numpy()
        wr = b._state16()
        msg = f"  a{i} epochs {None if ep is None else list(ep)} ref fits {list(k[f'it{it}_a{i}_fits'])} imit {int(k[f'it{it}_a{i}_imitation'])}"
        msg += f" init {b.model_initialised}/{bool(k[f'it{it}_a{i}_init'])} torch_state_equal {np.array_equal(ts, k[f'it{it}_a{i}_torch_state'])}"
        if f"it{it}_a{i}_winrate_model" in k:
            msg += f" wr maxabs {np.max(np.abs(wr[:4] - k[f'it{it}_a{i}_winrate_model'])):.2e}"
        for name in ("bidding_policy", "model"):
            if f"it{it}_a{i}_{name}" in k:
                ref = k[f"it{it}_a{i}_{name}"]
                if ref.size == 24:  # BidShadingPolicy: shared (6), mu hidden (6), mu out (3), sigma hidden (6), sigma out (3)
                    ref = np.concatenate([ref[0:6], ref[12:15], ref[21:24]])
                msg += f" pol maxabs {np.max(np.abs(wr[4:] - ref)):.2e}"
        print(msg, flush=True)
        a.clear_utility()
        a.clear_logs()
    auction.clear_revenue()
