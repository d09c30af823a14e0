#!/usr/bin/env python3 -B
"""Golden-vector generator (TEST INFRASTRUCTURE; runs only in the dev container).

Imports the reference AuctionGym (`/root/reference/src`, read-only) with harness-only
shims and records what its hot path computes on fixed seeds, so that the oracle
(`oracle/`) and the HIP path can be pinned against the reference's own outputs.
Nothing from the reference is copied: the outputs written here are data
(inputs + expected outputs) in `tests/golden/*.npz` / `*.json`.

Shims (nothing under /root/reference is modified; run with `python3 -B`):
  * numba is absent -> `numba.jit` stub. Default "numba-faithful": the sigmoid
    of `src/Models.py:10-12` evaluated with libm `exp` per element (what the
    pinned numba 0.55.1, requirements.txt:7, compiles to). This is the exp the
    oracle and the HIP kernels restate.
  * seaborn is absent -> empty module (plots only, src/main.py:7).
  * matplotlib -> Agg backend.

Draw-order replay: alongside the reference rng we advance a CLONE of the same
PCG64 Generator in the order this repo's replay inputs assume
(src/Auction.py:30 integers(1,2) -> no draw when max_slots == 1;
 :33 normal(0, var, E); :42 choice(N, P, replace=False); per-participant
 bidder draws (none for TruthfulBidder); :65 binomial(1, p) -> one next_double)
and assert after every round that the clone's state equals the reference's.
That pins SURVEY §8 a2/a3 on every recorded round.

Usage:  python3 -B tests/golden/make_golden.py [--full]
"""
import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np

REF_SRC = "/root/reference/src"
REF_CFG = "/root/reference/config"
OUT = os.path.dirname(os.path.abspath(__file__))


def install_shims():
    nb = types.ModuleType("numba")
    # libm exp called per element through ctypes (math.exp would raise on overflow,
    # C exp returns inf, as the numba-compiled loop does).
    import ctypes
    _libm = ctypes.CDLL("libm.so.6")
    _libm.exp.restype = ctypes.c_double
    _libm.exp.argtypes = [ctypes.c_double]
    _e = np.frompyfunc(_libm.exp, 1, 1)

    def jit(*a, **k):
        def deco(f):
            def sigmoid(x):
                x = np.asarray(x, np.float64)
                return 1.0 / (1.0 + _e(-x).astype(np.float64))
            return sigmoid
        return deco

    nb.jit = jit
    sys.modules["numba"] = nb
    sns = types.ModuleType("seaborn")
    sns.lineplot = lambda *a, **k: None  # plots only (src/main.py:239-326)
    sys.modules["seaborn"] = sns
    import matplotlib
    matplotlib.use("Agg")
    import torch
    torch.manual_seed(0)

    class _RP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)

    torch.optim.lr_scheduler.ReduceLROnPlateau = _RP
    sys.path.insert(0, REF_SRC)


def write_cfg(cfg):
    fd, path = tempfile.mkstemp(suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(cfg, f)
    return path


def load_cfg(name, **over):
    with open(os.path.join(REF_CFG, name)) as f:
        cfg = json.load(f)
    cfg.update(over)
    return cfg


def oracle_truthful_cfg(n_agents, n_items, P, allocation, seed, E=5, OE=4, var=1.0):
    return {
        "random_seed": seed, "num_runs": 1, "num_iter": 1, "rounds_per_iter": 0,
        "num_participants_per_round": P, "embedding_size": E, "embedding_var": var,
        "obs_embedding_size": OE, "allocation": allocation,
        "agents": [{"name": "Truthful Oracle", "num_copies": n_agents, "num_items": n_items,
                    "allocator": {"type": "OracleAllocator", "kwargs": {}},
                    "bidder": {"type": "TruthfulBidder", "kwargs": {}}}],
        "output_dir": "/tmp/ag_golden_unused/",
    }


def _bidder_kind(b):
    return type(b).__name__


def capture(cfg, rounds, torch_seed=0, keep=False):
    """Run `rounds` reference rounds (one iteration) and record replay inputs + outputs.

    Replay inputs beyond ctx/part/u, per (round, slot):
      gamma_raw  the raw rng.normal(prev_gamma, gamma_sigma) draw of an uninitialised shading
                 bidder (src/Bidder.py:51,177,354,461), NaN for bidders that draw nothing;
      ts_noise   [K][OE+1] float32 output of torch.normal in PyTorchLogisticRegression.forward
                 (src/Models.py:31) for Thompson-sampling agents, 0 otherwise.
    """
    import main as M
    import torch
    path = write_cfg(cfg)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     E, var, OE) = M.parse_config(path)
    os.unlink(path)
    torch.manual_seed(torch_seed)
    agents = M.instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
    auction, _, _, _ = M.instantiate_auction(rng, config, agents2items, agents2item_values,
                                             agents, max_slots, E, var, OE)
    N = len(agents)
    P = config["num_participants_per_round"]
    names = [a.name for a in agents]
    # per-agent item counts (src/main.py:61,66): catalogues padded to the largest K with
    # value-0 rows (num_items in the meta says which rows are the agent's own)
    num_items = [len(agents2item_values[n]) for n in names]
    K = max(num_items)
    D = agents2items[names[0]].shape[1]
    items = np.zeros((N, K, D))                                 # [N][K][D]
    values = np.zeros((N, K))                                   # [N][K]
    for i, n in enumerate(names):
        items[i, :num_items[i]] = agents2items[n]
        values[i, :num_items[i]] = agents2item_values[n]
    is_ts = [type(a.allocator).__name__ == "PyTorchLogisticRegressionAllocator" for a in agents]
    Do = None
    ts_m = ts_q = None
    if any(is_ts):
        Do = agents[is_ts.index(True)].allocator.response_model.m.shape[1]
        ts_m = np.zeros((N, K, Do), np.float32)
        ts_q = np.ones((N, K, Do), np.float32)
        for i, a in enumerate(agents):
            if is_ts[i]:
                ts_m[i, :num_items[i]] = a.allocator.response_model.m.detach().numpy()
                ts_q[i, :num_items[i]] = a.allocator.response_model.q.numpy()
    shading = [hasattr(a.bidder, "prev_gamma") for a in agents]

    clone = np.random.Generator(np.random.PCG64())
    clone.bit_generator.state = rng.bit_generator.state

    alloc_log = []
    orig = auction.allocation.allocate

    def wrapped(bids, num_slots):
        w, p, s = orig(bids, num_slots)
        alloc_log.append((np.array(bids, np.float64), np.array(w), np.array(p), np.array(s)))
        return w, p, s

    auction.allocation.allocate = wrapped
    noise_log = []
    orig_normal = torch.normal

    def rec_normal(*a, **k):
        t = orig_normal(*a, **k)
        noise_log.append(t.detach().numpy().copy())
        return t

    torch.normal = rec_normal

    ctx = np.zeros((rounds, E))
    part = np.zeros((rounds, P), np.int32)
    u = np.zeros(rounds)
    gamma_raw = np.full((rounds, P), np.nan)
    ts_noise = np.zeros((rounds, P, K, Do), np.float32) if Do else None
    rec = {k: np.zeros((rounds, P)) for k in
           ("bid", "est_ctr", "true_ctr", "best_ev", "value", "price", "second_price", "gamma",
            "propensity")}
    item = np.zeros((rounds, P), np.int32)
    won = np.zeros((rounds, P), np.int8)
    outcome_slot = np.zeros((rounds, P), np.int8)
    winner = np.full(rounds, -1, np.int32)
    price = np.full(rounds, np.nan)
    second = np.full(rounds, np.nan)
    outcome = np.zeros(rounds, np.int8)

    try:
        for r in range(rounds):
            # replay order (see module docstring)
            c = clone.normal(0, var, size=E)
            pa = clone.choice(N, P, replace=False)
            for s_, a_ in enumerate(pa):
                b = agents[a_].bidder
                if shading[a_] and not getattr(b, "model_initialised", False):
                    gamma_raw[r, s_] = clone.normal(b.prev_gamma, b.gamma_sigma)
            uu = clone.random()
            n0 = len(noise_log)
            auction.simulate_opportunity()
            assert clone.bit_generator.state == rng.bit_generator.state, f"draw order diverged at round {r}"
            ctx[r] = c
            part[r] = pa
            u[r] = uu
            nts = [s_ for s_, a_ in enumerate(pa) if is_ts[a_] and agents[a_].allocator.thompson_sampling]
            assert len(noise_log) - n0 == len(nts)
            for j, s_ in enumerate(nts):
                ts_noise[r, s_, :num_items[pa[s_]]] = noise_log[n0 + j]
            for s, a in enumerate(pa):
                lg = agents[a].logs[-1]
                rec["bid"][r, s] = lg.bid
                rec["est_ctr"][r, s] = lg.estimated_CTR
                rec["true_ctr"][r, s] = lg.true_CTR
                rec["best_ev"][r, s] = lg.best_expected_value
                rec["value"][r, s] = lg.value
                rec["price"][r, s] = lg.price
                rec["second_price"][r, s] = lg.second_price
                if shading[a]:
                    g = agents[a].bidder.gammas[-1]
                    rec["gamma"][r, s] = float(g)
                    pr = getattr(agents[a].bidder, "propensities", [np.nan])[-1] \
                        if hasattr(agents[a].bidder, "propensities") else np.nan
                    rec["propensity"][r, s] = float(pr)
                else:
                    rec["gamma"][r, s] = np.nan
                    rec["propensity"][r, s] = np.nan
                item[r, s] = lg.item
                won[r, s] = bool(lg.won)
                outcome_slot[r, s] = bool(lg.outcome)
            bids, w, p, s2 = alloc_log[-1]
            assert np.array_equal(bids, rec["bid"][r])
            winner[r] = w[0]
            if len(p):
                price[r] = p[0]
            if len(s2):
                second[r] = s2[0]
            if len(p):
                outcome[r] = outcome_slot[r, w[0]]
    finally:
        torch.normal = orig_normal

    agg = {
        "net_utility": [a.net_utility for a in agents],
        "gross_utility": [a.gross_utility for a in agents],
        "revenue": auction.revenue,
        "allocation_regret": [float(a.get_allocation_regret()) for a in agents],
        "estimation_regret": [float(a.get_estimation_regret()) for a in agents],
        "overbid_regret": [float(a.get_overbid_regret()) for a in agents],
        "underbid_regret": [float(a.get_underbid_regret()) for a in agents],
        "ctr_rmse": [float(a.get_CTR_RMSE()) for a in agents],
        "ctr_bias": [float(a.get_CTR_bias()) if any(o.won for o in a.logs) else float("nan")
                     for a in agents],
        "mean_best_ev": [float(np.mean([o.best_expected_value for o in a.logs]))
                         if a.logs else float("nan") for a in agents],
        "n_logs": [len(a.logs) for a in agents],
    }
    arrays = dict(items=items, values=values, ctx=ctx, part=part, u=u, item=item, won=won,
                  winner=winner, price=price, second_price=second, outcome=outcome,
                  gamma_raw=gamma_raw, **{"slot_" + k: v for k, v in rec.items()})
    if Do:
        arrays.update(ts_noise=ts_noise, ts_m=ts_m, ts_q=ts_q)
    meta = dict(N=N, P=P, K=K, E=E, OE=OE, var=var, rounds=rounds,
                allocation=config["allocation"], seed=config["random_seed"], torch_seed=torch_seed,
                allocators=[type(a.allocator).__name__ for a in agents],
                bidders=[_bidder_kind(a.bidder) for a in agents],
                bidder_kwargs=[c["bidder"]["kwargs"] for c in agent_configs],
                ts_dim=Do, num_items=num_items)
    if keep:
        return arrays, agg, meta, (agents, auction, rng)
    return arrays, agg, meta


def save_capture(name, arrays, agg, meta):
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
    with open(os.path.join(OUT, name + ".json"), "w") as f:
        json.dump({"meta": meta, "aggregates": agg}, f, indent=1)
    print("wrote", name, {k: v.shape for k, v in arrays.items()})


def alloc_kats():
    """Reference FirstPrice/SecondPrice.allocate on random and tied bid rows."""
    import AuctionAllocation as AA
    g = np.random.default_rng(1234)
    out = {}
    for P in (1, 2, 3, 4, 8, 32, 64, 100):
        rows = [g.lognormal(0.1, 0.2, P) * g.random(P) for _ in range(48)]
        # ties: all-equal, all-zero, tie at top, tie at second, duplicates of zeros
        rows.append(np.zeros(P))
        rows.append(np.full(P, 0.25))
        b = g.random(P); b[P // 2] = b.max(); rows.append(b)
        b = g.random(P); b[-1] = b.max(); rows.append(b)
        b = g.random(P) * (g.random(P) < 0.5); rows.append(b)
        if P >= 2:
            b = g.random(P); srt = np.sort(b); b[b == srt[-2]] = 0.0; b[0] = srt[-1] if P > 1 else b[0]
            rows.append(b)
        bids = np.stack(rows)
        for mech in ("FirstPrice", "SecondPrice"):
            m = getattr(AA, mech)()
            W, PR, SP = [], [], []
            for row in bids:
                w, p, s = m.allocate(row.copy(), 1)
                W.append(int(w[0]))
                PR.append(float(p[0]) if len(p) else np.nan)
                SP.append(float(s[0]) if len(s) else np.nan)
            out[f"{mech}_P{P}_winner"] = np.array(W, np.int32)
            out[f"{mech}_P{P}_price"] = np.array(PR)
            out[f"{mech}_P{P}_second_price"] = np.array(SP)
        out[f"P{P}_bids"] = bids
    np.savez_compressed(os.path.join(OUT, "alloc_kat.npz"), **out)
    print("wrote alloc_kat", len(out))


def lrts_update_kat(agents, out_name):
    """LR-TS Agent.update (src/Agent.py:79-94 -> src/BidderAllocation.py:29-65) on the logs of
    the captured iteration: inputs, the loss and gradient of the first epoch (the model's own
    loss/backward), the per-epoch loss trajectory (recorded by the scheduler shim), and the
    updated m, q, prev_m."""
    import torch
    import BidderAllocation as BA
    traj = []

    class RecRP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)

        def step(self, metrics, *a, **k):
            traj.append(float(metrics))
            return super().step(metrics, *a, **k)

    saved = torch.optim.lr_scheduler.ReduceLROnPlateau
    torch.optim.lr_scheduler.ReduceLROnPlateau = RecRP
    out = {}
    try:
        for i, a in enumerate(agents):
            if not isinstance(a.allocator, BA.PyTorchLogisticRegressionAllocator):
                continue
            rm = a.allocator.response_model
            contexts = np.array(list(opp.context for opp in a.logs))
            items = np.array(list(opp.item for opp in a.logs))
            outcomes = np.array(list(opp.outcome for opp in a.logs))
            won = np.array(list(opp.won for opp in a.logs))
            X, A, y = contexts[won], items[won], outcomes[won]
            out[f"a{i}_X"] = X
            out[f"a{i}_A"] = A.astype(np.int64)
            out[f"a{i}_y"] = y.astype(np.float64)
            out[f"a{i}_m0"] = rm.m.detach().numpy().copy()
            out[f"a{i}_prevm0"] = rm.prev_iter_m.numpy().copy()
            out[f"a{i}_q0"] = rm.q.numpy().copy()
            # epoch-0 loss and gradient through the reference's own model code
            Xt, At, yt = torch.Tensor(X), torch.LongTensor(A), torch.Tensor(y)
            rm.zero_grad()
            loss = rm.loss(torch.squeeze(rm.predict_item(Xt, At)), yt)
            loss.backward()
            out[f"a{i}_loss0"] = np.array(float(loss.item()))
            out[f"a{i}_grad0"] = rm.m.grad.detach().numpy().copy()
            rm.zero_grad()
            traj.clear()
            a.update(iteration=0)
            out[f"a{i}_losses"] = np.array(traj, np.float64)
            out[f"a{i}_m1"] = rm.m.detach().numpy().copy()
            out[f"a{i}_q1"] = rm.q.numpy().copy()
            print("lrts update agent", i, "samples", len(y), "epochs", len(traj), flush=True)
    finally:
        torch.optim.lr_scheduler.ReduceLROnPlateau = saved
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def dr_update_kat(out_name="dr_update_kat", rounds=2048):
    """DoublyRobustBidder.update (src/Bidder.py:473-615; src/Models.py:51-218) on the logs of
    FP_DR_TS.json's first iteration, through the reference's own classes: the update's
    inputs, the models' initial parameters, epoch-0 loss and gradients of the three fits
    (win-rate BCE, policy imitation MSE, DR policy loss at its starting point with the
    recorded torch RNG state), the per-epoch scheduler losses of the two scheduled fits, the
    torch RNG state at the start of the DR fit (its per-epoch rsample noise), and the
    parameters after each fit."""
    import copy

    import torch
    import Models
    _, _, _, (agents, _, _) = capture(load_cfg("FP_DR_TS.json"), rounds, keep=True)
    recs = []

    class RecRP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)
            self.rec = {"rng": torch.get_rng_state().clone(), "losses": []}
            recs.append(self.rec)

        def step(self, metrics, *a, **k):
            self.rec["losses"].append(float(metrics))
            return super().step(metrics, *a, **k)

    init_snap = {}
    orig_init = Models.BidShadingContextualBandit.initialise_policy

    def rec_init(self, X, gammas):
        orig_init(self, X, gammas)
        init_snap["params"] = [p.detach().numpy().copy() for p in self.parameters()]

    def params(mod):
        return [p.detach().numpy().copy() for p in mod.parameters()]

    saved = torch.optim.lr_scheduler.ReduceLROnPlateau
    torch.optim.lr_scheduler.ReduceLROnPlateau = RecRP
    Models.BidShadingContextualBandit.initialise_policy = rec_init
    out = {}
    try:
        for i, ag in enumerate(agents):
            b = ag.bidder
            L = ag.logs
            est = np.array([o.estimated_CTR for o in L])
            vals = np.array([o.value for o in L])
            prices = np.array([o.price for o in L])
            outc = np.array([o.outcome for o in L])
            won = np.array([o.won for o in L])
            k = f"a{i}_"
            out[k + "est_ctr"], out[k + "value"], out[k + "price"] = est, vals, prices
            out[k + "outcome"], out[k + "won"] = outc.astype(np.int8), won.astype(np.int8)
            out[k + "gamma"] = np.array([float(g) for g in b.gammas])
            out[k + "propensity"] = np.array([float(p) for p in b.propensities])
            for j, p in enumerate(params(b.winrate_model)):
                out[k + f"wr0_{j}"] = p
            for j, p in enumerate(params(b.bidding_policy)):
                out[k + f"pol0_{j}"] = p
            # epoch-0 KATs of the win-rate BCE fit and the imitation MSE, on the data the
            # update builds (src/Bidder.py:500-514, src/Models.py:114-121)
            X = np.hstack((est.reshape(-1, 1), vals.reshape(-1, 1), out[k + "gamma"].reshape(-1, 1)))
            Xn = X.copy()
            Xn[:, -1] = 0.0
            Xt = torch.Tensor(np.vstack((X, Xn)))
            y = won.astype(np.uint8).reshape(-1, 1)
            yt = torch.Tensor(np.concatenate((y, np.zeros_like(y))))
            wm = copy.deepcopy(b.winrate_model)
            loss = torch.nn.BCELoss()(wm(Xt), yt)
            loss.backward()
            out[k + "wr_loss0"] = np.array(loss.item())
            for j, p in enumerate(wm.parameters()):
                out[k + f"wr_grad0_{j}"] = p.grad.numpy().copy()
            pol = copy.deepcopy(b.bidding_policy)
            Xc = torch.Tensor(np.hstack((est.reshape(-1, 1), vals.reshape(-1, 1))))
            gt = torch.Tensor(b.gammas)
            sp = torch.nn.Softplus()
            mu = sp(pol.mu_linear_out(sp(pol.shared_linear(Xc))))
            sg = sp(pol.sigma_linear_out(sp(pol.shared_linear(Xc))))
            crit = torch.nn.MSELoss()
            loss = crit(mu.squeeze(), gt) + crit(sg.squeeze(), torch.ones_like(gt) * .05)
            loss.backward()
            out[k + "init_loss0"] = np.array(loss.item())
            for j, p in enumerate(pol.parameters()):
                out[k + f"init_grad0_{j}"] = p.grad.numpy().copy()
            recs.clear()
            init_snap.clear()
            ag.update(iteration=0)  # LR-TS allocator update, then the DR bidder's
            # recs: [LR-TS allocator, win-rate fit, DR policy fit]
            assert len(recs) == 3, len(recs)
            out[k + "wr_losses"] = np.array(recs[1]["losses"])
            out[k + "dr_losses"] = np.array(recs[2]["losses"])
            out[k + "dr_rng_state"] = recs[2]["rng"].numpy()
            for j, p in enumerate(init_snap["params"]):
                out[k + f"pol_init_{j}"] = p
            for j, p in enumerate(params(b.winrate_model)):
                out[k + f"wr1_{j}"] = p
            for j, p in enumerate(params(b.bidding_policy)):
                out[k + f"pol1_{j}"] = p
            # epoch-0 KAT of the DR loss at its starting point (post-imitation policy, fitted
            # win-rate model, the RNG state the fit started from)
            after = torch.get_rng_state()
            pol = copy.deepcopy(b.bidding_policy)
            with torch.no_grad():
                for p, v in zip(pol.parameters(), init_snap["params"]):
                    p.copy_(torch.from_numpy(v))
            W = b.winrate_model(torch.Tensor(X)).squeeze().detach().numpy()
            util = np.zeros_like(vals)
            util[won] = vals[won] * outc[won] - prices[won]
            est_u = W * (est * vals - est * vals * out[k + "gamma"])
            out[k + "util"], out[k + "est_util"] = util, est_u
            torch.set_rng_state(recs[2]["rng"])
            loss = pol.loss(Xc, gt, torch.clip(torch.Tensor(b.propensities), min=1e-15), torch.Tensor(util),
                            utility_estimates=torch.Tensor(est_u), winrate_model=b.winrate_model,
                            importance_weight_clipping_eps=50.0)
            loss.backward()
            out[k + "dr_loss0"] = np.array(loss.item())
            for j, p in enumerate(pol.parameters()):
                out[k + f"dr_grad0_{j}"] = p.grad.numpy().copy()
            torch.set_rng_state(after)
            print("dr update agent", i, "n", len(L), "wr epochs", len(out[k + "wr_losses"]),
                  "dr epochs", len(out[k + "dr_losses"]), flush=True)
    finally:
        torch.optim.lr_scheduler.ReduceLROnPlateau = saved
        Models.BidShadingContextualBandit.initialise_policy = orig_init
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def learner_update_kat(cfg_name, out_name, rounds=2048):
    """ValueLearningBidder (FP_DM_TS.json, inference 'policy') and PolicyLearningBidder
    (FP_IPS_TS.json, loss 'PPO') .update (src/Bidder.py:204-325, :364-431) on the logs of the
    config's first iteration, through the reference's own classes: the update's inputs, the
    models' parameters before / after, every scheduled fit's per-epoch losses and the torch
    RNG state it started from (the DM policy fit's per-epoch rsample noise), the imitation
    result (first PolicyLearningBidder update), and the torch RNG state after the update
    (PolicyLearningBidder draws one rsample per record after its fit, :423)."""
    import torch
    import Models
    _, _, _, (agents, _, _) = capture(load_cfg(cfg_name), rounds, keep=True)
    recs = []

    class RecRP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)
            self.rec = {"rng": torch.get_rng_state().clone(), "losses": []}
            recs.append(self.rec)

        def step(self, metrics, *a, **k):
            self.rec["losses"].append(float(metrics))
            return super().step(metrics, *a, **k)

    init_snap = {}
    orig_init = Models.BidShadingContextualBandit.initialise_policy

    def rec_init(self, X, gammas):
        orig_init(self, X, gammas)
        init_snap["params"] = [p.detach().numpy().copy() for p in self.parameters()]

    def params(mod):
        return [p.detach().numpy().copy() for p in mod.parameters()]

    mse_log = []

    class RecMSE(torch.nn.MSELoss):  # the imitation's two MSE terms per epoch (no scheduler)
        def forward(self, a, b):
            r = super().forward(a, b)
            mse_log.append(r.detach().clone())
            return r

    saved = torch.optim.lr_scheduler.ReduceLROnPlateau
    saved_mse = torch.nn.MSELoss
    torch.optim.lr_scheduler.ReduceLROnPlateau = RecRP
    torch.nn.MSELoss = RecMSE
    Models.BidShadingContextualBandit.initialise_policy = rec_init
    out = {}
    try:
        for i, ag in enumerate(agents):
            b = ag.bidder
            L = ag.logs
            k = f"a{i}_"
            mse_log.clear()
            out[k + "est_ctr"] = np.array([o.estimated_CTR for o in L])
            out[k + "value"] = np.array([o.value for o in L])
            out[k + "price"] = np.array([o.price for o in L])
            out[k + "outcome"] = np.array([o.outcome for o in L]).astype(np.int8)
            won = np.array([o.won for o in L])
            out[k + "won"] = won.astype(np.int8)
            out[k + "gamma"] = np.array([float(g) for g in b.gammas])
            out[k + "propensity"] = np.array([float(p) for p in b.propensities])
            util = np.zeros(len(L))
            util[won] = out[k + "value"][won] * out[k + "outcome"][won] - out[k + "price"][won]
            out[k + "util"] = util
            mods = {"wr": getattr(b, "winrate_model", None),
                    "pol": getattr(b, "bidding_policy", None) or getattr(b, "model", None)}
            for name, mod in mods.items():
                if mod is not None:
                    for j, p in enumerate(params(mod)):
                        out[k + f"{name}0_{j}"] = p
            recs.clear()
            init_snap.clear()
            ag.update(iteration=0)  # LR-TS allocator update, then the bidder's
            out[k + "rng_after"] = torch.get_rng_state().numpy()
            fits = recs[1:]  # recs[0]: the LR-TS allocator's scheduler
            for j, r in enumerate(fits):
                out[k + f"fit{j}_losses"] = np.array(r["losses"])
                out[k + f"fit{j}_rng"] = r["rng"].numpy()
            if init_snap:
                for j, p in enumerate(init_snap["params"]):
                    out[k + f"pol_init_{j}"] = p
                out[k + "init_losses"] = np.array([(mse_log[2 * e] + mse_log[2 * e + 1]).item()
                                                   for e in range(len(mse_log) // 2)])
            if hasattr(b, "model"):  # every PolicyLearningBidder loss at the imitation result
                import copy
                Xc = torch.Tensor(np.hstack((out[k + "est_ctr"].reshape(-1, 1), out[k + "value"].reshape(-1, 1))))
                gt = torch.Tensor(out[k + "gamma"])
                pr = torch.clip(torch.Tensor(out[k + "propensity"]), min=1e-15)
                for name in ("REINFORCE", "REINFORCE_offpolicy", "TRPO", "PPO"):
                    m = copy.deepcopy(b.model)
                    with torch.no_grad():
                        for p, v in zip(m.parameters(), init_snap["params"]):
                            p.copy_(torch.from_numpy(v))
                    m.loss_name = name
                    loss = m.loss(Xc, gt, pr, torch.Tensor(util), importance_weight_clipping_eps=50.0)
                    loss.backward()
                    out[k + f"loss0_{name}"] = np.array(loss.item())
                    out[k + f"grad0_{name}"] = np.concatenate([p.grad.numpy().ravel() for p in m.parameters()])
            for name, mod in mods.items():
                if mod is not None:
                    for j, p in enumerate(params(mod)):
                        out[k + f"{name}1_{j}"] = p
            print(cfg_name, "agent", i, "n", len(L), "fits", [len(r["losses"]) for r in fits], flush=True)
    finally:
        torch.optim.lr_scheduler.ReduceLROnPlateau = saved
        torch.nn.MSELoss = saved_mse
        Models.BidShadingContextualBandit.initialise_policy = orig_init
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def learner_driver_kat(cfg_name, out_name, rounds, iters, torch_seed=0):
    """The reference's driver loop (src/main.py:113-155) on a learning-bidder config for
    `iters` iterations of `rounds` rounds (torch seeded with torch_seed before the agents
    are built), recording per iteration the revenue, net and gross utilities, and after
    every agent's update its bidder's parameters, the scheduled fits' epochs, the
    imitation's epochs and the torch generator state; plus the numpy Generator state after
    each iteration's rounds."""
    import torch
    import main as M
    cfg = load_cfg(cfg_name, num_runs=1, num_iter=iters, rounds_per_iter=rounds)
    path = write_cfg(cfg)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     E, var, OE) = M.parse_config(path)
    os.unlink(path)
    torch.manual_seed(torch_seed)
    agents = M.instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
    auction, num_iter, rpi, _ = M.instantiate_auction(rng, config, agents2items, agents2item_values,
                                                      agents, max_slots, E, var, OE)
    recs, mse_n = [], [0]

    class RecRP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)
            self.n = 0
            recs.append(self)

        def step(self, metrics, *a, **k):
            self.n += 1
            return super().step(metrics, *a, **k)

    class RecMSE(torch.nn.MSELoss):
        def forward(self, a, b):
            mse_n[0] += 1
            return super().forward(a, b)

    saved, saved_mse = torch.optim.lr_scheduler.ReduceLROnPlateau, torch.nn.MSELoss
    torch.optim.lr_scheduler.ReduceLROnPlateau, torch.nn.MSELoss = RecRP, RecMSE
    out = {"cfg": np.array(json.dumps(cfg))}
    try:
        for it in range(num_iter):
            for _ in range(rpi):
                auction.simulate_opportunity()
            out[f"it{it}_revenue"] = np.array(auction.revenue)
            out[f"it{it}_net"] = np.array([a.net_utility for a in agents])
            out[f"it{it}_gross"] = np.array([a.gross_utility for a in agents])
            out[f"it{it}_np_state"] = np.array(json.dumps(rng.bit_generator.state))
            for i, a in enumerate(agents):
                recs.clear()
                mse_n[0] = 0
                a.update(iteration=it)
                b = a.bidder
                out[f"it{it}_a{i}_fits"] = np.array([r.n for r in recs[1:]])  # recs[0]: LR-TS
                out[f"it{it}_a{i}_imitation"] = np.array(mse_n[0] // 2)
                for name in ("winrate_model", "bidding_policy", "model"):
                    mod = getattr(b, name, None)
                    if mod is not None:
                        out[f"it{it}_a{i}_{name}"] = np.concatenate(
                            [p.detach().numpy().ravel() for p in mod.parameters()])
                out[f"it{it}_a{i}_init"] = np.array(bool(b.model_initialised))
                out[f"it{it}_a{i}_torch_state"] = torch.get_rng_state().numpy()
                a.clear_utility()
                a.clear_logs()
            auction.clear_revenue()
            print(cfg_name, "iteration", it, "revenue", out[f"it{it}_revenue"],
                  [list(out[f"it{it}_a{i}_fits"]) for i in range(len(agents))], flush=True)
    finally:
        torch.optim.lr_scheduler.ReduceLROnPlateau, torch.nn.MSELoss = saved, saved_mse
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def later_update_kat(cfg_name, out_name, rounds, iters, torch_seed=0):
    """Every Agent.update of the reference's driver loop (src/main.py:113-155) on `cfg_name`
    for `iters` iterations of `rounds` rounds, recorded at its inputs and outputs so that the
    oracle can be run from EXACTLY the reference's state at iterations >= 1 (the verdict's
    "pin later-iteration updates"): per iteration and agent, the LR-TS allocator's won samples
    and posterior before / after with its per-epoch losses, and (learning bidders) the logged
    records, the models before / after, every scheduled fit's per-epoch losses and the torch
    generator state it started from (the DR / DM policy fit's per-epoch rsample noise)."""
    import torch
    import main as M
    import BidderAllocation as BA
    cfg = load_cfg(cfg_name, num_runs=1, num_iter=iters, rounds_per_iter=rounds)
    path = write_cfg(cfg)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     E, var, OE) = M.parse_config(path)
    os.unlink(path)
    torch.manual_seed(torch_seed)
    agents = M.instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
    auction, num_iter, rpi, _ = M.instantiate_auction(rng, config, agents2items, agents2item_values,
                                                      agents, max_slots, E, var, OE)
    recs = []

    class RecRP(torch.optim.lr_scheduler.ReduceLROnPlateau):
        def __init__(self, *a, verbose=None, **k):
            super().__init__(*a, **k)
            self.rec = {"rng": torch.get_rng_state().clone(), "losses": []}
            recs.append(self.rec)

        def step(self, metrics, *a, **k):
            self.rec["losses"].append(float(metrics))
            return super().step(metrics, *a, **k)

    def params(mod):
        return np.concatenate([p.detach().numpy().ravel() for p in mod.parameters()])

    saved = torch.optim.lr_scheduler.ReduceLROnPlateau
    torch.optim.lr_scheduler.ReduceLROnPlateau = RecRP
    out = {"cfg": np.array(json.dumps(cfg))}
    try:
        for it in range(num_iter):
            for _ in range(rpi):
                auction.simulate_opportunity()
            for i, a in enumerate(agents):
                k = f"it{it}_a{i}_"
                L = a.logs
                won = np.array([o.won for o in L], bool)
                out[k + "won"] = won.astype(np.int8)
                lrts = isinstance(a.allocator, BA.PyTorchLogisticRegressionAllocator)
                if lrts:
                    rm = a.allocator.response_model
                    ctx = np.array([o.context for o in L])
                    out[k + "X"] = ctx[won]
                    out[k + "A"] = np.array([o.item for o in L], np.int64)[won]
                    out[k + "y"] = np.array([o.outcome for o in L], np.float64)[won]
                    out[k + "m0"] = rm.m.detach().numpy().copy()
                    out[k + "prevm0"] = rm.prev_iter_m.numpy().copy()
                    out[k + "q0"] = rm.q.numpy().copy()
                b = a.bidder
                learner = hasattr(b, "winrate_model") or hasattr(b, "bidding_policy")
                if learner:
                    out[k + "est_ctr"] = np.array([o.estimated_CTR for o in L])
                    out[k + "value"] = np.array([o.value for o in L])
                    out[k + "price"] = np.array([o.price for o in L])
                    out[k + "outcome"] = np.array([o.outcome for o in L], np.int8)
                    out[k + "gamma"] = np.array([float(g) for g in b.gammas])
                    if hasattr(b, "propensities"):
                        out[k + "propensity"] = np.array([float(p) for p in b.propensities])
                    out[k + "init0"] = np.array(bool(getattr(b, "model_initialised", False)))
                    for name in ("winrate_model", "bidding_policy"):
                        if getattr(b, name, None) is not None:
                            out[k + name + "0"] = params(getattr(b, name))
                recs.clear()
                a.update(iteration=it)
                fits = [r for r in recs]
                if lrts:
                    lr = fits.pop(0)
                    out[k + "lrts_losses"] = np.array(lr["losses"])
                    out[k + "m1"] = rm.m.detach().numpy().copy()
                    out[k + "q1"] = rm.q.numpy().copy()
                for j, r in enumerate(fits):
                    out[k + f"fit{j}_losses"] = np.array(r["losses"])
                    out[k + f"fit{j}_rng"] = r["rng"].numpy()
                if learner:
                    for name in ("winrate_model", "bidding_policy"):
                        if getattr(b, name, None) is not None:
                            out[k + name + "1"] = params(getattr(b, name))
                a.clear_utility()
                a.clear_logs()
            auction.clear_revenue()
            print(cfg_name, "iteration", it, flush=True)
    finally:
        torch.optim.lr_scheduler.ReduceLROnPlateau = saved
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def search_bid_kat(out_name="search_bid_kat", rounds=1000, bids=4000):
    """ValueLearningBidder 'search' bids (src/Bidder.py:180-196) of FP_DM_Oracle's agents after
    their first update, through the reference's own bid(): per call the (value, estimated
    CTR) given, the 128-point grid it drew (the same draws from a clone of its Generator) and
    the gamma it chose, with the agent's win-rate parameters."""
    import torch
    import main as M
    cfg = load_cfg("FP_DM_Oracle.json", num_runs=1, num_iter=1, rounds_per_iter=rounds)
    path = write_cfg(cfg)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     E, var, OE) = M.parse_config(path)
    os.unlink(path)
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
    auction, _, rpi, _ = M.instantiate_auction(rng, config, agents2items, agents2item_values,
                                               agents, max_slots, E, var, OE)
    for _ in range(rpi):
        auction.simulate_opportunity()
    out = {}
    g = np.random.default_rng(11)
    for i, a in enumerate(agents):
        a.update(iteration=0)
        b = a.bidder
        assert b.model_initialised
        out[f"a{i}_wr"] = np.concatenate([p.detach().numpy().ravel() for p in b.winrate_model.parameters()])
        vals = g.lognormal(0.1, 0.2, bids)
        ctrs = 1.0 / (1.0 + np.exp(-g.normal(-3.0, 1.0, bids)))
        gammas, out_bids = np.zeros(bids), np.zeros(bids)
        # each bid draws exactly its 128 grid points from the shared Generator: the grids
        # are regenerated from this state by the test
        out[f"a{i}_rng_state"] = np.array(json.dumps(b.rng.bit_generator.state))
        for j in range(bids):
            out_bids[j] = b.bid(vals[j], None, ctrs[j])
            gammas[j] = b.gammas[-1]
        out[f"a{i}_value"], out[f"a{i}_ctr"] = vals, ctrs
        out[f"a{i}_gamma"], out[f"a{i}_bid"] = gammas, out_bids
        print("search bids agent", i, "gamma mean", gammas.mean(), flush=True)
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


def sigmoid_kats():
    """Reference sigmoid (numba-faithful shim) on OracleAllocator-shaped dots."""
    import Models
    g = np.random.default_rng(7)
    z = np.concatenate([g.normal(0, 4, 20000), g.uniform(-745, 710, 2000),
                        np.array([0.0, -0.0, 1e-300, -1e-300, 36.0, -36.0, 709.0, -709.0, -745.0, 40.0])])
    np.savez_compressed(os.path.join(OUT, "sigmoid_kat.npz"), z=z, sigmoid=Models.sigmoid(z))
    print("wrote sigmoid_kat")


def full_run_aggregates(cfg_name, runs=None, iters=None, rounds=None):
    """SP_Oracle as shipped: per-iteration revenue / net / gross / regrets (src/main.py:113-155 loop)."""
    import main as M
    cfg = load_cfg(cfg_name)
    if runs is not None:
        cfg["num_runs"] = runs
    if iters is not None:
        cfg["num_iter"] = iters
    if rounds is not None:
        cfg["rounds_per_iter"] = rounds
    path = write_cfg(cfg)
    (rng, config, agent_configs, agents2items, agents2item_values, num_runs, max_slots,
     E, var, OE) = M.parse_config(path)
    os.unlink(path)
    res = []
    for run in range(num_runs):
        agents = M.instantiate_agents(rng, agent_configs, agents2item_values, agents2items)
        auction, num_iter, rpi, _ = M.instantiate_auction(rng, config, agents2items, agents2item_values,
                                                          agents, max_slots, E, var, OE)
        for i in range(num_iter):
            for _ in range(rpi):
                auction.simulate_opportunity()
            row = {"run": run, "iter": i, "revenue": auction.revenue,
                   "net": [a.net_utility for a in agents], "gross": [a.gross_utility for a in agents],
                   "allocation_regret": [float(a.get_allocation_regret()) for a in agents],
                   "estimation_regret": [float(a.get_estimation_regret()) for a in agents],
                   "overbid_regret": [float(a.get_overbid_regret()) for a in agents],
                   "underbid_regret": [float(a.get_underbid_regret()) for a in agents],
                   "ctr_rmse": [float(a.get_CTR_RMSE()) for a in agents],
                   "mean_best_ev": [float(np.mean([o.best_expected_value for o in a.logs])) for a in agents]}
            res.append(row)
            for a in agents:
                a.update(iteration=i)
                a.clear_utility()
                a.clear_logs()
            auction.clear_revenue()
            print(cfg_name, run, i, row["revenue"], flush=True)
    return {"config": cfg, "iterations": res}


EMPIRICAL_CASES = (  # (gamma_sigma, init_gamma, P, allocation, seed, rounds)
    (0.05, 0.9, 2, "FirstPrice", 15, 2048),
    (0.2, 0.6, 3, "FirstPrice", 16, 4096),
    (0.5, 1.0, 2, "SecondPrice", 17, 4096),
)


def empirical_update_kat(out_name="empirical_update_kat", iters=3):
    """EmpiricalShadedBidder.update (src/Bidder.py:60-147) through the reference's own driver
    loop (src/main.py:113-155): per case and iteration, every agent's inputs to the update
    (gammas, and the utilities it computes from the logs) and prev_gamma before / after."""
    import main as M
    out = {}
    for ci, (sigma, init, P, alloc, seed, rounds) in enumerate(EMPIRICAL_CASES):
        cfg = oracle_truthful_cfg(6, 12, P, alloc, seed=seed)
        cfg["agents"][0]["bidder"] = {"type": "EmpiricalShadedBidder",
                                      "kwargs": {"gamma_sigma": sigma, "init_gamma": init}}
        cfg["rounds_per_iter"], cfg["num_iter"] = rounds, iters
        out[f"c{ci}_cfg"] = np.array(json.dumps(cfg))
        path = write_cfg(cfg)
        (rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE) = M.parse_config(path)
        os.unlink(path)
        agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
        auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
        for it in range(iters):
            for _ in range(rounds):
                auction.simulate_opportunity()
            out[f"c{ci}_it{it}_revenue"] = np.array(auction.revenue)
            out[f"c{ci}_it{it}_net"] = np.array([a.net_utility for a in agents])
            for i, a in enumerate(agents):
                won = np.array([o.won for o in a.logs])
                util = np.zeros(len(a.logs))
                vals = np.array([o.value for o in a.logs])
                outc = np.array([o.outcome for o in a.logs])
                pr = np.array([o.price for o in a.logs])
                util[won] = vals[won] * outc[won] - pr[won]
                k = f"c{ci}_it{it}_a{i}"
                out[k + "_gammas"] = np.array(a.bidder.gammas, np.float64)
                out[k + "_util"] = util
                out[k + "_pg0"] = np.array(float(a.bidder.prev_gamma))
                a.update(iteration=it)
                out[k + "_pg1"] = np.array(float(a.bidder.prev_gamma))
                a.clear_utility()
                a.clear_logs()
            auction.clear_revenue()
            print("empirical", ci, it, [float(out[f"c{ci}_it{it}_a{i}_pg1"]) for i in range(6)], flush=True)
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


MEMORY_CASES = {
    # name: (population, memory, rounds, iterations, allocation, seed)
    "empirical": ("empirical", 300, 1000, 4, "FirstPrice", 31),
    "lrts": ("lrts", 150, 1000, 3, "SecondPrice", 32),
}


def memory_driver_kat(out_name="memory_driver_kat"):
    """Agent(memory=M) (src/Agent.py:124-129; 'memory' in an agent config, src/main.py:87)
    through the reference's own driver loop (src/main.py:113-155): per iteration the revenue,
    the utilities and, after every agent's update (before clear_logs), the metrics main.py
    records over its logs -- which carry the last M records of the previous iteration -- the
    log count and the learner's new state (prev_gamma / LR-TS m)."""
    import torch
    import main as M
    out = {}
    for name, (pop, mem, rounds, iters, alloc, seed) in MEMORY_CASES.items():
        if pop == "empirical":
            cfg = oracle_truthful_cfg(6, 12, 2, alloc, seed=seed)
            cfg["agents"][0]["bidder"] = {"type": "EmpiricalShadedBidder",
                                          "kwargs": {"gamma_sigma": 0.05, "init_gamma": 0.9}}
        else:
            cfg = load_cfg("SP_Truthful_TS.json", random_seed=seed, allocation=alloc)
        cfg["agents"][0]["memory"] = mem
        cfg["rounds_per_iter"], cfg["num_iter"], cfg["num_runs"] = rounds, iters, 1
        out[f"{name}_cfg"] = np.array(json.dumps(cfg))
        path = write_cfg(cfg)
        (rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE) = M.parse_config(path)
        os.unlink(path)
        torch.manual_seed(0)
        agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
        auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
        for it in range(iters):
            for _ in range(rounds):
                auction.simulate_opportunity()
            k = f"{name}_it{it}"
            out[k + "_revenue"] = np.array(auction.revenue)
            out[k + "_net"] = np.array([a.net_utility for a in agents])
            out[k + "_gross"] = np.array([a.gross_utility for a in agents])
            met = []
            for i, a in enumerate(agents):
                out[k + f"_a{i}_nlogs"] = np.array(len(a.logs))
                a.update(iteration=it)
                met.append([a.get_allocation_regret(), a.get_estimation_regret(), a.get_overbid_regret(),
                            a.get_underbid_regret(), a.get_CTR_RMSE(), a.get_CTR_bias(),
                            np.mean([o.best_expected_value for o in a.logs])])
                if pop == "empirical":
                    out[k + f"_a{i}_pg"] = np.array(float(a.bidder.prev_gamma))
                else:
                    out[k + f"_a{i}_m"] = a.allocator.response_model.m.detach().numpy().copy()
                a.clear_utility()
                a.clear_logs()
            out[k + "_metrics"] = np.array(met, np.float64)
            auction.clear_revenue()
            print("memory", name, it, float(out[k + "_revenue"]), flush=True)
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


INTERLEAVE_STEPS = (("sim", 600), ("upd", 0), ("sim", 300), ("upd", 0), ("upd", 1), ("clr", 1), ("clr", 0),
                    ("sim", 200), ("upd", 0), ("upd", 1), ("upd", 2), ("upd", 3), ("upd", 4), ("upd", 5),
                    ("sim", 150))


def interleave_kat(out_name="interleave_kat"):
    """Notebook-style use of the per-agent surface (src/Agent.py:79-94, :124-129): rounds
    simulated between one agent's update() and the others', a second update() of an agent's
    grown logs, clear_logs() of some agents only -- the sequence INTERLEAVE_STEPS on two
    populations (EmpiricalShadedBidders, FirstPrice: exact; SP_Truthful_TS LR-TS allocators:
    float32 torch fits). Recorded after every step: revenue, utilities, every agent's log count
    and learner state (prev_gamma / LR-TS m, q)."""
    import torch
    import main as M
    out = {"steps": np.array(json.dumps(INTERLEAVE_STEPS))}
    for name in ("empirical", "lrts"):
        if name == "empirical":
            cfg = oracle_truthful_cfg(6, 12, 2, "FirstPrice", seed=5)
            cfg["agents"][0]["bidder"] = {"type": "EmpiricalShadedBidder",
                                          "kwargs": {"gamma_sigma": 0.05, "init_gamma": 0.9}}
        else:
            cfg = load_cfg("SP_Truthful_TS.json", random_seed=5)
        cfg["num_runs"], cfg["num_iter"] = 1, 1
        out[f"{name}_cfg"] = np.array(json.dumps(cfg))
        path = write_cfg(cfg)
        (rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE) = M.parse_config(path)
        os.unlink(path)
        torch.manual_seed(0)
        agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
        auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
        for j, (op, arg) in enumerate(INTERLEAVE_STEPS):
            if op == "sim":
                for _ in range(arg):
                    auction.simulate_opportunity()
            elif op == "upd":
                agents[arg].update(iteration=j)
            else:
                agents[arg].clear_logs()
            k = f"{name}_s{j}"
            out[k + "_revenue"] = np.array(auction.revenue)
            out[k + "_net"] = np.array([a.net_utility for a in agents])
            out[k + "_nlogs"] = np.array([len(a.logs) for a in agents])
            if name == "empirical":
                out[k + "_pg"] = np.array([float(a.bidder.prev_gamma) for a in agents])
            else:
                out[k + "_m"] = np.stack([a.allocator.response_model.m.detach().numpy().copy() for a in agents])
                out[k + "_q"] = np.stack([a.allocator.response_model.q.detach().numpy().copy() for a in agents])
        print("interleave", name, float(out[k + "_revenue"]), flush=True)
    np.savez_compressed(os.path.join(OUT, out_name + ".npz"), **out)


CSV_CASES = {
    # name: config overrides on oracle_truthful_cfg(...) (both populations run end to end on
    # the GPU path, so main.py's CSV files can be compared cell by cell)
    "sp_oracle": (dict(n_agents=6, n_items=12, P=2, allocation="SecondPrice", seed=0), None),
    "fp_empirical": (dict(n_agents=6, n_items=12, P=2, allocation="FirstPrice", seed=21),
                     {"type": "EmpiricalShadedBidder", "kwargs": {"gamma_sigma": 0.05, "init_gamma": 0.9}}),
}


def csv_outputs(runs=2, iters=3, rounds=2000):
    """The reference's own __main__ (src/main.py:157-345) on small configs; its CSV files are
    the fixtures (tests/golden/csv/<case>/), with the config used."""
    import runpy
    import shutil
    for name, (kw, bidder) in CSV_CASES.items():
        cfg = oracle_truthful_cfg(**kw)
        if bidder:
            cfg["agents"][0]["bidder"] = bidder
        cfg.update(num_runs=runs, num_iter=iters, rounds_per_iter=rounds)
        work = tempfile.mkdtemp()
        cfg["output_dir"] = os.path.join(work, "out")
        path = os.path.join(work, "cfg.json")
        with open(path, "w") as f:
            json.dump(cfg, f)
        argv = sys.argv
        sys.argv = ["main.py", path]
        try:
            runpy.run_path(os.path.join(REF_SRC, "main.py"), run_name="__main__")
        finally:
            sys.argv = argv
        dst = os.path.join(OUT, "csv", name)
        os.makedirs(dst, exist_ok=True)
        for f in os.listdir(cfg["output_dir"]):
            if f.endswith(".csv"):
                shutil.copy(os.path.join(cfg["output_dir"], f), dst)
        cfg["output_dir"] = "OUTPUT_DIR"
        with open(os.path.join(dst, "config.json"), "w") as f:
            json.dump(cfg, f, indent=1)
        shutil.rmtree(work)
        print("csv", name, sorted(os.listdir(dst)), flush=True)


def ragged_items_capture(out_name="ragged_items_r2048", rounds=2048):
    """Agents with their own num_items (src/main.py:61,66): 3 Oracle agents with 12 items, 3
    LR-TS (Thompson sampling) agents with 9, 2 with 6 and 1 with 13 -- the sgemv block /
    remainder rows and the catalogue draw order follow each agent's count. The config travels
    in the fixture's meta."""
    cfg = load_cfg("SP_Truthful_TS.json")
    base = cfg["agents"][0]
    orc = {"type": "OracleAllocator", "kwargs": {}}

    def lrts(k):
        return {"type": base["allocator"]["type"], "kwargs": dict(base["allocator"]["kwargs"], num_items=k)}
    cfg["agents"] = [dict(base, name="Oracle 12", num_copies=3, num_items=12, allocator=orc),
                     dict(base, name="TS 9", num_copies=3, num_items=9, allocator=lrts(9)),
                     dict(base, name="TS 6", num_copies=2, num_items=6, allocator=lrts(6)),
                     dict(base, name="TS 13", num_items=13, allocator=lrts(13))]
    cfg["agents"][3].pop("num_copies", None)
    cfg["output_dir"] = "/tmp/ag_golden_unused/"
    a, g, m = capture(cfg, rounds)
    m["config"] = cfg
    save_capture(out_name, a, g, m)


def mixed_ts_flags_capture(out_name="sp_ts_mixed_flags_r2048", rounds=2048):
    """SP_Truthful_TS with thompson_sampling set per allocator (src/BidderAllocation.py:24-26):
    4 LR-TS agents sample, 4 bid from their MAP estimates (estimate_CTR(sample=False),
    src/BidderAllocation.py:67-68). The config travels in the fixture's meta."""
    cfg = load_cfg("SP_Truthful_TS.json")
    base = cfg["agents"][0]
    cfg["agents"] = [dict(base, name="Truthful TS", num_copies=4),
                     dict(base, name="Truthful MAP", num_copies=4,
                          allocator={"type": base["allocator"]["type"],
                                     "kwargs": dict(base["allocator"]["kwargs"], thompson_sampling=False)})]
    cfg["output_dir"] = "/tmp/ag_golden_unused/"
    a, g, m = capture(cfg, rounds)
    m["config"] = cfg
    save_capture(out_name, a, g, m)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also run SP_Oracle as shipped (3x20x10k rounds, ~1 min)")
    ap.add_argument("--which", choices=["dm", "ips", "dr", "dmo", "search"], help="with --only learners/drivers: one config")
    ap.add_argument("--only", choices=["empirical", "csv", "dr", "learners", "drivers", "memory", "later", "mixedts", "ragged",
                                       "interleave"],
                    help="regenerate one fixture family only")
    args = ap.parse_args()
    install_shims()
    if args.only == "interleave":
        interleave_kat()
        return
    if args.only == "mixedts":
        mixed_ts_flags_capture()
        return
    if args.only == "ragged":
        ragged_items_capture()
        return
    if args.only == "memory":
        memory_driver_kat()
        return
    if args.only == "later":
        later_update_kat("SP_Truthful_TS.json", "sp_ts_later_kat", rounds=2000, iters=3)
        later_update_kat("FP_DR_TS.json", "dr_later_kat", rounds=1000, iters=3)
        return
    if args.only == "empirical":
        empirical_update_kat()
        return
    if args.only == "csv":
        csv_outputs()
        return
    if args.only == "dr":
        dr_update_kat()
    if args.only == "drivers":
        if args.which in (None, "search"):
            search_bid_kat()
        for cfg_name, tag in (("FP_DR_TS.json", "dr"), ("FP_DM_TS.json", "dm"), ("FP_IPS_TS.json", "ips"),
                              ("FP_DM_Oracle.json", "dmo")):
            if args.which in (None, tag):
                learner_driver_kat(cfg_name, f"{tag}_driver_kat", rounds=1000, iters=3)
        return
    if args.only == "learners":
        if args.which in (None, "dm"):
            learner_update_kat("FP_DM_TS.json", "dm_update_kat")
        if args.which in (None, "ips"):
            learner_update_kat("FP_IPS_TS.json", "ips_update_kat")
        return

    sigmoid_kats()
    alloc_kats()

    # 1. SP_Oracle.json exactly as shipped (seed 0, N=6, P=2, K=12, E=5): first 4096 rounds of run 0.
    a, g, m = capture(load_cfg("SP_Oracle.json"), 4096)
    save_capture("sp_oracle_r4096", a, g, m)
    # 2. FirstPrice, 8 truthful Oracle agents, P=3 (FP charges, 3-way allocation).
    a, g, m = capture(oracle_truthful_cfg(8, 12, 3, "FirstPrice", seed=11), 2048)
    save_capture("fp_oracle_n8_p3", a, g, m)
    # 3. SecondPrice, 32 agents, P=8 (wider auctions, the Mixed-population width).
    a, g, m = capture(oracle_truthful_cfg(32, 12, 8, "SecondPrice", seed=12), 2048)
    save_capture("sp_oracle_n32_p8", a, g, m)
    # 4. P=1 edge: prices empty -> nobody charged, no revenue, U still drawn (src/Auction.py:65-74).
    a, g, m = capture(oracle_truthful_cfg(4, 12, 1, "SecondPrice", seed=13), 256)
    save_capture("sp_oracle_n4_p1", a, g, m)
    # 5. Non-default catalogue shape: K=5 items, E=5.
    a, g, m = capture(oracle_truthful_cfg(5, 5, 2, "FirstPrice", seed=14), 1024)
    save_capture("fp_oracle_n5_k5", a, g, m)

    # 6. SP_Truthful_TS.json as shipped: LR-TS Thompson sampling (torch seeded 0, noise
    #    recorded), 2048 rounds of iteration 0, then the LR-TS update KATs on those logs.
    a, g, m, (agents, _, _) = capture(load_cfg("SP_Truthful_TS.json"), 2048, keep=True)
    save_capture("sp_ts_r2048", a, g, m)
    lrts_update_kat(agents, "sp_ts_update_kat")
    # 7. Learned bidders in their first (uninitialised) iteration: Gaussian shading draws.
    for cfg_name, tag in (("FP_DR_TS.json", "fp_dr_ts_r1024"), ("FP_DM_TS.json", "fp_dm_ts_r1024"),
                          ("FP_IPS_TS.json", "fp_ips_ts_r1024"), ("FP_DM_Oracle.json", "fp_dm_oracle_r1024")):
        a, g, m = capture(load_cfg(cfg_name), 1024)
        save_capture(tag, a, g, m)
    # 8. EmpiricalShadedBidder with Oracle CTRs (clipped Gaussian shading, src/Bidder.py:38-58).
    cfg = oracle_truthful_cfg(6, 12, 2, "FirstPrice", seed=15)
    cfg["agents"][0]["bidder"] = {"type": "EmpiricalShadedBidder",
                                  "kwargs": {"gamma_sigma": 0.05, "init_gamma": 0.9}}
    a, g, m = capture(cfg, 2048)
    save_capture("fp_empirical_r2048", a, g, m)
    # 9. EmpiricalShadedBidder.update over three iterations of three populations.
    empirical_update_kat()
    # 10. main.py's CSV outputs (SP_Oracle-shaped and EmpiricalShaded, 2 runs x 3 iterations).
    csv_outputs()
    # 11. DoublyRobustBidder.update KATs (FP_DR_TS.json, iteration 0).
    dr_update_kat()

    if args.full:
        agg = full_run_aggregates("SP_Oracle.json")
        with open(os.path.join(OUT, "sp_oracle_full_run.json"), "w") as f:
            json.dump(agg, f)
        print("wrote sp_oracle_full_run.json")


if __name__ == "__main__":
    main()
