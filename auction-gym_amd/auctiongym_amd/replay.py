"""Replay-mode inputs: the reference's per-round random draws, in its order.

src/Auction.py draws, per round, from the ONE numpy Generator shared by everything
(src/main.py:29): integers(1, max_slots + 1) (:30; consumes nothing when max_slots == 1),
normal(0, embedding_var, E) (:33), choice(N, P, replace=False) (:42), then, after the
bids, binomial(1, CTR[winner]) (:65), which for n = 1 consumes exactly one next_double U.
TruthfulBidder / OracleAllocator draw nothing in between. Drawing U with rng.random()
leaves the Generator in the same state as the reference after every round
(tests/golden/make_golden.py asserts that on every captured round), so a batch of
rounds can be drawn up front and resolved on the GPU.

Populations with shading bidders or Thompson-sampling allocators draw more per round, in
slot order after the participants (src/Agent.py:44-53): a shading bidder in its
uninitialised state draws rng.normal(prev_gamma, gamma_sigma) (src/Bidder.py:51, 177, 354,
461); an LR-TS allocator draws torch.normal(0, 1/sqrt(q)) from torch's own global
generator (src/Models.py:31). draw_round_population makes the same calls in the same order.

(The one exception: numpy's binomial draws nothing when p == 0.0 exactly, i.e. when a
winner's sigmoid underflows to 0, which needs items . ctx < -745.)
"""
import numpy as np
import torch


def draw_round(rng, num_agents, num_participants, embedding_size, embedding_var, max_slots=1):
    rng.integers(1, max_slots + 1)
    ctx = rng.normal(0, embedding_var, size=embedding_size)
    part = rng.choice(num_agents, num_participants, replace=False)
    u = rng.random()
    return ctx, part, u


def draw_rounds(rng, B, num_agents, num_participants, embedding_size, embedding_var, max_slots=1):
    """B rounds -> SoA host arrays ctx [E][B] float64, part [P][B] int32, u [B] float64."""
    ctx = np.empty((embedding_size, B))
    part = np.empty((num_participants, B), np.int32)
    u = np.empty(B)
    for r in range(B):
        c, p, uu = draw_round(rng, num_agents, num_participants, embedding_size, embedding_var,
                              max_slots)
        ctx[:, r] = c
        part[:, r] = p
        u[r] = uu
    return ctx, part, u


def draw_round_population(rng, num_agents, num_participants, embedding_size, embedding_var,
                          shading, ts_models, max_slots=1, policy=None, search=None):
    """One round of a general population. shading[a] = (prev_gamma, gamma_sigma) of a shading
    bidder in its uninitialised state (else None); ts_models[a] = the LR-TS model whose
    Thompson draw the round makes (else None); policy[a] = True for a learning bidder bidding
    from its fitted policy, whose rsample draws one standard normal from torch's generator
    (src/Models.py:87-88 / :160-161, via torch.distributions.Normal.rsample); search[a] = True
    for a ValueLearningBidder bidding by search, which draws rng.uniform(0.1, 1.0, 128) and
    sorts it (src/Bidder.py:184-186). Returns ctx [E], part [P], gamma_raw [P] (NaN where
    nothing is drawn), u, ts_noise [P][K*Do] float32 or None, policy_eps [P] float32 (0
    where nothing is drawn) or None, gamma_grid [P][128] (0 where nothing is drawn) or
    None."""
    rng.integers(1, max_slots + 1)
    ctx = rng.normal(0, embedding_var, size=embedding_size)
    part = rng.choice(num_agents, num_participants, replace=False)
    gamma_raw = np.full(num_participants, np.nan)
    noise = None
    eps = None
    grid = None
    for s, a in enumerate(part):
        m = ts_models[a]
        if m is not None:  # Agent.select_item: the allocator's Thompson draw first
            z = m.sample_noise().numpy().ravel()
            if noise is None:
                noise = np.zeros((num_participants, z.size), np.float32)
            noise[s] = z
        if policy is not None and policy[a]:  # then the bidder's
            if eps is None:
                eps = np.zeros(num_participants, np.float32)
            eps[s] = torch.empty(1).normal_().item()
            continue
        if search is not None and search[a]:
            if grid is None:
                grid = np.zeros((num_participants, 128))
            gg = rng.uniform(0.1, 1.0, size=128)
            gg.sort()
            grid[s] = gg
            continue
        sh = shading[a]
        if sh is not None:
            gamma_raw[s] = rng.normal(sh[0], sh[1])
    u = rng.random()
    return ctx, part, gamma_raw, u, noise, eps, grid
