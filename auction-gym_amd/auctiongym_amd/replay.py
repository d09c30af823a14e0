"""Replay-mode inputs: the reference's per-round random draws, in its order.

src/Auction.py draws, per round, from the ONE numpy Generator shared by everything
(src/main.py:29): integers(1, max_slots + 1) (:30; consumes nothing when max_slots == 1),
normal(0, embedding_var, E) (:33), choice(N, P, replace=False) (:42), then, after the
bids, binomial(1, CTR[winner]) (:65), which for n = 1 consumes exactly one next_double U.
TruthfulBidder / OracleAllocator draw nothing in between. Drawing U with rng.random()
leaves the Generator in the same state as the reference after every round
(tests/golden/make_golden.py asserts that on every captured round), so a batch of
rounds can be drawn up front and resolved on the GPU.

(The one exception: numpy's binomial draws nothing when p == 0.0 exactly, i.e. when a
winner's sigmoid underflows to 0, which needs items . ctx < -745.)
"""
import numpy as np


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
