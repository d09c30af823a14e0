"""Auction: the surface of src/Auction.py:9-77, executed as batched HIP kernels.

Rounds within an iteration are independent given agent state (agent state changes only
in Agent.update, between iterations), so the round loop is a data-parallel batch:

* `simulate_opportunity()` -- the reference's per-round call. It draws the round's
  random inputs from the shared numpy Generator in the reference's order (src/Auction.py:
  30, 33, 42, then the one next_double binomial consumes at :65) and queues them; the
  queued rounds run as ONE fused kernel launch the first time anything reads state
  (net_utility, revenue, update, ...). Same draws, same results, one launch.
* `simulate_batch(B)` -- the same, for B rounds at once.
* `simulate_synthetic(B, seed)` -- B rounds whose inputs are generated on the GPU
  (Philox4x32-10 keyed by the global auction index); the rng is not touched.
"""
import numpy as np
import torch

from . import Agent as _agent_mod
from . import _lib
from .engine import AuctionEngine
from .replay import draw_round

C = _agent_mod.C


class Auction:
    """Base class for auctions (src/Auction.py:9-26)."""

    FLUSH_ROUNDS = 1 << 20

    def __init__(self, rng, allocation, agents, agent2items, agents2item_values, max_slots,
                 embedding_size, embedding_var, obs_embedding_size, num_participants_per_round):
        self.rng = rng
        self.allocation = allocation
        self.agents = agents
        self.max_slots = max_slots
        self.agent2items = agent2items
        self.agents2item_values = agents2item_values
        self.embedding_size = embedding_size
        self.embedding_var = embedding_var
        self.obs_embedding_size = obs_embedding_size
        self.num_participants_per_round = num_participants_per_round
        if max_slots != 1:
            raise NotImplementedError("max_slots must be 1 (src/main.py:37)")

        ks = {len(agents2item_values[a.name]) for a in agents}
        if len(ks) != 1:
            raise NotImplementedError("all agents must have the same num_items")
        K = ks.pop()
        for a in agents:
            if a.allocator.kind is None or a.bidder.kind is None:
                raise NotImplementedError(
                    f"agent {a.name!r}: {type(a.allocator).__name__} + {type(a.bidder).__name__} "
                    "is not on the GPU path yet (built: OracleAllocator + TruthfulBidder)")
        self._engine = AuctionEngine(len(agents), num_participants_per_round, K, embedding_size,
                                     obs_embedding_size, allocation.code, embedding_var)
        self._engine.set_agent_kinds([a.allocator.kind for a in agents],
                                     [a.bidder.kind for a in agents])
        self._values = np.stack([np.asarray(agents2item_values[a.name], np.float64) for a in agents])
        self._engine.load_catalog(np.stack([np.asarray(agent2items[a.name], np.float64)
                                            for a in agents]), self._values)
        for i, a in enumerate(agents):
            a._attach(self, i)
        self._revenue_fx = 0
        self._pending_ctx, self._pending_part, self._pending_u = [], [], []
        self._log_batches = []
        self._log_base = 0
        self._logged_rounds = 0
        self.keep_logs = True

    # ------------------------------------------------------------------ rounds
    def _draw_round(self):
        ctx, part, u = draw_round(self.rng, len(self.agents), self.num_participants_per_round,
                                  self.embedding_size, self.embedding_var, self.max_slots)
        self._pending_ctx.append(ctx)
        self._pending_part.append(part)
        self._pending_u.append(u)

    def simulate_opportunity(self):
        """One round (src/Auction.py:28-74), queued into the next batched launch."""
        self._draw_round()
        if len(self._pending_u) >= self.FLUSH_ROUNDS:
            self._flush()

    def simulate_batch(self, B):
        """B rounds with the reference's draws, run as one batch."""
        for _ in range(int(B)):
            self._draw_round()
            if len(self._pending_u) >= self.FLUSH_ROUNDS:
                self._flush()
        self._flush()

    def simulate_synthetic(self, B, seed, first_auction=0):
        """B rounds with on-device Philox inputs (throughput mode; parity via the oracle)."""
        self._flush()
        eng = self._engine
        inp = eng.alloc_inputs(int(B))
        eng.generate(seed, first_auction, inp)
        self._run(inp)

    # ------------------------------------------------------------------ engine
    def _flush(self):
        if not self._pending_u:
            return
        d = self._engine.device
        ctx = torch.from_numpy(np.ascontiguousarray(np.array(self._pending_ctx, np.float64).T)).to(d)
        part = torch.from_numpy(np.ascontiguousarray(np.array(self._pending_part, np.int32).T)).to(d)
        u = torch.from_numpy(np.array(self._pending_u, np.float64)).to(d)
        self._pending_ctx, self._pending_part, self._pending_u = [], [], []
        self._run({"ctx": ctx, "part": part, "u": u})

    def _run(self, inp):
        eng = self._engine
        B = inp["u"].shape[0]
        out = eng.alloc_outputs(B)
        cnt = eng.new_counters()
        max_b = 2048 * 8192
        for lo in range(0, B, max_b):
            hi = min(B, lo + max_b)
            sl_in = {"ctx": inp["ctx"][:, lo:hi].contiguous(), "part": inp["part"][:, lo:hi].contiguous(),
                     "u": inp["u"][lo:hi]}
            sl_out = {k: (v[:, lo:hi] if v.dim() == 2 else v[lo:hi]) for k, v in out.items()}
            if hi - lo != B:  # kernels need contiguous slices
                sl_out = {k: torch.empty_like(v) for k, v in sl_out.items()}
            eng.simulate(sl_in, sl_out, cnt)
            if hi - lo != B:
                for k, v in out.items():
                    (v[:, lo:hi] if v.dim() == 2 else v[lo:hi]).copy_(sl_out[k])
        limbs = cnt.cpu().numpy()
        paid = 0
        for a, agent in enumerate(self.agents):
            for c in range(_lib.NUM_COUNTERS):
                L = limbs[a, c]
                v = int(L[0]) + (int(L[1]) << 42) + (int(L[2]) << 84)
                agent._fx[c] += v
                if c == C["paid"]:
                    paid += v
        self._revenue_fx += paid
        if self.keep_logs:
            self._log_batches.append((inp["part"], out))
        self._logged_rounds += B

    # ------------------------------------------------------------------ logs
    def _log_rounds(self):
        """Rounds run so far; drops the device log buffers once every agent cleared them."""
        self._flush()
        if all(a._log_start >= self._logged_rounds for a in self.agents):
            self._log_batches = []
            self._log_base = self._logged_rounds
        return self._logged_rounds

    def _materialise_logs(self, agent_index, start_round):
        return _agent_mod.materialise(self._log_batches, agent_index,
                                      start_round - self._log_base, self._values)

    # ------------------------------------------------------------------ revenue
    @property
    def revenue(self):
        self._flush()
        return _agent_mod.fx_to_float(self._revenue_fx)

    def clear_revenue(self):
        self._flush()
        self._revenue_fx = 0
