"""Auction: the surface of src/Auction.py:9-77, executed as batched HIP kernels.

Rounds within an iteration are independent given agent state (agent state changes only
in Agent.update, between iterations), so the round loop is a data-parallel batch:

* `simulate_opportunity()` -- the reference's per-round call. It draws the round's
  random inputs in the reference's order (src/Auction.py:30, 33, 42; the bidders' and
  Thompson samplers' draws in slot order; then the one next_double binomial consumes at
  :65) and queues them; the queued rounds run as ONE fused kernel launch the first time
  anything reads state (net_utility, revenue, update, ...). Same draws, same results.
* `simulate_batch(B)` -- the same, for B rounds at once.
* `simulate_synthetic(B, seed)` -- B rounds whose inputs are generated on the GPU
  (Philox4x32-10 keyed by the global auction index); the rng is not touched.

Agent.update of learning plugins (src/Agent.py:79-94) runs on the GPU too: the won
samples of LR-TS agents are collected on the device after every batch
(ag_lrts_collect), and the first LR-TS agent's update() trains every LR-TS agent of the
auction in one launch (ag_lrts_update; the agents' updates are independent, so batching
them is the reference's per-agent loop, src/main.py:127-152).
"""
import warnings

import numpy as np
import torch

from . import Agent as _agent_mod
from . import _lib
from .engine import TORCH_NORMAL_AVX2, AuctionEngine
from .replay import draw_round, draw_round_population, draw_rounds_native, draw_rounds_native_population

C = _agent_mod.C


class Auction:
    """Base class for auctions (src/Auction.py:9-26)."""

    FLUSH_ROUNDS = 1 << 20
    FLUSH_ROUNDS_TS = 1 << 16  # Thompson-sampling rounds carry K*(OE+1) floats per slot

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

        # each agent's own num_items (src/main.py:61,66): catalogues padded to the largest K
        # with value-0 rows (ag_set_agent_items)
        self._num_items = np.array([len(agents2item_values[a.name]) for a in agents], np.int32)
        K = int(self._num_items.max())
        N = len(agents)
        D = embedding_size + 1
        if K == 1 or (D >= 8 and K % 4 != 0):
            # the true CTRs restate numpy's items @ context in OpenBLAS dgemv_t's order, which
            # tests/test_oracle_golden.py pins for K >= 2 with D <= 7 or K % 4 == 0; for other
            # shapes numpy runs other kernels (ddot for K = 1, CPU-dependent remainder kernels)
            warnings.warn(f"catalogue shape K={K}, E+1={D}: bit-exact parity of the true CTRs with the "
                          "reference's numpy dot is unpinned for this shape (DESIGN.md section 5)", stacklevel=2)
        for a in agents:
            if a.allocator.kind is None or a.bidder.kind is None:
                raise NotImplementedError(
                    f"agent {a.name!r}: {type(a.allocator).__name__} + {type(a.bidder).__name__} "
                    "is not on the GPU path")
        ak = np.array([a.allocator.kind for a in agents], np.int32)
        bk = np.array([a.bidder.kind for a in agents], np.int32)
        self._shading = bk != _lib.BIDDER_TRUTHFUL
        self._lrts = ak == _lib.ALLOCATOR_LRTS
        self._engine = eng = AuctionEngine(N, num_participants_per_round, K, embedding_size,
                                           obs_embedding_size, allocation.code, embedding_var)
        pg = np.array([getattr(a.bidder, "prev_gamma", 1.0) for a in agents], np.float64)
        gs = np.array([getattr(a.bidder, "gamma_sigma", 1.0) for a in agents], np.float64)
        eng.set_agent_params(ak, bk, pg if self._shading.any() else None,
                             gs if self._shading.any() else None)
        self._values = np.zeros((N, K))
        items = np.zeros((N, K, embedding_size + 1))
        for i, a in enumerate(agents):
            self._values[i, :self._num_items[i]] = agents2item_values[a.name]
            items[i, :self._num_items[i]] = agent2items[a.name]
        if (self._num_items < K).any():
            eng.set_agent_items(self._num_items)
        eng.load_catalog(items, self._values)
        self._ts = False
        self._ts_agent = np.zeros(len(agents), bool)
        if self._lrts.any():
            lr = [a.allocator for a in agents if a.allocator.kind == _lib.ALLOCATOR_LRTS]
            for i, a in enumerate(agents):
                al = a.allocator
                if al.kind != _lib.ALLOCATOR_LRTS:
                    continue
                if al.embedding_size != obs_embedding_size or al.num_items != self._num_items[i]:
                    raise ValueError(
                        f"PyTorchLogisticRegressionAllocator(embedding_size={al.embedding_size}, "
                        f"num_items={al.num_items}) must model the observed context "
                        f"(obs_embedding_size={obs_embedding_size}) and the agent's {self._num_items[i]} items")
            # thompson_sampling is per allocator (src/BidderAllocation.py:24-26, :67-68): the
            # kernel runs in sampling mode when any LR-TS agent samples; an agent that does not
            # sample gets zero noise, so its "sampled" CTRs are its MAP CTRs (m + 0 = m) and it
            # bids exactly as the reference's sample=False forward (src/Agent.py:29-42)
            self._ts_agent = np.array([bool(self._lrts[i] and a.allocator.thompson_sampling)
                                       for i, a in enumerate(agents)])
            self._ts = bool(self._ts_agent.any())
            self._load_lrts()
        self._learning = np.isin(bk, (_lib.BIDDER_VALUE_LEARNING, _lib.BIDDER_POLICY_LEARNING,
                                      _lib.BIDDER_DOUBLY_ROBUST))
        if self._learning.any():
            self._load_learners()
        for i, a in enumerate(agents):
            a._attach(self, i)
        self._charged = num_participants_per_round >= 2  # P == 1: nobody charged (src/Auction.py:68)
        self._first_price = allocation.code == _lib.FIRST_PRICE
        self._revenue_fx = 0
        self._pending = []
        self._log_batches = []
        self._log_base = 0
        self._logged_rounds = 0
        self.keep_logs = True
        # Agent.update bookkeeping (see _update_agent)
        self._empirical = bk == _lib.BIDDER_EMPIRICAL_SHADED
        self._shading_rec = self._empirical | self._learning  # agents whose records are kept
        self._learner = self._lrts | self._shading_rec
        self._stores = {}                       # device record stores, by learner family
        self._bounds = {"lrts": 0, "shading": 0}  # upper bounds of the records they hold
        # LR-TS updates deferred until something needs their result (_settle_lrts), so that
        # the agents updated one after the other train in one launch
        self._lrts_pending = np.zeros(N, bool)
        self._lrts_drop = np.zeros(N, bool)  # cleared agents whose won samples go at the settle

    def _load_lrts(self):
        K, Do = self._engine.K, self.obs_embedding_size + 1
        shape = (len(self.agents), K, Do)
        m, q, pm = np.zeros(shape, np.float32), np.ones(shape, np.float32), np.zeros(shape, np.float32)
        for i, a in enumerate(self.agents):
            if self._lrts[i]:
                rm = a.allocator.response_model
                k = self._num_items[i]  # rows beyond the agent's own items: m = prev_m = 0, q = 1
                m[i, :k], q[i, :k], pm[i, :k] = rm.m.numpy(), rm.q.numpy(), rm.prev_iter_m.numpy()
        self._engine.load_lrts(m, q, pm, thompson_sampling=self._ts)

    def _load_learners(self):
        """Learning bidders' models and modes onto the device (ag_set_dr_state,
        ag_set_bidder_modes)."""
        N = len(self.agents)
        st = np.zeros((N, 16), np.float32)
        init = np.zeros(N, np.int32)
        modes = np.zeros(N, np.int32)
        for i, a in enumerate(self.agents):
            if self._learning[i]:
                st[i] = a.bidder._state16()
                init[i] = a.bidder._learner_state()
                modes[i] = a.bidder._mode()
        self._engine.set_dr_state(st, init)
        self._engine.set_bidder_modes(modes)

    # ------------------------------------------------------------------ rounds
    def _draw_round(self):
        N, P = len(self.agents), self.num_participants_per_round
        if not (self._shading.any() or (self._lrts.any() and self._ts)):
            ctx, part, u = draw_round(self.rng, N, P, self.embedding_size, self.embedding_var,
                                      self.max_slots)
            self._pending.append((ctx, part, u, None, None, None, None))
            return
        shading, models, policy, search = self._population_draws()
        ctx, part, g, u, noise, eps, grid = draw_round_population(
            self.rng, N, P, self.embedding_size, self.embedding_var, shading, models, self.max_slots,
            policy, search, kdo_max=self._engine.K * (self.obs_embedding_size + 1))
        self._pending.append((ctx, part, u, g, noise, eps, grid))

    def _flush_limit(self):
        return self.FLUSH_ROUNDS_TS if (self._lrts.any() and self._ts) else self.FLUSH_ROUNDS

    def simulate_opportunity(self):
        """One round (src/Auction.py:28-74), queued into the next batched launch."""
        self._settle_lrts()
        self._draw_round()
        if len(self._pending) >= self._flush_limit():
            self._flush()

    def _population_draws(self):
        """Per agent: shading (prev_gamma, gamma_sigma) or None, the LR-TS model making a
        Thompson draw or None, and the learning bidders' policy / search flags (None: no such
        bidder) -- what draw_round_population takes; fixed between updates."""
        shading = [(a.bidder.prev_gamma, a.bidder.gamma_sigma) if self._shading[i] else None
                   for i, a in enumerate(self.agents)]
        models = [a.allocator.response_model if self._ts_agent[i] else None for i, a in enumerate(self.agents)]
        policy = search = None
        if self._learning.any():
            ls = [a.bidder._learner_state() if self._learning[i] else 0 for i, a in enumerate(self.agents)]
            policy = [x == _lib.LEARNER_POLICY for x in ls]
            search = [x == _lib.LEARNER_SEARCH for x in ls]
        return shading, models, policy, search

    # torch CPU builds whose float normal_ of >= 16 elements runs the kernel ag_replay.cpp
    # restates (engine.TORCH_NORMAL_AVX2; the learner fits' draws are gated the same way in
    # engine.torch_normal_epochs)
    _TORCH_NORMAL_AVX2 = TORCH_NORMAL_AVX2

    def _native_draws(self):
        """True when the draws can be made in C for a whole batch: numpy's Generator on PCG64
        (ag_replay_draw / ag_replay_draw_population restate it, and torch's CPU generator for
        the Thompson and rsample draws). Thompson draws are restated for torch's >= 16-element
        vectorised normal kernel only: a sampling LR-TS agent with K*(OE+1) < 16 (torch's
        scalar path) or a torch build without that kernel keeps the per-round loop."""
        if not isinstance(self.rng.bit_generator, np.random.PCG64):
            return False
        if self._lrts.any() and self._ts:
            if torch.backends.cpu.get_cpu_capability() not in self._TORCH_NORMAL_AVX2:
                return False
            kdo = self._num_items * (self.obs_embedding_size + 1)
            if (kdo[self._ts_agent] < 16).any():
                return False
        return True

    NATIVE_ROUNDS = 1 << 20
    NATIVE_ROUNDS_TS = 1 << 18  # Thompson noise: P * K*(OE+1) floats per round on the host

    def simulate_batch(self, B):
        """B rounds with the reference's draws, run as one batch. With numpy's PCG64 generator
        every draw is made in C for the whole batch (replay.draw_rounds_native /
        draw_rounds_native_population: the same numbers and the same numpy and torch generator
        states afterwards as the per-round loop); otherwise the per-round Python loop."""
        B = int(B)
        self._settle_lrts()
        if not self._native_draws():
            for _ in range(B):
                self._draw_round()
                if len(self._pending) >= self._flush_limit():
                    self._flush()
            self._flush()
            return
        self._flush()
        N, P = len(self.agents), self.num_participants_per_round
        shading, models, policy, search = self._population_draws()
        torch_or_grid = (any(m is not None for m in models) or (policy is not None and any(policy))
                         or (search is not None and any(search)))
        # Thompson draws hold P * (K*Do + 16) floats of uniforms per round on the host before the
        # transforms (plus the tiled noise): bounded per chunk, whatever P
        step = (max(1 << 12, (self.NATIVE_ROUNDS_TS * 2) // P) if (self._lrts.any() and self._ts)
                else self.NATIVE_ROUNDS)
        d = self._engine.device
        for lo in range(0, B, step):
            n = min(step, B - lo)
            if torch_or_grid:
                ctx, part, g, u, noise, eps, grid = draw_rounds_native_population(
                    self.rng, n, N, P, self.embedding_size, self.embedding_var,
                    shading if self._shading.any() else None, models, self.max_slots, policy, search,
                    kdo_max=self._engine.K * (self.obs_embedding_size + 1))
            else:
                ctx, part, u, g = draw_rounds_native(self.rng, n, N, P, self.embedding_size, self.embedding_var,
                                                     self.max_slots, shading if self._shading.any() else None)
                noise = eps = grid = None
            inp = {"ctx": torch.from_numpy(ctx).to(d), "part": torch.from_numpy(part).to(d),
                   "u": torch.from_numpy(u).to(d)}
            if self._shading.any():
                inp["gamma_raw"] = torch.from_numpy(g).to(d)
            if self._learning.any():
                inp["policy_eps"] = (torch.from_numpy(eps).to(d) if eps is not None else
                                     torch.zeros((P, n), dtype=torch.float32, device=d))
                if grid is not None:
                    inp["gamma_grid"] = torch.from_numpy(grid).to(d)
            if self._lrts.any() and self._ts:
                inp["ts_noise"] = torch.from_numpy(noise).to(d)
            self._run(inp)

    def simulate_synthetic(self, B, seed, first_auction=0):
        """B rounds with on-device Philox inputs (throughput mode; parity via the oracle)."""
        self._settle_lrts()
        self._flush()
        eng = self._engine
        inp = eng.alloc_inputs(int(B))
        eng.generate(seed, first_auction, inp)
        if "gamma_raw" in inp or "ts_noise" in inp:
            eng.generate_noise(seed, first_auction, inp)
        if "ts_noise" in inp and not self._ts_agent[self._lrts].all():
            # LR-TS agents that do not sample: zero noise in their slots ([P][T][K*Do][64] tiles)
            P, T = inp["ts_noise"].shape[0], inp["ts_noise"].shape[1]
            keep = torch.from_numpy(self._ts_agent).to(eng.device)[inp["part"].long()]  # [P][B]
            pad = torch.zeros((P, T * 64), dtype=torch.bool, device=eng.device)
            pad[:, :int(B)] = keep
            inp["ts_noise"].mul_(pad.view(P, T, 1, 64).to(inp["ts_noise"].dtype))
        if "gamma_grid" in inp:
            eng.generate_search_grid(seed, first_auction, inp)
        self._run(inp)

    # ------------------------------------------------------------------ engine
    def _flush(self):
        if not self._pending:
            return
        d, P = self._engine.device, self.num_participants_per_round
        rows, self._pending = self._pending, []
        B = len(rows)
        ctx = np.empty((self.embedding_size, B))
        part = np.empty((P, B), np.int32)
        u = np.empty(B)
        for r, (c, p, uu, _, _, _, _) in enumerate(rows):
            ctx[:, r], part[:, r], u[r] = c, p, uu
        inp = {"ctx": torch.from_numpy(ctx).to(d), "part": torch.from_numpy(part).to(d),
               "u": torch.from_numpy(u).to(d)}
        if self._shading.any():
            g = np.stack([row[3] for row in rows], axis=1)
            inp["gamma_raw"] = torch.from_numpy(np.ascontiguousarray(g)).to(d)
        if self._learning.any():
            e = np.zeros((P, B), np.float32)
            for r, row in enumerate(rows):
                if row[5] is not None:
                    e[:, r] = row[5]
            inp["policy_eps"] = torch.from_numpy(e).to(d)
            if any(row[6] is not None for row in rows):
                gg = np.zeros((P, 128, B))
                for r, row in enumerate(rows):
                    if row[6] is not None:
                        gg[:, :, r] = row[6]
                inp["gamma_grid"] = torch.from_numpy(gg).to(d)
        if self._lrts.any() and self._ts:
            KDo = self._engine.K * (self.obs_embedding_size + 1)
            z = np.zeros((B, P, KDo), np.float32)
            for r, row in enumerate(rows):
                if row[4] is not None:
                    z[r] = row[4]
            inp["ts_noise"] = torch.from_numpy(AuctionEngine.tile_ts_noise(z)).to(d)
        self._run(inp)

    def _run(self, inp):
        eng = self._engine
        B = inp["u"].shape[0]
        out = eng.alloc_outputs(B)
        cnt = eng.new_counters()
        max_b = 2048 * 8192
        for lo in range(0, B, max_b):
            hi = min(B, lo + max_b)
            if hi - lo == B:
                sl_in, sl_out = inp, out
            else:  # kernels need contiguous SoA slices
                sl_in = {k: (v[..., lo:hi].contiguous() if k != "ts_noise"
                             else v[:, lo // 64:(hi + 63) // 64].contiguous()) for k, v in inp.items()}
                sl_out = {k: torch.empty(v[..., lo:hi].shape, dtype=v.dtype, device=v.device)
                          for k, v in out.items()}
            eng.simulate(sl_in, sl_out, cnt)
            if self._learner.any():
                self._collect(sl_in, sl_out, hi - lo, self._logged_rounds + lo)
            if sl_out is not out:
                for k, v in out.items():
                    v[..., lo:hi].copy_(sl_out[k])
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
            self._log_batches.append((inp["part"], out, inp["ctx"]))
        self._logged_rounds += B

    # ------------------------------------------------------------------ Agent.update
    # Learners (LR-TS allocators, EmpiricalShadedBidder and the learning bidders) update from
    # their current logs. Their records are collected on the device after every batch into
    # append-only stores (one per learner family); an agent's clear_logs() removes its records
    # (keeping the last M with memory = M), so the stores always hold every learner's current
    # logs and each update() trains that agent alone on them, at its own call -- as the
    # reference does (src/Agent.py:79-94, src/main.py:127-152): rounds may be simulated between
    # updates, and an update may be repeated.
    _CAP_KEY = {"lrts": "key", "shading": "agent"}

    def _grow(self, name, need, make):
        """The `name` store with room for `need` records (grown by copying)."""
        old = self._stores.get(name)
        cap = old[self._CAP_KEY[name]].shape[0] if old is not None else 0
        if cap >= need:
            return old
        st = make(max(need, 2 * cap, 1 << 14))
        if old is not None:
            n = self._bounds[name]
            for k, v in old.items():
                if k == "count":
                    st[k].copy_(v)
                else:
                    st[k][..., :n].copy_(v[..., :n])
        self._stores[name] = st
        return st

    def _collect(self, inp, out, B, first_auction):
        eng = self._engine
        if self._lrts.any():
            need = self._bounds["lrts"] + B
            st = self._grow("lrts", need, eng.new_lrts_samples)
            eng.lrts_collect(inp, out, st)
            self._bounds["lrts"] = need
        if self._shading_rec.any():
            need = self._bounds["shading"] + B * self.num_participants_per_round
            learning = bool(self._learning.any())
            st = self._grow("shading", need, lambda cap: eng.new_shading_samples(cap, learning=learning))
            eng.shading_collect(inp, out, st, first_auction=first_auction)
            self._bounds["shading"] = need

    def _update_agent(self, index, iteration):
        """Agent.update (src/Agent.py:79-94) of agent `index` on the GPU, on its current logs: its
        allocator's update (LR-TS: the resumable update of this agent alone, ag_lrts_rp_*), then
        its bidder's (EmpiricalShadedBidder: ag_empirical_update_agents; the learning bidders:
        learner_update)."""
        if not self._learner[index]:
            return
        self._flush()
        eng = self._engine
        ag = self.agents[index]
        mask = np.zeros(len(self.agents), np.int32)
        mask[index] = 1
        if self._lrts[index]:
            # deferred: trained with the other LR-TS agents' updates at the next round, posterior
            # read or repeated update (_settle_lrts); on the samples it holds now (rounds cannot
            # be added before the settle), so the result is this call's
            if self._lrts_pending[index]:
                self._settle_lrts()
            self._lrts_pending[index] = True
            ag.allocator._settle = self._settle_lrts
        if self._empirical[index]:
            st = self._stores.get("shading") or eng.new_shading_samples(1, learning=bool(self._learning.any()))
            pg = eng.empirical_update(st, agents=mask)
            ag.bidder.prev_gamma = float(pg[index])
        if self._learning[index]:
            self._update_learner(index)

    def _update_learner(self, index):
        """One learning bidder's update (ag_bidder_update with a one-agent mask)."""
        eng = self._engine
        st = self._stores.get("shading") or eng.new_shading_samples(1, learning=True)
        learner_update(eng, st, index, self.agents[index].bidder, self.agents[index].name)

    def _settle_lrts(self):
        """The deferred LR-TS updates (_update_agent), trained together: every LR-TS agent's in
        one persistent launch (ag_lrts_update) when all of them are pending -- the reference's
        main loop updates every agent each iteration --, otherwise the pending ones alone
        (_lrts_train, the resumable update with their mask). Each agent trains on its own won
        samples, exact sums: the same posteriors and epochs as one update per call
        (tools/dropin_update_cost.py checks it; 747 -> 79 ms for configs[1]'s 8 agents,
        profiles/r05z_dropin_update.log). Then the won samples of the agents cleared meanwhile
        leave the store."""
        if not self._lrts_pending.any():
            return
        idx = np.flatnonzero(self._lrts_pending)
        mask = self._lrts_pending.astype(np.int32)
        self._lrts_pending[:] = False
        for i in idx:
            self.agents[i].allocator._settle = None
        eng = self._engine
        st = self._stores.get("lrts") or eng.new_lrts_samples(1)
        if np.array_equal(mask.astype(bool), self._lrts):
            ep = eng.lrts_update(st)
        else:
            ep = _lrts_train(eng, st, mask)
        m, q, pm = eng.lrts_state()
        for i in idx:
            al = self.agents[i].allocator
            rm = al.response_model
            k = self._num_items[i]  # the agent's own rows
            rm.m, rm.q, rm.prev_iter_m = (torch.from_numpy(np.ascontiguousarray(x[i, :k])) for x in (m, q, pm))
            al.epochs = int(ep[i])
        if self._lrts_drop.any():
            drop = self._lrts_drop.copy()
            self._lrts_drop[:] = False
            self._drop_records("lrts", drop)

    def _drop_records(self, name, drop):
        """Remove the records of the agents `drop` (bool [N]) from the device store `name`."""
        st = self._stores.get(name)
        if st is None:
            return
        n = min(int(st["count"][0].item()), self._bounds[name])
        agent = (((st["key"][:n].to(torch.int64) >> 16) & 0xFFFF) if name == "lrts"
                 else st["agent"][:n].to(torch.int64))
        keep = ~torch.from_numpy(drop).to(agent.device)[agent]
        m = int(keep.sum().item())
        if m < n:
            for k, v in st.items():
                if k != "count":
                    v[..., :m] = v[..., :n][..., keep]
        st["count"][0] = m
        self._bounds[name] = m

    def _cleared_logs(self, index):
        """Agent.clear_logs (src/Agent.py:124-129) of agent `index`: its records leave the device
        stores; with memory = M the last M go back (the records its next update trains on and its
        metrics read, src/Agent.py:81-94). The won samples of an agent whose LR-TS update is
        still deferred leave at the settle (it trains on them)."""
        if not self._learner[index]:
            return
        self._flush()
        cols = self.agents[index]._kept
        if cols is not None:  # memory: the kept samples go back now, so the update runs first
            self._settle_lrts()
        drop = np.zeros(len(self.agents), bool)
        drop[index] = True
        for name in list(self._stores):
            if name == "lrts" and self._lrts_pending[index]:
                self._lrts_drop[index] = True
                continue
            self._drop_records(name, drop)
        if cols is not None:
            self._append_kept(index, cols)

    def _append_kept(self, i, cols):
        """Agent(memory=M): the M records agent i kept (src/Agent.py:128) back into the device
        stores -- LR-TS won samples as ag_lrts_collect writes them, shading records with their
        log order -- so its next update trains on them and the new rounds' records."""
        eng, d = self._engine, self._engine.device
        if self._lrts[i]:
            w = cols["won"].astype(bool)
            if w.any():
                key = ((np.int64(i) << 16) | (cols["item"][w] << 1) | cols["outcome"][w].astype(np.int64))
                key = key.astype(np.uint32).view(np.int32)
                x = np.ascontiguousarray(cols["context"][w].astype(np.float32).T)
                n0, k = self._bounds["lrts"], len(key)
                st = self._grow("lrts", n0 + k, eng.new_lrts_samples)
                st["key"][n0:n0 + k] = torch.from_numpy(key).to(d)
                st["x"][:, n0:n0 + k] = torch.from_numpy(x).to(d)
                st["count"][0] = n0 + k
                self._bounds["lrts"] = n0 + k
        if self._shading_rec[i]:
            k = len(cols["item"])
            won = cols["won"].astype(bool)
            util = np.where(won, cols["value"] * cols["outcome"].astype(np.float64) - cols["price"], 0.0)
            learning = bool(self._learning.any())
            n0 = self._bounds["shading"]
            st = self._grow("shading", n0 + k, lambda cap: eng.new_shading_samples(cap, learning=learning))
            fields = {"agent": np.full(k, i, np.int32), "gamma": cols["gamma"], "utility": util,
                      "ctr": cols["est_ctr"], "value": cols["value"], "propensity": cols["propensity"],
                      "won": won.astype(np.uint8), "order": cols["order"]}
            for f, v in fields.items():
                if f in st:
                    st[f][n0:n0 + k] = torch.from_numpy(np.ascontiguousarray(v)).to(device=d, dtype=st[f].dtype)
            st["count"][0] = n0 + k
            self._bounds["shading"] = n0 + k

    def _agent_columns(self, index, start_round):
        """Agent(memory=M): columns of agent `index`'s records since start_round (host)."""
        self._flush()
        if not self.keep_logs:
            raise NotImplementedError("Agent(memory>0) needs the auction's logs (keep_logs=True)")
        oe = None if self.agents[index].allocator.kind == _lib.ALLOCATOR_ORACLE else self.obs_embedding_size
        return _agent_mod.agent_columns(self._log_batches, index, start_round - self._log_base, self._values,
                                        self.num_participants_per_round, self._log_base, obs=oe)

    # ------------------------------------------------------------------ logs
    def _log_rounds(self):
        """Rounds run so far; drops the device log buffers once every agent cleared them."""
        self._flush()
        if all(a._log_start >= self._logged_rounds for a in self.agents):
            self._log_batches = []
            self._log_base = self._logged_rounds
        return self._logged_rounds

    def _materialise_logs(self, agent_index, start_round):
        # the context an agent bid on (src/Agent.py:55): the true context for an
        # OracleAllocator agent, the observed one for the others (src/Auction.py:44-49)
        oe = None if self.agents[agent_index].allocator.kind == _lib.ALLOCATOR_ORACLE else self.obs_embedding_size
        return _agent_mod.materialise(self._log_batches, agent_index,
                                      start_round - self._log_base, self._values, obs=oe)

    # ------------------------------------------------------------------ revenue
    @property
    def revenue(self):
        self._flush()
        return _agent_mod.fx_to_float(self._revenue_fx)

    def clear_revenue(self):
        self._flush()
        self._revenue_fx = 0


def _lrts_train(eng, store, mask, launches=256):
    """PyTorchLogisticRegressionAllocator.update of the LR-TS agents of `mask` alone on the
    store's samples (the resumable per-epoch update, ag_lrts_rp_*, one process): the other
    agents' posteriors stay as they are. Returns epochs [N]."""
    eng.lrts_rp_begin(store, agents=mask)
    while True:
        eng.lrts_rp_epoch(launches)
        if eng.lrts_rp_poll() == 0:
            break
    return eng.lrts_rp_end()


NOISE_WINDOW_FLOATS = 1 << 26  # host-drawn rsample noise per window (256 MB)


def learner_update(eng, store, index, bidder, name):
    """Bidder.update of the learning bidder at engine slot `index` from the records of the
    device store, the bidder's host mirror refreshed afterwards. The DR and ValueLearning
    'policy' fits draw one rsample per record per epoch from torch's global generator
    (src/Models.py:160, :87): they train as the resumable update (ag_bidder_rp_*, run in
    persistent launches), fed the reference's draws window by window -- made in C from the
    generator's state (ag_torch_normal_epochs: torch's own normal kernels, the same numbers) --
    so the fit runs once, however long; the generator is then left exactly where the
    reference's is after the update (its fit's epochs drawn, plus the rsample of every record
    after DR / PolicyLearning fits, src/Bidder.py:605, :423). Returns the epochs [3] the fits
    ran."""
    b = bidder
    n = int(eng.shading_counts(store)[index])
    mask = np.zeros(eng.N, np.int32)
    mask[index] = 1
    noisy = b.kind == _lib.BIDDER_DOUBLY_ROBUST or (b.kind == _lib.BIDDER_VALUE_LEARNING
                                                     and b.inference == "policy")
    if noisy and n > 0:
        ep, stat = _fit_with_torch_noise(eng, store, mask, index, n)
    else:
        ep, stat = eng.bidder_update(store, None, np.zeros(eng.N, np.int64), 0, agents=mask)
    state, init = eng.dr_state()
    b._load_state16(state[index])
    b.model_initialised = bool(init[index] != _lib.LEARNER_UNINITIALISED)
    b.epochs = ep[index].copy()
    if stat[index] == 1:
        print(f"! Fallback for {name}")
    if b.kind in (_lib.BIDDER_DOUBLY_ROBUST, _lib.BIDDER_POLICY_LEARNING) and n > 0:
        torch.empty(n).normal_()  # pred_gammas = policy(X) after the fit
    return ep[index].copy()


def _fit_with_torch_noise(eng, store, mask, index, n):
    """One agent's update with the reference's torch rsample draws, single pass: windows of
    W policy-fit epochs drawn from the generator state as the fit reaches them; the fits run
    in persistent launches (ag_bidder_rp_run) that stop at a window's end."""
    from .engine import torch_normal_epochs
    W = int(min(4096, max(16, NOISE_WINDOW_FLOATS // n)))
    state = torch.get_rng_state().numpy().copy()  # advanced window by window
    w0, w_state = 0, state.copy()                 # the window's first epoch and its generator
    eng.bidder_rp_begin(store, agents=mask)
    win = torch.from_numpy(torch_normal_epochs(state, n, W)).to(eng.device)
    eng.bidder_rp_noise(win, n, w0, W)
    while True:
        eng.bidder_rp_run()
        fit, ep, need = eng.bidder_rp_poll()
        if fit[index] < 0:
            break
        if need[index] >= 0:  # the policy fit reached the end of the window: the next one
            w0, w_state = int(need[index]), state.copy()
            win = torch.from_numpy(torch_normal_epochs(state, n, W)).to(eng.device)
            eng.bidder_rp_noise(win, n, w0, W)
    ep, stat = eng.bidder_rp_end()
    # the generator after exactly the fit's epochs: the last window's start + its used epochs
    used = int(ep[index, 2]) - w0
    if used > 0:
        torch_normal_epochs(w_state, n, used)
    torch.set_rng_state(torch.from_numpy(w_state))
    return ep, stat
