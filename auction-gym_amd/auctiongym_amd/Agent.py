"""Agent: the surface of src/Agent.py:8-129 over the batched engine.

Per-round effects (charge / set_price / log append, src/Agent.py:44-77) happen inside the
fused kernel; what an Agent keeps is its exact fixed-point counter sums (include/
auctiongym.h AG_C_*). Every getter first flushes the auction's pending rounds, so code
written against the reference (read net_utility after the round loop, call update, clear)
sees the same values.
"""
import math

import numpy as np

from . import _lib
from .Impression import ImpressionOpportunity

C = {name: i for i, name in enumerate(_lib.COUNTERS)}
_UTILITY = (C["net"], C["gross"])
_LOGS = tuple(i for n, i in C.items() if n not in ("net", "gross", "paid"))


def fx_to_float(v):
    """Exact fixed-point integer (units of 2^-36) -> correctly rounded float."""
    return math.ldexp(float(v), -_lib.FX_FRAC_BITS) if abs(v) < (1 << 1000) else float("inf")


class Agent:
    """An agent representing an advertiser (src/Agent.py:8-27)."""

    def __init__(self, rng, name, num_items, item_values, allocator, bidder, memory=0):
        self.rng = rng
        self.name = name
        self.num_items = num_items
        self.item_values = item_values
        self.allocator = allocator
        self.bidder = bidder
        if memory:
            raise NotImplementedError("Agent(memory>0): log memory across iterations is not "
                                      "implemented on the GPU path yet")
        self.memory = memory
        self._auction = None
        self._index = None
        self._fx = [0] * _lib.NUM_COUNTERS
        self._log_start = 0
        self._call_logs = []

    # engine plumbing --------------------------------------------------------
    def _attach(self, auction, index):
        self._auction = auction
        self._index = index

    def _sync(self):
        if self._auction is not None:
            self._auction._flush()

    def _get(self, name):
        self._sync()
        return fx_to_float(self._fx[C[name]])

    # reference attributes ----------------------------------------------------
    @property
    def net_utility(self):
        return self._get("net")

    @property
    def gross_utility(self):
        return self._get("gross")

    @property
    def logs(self):
        """Materialised ImpressionOpportunity records of the current iteration: the auction's
        rounds (from the device SoA outputs), then any per-call Agent.bid records."""
        self._sync()
        recs = [] if self._auction is None else self._auction._materialise_logs(self._index, self._log_start)
        return recs + self._call_logs

    # the per-call surface (src/Agent.py:29-68): one request through the GPU plugins
    def select_item(self, context):
        """src/Agent.py:29-42: the allocator's CTR estimates (ag_estimate_ctr), the first
        argmax of CTR * value, and for Thompson sampling the MAP CTR of that item."""
        from .BidderAllocation import PyTorchLogisticRegressionAllocator
        estim = self.allocator.estimate_CTR(context)
        best = int(np.argmax(estim * self.item_values))
        if type(self.allocator) is PyTorchLogisticRegressionAllocator and self.allocator.thompson_sampling:
            return best, self.allocator.estimate_CTR(context, sample=False)[best]
        return best, estim[best]

    def bid(self, context):
        """src/Agent.py:44-68: select_item, the bidder's bid (ag_bid for shading bidders), and
        the log record (kept with this agent's logs until clear_logs)."""
        best, ctr = self.select_item(context)
        value = self.item_values[best]
        b = self.bidder.bid(value, context, ctr)
        self._call_logs.append(ImpressionOpportunity(
            context=context, item=best, value=value, bid=b, best_expected_value=0.0, true_CTR=0.0,
            estimated_CTR=ctr, price=0.0, second_price=0.0, outcome=False, won=False))
        return b, best

    def update(self, iteration, plot=False, figsize=(8, 5), fontsize=14):
        """src/Agent.py:79-94. Oracle / Truthful updates are no-ops (src/BidderAllocation.py:
        17-18, src/Bidder.py:21-22); every learner trains on the GPU from the device record
        stores of its rounds (Auction._update_agent): the LR-TS allocator on its won samples
        (ag_lrts_update), EmpiricalShadedBidder (ag_empirical_update) and the learning bidders
        (ag_bidder_update) on all of its records."""
        self._sync()
        if self._auction is not None:
            self._auction._update_agent(self._index, iteration)

    def get_allocation_regret(self):
        return self._get("allocation_regret")

    def get_estimation_regret(self):
        return self._get("estimation_regret")

    def get_overbid_regret(self):
        return self._get("overbid_regret")

    def get_underbid_regret(self):
        return self._get("underbid_regret")

    def get_CTR_RMSE(self):
        n = self._fx[C["n_logs"]]
        return math.sqrt(self._get("ctr_sqerr") / fx_to_float(n)) if n else float("nan")

    def get_CTR_bias(self):
        self._sync()
        n = self._fx[C["n_won"]]
        return self._get("ctr_bias_sum") / fx_to_float(n) if n else float("nan")

    def get_mean_best_expected_value(self):
        """np.mean(opp.best_expected_value for opp in logs) (src/main.py:147)."""
        self._sync()
        n = self._fx[C["n_logs"]]
        return self._get("best_ev_sum") / fx_to_float(n) if n else float("nan")

    def num_logs(self):
        self._sync()
        return int(round(fx_to_float(self._fx[C["n_logs"]])))

    def clear_utility(self):
        self._sync()
        for i in _UTILITY:
            self._fx[i] = 0

    def clear_logs(self):
        self._sync()
        for i in _LOGS:
            self._fx[i] = 0
        if self._auction is not None:
            self._log_start = self._auction._log_rounds()
            self._auction._cleared_logs(self._index)
        self._call_logs = self._call_logs[-self.memory:] if self.memory else []
        self.bidder.clear_logs(memory=self.memory)

    def __repr__(self):
        return f"Agent({self.name!r})"


def _records(part, out, ctx, agent, first_round, values, obs=None):
    """Build ImpressionOpportunity rows of `agent` from host copies of one batch. ctx [E][B]:
    the record's context is the true context + intercept, or (obs = OE) its first OE entries
    + intercept (src/Auction.py:33-36)."""
    recs = []
    P, B = part.shape
    for r in range(B):
        for s in range(P):
            if part[s, r] != agent:
                continue
            charged = P >= 2
            won = charged and out["winner"][r] == s
            it = int(out["item"][s, r])
            c = ctx[:, r] if obs is None else ctx[:obs, r]
            recs.append(ImpressionOpportunity(
                context=np.concatenate((c, [1.0])), item=it, value=float(values[agent][it]),
                bid=float(out["bid"][s, r]),
                best_expected_value=float(out["best_ev"][s, r]),
                true_CTR=float(out["true_ctr"][s, r]), estimated_CTR=float(out["est_ctr"][s, r]),
                price=float(out["price"][r]) if charged else 0.0,
                second_price=float(out["second_price"][r]) if won else 0.0,
                outcome=bool(out["outcome"][r]) if won else False, won=bool(won)))
    return recs


def materialise(batches, agent, start_round, values, obs=None):
    recs = []
    base = 0
    for part, out, ctx in batches:
        B = part.shape[1]
        if base + B > start_round:
            p = part.cpu().numpy()
            c = ctx.cpu().numpy()
            o = {k: v.cpu().numpy() for k, v in out.items()}
            lo = max(0, start_round - base)
            if lo:
                p, c = p[:, lo:], c[:, lo:]
                o = {k: (v[:, lo:] if v.ndim == 2 else v[lo:]) for k, v in o.items()}
            recs.extend(_records(p, o, c, agent, base + lo, values, obs))
        base += B
    return recs


__all__ = ["Agent", "fx_to_float", "materialise"]
