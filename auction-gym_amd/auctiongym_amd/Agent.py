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
        self.memory = int(memory)
        self._kept = None  # Agent(memory=M): columns of the M records kept by clear_logs
        self._auction = None
        self._index = None
        self._fx = [0] * _lib.NUM_COUNTERS
        self._log_start = 0
        self._call_logs = []
        self._kept_calls = None  # memory=M: columns of the per-call records clear_logs kept

    # engine plumbing --------------------------------------------------------
    def _attach(self, auction, index):
        self._auction = auction
        self._index = index

    def _sync(self):
        if self._auction is not None:
            self._auction._flush()

    def _get(self, name):
        self._sync()
        return fx_to_float(self._fx[C[name]] + self._call_terms().get(C[name], 0))

    def _call_terms(self):
        """Exact log-counter terms of the per-call records (Agent.bid outside an Auction, their
        prices / outcomes set by charge / set_price / set_true_CTR), as the kernels add them."""
        if not self._call_logs:
            return {}
        return log_counter_terms(columns_from_records(self._call_logs), True, True)

    def _count(self, name):
        return self._fx[C[name]] + self._call_terms().get(C[name], 0)

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
        kept = records_from_columns(self._kept) if self._kept is not None else []
        kept_calls = records_from_columns(self._kept_calls) if self._kept_calls is not None else []
        return kept + recs + kept_calls + self._call_logs

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

    def charge(self, price, second_price, outcome):
        """src/Agent.py:70-74: the last per-call record won at `price`; utilities updated
        (exact fixed-point terms, as the kernels add them: gross += value * outcome, paid +=
        price)."""
        if not self._call_logs:
            raise IndexError("list index out of range")  # the reference's self.logs[-1]
        rec = self._call_logs[-1]
        rec.set_price_outcome(price, second_price, outcome, won=True)
        g = _fx([rec.value * float(outcome)])
        paid = _fx([price])
        self._fx[C["gross"]] += g
        self._fx[C["paid"]] += paid
        self._fx[C["net"]] += g - paid

    def set_price(self, price):
        """src/Agent.py:76-77."""
        if not self._call_logs:
            raise IndexError("list index out of range")
        self._call_logs[-1].set_price(price)

    def update(self, iteration, plot=False, figsize=(8, 5), fontsize=14):
        """src/Agent.py:79-94. Oracle / Truthful updates are no-ops (src/BidderAllocation.py:
        17-18, src/Bidder.py:21-22); every learner trains on the GPU from the device record
        stores of its rounds (Auction._update_agent): the LR-TS allocator on its won samples
        (ag_lrts_update), EmpiricalShadedBidder (ag_empirical_update) and the learning bidders
        (ag_bidder_update) on all of its records."""
        self._sync()
        if self._call_logs or self._kept_calls is not None:
            if self._auction is not None:
                raise NotImplementedError(
                    "Agent.update on per-call Agent.bid records of an agent that also takes part in a "
                    "batched Auction: update one or the other")
            self._update_call_logs(iteration, plot, figsize, fontsize)
        elif self._auction is not None:
            self._auction._update_agent(self._index, iteration)

    def _update_call_logs(self, iteration, plot, figsize, fontsize):
        """src/Agent.py:79-94 over the per-call records (kept ones first): the allocator on the
        won records, the bidder on all of them, through the plugins' GPU updates."""
        recs = (records_from_columns(self._kept_calls) if self._kept_calls is not None else []) + self._call_logs
        contexts = np.array([o.context for o in recs])
        items = np.array([o.item for o in recs])
        values = np.array([o.value for o in recs])
        bids = np.array([o.bid for o in recs])
        prices = np.array([o.price for o in recs])
        outcomes = np.array([o.outcome for o in recs])
        est = np.array([o.estimated_CTR for o in recs])
        won = np.array([o.won for o in recs])
        self.allocator.update(contexts[won], items[won], outcomes[won], iteration, plot, figsize, fontsize, self.name)
        self.bidder.update(contexts, values, bids, prices, outcomes, est, won, iteration, plot, figsize, fontsize,
                           self.name)

    def get_allocation_regret(self):
        return self._get("allocation_regret")

    def get_estimation_regret(self):
        return self._get("estimation_regret")

    def get_overbid_regret(self):
        return self._get("overbid_regret")

    def get_underbid_regret(self):
        return self._get("underbid_regret")

    def get_CTR_RMSE(self):
        n = self._count("n_logs")
        return math.sqrt(self._get("ctr_sqerr") / fx_to_float(n)) if n else float("nan")

    def get_CTR_bias(self):
        self._sync()
        n = self._count("n_won")
        return self._get("ctr_bias_sum") / fx_to_float(n) if n else float("nan")

    def get_mean_best_expected_value(self):
        """np.mean(opp.best_expected_value for opp in logs) (src/main.py:147)."""
        self._sync()
        n = self._count("n_logs")
        return self._get("best_ev_sum") / fx_to_float(n) if n else float("nan")

    def num_logs(self):
        self._sync()
        return int(round(fx_to_float(self._count("n_logs"))))

    def clear_utility(self):
        self._sync()
        for i in _UTILITY:
            self._fx[i] = 0

    def clear_logs(self):
        """src/Agent.py:124-129: the logs are emptied, or with memory = M the last M records
        are kept -- they stay in this agent's metrics (their exact counter terms, recomputed
        on the host from the kept columns) and in the records its next update trains on (the
        device record stores are rebuilt from them, Auction._cleared_logs)."""
        self._sync()
        if self.memory and self._auction is not None:
            cols = self._auction._agent_columns(self._index, self._log_start)
            if self._kept is not None:
                cols = concat_columns(self._kept, cols)
            self._kept = take_last(cols, self.memory)
            terms = log_counter_terms(self._kept, self._auction._charged, self._auction._first_price)
            for i in _LOGS:
                self._fx[i] = terms.get(i, 0)
        else:
            for i in _LOGS:
                self._fx[i] = 0
        if self._auction is not None:
            self._log_start = self._auction._log_rounds()
            self._auction._cleared_logs(self._index)
        if self._call_logs:  # per-call records: the last M kept (src/Agent.py:124-129)
            cols = columns_from_records(self._call_logs)
            if self._kept_calls is not None:
                cols = concat_columns(self._kept_calls, cols)
            self._kept_calls = take_last(cols, self.memory) if self.memory else None
        if self._kept_calls is not None:  # kept records stay in the metrics, new ones or not
            terms = log_counter_terms(self._kept_calls, True, True)
            for i in _LOGS:
                self._fx[i] += terms.get(i, 0)
        self._call_logs = []
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


# ---- Agent(memory=M): the kept records as columns ------------------------------------
COLUMNS = ("context", "item", "value", "bid", "best_ev", "true_ctr", "est_ctr", "price", "second_price",
           "outcome", "won", "gamma", "propensity", "order")


def agent_columns(batches, agent, start_round, values, P, log_base, obs=None):
    """Columns of `agent`'s records from round start_round on (log order: round, then slot):
    the ImpressionOpportunity fields plus what the learners' record stores hold (gamma,
    propensity; order = global round index * P + slot, ag_shading_samples.order)."""
    parts = {k: [] for k in COLUMNS}
    base = 0
    for part, out, ctx in batches:
        B = part.shape[1]
        if base + B > start_round:
            lo = max(0, start_round - base)
            p = part[:, lo:].cpu().numpy()
            r, s = np.nonzero(p.T == agent)  # row-major over [round][slot]: log order
            if len(r):
                o = {k: v.cpu().numpy() for k, v in out.items()}
                rr = r + lo
                charged = P >= 2
                won = (o["winner"][rr] == s) if charged else np.zeros(len(r), bool)
                c = ctx.cpu().numpy()[:, rr].T
                c = c if obs is None else c[:, :obs]
                item = o["item"][s, rr]
                parts["context"].append(np.concatenate([c, np.ones((len(r), 1))], axis=1))
                parts["item"].append(item.astype(np.int64))
                parts["value"].append(np.asarray(values[agent], np.float64)[item])
                parts["bid"].append(o["bid"][s, rr])
                parts["best_ev"].append(o["best_ev"][s, rr])
                parts["true_ctr"].append(o["true_ctr"][s, rr])
                parts["est_ctr"].append(o["est_ctr"][s, rr])
                parts["price"].append(o["price"][rr] if charged else np.zeros(len(r)))
                parts["second_price"].append(np.where(won, o["second_price"][rr], 0.0) if charged
                                             else np.zeros(len(r)))
                parts["outcome"].append(np.where(won, o["outcome"][rr] != 0, False))
                parts["won"].append(won)
                nan = np.full(len(r), np.nan)
                parts["gamma"].append(o["gamma"][s, rr] if "gamma" in o else nan)
                parts["propensity"].append(o["propensity"][s, rr] if "propensity" in o else nan)
                parts["order"].append(((log_base + base + rr).astype(np.int64)) * P + s)
        base += B
    return {k: (np.concatenate(v) if v else None) for k, v in parts.items()}


def _ncols(cols):
    return 0 if cols is None or cols["item"] is None else len(cols["item"])


def concat_columns(a, b):
    if _ncols(a) == 0:
        return b
    if _ncols(b) == 0:
        return a
    return {k: np.concatenate([a[k], b[k]]) for k in COLUMNS}


def take_last(cols, m):
    n = _ncols(cols)
    if n == 0:
        return None
    return {k: v[max(0, n - m):] for k, v in cols.items()}


def records_from_columns(cols):
    n = _ncols(cols)
    return [ImpressionOpportunity(
        context=cols["context"][j].copy(), item=int(cols["item"][j]), value=float(cols["value"][j]),
        bid=float(cols["bid"][j]), best_expected_value=float(cols["best_ev"][j]),
        true_CTR=float(cols["true_ctr"][j]), estimated_CTR=float(cols["est_ctr"][j]),
        price=float(cols["price"][j]), second_price=float(cols["second_price"][j]),
        outcome=bool(cols["outcome"][j]), won=bool(cols["won"][j])) for j in range(n)]


def columns_from_records(recs):
    """Columns (COLUMNS) of ImpressionOpportunity records (per-call records; no gamma /
    propensity / order: those live in the bidder's own lists)."""
    n = len(recs)
    if n == 0:
        return None
    nan = np.full(n, np.nan)
    return {"context": np.array([np.asarray(o.context, np.float64) for o in recs]),
            "item": np.array([o.item for o in recs], np.int64),
            "value": np.array([o.value for o in recs], np.float64),
            "bid": np.array([o.bid for o in recs], np.float64),
            "best_ev": np.array([o.best_expected_value for o in recs], np.float64),
            "true_ctr": np.array([o.true_CTR for o in recs], np.float64),
            "est_ctr": np.array([o.estimated_CTR for o in recs], np.float64),
            "price": np.array([o.price for o in recs], np.float64),
            "second_price": np.array([o.second_price for o in recs], np.float64),
            "outcome": np.array([bool(o.outcome) for o in recs]), "won": np.array([bool(o.won) for o in recs]),
            "gamma": nan, "propensity": nan.copy(), "order": np.arange(n, dtype=np.int64)}


def _fx(x):
    """The kernels' per-record rounding (ag_sim.h to_fx): x * 2^36 to nearest-even as an
    integer, terms with |x| >= 2^26 (or non-finite) dropped."""
    x = np.asarray(x, np.float64)
    ok = np.abs(x) < 2.0 ** 26
    r = np.rint(np.where(ok, x, 0.0) * 2.0 ** 36).astype(np.int64)
    return sum(int(v) for v in r)


def log_counter_terms(cols, charged, first_price):
    """Exact fixed-point sums of the log counters (src/Agent.py:96-118 terms, as the simulate
    kernels add them per record) over the kept records."""
    n = _ncols(cols)
    if n == 0:
        return {}
    won = cols["won"].astype(bool)
    val, bid, tru, est, bev = (cols[k] for k in ("value", "bid", "true_ctr", "est_ctr", "best_ev"))
    lp = cols["price"] if charged else np.zeros(n)
    tv = tru * val
    t = {C["allocation_regret"]: _fx(bev - tv), C["estimation_regret"]: _fx(est * val - tv),
         C["underbid_regret"]: _fx(((lp - bid) * (lp < tv).astype(np.float64))[~won]),
         C["ctr_sqerr"]: _fx((tru - est) * (tru - est)), C["best_ev_sum"]: _fx(bev),
         C["ctr_bias_sum"]: _fx((est / np.where(won, tru, 1.0))[won]),
         C["n_logs"]: n << _lib.FX_FRAC_BITS, C["n_won"]: int(won.sum()) << _lib.FX_FRAC_BITS,
         C["overbid_regret"]: _fx((lp - cols["second_price"])[won]) if first_price else 0}
    return t


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


__all__ = ["Agent", "fx_to_float", "materialise", "agent_columns"]
