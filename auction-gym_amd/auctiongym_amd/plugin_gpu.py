"""The per-call plugin surface on the GPU: estimate_CTR, bid and the plugin-level update of
ONE plugin object, called the way the reference's own code and notebooks call them
(src/BidderAllocation.py, src/Bidder.py, src/Agent.py:29-94), outside a batched Auction.

Each plugin owns a one-agent engine (an ag_ctx with N = P = 1) that holds a copy of the
plugin's host state -- catalogue, LR-TS posterior, shading parameters, learner models --
refreshed before every call, so the answer is the plugin's current state's. The calls go
through the same device code as the batched path (ag_estimate_ctr, ag_bid, ag_lrts_update,
ag_empirical_update, ag_bidder_update): a per-call answer equals what the fused simulate
kernel computes for the same participant. The random draws the reference makes inside
these calls (numpy rng, torch's global generator) are made here, on the host, with the same
calls in the same order, and passed in.
"""
import numpy as np
import torch

from . import _lib

_ENGINES = {}


def _drop(key):
    e = _ENGINES.pop(key, None)
    if e is not None:
        try:
            e[2].close()
        except Exception:  # interpreter shutdown: the runtime may already be gone
            pass


def _engine(owner, K, E, OE):
    """The owner's one-agent engine (created on first use; re-created if its shape changes).
    Held by id with only a weak reference to the owner: when the plugin is collected its
    engine (the ag_ctx with its device catalogue and learner workspaces) is closed."""
    import weakref

    from .engine import AuctionEngine
    key = id(owner)
    shape = (K, E, OE)
    e = _ENGINES.get(key)
    if e is None or e[0]() is not owner or e[1] != shape:
        if e is not None:
            e[3].detach()
            _drop(key)
        eng = AuctionEngine(1, 1, K, E, OE, _lib.SECOND_PRICE, 1.0)
        _ENGINES[key] = (weakref.ref(owner), shape, eng, weakref.finalize(owner, _drop, key))
        return eng
    return e[2]


# ------------------------------------------------------------------------------ allocators
def oracle_estimate_ctr(alloc, context):
    """OracleAllocator.estimate_CTR(context) (src/BidderAllocation.py:81-82): context is the
    true context with its intercept [E+1]; returns float64 [K]."""
    items = np.asarray(alloc.item_embeddings, np.float64)
    if items.ndim != 2:
        raise ValueError("OracleAllocator.estimate_CTR: update_item_embeddings first")
    K, D = items.shape
    x = np.asarray(context, np.float64).reshape(-1)
    if x.shape[0] != D:
        raise ValueError(f"OracleAllocator.estimate_CTR: context has {x.shape[0]} entries, the "
                         f"item embeddings {D}")
    eng = _engine(alloc, K, D - 1, D - 1)
    eng.load_catalog(items[None], np.ones((1, K)))
    return eng.estimate_ctr(0, x[None])[0].cpu().numpy()


def _lrts_engine(alloc):
    rm = alloc.response_model
    K, Do = rm.m.shape
    eng = _engine(alloc, K, Do - 1, Do - 1)
    eng.set_agent_params(np.array([_lib.ALLOCATOR_LRTS], np.int32), np.array([_lib.BIDDER_TRUTHFUL], np.int32))
    eng.load_lrts(rm.m.detach().numpy()[None], rm.q.detach().numpy()[None], rm.prev_iter_m.detach().numpy()[None],
                  thompson_sampling=bool(alloc.thompson_sampling))
    return eng


def lrts_estimate_ctr(alloc, context, sample=True):
    """PyTorchLogisticRegressionAllocator.estimate_CTR(context, sample) (src/BidderAllocation.py:
    67-68): context is the observed context with its intercept [OE+1]. With Thompson sampling
    the posterior draw is torch.normal(0, 1/sqrt(q)) from torch's global generator, the call
    src/Models.py:31 makes; returns float32 [K] as the reference does."""
    eng = _lrts_engine(alloc)
    x = np.asarray(context, np.float64).reshape(1, -1)
    noise = None
    if alloc.thompson_sampling and sample:
        noise = alloc.response_model.sample_noise().numpy()[None]
    return eng.estimate_ctr(0, x, noise)[0].cpu().numpy().astype(np.float32)


def lrts_update(alloc, contexts, items, outcomes):
    """PyTorchLogisticRegressionAllocator.update (src/BidderAllocation.py:29-65) on the GPU
    trainer (ag_lrts_update) from the reference's arrays; the host model is refreshed.
    Returns the epochs run (0: fewer than 2 samples, nothing trained, as the reference)."""
    eng = _lrts_engine(alloc)
    X = np.asarray(contexts, np.float64)
    A = np.asarray(items, np.int64).reshape(-1)
    y = np.asarray(outcomes).reshape(-1)
    n = A.shape[0]
    if n < 2:
        return 0
    K, Do = alloc.response_model.m.shape
    if X.shape != (n, Do):
        raise ValueError(f"contexts must be [{n}][{Do}] (the observed context with its intercept)")
    st = eng.new_lrts_samples(n)
    key = (A.astype(np.uint32) << 1) | (y != 0).astype(np.uint32)  # agent 0
    st["key"].copy_(torch.from_numpy(key.astype(np.int64).astype(np.int32)))
    st["x"].copy_(torch.from_numpy(np.ascontiguousarray(X.T.astype(np.float32))))  # torch.Tensor(X)
    st["count"].fill_(n)
    ep = eng.lrts_update(st)
    m, q, pm = eng.lrts_state()
    rm = alloc.response_model
    rm.m, rm.q, rm.prev_iter_m = torch.from_numpy(m[0].copy()), torch.from_numpy(q[0].copy()), \
        torch.from_numpy(pm[0].copy())
    alloc.epochs = int(ep[0])
    return alloc.epochs


# -------------------------------------------------------------------------------- bidders
def _bidder_engine(bidder):
    eng = _engine(bidder, 1, 1, 1)
    kind = np.array([bidder.kind], np.int32)
    shading = bidder.kind != _lib.BIDDER_TRUTHFUL
    eng.set_agent_params(np.array([_lib.ALLOCATOR_ORACLE], np.int32), kind,
                         np.array([float(bidder.prev_gamma)]) if shading else None,
                         np.array([float(bidder.gamma_sigma)]) if shading else None)
    if bidder.kind >= _lib.BIDDER_VALUE_LEARNING:
        eng.set_dr_state(bidder._state16()[None], np.array([bidder._learner_state()], np.int32))
        eng.set_bidder_modes(np.array([bidder._mode()], np.int32))
    return eng


def shading_bid(bidder, value, estimated_ctr):
    """Bidder.bid(value, context, estimated_CTR) of a shading / learning bidder (src/Bidder.py:
    47-58, :171-208, :348-367, :455-475): the draw its state makes (numpy rng, or torch's
    generator for a fitted policy), then the bid rule on the GPU. Appends gamma and the
    propensity to the bidder's lists as the reference does; returns the bid (float)."""
    eng = _bidder_engine(bidder)
    state = bidder._learner_state() if bidder.kind >= _lib.BIDDER_VALUE_LEARNING else _lib.LEARNER_UNINITIALISED
    g_raw = eps = grid = None
    if state == _lib.LEARNER_POLICY:
        eps = np.array([torch.empty(1).normal_().item()], np.float32)  # dist.rsample() (src/Models.py:87, :160)
    elif state == _lib.LEARNER_SEARCH:
        gg = bidder.rng.uniform(0.1, 1.0, size=128)  # src/Bidder.py:185-186
        gg.sort()
        grid = gg[None]
    else:
        g_raw = np.array([bidder.rng.normal(bidder.prev_gamma, bidder.gamma_sigma)])  # src/Bidder.py:51, :177, ...
    b, g, p = eng.bid(0, np.array([float(value)]), np.array([float(estimated_ctr)]), g_raw, eps, grid)
    b, g, p = float(b[0]), float(g[0]), float(p[0])
    bidder.gammas.append(g)
    if hasattr(bidder, "propensities"):
        bidder.propensities.append(p)
    return b


def _shading_store(eng, gammas, values, prices, outcomes, estimated_ctrs, won_mask, propensities, learning):
    values = np.asarray(values, np.float64).reshape(-1)
    n = values.shape[0]
    gammas = np.asarray([float(g) for g in gammas], np.float64)
    if gammas.shape[0] != n:
        raise ValueError(f"the bidder logged {gammas.shape[0]} bids but update got {n} records")
    won = np.asarray(won_mask, bool).reshape(-1)
    util = np.zeros(n)
    util[won] = values[won] * np.asarray(outcomes, np.float64).reshape(-1)[won] - \
        np.asarray(prices, np.float64).reshape(-1)[won]  # src/Bidder.py:62-63, :474-476
    st = eng.new_shading_samples(max(n, 1), learning=learning)
    if n:
        st["agent"][:n] = 0
        st["gamma"][:n].copy_(torch.from_numpy(gammas))
        st["utility"][:n].copy_(torch.from_numpy(util))
        if learning:
            st["ctr"][:n].copy_(torch.from_numpy(np.asarray(estimated_ctrs, np.float64).reshape(-1)))
            st["value"][:n].copy_(torch.from_numpy(values))
            st["propensity"][:n].copy_(torch.from_numpy(np.asarray([float(p) for p in propensities], np.float64)))
            st["won"][:n].copy_(torch.from_numpy(won.astype(np.uint8)))
            st["order"][:n].copy_(torch.arange(n, dtype=torch.int64))
    st["count"].fill_(n)
    return st


def empirical_update(bidder, values, prices, outcomes, won_mask):
    """EmpiricalShadedBidder.update (src/Bidder.py:60-147) on the GPU (ag_empirical_update)
    from the reference's arrays and the bidder's logged gammas; sets prev_gamma."""
    eng = _bidder_engine(bidder)
    st = _shading_store(eng, bidder.gammas, values, prices, outcomes, None, won_mask, None, learning=False)
    bidder.prev_gamma = float(eng.empirical_update(st)[0])
    return bidder.prev_gamma


def learner_update_call(bidder, values, prices, outcomes, estimated_ctrs, won_mask, name):
    """ValueLearningBidder / PolicyLearningBidder / DoublyRobustBidder.update (src/Bidder.py:
    204-325, :364-431, :473-615) on the GPU trainer (ag_bidder_update) from the reference's
    arrays and the bidder's logged gammas / propensities; the host models are refreshed."""
    from .Auction import learner_update
    eng = _bidder_engine(bidder)
    st = _shading_store(eng, bidder.gammas, values, prices, outcomes, estimated_ctrs, won_mask,
                        bidder.propensities, learning=True)
    return learner_update(eng, st, 0, bidder, name)
