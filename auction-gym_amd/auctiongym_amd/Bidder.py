"""Bidder plugins: the surface of src/Bidder.py:15-35 (+ the learned bidders' names).

Bidders are descriptors here: `kind` selects the bid rule the fused kernel applies per
participant. TruthfulBidder (bid = value * estimated CTR, src/Bidder.py:34-35) is built;
the shading / learning bidders keep their constructors so configs parse, and the engine
refuses them with NotImplementedError until their kernels land (f).
"""
from . import _lib


class Bidder:
    """Bidder base class (src/Bidder.py:15-25)."""

    kind = None

    def __init__(self, rng):
        self.rng = rng
        self.truthful = False

    def update(self, contexts, values, bids, prices, outcomes, estimated_CTRs, won_mask, iteration,
               plot, figsize, fontsize, name):
        pass

    def clear_logs(self, memory):
        pass


class TruthfulBidder(Bidder):
    """A bidder that bids truthfully: value * estimated CTR (src/Bidder.py:28-35)."""

    kind = _lib.BIDDER_TRUTHFUL

    def __init__(self, rng):
        super().__init__(rng)
        self.truthful = True

    def bid(self, value, context, estimated_CTR):
        return value * estimated_CTR


class _NotYetBuilt(Bidder):
    kind = None

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, **kw):
        super().__init__(rng)
        self.gamma_sigma = gamma_sigma
        self.prev_gamma = init_gamma
        self.kwargs = kw
        self.gammas = []


class EmpiricalShadedBidder(_NotYetBuilt):
    """src/Bidder.py:38-153 (not yet on the GPU path)."""


class ValueLearningBidder(_NotYetBuilt):
    """src/Bidder.py:156-333 (not yet on the GPU path)."""

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, inference="search"):
        assert inference in ["search", "policy"]
        super().__init__(rng, gamma_sigma, init_gamma, inference=inference)


class PolicyLearningBidder(_NotYetBuilt):
    """src/Bidder.py:336-439 (not yet on the GPU path)."""

    def __init__(self, rng, gamma_sigma, loss, init_gamma=1.0):
        super().__init__(rng, gamma_sigma, init_gamma, loss=loss)


class DoublyRobustBidder(_NotYetBuilt):
    """src/Bidder.py:442-623 (not yet on the GPU path)."""
