"""Bidder plugins: the surface of src/Bidder.py:15-35 (+ the shading bidders).

Bidders are descriptors here: `kind` selects the bid rule the fused kernel applies per
participant. TruthfulBidder (bid = value * estimated CTR, src/Bidder.py:34-35) is
complete. The shading bidders bid on the GPU in their uninitialised state -- gamma ~
N(prev_gamma, gamma_sigma), clipped to [0, 1] for EmpiricalShadedBidder (src/Bidder.py:
47-58), unclipped with its Gaussian propensity for the learning bidders (:174-179,
:351-356, :458-463) -- which is every bid of their first iteration; their update()
is not built yet (Agent.update raises NotImplementedError).
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


class _ShadingBidder(Bidder):
    kind = None

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, **kw):
        super().__init__(rng)
        self.gamma_sigma = gamma_sigma
        self.prev_gamma = init_gamma
        self.kwargs = kw
        self.gammas = []


class EmpiricalShadedBidder(_ShadingBidder):
    """src/Bidder.py:38-153."""

    kind = _lib.BIDDER_EMPIRICAL_SHADED


class ValueLearningBidder(_ShadingBidder):
    """src/Bidder.py:156-333 (uninitialised state)."""

    kind = _lib.BIDDER_VALUE_LEARNING

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, inference="search"):
        assert inference in ["search", "policy"]
        super().__init__(rng, gamma_sigma, init_gamma, inference=inference)


class PolicyLearningBidder(_ShadingBidder):
    """src/Bidder.py:336-439 (uninitialised state)."""

    kind = _lib.BIDDER_POLICY_LEARNING

    def __init__(self, rng, gamma_sigma, loss, init_gamma=1.0):
        super().__init__(rng, gamma_sigma, init_gamma, loss=loss)


class DoublyRobustBidder(_ShadingBidder):
    """src/Bidder.py:442-623 (uninitialised state)."""

    kind = _lib.BIDDER_DOUBLY_ROBUST
