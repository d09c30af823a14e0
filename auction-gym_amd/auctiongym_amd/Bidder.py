"""Bidder plugins: the surface of src/Bidder.py:15-35 (+ the shading bidders).

Bidders are descriptors here: `kind` selects the bid rule the fused kernel applies per
participant. TruthfulBidder (bid = value * estimated CTR, src/Bidder.py:34-35) is
complete. The shading bidders bid on the GPU in their uninitialised state -- gamma ~
N(prev_gamma, gamma_sigma), clipped to [0, 1] for EmpiricalShadedBidder (src/Bidder.py:
47-58), unclipped with its Gaussian propensity for the learning bidders (:174-179,
:351-356, :458-463) -- which is every bid of their first iteration. The learning bidders (ValueLearning, PolicyLearning,
DoublyRobust) keep host mirrors of their models; their update() trains on the GPU and from
then on they bid from the fitted policy inside the simulate kernel.
"""
import numpy as np
import torch

from . import _lib


class Bidder:
    """Bidder base class (src/Bidder.py:15-25)."""

    kind = None

    def __init__(self, rng):
        self.rng = rng
        self.truthful = False

    def update(self, contexts, values, bids, prices, outcomes, estimated_CTRs, won_mask, iteration,
               plot=False, figsize=(8, 5), fontsize=14, name=""):
        """The reference's base update is a no-op (src/Bidder.py:21-22); TruthfulBidder inherits
        it. The shading and learning bidders override it (GPU updates)."""
        if self.kind is None:
            raise NotImplementedError(f"{type(self).__name__}.update: not a built plugin")

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

    def bid(self, value, context, estimated_CTR):
        """Bidder.bid (src/Bidder.py:47-58, :171-208, :348-367, :455-475) as one call: the draw
        of the bidder's state on the host (numpy rng / torch generator, the reference's
        calls), the bid rule on the GPU (ag_bid); gamma (and the propensity) are logged."""
        from .plugin_gpu import shading_bid
        return shading_bid(self, value, estimated_CTR)


class EmpiricalShadedBidder(_ShadingBidder):
    """src/Bidder.py:38-153."""

    kind = _lib.BIDDER_EMPIRICAL_SHADED

    def update(self, contexts, values, bids, prices, outcomes, estimated_CTRs, won_mask, iteration,
               plot=False, figsize=(8, 5), fontsize=14, name=""):
        """src/Bidder.py:60-147 called directly: the GPU update (ag_empirical_update) of the
        logged gammas against these utilities; sets prev_gamma."""
        from .plugin_gpu import empirical_update
        empirical_update(self, values, prices, outcomes, won_mask)

    def clear_logs(self, memory):
        self.gammas = self.gammas[-memory:] if memory else []


def _linear(n_in, n_out):
    """torch.nn.Linear(n_in, n_out)'s default initialisation (kaiming-uniform weight, uniform
    bias), drawn from torch's global generator as the reference's constructors draw it.
    Returns (weight [n_out][n_in], bias [n_out]) float32 numpy."""
    lin = torch.nn.Linear(n_in, n_out, bias=True)
    return lin.weight.detach().numpy().copy(), lin.bias.detach().numpy().copy()


class _LearningBidder(_ShadingBidder):
    """Host mirror of a learning bidder's models (the device holds the live copy).

    `winrate` = PyTorchWinRateEstimator (src/Models.py:51-62): Linear(3, 1) + sigmoid;
    `policy` = the 12 parameters on the policy's forward path, in parameters() order:
    shared W [2][2], b [2]; mu W [1][2], b [1]; sigma W [1][2], b [1] (src/Models.py:64-104,
    :92-164). Constructors draw their initial values in the reference's order."""

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, **kw):
        super().__init__(rng, gamma_sigma, init_gamma, **kw)
        self.propensities = []
        self.model_initialised = False
        self.winrate = None
        self.policy = None

    def _state16(self):
        """float32 [16]: win-rate weight (3), bias, then the policy's 12 parameters."""
        st = np.zeros(16, np.float32)
        if self.winrate is not None:
            st[:3], st[3] = self.winrate[0].ravel(), self.winrate[1][0]
        if self.policy is not None:
            st[4:] = np.concatenate([p.ravel() for p in self.policy])
        return st

    def _load_state16(self, st):
        st = np.asarray(st, np.float32)
        if self.winrate is not None:
            self.winrate = (st[:3].reshape(1, 3).copy(), st[3:4].copy())
        if self.policy is not None:
            shapes = [(2, 2), (2,), (1, 2), (1,), (1, 2), (1,)]
            out, o = [], 4
            for sh in shapes:
                k = int(np.prod(sh))
                out.append(st[o:o + k].reshape(sh).copy())
                o += k
            self.policy = out

    def _learner_state(self):
        """ag_learner_state the agent bids from."""
        if not self.model_initialised:
            return _lib.LEARNER_UNINITIALISED
        return _lib.LEARNER_SEARCH if getattr(self, "inference", None) == "search" else _lib.LEARNER_POLICY

    def update(self, contexts, values, bids, prices, outcomes, estimated_CTRs, won_mask, iteration,
               plot=False, figsize=(8, 5), fontsize=14, name=""):
        """The bidder's update (src/Bidder.py:204-325, :364-431, :473-615) called directly: the
        GPU trainer (ag_bidder_update) on the logged gammas / propensities and these arrays."""
        from .plugin_gpu import learner_update_call
        learner_update_call(self, values, prices, outcomes, estimated_CTRs, won_mask, name)

    def clear_logs(self, memory):
        if not memory:
            self.gammas = []
            self.propensities = []
        else:
            self.gammas = self.gammas[-memory:]
            self.propensities = self.propensities[-memory:]


class ValueLearningBidder(_LearningBidder):
    """Bid shading by value learning (src/Bidder.py:156-333): a win-rate model
    P(win | CTR, value, gamma) and, with inference 'policy', a Gaussian shading policy
    trained to maximise the predicted utility. Uninitialised it bids gamma ~ N(prev_gamma,
    gamma_sigma); fitted it bids from its policy ('policy') or by a 128-point search of the
    win-rate model's utility ('search'). Its update is the GPU trainer (ag_bidder_update)."""

    kind = _lib.BIDDER_VALUE_LEARNING

    def __init__(self, rng, gamma_sigma, init_gamma=1.0, inference="search"):
        assert inference in ["search", "policy"]
        super().__init__(rng, gamma_sigma, init_gamma, inference=inference)
        self.inference = inference
        self.winrate = _linear(3, 1)
        if inference == "policy":  # BidShadingPolicy: shared, mu hidden, mu out, sigma hidden, sigma out
            shared, _, mu, _, sigma = (_linear(2, 2), _linear(2, 2), _linear(2, 1), _linear(2, 2),
                                       _linear(2, 1))
            self.policy = [shared[0], shared[1], mu[0], mu[1], sigma[0], sigma[1]]

    def _mode(self):
        return _lib.VL_POLICY if self.inference == "policy" else _lib.VL_SEARCH


class PolicyLearningBidder(_LearningBidder):
    """Bid shading by off-policy policy learning (src/Bidder.py:336-439):
    BidShadingContextualBandit with the REINFORCE / off-policy REINFORCE / TRPO / PPO loss.
    Its update is the GPU trainer (ag_bidder_update)."""

    kind = _lib.BIDDER_POLICY_LEARNING

    def __init__(self, rng, gamma_sigma, loss, init_gamma=1.0):
        super().__init__(rng, gamma_sigma, init_gamma, loss=loss)
        if loss not in _lib.PL_LOSSES:
            raise NotImplementedError(f"PolicyLearningBidder(loss={loss!r}): "
                                      f"one of {sorted(_lib.PL_LOSSES)} is built")
        self.loss = loss
        shared, mu, sigma = _linear(2, 2), _linear(2, 1), _linear(2, 1)
        self.policy = [shared[0], shared[1], mu[0], mu[1], sigma[0], sigma[1]]

    def _mode(self):
        return _lib.PL_LOSSES[self.loss]


class DoublyRobustBidder(_LearningBidder):
    """Bid shading with a doubly robust policy estimator (src/Bidder.py:442-623): win-rate
    model + BidShadingContextualBandit('Doubly Robust'). Its update is the GPU trainer."""

    kind = _lib.BIDDER_DOUBLY_ROBUST

    def __init__(self, rng, gamma_sigma, init_gamma=1.0):
        super().__init__(rng, gamma_sigma, init_gamma)
        self.winrate = _linear(3, 1)
        shared, mu, sigma = _linear(2, 2), _linear(2, 1), _linear(2, 1)
        self.policy = [shared[0], shared[1], mu[0], mu[1], sigma[0], sigma[1]]

    def _mode(self):
        return 0
