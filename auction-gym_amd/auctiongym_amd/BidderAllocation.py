"""Allocator plugins: the surface of src/BidderAllocation.py:11-82.

OracleAllocator's estimate_CTR (sigmoid(items @ ctx), src/BidderAllocation.py:81-82) runs
inside the fused simulate kernel with the reference's exact FP64 arithmetic.
PyTorchLogisticRegressionAllocator's Thompson-sampling forward (src/Models.py:28-33) runs
there too, and its update (src/BidderAllocation.py:29-65) is the GPU training kernel of
ag_lrts_update, batched over every LR-TS agent of the auction (Agent.update). The model
tensors here are host mirrors of the device posterior, refreshed after each update.
"""
import torch

from . import _lib


class Allocator:
    """Base class for an allocator (src/BidderAllocation.py:11-18)."""

    kind = None

    def __init__(self, rng):
        self.rng = rng

    def update(self, contexts, items, outcomes, iteration, plot, figsize, fontsize, name):
        """The reference's base update is a no-op (src/BidderAllocation.py:17-18); OracleAllocator
        inherits it. PyTorchLogisticRegressionAllocator overrides it (GPU trainer)."""
        if self.kind is None:
            raise NotImplementedError(f"{type(self).__name__}.update: not a built plugin")


class OracleAllocator(Allocator):
    """An allocator that acts on the true P(click) (src/BidderAllocation.py:71-82)."""

    kind = _lib.ALLOCATOR_ORACLE

    def __init__(self, rng):
        self.item_embeddings = None
        super().__init__(rng)

    def update_item_embeddings(self, item_embeddings):
        self.item_embeddings = item_embeddings

    def estimate_CTR(self, context):
        """sigmoid(item_embeddings @ context) (src/BidderAllocation.py:81-82) on the GPU, with
        the simulate kernels' exact FP64 arithmetic (ag_estimate_ctr)."""
        from .plugin_gpu import oracle_estimate_ctr
        return oracle_estimate_ctr(self, context)


class PyTorchLogisticRegression:
    """Parameters of src/Models.py:18-26: m [K][n_dim+1] ~ N(0, 1) (drawn from torch's global
    generator exactly as the reference's constructor does), prev_iter_m = m, q = 1."""

    def __init__(self, n_dim, n_items):
        self.m = torch.empty(n_items, n_dim + 1)
        torch.nn.init.normal_(self.m, mean=0.0, std=1.0)
        self.prev_iter_m = self.m.detach().clone()
        self.q = torch.ones((n_items, n_dim + 1))

    def sample_noise(self):
        """The Thompson-sampling draw of src/Models.py:31 (same torch call, same stream)."""
        return torch.normal(mean=0.0, std=1.0 / torch.sqrt(self.q))


class PyTorchLogisticRegressionAllocator(Allocator):
    """Bayesian logistic regression with Thompson sampling (src/BidderAllocation.py:21-68)."""

    kind = _lib.ALLOCATOR_LRTS

    def __init__(self, rng, embedding_size, num_items, thompson_sampling=True):
        # an Auction defers this allocator's update to train it together with the other LR-TS
        # agents' (Auction._settle_lrts); reading the posterior or the epochs runs it first
        self._settle = None
        self.response_model = PyTorchLogisticRegression(n_dim=embedding_size, n_items=num_items)
        self.thompson_sampling = thompson_sampling
        self.embedding_size = embedding_size
        self.num_items = num_items
        self.epochs = None  # epochs run by the last update (None: not updated yet)
        super().__init__(rng)

    @property
    def response_model(self):
        if self._settle is not None:
            self._settle()
        return self._response_model

    @response_model.setter
    def response_model(self, model):
        self._response_model = model

    @property
    def epochs(self):
        if self._settle is not None:
            self._settle()
        return self._epochs

    @epochs.setter
    def epochs(self, n):
        self._epochs = n

    def estimate_CTR(self, context, sample=True):
        """src/BidderAllocation.py:67-68 on the GPU (ag_estimate_ctr): float32 CTRs [K] of the
        observed context (with its intercept); with Thompson sampling (and sample=True) the
        posterior draw is torch.normal(0, 1/sqrt(q)) from torch's global generator."""
        from .plugin_gpu import lrts_estimate_ctr
        return lrts_estimate_ctr(self, context, sample=sample)

    def update(self, contexts, items, outcomes, iteration, plot=False, figsize=(8, 5), fontsize=14, name=""):
        """src/BidderAllocation.py:29-65 called directly (outside an Auction, whose Agent.update
        batches every LR-TS agent): the GPU trainer (ag_lrts_update) on these samples."""
        from .plugin_gpu import lrts_update
        lrts_update(self, contexts, items, outcomes)
