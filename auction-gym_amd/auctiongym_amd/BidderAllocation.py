"""Allocator plugins: the surface of src/BidderAllocation.py:11-82.

OracleAllocator's estimate_CTR (sigmoid(items @ ctx), src/BidderAllocation.py:81-82) runs
inside the fused simulate kernel with the reference's exact FP64 arithmetic.
PyTorchLogisticRegressionAllocator keeps its constructor so configs parse; the engine
refuses it with NotImplementedError until the LR-TS kernels land.
"""
from . import _lib


class Allocator:
    """Base class for an allocator (src/BidderAllocation.py:11-18)."""

    kind = None

    def __init__(self, rng):
        self.rng = rng

    def update(self, contexts, items, outcomes, iteration, plot, figsize, fontsize, name):
        pass


class OracleAllocator(Allocator):
    """An allocator that acts on the true P(click) (src/BidderAllocation.py:71-82)."""

    kind = _lib.ALLOCATOR_ORACLE

    def __init__(self, rng):
        self.item_embeddings = None
        super().__init__(rng)

    def update_item_embeddings(self, item_embeddings):
        self.item_embeddings = item_embeddings


class PyTorchLogisticRegressionAllocator(Allocator):
    """Bayesian logistic regression with Thompson sampling (src/BidderAllocation.py:21-68);
    not yet on the GPU path."""

    kind = None

    def __init__(self, rng, embedding_size, num_items, thompson_sampling=True):
        super().__init__(rng)
        self.embedding_size = embedding_size
        self.num_items = num_items
        self.thompson_sampling = thompson_sampling
