"""Plugin kinds of a population: the codes the kernels dispatch on per participant
(include/auctiongym.h ag_allocator_kind / ag_bidder_kind)."""
import numpy as np

ALLOCATOR_KINDS = {"OracleAllocator": 0, "PyTorchLogisticRegressionAllocator": 1}
BIDDER_KINDS = {"TruthfulBidder": 0, "EmpiricalShadedBidder": 1, "ValueLearningBidder": 2,
                "PolicyLearningBidder": 3, "DoublyRobustBidder": 4}


def kinds_from_names(allocators, bidders, bidder_kwargs=None):
    """Class names (+ bidder kwargs) -> (alloc_kind, bid_kind, prev_gamma, gamma_sigma)."""
    n = len(allocators)
    ak = np.array([ALLOCATOR_KINDS[a] for a in allocators], np.int32)
    bk = np.array([BIDDER_KINDS[b] for b in bidders], np.int32)
    pg = np.ones(n)
    gs = np.ones(n)
    for i, kw in enumerate(bidder_kwargs or [{}] * n):
        pg[i] = float(kw.get("init_gamma", 1.0))
        gs[i] = float(kw.get("gamma_sigma", 1.0))
    return ak, bk, pg, gs
