"""Allocation mechanisms: the plugin surface of src/AuctionAllocation.py:3-34.

`allocate(bids, num_slots)` keeps the reference signature and return types for one
auction; `allocate_batch(bids)` is the native form: bids [P][B] in HBM -> winners,
prices, second prices for B auctions in one kernel (ag_allocate). Both run on the GPU.
Ties go to the lowest slot (SURVEY §8 a13').
"""
import numpy as np
import torch

from . import _lib


class AllocationMechanism:
    """Base class for allocation mechanisms (src/AuctionAllocation.py:3-9)."""

    code = None
    _engines = {}

    def __init__(self):
        pass

    def _engine(self, P):
        from .engine import AuctionEngine
        key = (type(self), P)
        eng = AllocationMechanism._engines.get(key)
        if eng is None:
            eng = AuctionEngine(P, P, 1, 1, 0, self.code)
            AllocationMechanism._engines[key] = eng
        return eng

    def allocate_batch(self, bids):
        """bids: float64 [P][B] device tensor -> (winner int32 [B], price [B], second [B]).
        P == 1: nobody is charged (SecondPrice price and every second price are NaN)."""
        return self._engine(int(bids.shape[0])).allocate(bids)

    def allocate(self, bids, num_slots):
        """One auction, reference return types: (winners int64[S], prices[<=S], second[<=S])."""
        if num_slots != 1:
            raise NotImplementedError("multi-slot allocation is not supported (src/main.py:37)")
        b = np.asarray(bids, np.float64).reshape(-1, 1)
        P = b.shape[0]
        dev = torch.from_numpy(np.ascontiguousarray(b)).cuda()
        w, p, s = self.allocate_batch(dev)
        w, p, s = int(w.item()), float(p.item()), float(s.item())
        winners = np.array([w], dtype=np.int64)
        prices = np.array([] if np.isnan(p) else [p])
        second = np.array([] if (P < 2 or np.isnan(s)) else [s])
        return winners, prices, second


class FirstPrice(AllocationMechanism):
    """(Generalised) First-Price Allocation (src/AuctionAllocation.py:11-23)."""
    code = _lib.FIRST_PRICE


class SecondPrice(AllocationMechanism):
    """(Generalised) Second-Price Allocation (src/AuctionAllocation.py:26-34)."""
    code = _lib.SECOND_PRICE
