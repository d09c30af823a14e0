"""auctiongym_amd -- MI355X-native batched AuctionGym hot path.

Drop-in for the reference's plugin surface (src/{Auction,Agent,AuctionAllocation,Bidder,
BidderAllocation,Impression,main}.py) over HIP kernels reached through the C-ABI in
include/auctiongym.h (libauctiongym_hip.so, built by `make -C auction-gym_amd`).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
__version__ = "0.1.0"
