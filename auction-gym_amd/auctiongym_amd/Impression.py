"""Per-(round, participant) log record (src/Impression.py:4-31).

On the GPU path logs are structure-of-arrays device buffers (ag_batch_out); this record
type is only materialised when a caller iterates `Agent.logs` (compatibility / debugging).
"""
from dataclasses import dataclass

import numpy as np


@dataclass
class ImpressionOpportunity:
    __slots__ = ["context", "item", "value", "bid", "best_expected_value", "true_CTR",
                 "estimated_CTR", "price", "second_price", "outcome", "won"]

    context: np.ndarray
    item: int
    value: float
    bid: float
    best_expected_value: float
    true_CTR: float
    estimated_CTR: float
    price: float
    second_price: float
    outcome: bool
    won: bool
