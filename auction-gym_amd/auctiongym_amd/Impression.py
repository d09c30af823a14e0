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

    def set_true_CTR(self, best_expected_value, true_CTR):
        """src/Impression.py:21-23."""
        self.best_expected_value = best_expected_value
        self.true_CTR = true_CTR

    def set_price_outcome(self, price, second_price, outcome, won=True):
        """src/Impression.py:25-29."""
        self.price = price
        self.second_price = second_price
        self.outcome = outcome
        self.won = won

    def set_price(self, price):
        """src/Impression.py:31-32."""
        self.price = price
