"""Shared test setup: import paths, the `gpu` marker, fixture loaders.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, C-ABI symbol
table, gloo multi-process paths); `-m gpu` tests need an MI355X and call the HIP path
through the C-ABI, comparing it with the oracle (oracle/) and the golden vectors.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

CAPTURES = ("sp_oracle_r4096", "fp_oracle_n8_p3", "sp_oracle_n32_p8", "sp_oracle_n4_p1",
            "fp_oracle_n5_k5")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP path")


def load_capture(name):
    arrays = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    return arrays, meta["meta"], meta["aggregates"]


def mech_code(meta):
    return 0 if meta["allocation"] == "FirstPrice" else 1


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return torch.device("cuda", 0)
