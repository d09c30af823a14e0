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


POP_CAPTURES = ("sp_ts_r2048", "fp_dr_ts_r1024", "fp_dm_ts_r1024", "fp_ips_ts_r1024",
                "fp_dm_oracle_r1024", "fp_empirical_r2048", "sp_ts_mixed_flags_r2048",
                "ragged_items_r2048")


def pop_args(d, meta):
    """Population + replay inputs of a capture, in the oracle's keyword form."""
    from auctiongym_amd.population import kinds_from_names
    ak, bk, pg, gs = kinds_from_names(meta["allocators"], meta["bidders"], meta["bidder_kwargs"])
    return dict(alloc_kind=ak, bid_kind=bk, prev_gamma=pg, gamma_sigma=gs, OE=meta["OE"],
                ts_m=d.get("ts_m"), ts_noise=d.get("ts_noise"), gamma_raw=d["gamma_raw"],
                num_items=meta.get("num_items"))
