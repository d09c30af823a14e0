"""World-size-2 gloo runs of the multi-GPU path's host logic (CPU only): contiguous
global-index shards + the exact int64 limb all-reduce reproduce the single-process
counters bit for bit (the same functions bench.py uses over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _batch(B, N=6, P=2, E=5, K=12, seed=3):
    g = np.random.default_rng(seed)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ctx = g.normal(0, 1, (B, E))
    part = np.stack([g.choice(N, P, replace=False) for _ in range(B)]).astype(np.int32)
    u = g.random(B)
    return items, values, ctx, part, u


def _worker(rank, world, port, B, mech, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from auctiongym_amd.sharding import allreduce_counters, normalize_limbs, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    items, values, ctx, part, u = _batch(B)
    lo, hi = shard_range(B, rank, world)
    o = O.simulate(mech, items, values, ctx[lo:hi], part[lo:hi], u[lo:hi])
    limbs = torch.from_numpy(o["counters_fx"].copy())
    allreduce_counters(limbs)
    if rank == 0:
        np.save(out_path, normalize_limbs(limbs.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_counters_equal_single_process(tmp_path, oracle, world):
    B, mech = 30001, 1
    out = str(tmp_path / "limbs.npy")
    mp.spawn(_worker, args=(world, _free_port(), B, mech, out), nprocs=world, join=True)
    got = np.load(out)
    items, values, ctx, part, u = _batch(B)
    ref = oracle.simulate(mech, items, values, ctx, part, u)["counters_fx"]
    assert np.array_equal(got, ref)


def test_shard_ranges_cover_exactly():
    from auctiongym_amd.sharding import shard_range
    for total in (0, 1, 7, 1 << 24, 4_000_003):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))


def test_normalize_limbs_roundtrip():
    from auctiongym_amd.sharding import normalize_limbs
    g = np.random.default_rng(0)
    vals = [int(v) for v in g.integers(-(1 << 62), 1 << 62, 50)] + [0, -1, 1 << 100]
    # non-normalised: spread the value over the limbs arbitrarily, then normalise
    raw = np.array([[v - (5 << 42), 5, 0] if abs(v) < (1 << 62) else
                    [v & ((1 << 42) - 1), (v >> 42) & ((1 << 42) - 1), v >> 84] for v in vals], np.int64)
    n = normalize_limbs(raw)
    back = [int(a) + (int(b) << 42) + (int(c) << 84) for a, b, c in n]
    assert back == vals
    assert (n[:, 0] >= 0).all() and (n[:, 0] < (1 << 42)).all()
