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


def _lrts_worker(rank, world, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from auctiongym_amd.sharding import gather_records, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kat = np.load(os.path.join(ROOT, "tests", "golden", "sp_ts_update_kat.npz"))
    X, A, y = kat["a2_X"], kat["a2_A"], kat["a2_y"]
    lo, hi = shard_range(len(y), rank, world)          # this rank's share of the won samples
    key = (2 << 16) | (A[lo:hi].astype(np.int64) << 1) | (y[lo:hi] != 0)
    cap = hi - lo + 7
    st = {"key": torch.zeros(cap, dtype=torch.int32), "x": torch.zeros((5, cap), dtype=torch.float32),
          "count": torch.tensor([hi - lo], dtype=torch.int64)}
    st["key"][:hi - lo] = torch.from_numpy(key.astype(np.uint32).view(np.int32))
    st["x"][:, :hi - lo] = torch.from_numpy(X[lo:hi].astype(np.float32).T)
    g = gather_records(st)
    n = int(g["count"][0])
    k = g["key"][:n].numpy().view(np.uint32)
    xs = g["x"][:, :n].numpy().T
    m, pm, q, ep, _ = O.lrts_update(xs, (k >> 1) & 0x7FFF, k & 1, kat["a2_m0"], kat["a2_prevm0"], kat["a2_q0"])
    np.save(out_path + f".{rank}.npy", np.concatenate([m.ravel(), q.ravel(), [ep]]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_lrts_update_on_gathered_samples_is_rank_independent(tmp_path, oracle, world):
    """Each rank holds a shard of the won samples; after gather_records every rank trains on
    the same multiset: identical m, q, epochs on every rank, equal to one process training
    on all samples (exact sums: order-free)."""
    out = str(tmp_path / "lrts")
    mp.spawn(_lrts_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = [np.load(out + f".{r}.npy") for r in range(world)]
    kat = np.load(os.path.join(ROOT, "tests", "golden", "sp_ts_update_kat.npz"))
    m, pm, q, ep, _ = oracle.lrts_update(kat["a2_X"], kat["a2_A"], kat["a2_y"], kat["a2_m0"],
                                         kat["a2_prevm0"], kat["a2_q0"])
    want = np.concatenate([m.ravel(), q.ravel(), [ep]])
    for g in got:
        assert np.array_equal(g, want)


def _bidder_worker(rank, world, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from auctiongym_amd.sharding import gather_records, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kat = np.load(os.path.join(ROOT, "tests", "golden", "dm_update_kat.npz"))
    k = lambda s: kat[f"a2_{s}"]  # noqa: E731
    n = len(k("est_ctr"))
    lo, hi = shard_range(n, rank, world)  # this rank's auctions' records, in log order
    cap = hi - lo + 5
    st = {"agent": torch.zeros(cap, dtype=torch.int32), "order": torch.zeros(cap, dtype=torch.int64)}
    for f in ("gamma", "utility", "ctr", "value", "propensity"):
        st[f] = torch.zeros(cap, dtype=torch.float64)
    st["won"] = torch.zeros(cap, dtype=torch.uint8)
    st["count"] = torch.tensor([hi - lo], dtype=torch.int64)
    for f, v in (("gamma", k("gamma")), ("utility", k("util")), ("ctr", k("est_ctr")), ("value", k("value")),
                 ("propensity", k("propensity")), ("won", k("won").astype(np.uint8)),
                 ("order", np.arange(n, dtype=np.int64))):
        st[f][:hi - lo] = torch.from_numpy(np.ascontiguousarray(v[lo:hi]))
    g = gather_records(st)
    m = int(g["count"][0])
    idx = np.argsort(g["order"][:m].numpy(), kind="stable")  # the device's (agent, log order) sort
    col = {f: g[f][:m].numpy()[idx] for f in ("ctr", "value", "gamma", "won")}
    wr0 = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
    pol0 = np.concatenate([k(f"pol0_{i}").ravel() for i in (0, 1, 4, 5, 8, 9)])
    r = O.vl_update(col["ctr"], col["value"], col["gamma"], col["won"], wr0, pol0, False, None)
    np.save(out_path + f".{rank}.npy", np.concatenate([r["wr"], r["epochs"].astype(np.float32)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bidder_update_on_gathered_records_is_rank_independent(tmp_path, oracle, world):
    """Learning-bidder records (the store ag_bidder_update reads: ctr, value, gamma, won, log
    order, ...) sharded by auction over ranks and all-gathered: restored to log order, every
    rank fits the same ValueLearningBidder win-rate model, equal to one process on all the
    reference's records (FP_DM_TS KAT agent 2)."""
    out = str(tmp_path / "vl")
    mp.spawn(_bidder_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = [np.load(out + f".{r}.npy") for r in range(world)]
    kat = np.load(os.path.join(ROOT, "tests", "golden", "dm_update_kat.npz"))
    k = lambda s: kat[f"a2_{s}"]  # noqa: E731
    wr0 = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
    pol0 = np.concatenate([k(f"pol0_{i}").ravel() for i in (0, 1, 4, 5, 8, 9)])
    r = oracle.vl_update(k("est_ctr"), k("value"), k("gamma"), k("won"), wr0, pol0, False, None)
    want = np.concatenate([r["wr"], r["epochs"].astype(np.float32)])
    for g in got:
        assert np.array_equal(g, want)


# ---- agent-parallel learner updates (sharding.route_records / take_owned_rows: the path
# bench.py and sharding.*_agent_parallel take at N > 1)

def _lrts_agents_case():
    """The reference's SP_Truthful_TS won samples (agent 2's KAT) relabelled over 3 agents."""
    kat = np.load(os.path.join(ROOT, "tests", "golden", "sp_ts_update_kat.npz"))
    X, A, y = kat["a2_X"], kat["a2_A"], kat["a2_y"]
    agent = np.arange(len(y)) % 3
    return kat, X, A, y, agent


def _lrts_route_worker(rank, world, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from auctiongym_amd.sharding import owners, route_records, shard_range, take_owned_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kat, X, A, y, agent = _lrts_agents_case()
    lo, hi = shard_range(len(y), rank, world)  # this rank's auctions' won samples
    key = (agent[lo:hi].astype(np.int64) << 16) | (A[lo:hi].astype(np.int64) << 1) | (y[lo:hi] != 0)
    cap = hi - lo + 3
    st = {"key": torch.zeros(cap, dtype=torch.int32), "x": torch.zeros((5, cap), dtype=torch.float32),
          "count": torch.tensor([hi - lo], dtype=torch.int64)}
    st["key"][:hi - lo] = torch.from_numpy(key.astype(np.uint32).view(np.int32))
    st["x"][:, :hi - lo] = torch.from_numpy(X[lo:hi].astype(np.float32).T)
    own = owners([0, 1, 2], world)
    r = route_records(st, own)
    n = int(r["count"][0])
    k = r["key"][:n].numpy().view(np.uint32)
    xs = r["x"][:, :n].numpy().T
    ag = k >> 16
    assert set(ag.tolist()) <= {a for a, o in own.items() if o == rank}  # only owned agents arrive
    m = np.zeros((3,) + kat["a2_m0"].shape, np.float32)
    q = np.zeros_like(m)
    ep = np.zeros(3, np.int64)
    for a in range(3):
        if own[a] == rank:
            sel = ag == a
            m[a], _, q[a], ep[a], _ = O.lrts_update(xs[sel], (k[sel] >> 1) & 0x7FFF, k[sel] & 1, kat["a2_m0"],
                                                   kat["a2_prevm0"], kat["a2_q0"])
    m, q, ep = (take_owned_rows(v, own) for v in (m, q, ep))
    np.save(out_path + f".{rank}.npy", np.concatenate([m.ravel(), q.ravel(), ep.astype(np.float32)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_lrts_agent_parallel_update_equals_single_process(tmp_path, oracle, world):
    """Won samples of 3 LR-TS agents sharded by auction over ranks; each is routed to its
    agent's owner (all-to-all), owners train their agents, posteriors exchanged
    (all-gather): every rank ends with the single-process models bit for bit, and no rank
    trains an agent it does not own."""
    out = str(tmp_path / "lrts_ap")
    mp.spawn(_lrts_route_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    kat, X, A, y, agent = _lrts_agents_case()
    m = np.zeros((3,) + kat["a2_m0"].shape, np.float32)
    q = np.zeros_like(m)
    ep = np.zeros(3, np.int64)
    for a in range(3):
        s = agent == a
        m[a], _, q[a], ep[a], _ = oracle.lrts_update(X[s], A[s], y[s], kat["a2_m0"], kat["a2_prevm0"], kat["a2_q0"])
    want = np.concatenate([m.ravel(), q.ravel(), ep.astype(np.float32)])
    for r in range(world):
        assert np.array_equal(np.load(out + f".{r}.npy"), want)


def _dm_agents_case():
    kat = np.load(os.path.join(ROOT, "tests", "golden", "dm_update_kat.npz"))
    k = lambda s: kat[f"a2_{s}"]  # noqa: E731
    n = len(k("est_ctr"))
    agent = (np.arange(n) % 2).astype(np.int32)  # the reference's records split over 2 agents
    wr0 = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
    pol0 = np.concatenate([k(f"pol0_{i}").ravel() for i in (0, 1, 4, 5, 8, 9)])
    return k, n, agent, wr0, pol0


def _bidder_route_worker(rank, world, port, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    from auctiongym_amd.sharding import owners, route_records, shard_range, take_owned_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    k, n, agent, wr0, pol0 = _dm_agents_case()
    lo, hi = shard_range(n, rank, world)
    cap = hi - lo + 5
    st = {"agent": torch.zeros(cap, dtype=torch.int32), "order": torch.zeros(cap, dtype=torch.int64)}
    for f in ("gamma", "utility", "ctr", "value", "propensity"):
        st[f] = torch.zeros(cap, dtype=torch.float64)
    st["won"] = torch.zeros(cap, dtype=torch.uint8)
    st["count"] = torch.tensor([hi - lo], dtype=torch.int64)
    for f, v in (("agent", agent), ("gamma", k("gamma")), ("utility", k("util")), ("ctr", k("est_ctr")),
                 ("value", k("value")), ("propensity", k("propensity")), ("won", k("won").astype(np.uint8)),
                 ("order", np.arange(n, dtype=np.int64))):
        st[f][:hi - lo] = torch.from_numpy(np.ascontiguousarray(v[lo:hi]))
    own = owners([1, 0], world)  # owner order need not follow agent order
    r = route_records(st, own)
    m = int(r["count"][0])
    ag = r["agent"][:m].numpy()
    assert set(ag.tolist()) <= {a for a, o in own.items() if o == rank}
    wr = np.zeros((2, 4), np.float32)
    ep = np.zeros((2, 3), np.int32)
    for a in range(2):
        if own[a] != rank:
            continue
        sel = np.nonzero(ag == a)[0]
        idx = sel[np.argsort(r["order"][:m].numpy()[sel], kind="stable")]  # the trainer's log-order sort
        col = {f: r[f][:m].numpy()[idx] for f in ("ctr", "value", "gamma", "won")}
        res = O.vl_update(col["ctr"], col["value"], col["gamma"], col["won"], wr0, pol0, False, None)
        wr[a], ep[a] = res["wr"], res["epochs"]
    wr, ep = take_owned_rows(wr, own), take_owned_rows(ep, own)
    np.save(out_path + f".{rank}.npy", np.concatenate([wr.ravel(), ep.ravel().astype(np.float32)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bidder_agent_parallel_update_equals_single_process(tmp_path, oracle, world):
    """Learning-bidder records of 2 agents sharded by auction; routed to their owners, who
    restore log order and fit; models exchanged: every rank holds the single-process win-rate
    models and epochs (FP_DM_TS KAT records). With world 3 one rank owns nothing."""
    out = str(tmp_path / "vl_ap")
    mp.spawn(_bidder_route_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    k, n, agent, wr0, pol0 = _dm_agents_case()
    wr = np.zeros((2, 4), np.float32)
    ep = np.zeros((2, 3), np.int32)
    for a in range(2):
        s = agent == a
        res = oracle.vl_update(k("est_ctr")[s], k("value")[s], k("gamma")[s], k("won")[s], wr0, pol0, False, None)
        wr[a], ep[a] = res["wr"], res["epochs"]
    want = np.concatenate([wr.ravel(), ep.ravel().astype(np.float32)])
    for r in range(world):
        assert np.array_equal(np.load(out + f".{r}.npy"), want)


def _overflow_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
    from auctiongym_amd.sharding import gather_records, owners, route_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cap = 4 + rank  # ranks hold different capacities
    st = {"agent": torch.zeros(cap, dtype=torch.int32), "gamma": torch.zeros(cap, dtype=torch.float64),
          "count": torch.tensor([cap + 2 if rank == 1 else 2], dtype=torch.int64)}  # rank 1 overflowed
    res = []
    for fn in (lambda: gather_records(st), lambda: route_records(st, owners([0], world))):
        try:
            fn()
            res.append(0)
        except ValueError:
            res.append(1)
    ok = {"agent": torch.zeros(cap, dtype=torch.int32), "count": torch.tensor([3 + rank], dtype=torch.int64)}
    g = gather_records(ok)  # capacities below the largest count are padded, not refused
    res.append(int(g["count"][0]))
    np.save(out_path + f".{rank}.npy", np.array(res))
    dist.barrier()
    dist.destroy_process_group()


def test_store_overflow_raises_on_every_rank(tmp_path):
    """A rank whose record store overflowed makes gather_records / route_records raise on
    EVERY rank (no rank left waiting in a collective); stores smaller than another rank's
    count are padded."""
    out = str(tmp_path / "ovf")
    mp.spawn(_overflow_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert np.load(out + f".{r}.npy").tolist() == [1, 1, 7]


def _empty_route_worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
    from auctiongym_amd.sharding import owners, route_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cap = 6
    res = []

    def store(n):
        st = {"key": torch.zeros(cap, dtype=torch.int32), "x": torch.zeros((5, cap), dtype=torch.float32),
              "count": torch.tensor([n], dtype=torch.int64)}
        st["key"][:n] = torch.arange(n, dtype=torch.int32) % 2 << 16  # agents 0, 1
        st["x"][:, :n] = torch.arange(5 * n, dtype=torch.float32).reshape(5, n) + 100 * rank
        return st

    # (a) rank 0 holds no records; (b) every rank empty; (c) an empty owner list
    for st, own in ((store(0 if rank == 0 else 4), owners([0, 1], world)), (store(0), owners([0, 1], world)),
                    (store(3), {})):
        r = route_records(st, own)
        n = int(r["count"][0])
        res.append(n)
        res.append(float(r["x"][:, :n].sum()))
    np.save(out_path + f".{rank}.npy", np.array(res))
    dist.barrier()
    dist.destroy_process_group()


def test_route_records_with_empty_ranks(tmp_path):
    """route_records when a rank sends nothing (no records, none of an owned agent, no owners,
    every rank empty): no crash, no rank left waiting, the records that exist arrive."""
    out = str(tmp_path / "empty")
    mp.spawn(_empty_route_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = (np.load(out + f".{r}.npy").tolist() for r in range(2))
    # (a) rank 1's 4 records: agents 0 (owner 0) and 1 (owner 1), 2 each
    x1 = np.arange(20, dtype=np.float32).reshape(5, 4) + 100
    assert r0[:2] == [2, float(x1[:, 0::2].sum())] and r1[:2] == [2, float(x1[:, 1::2].sum())]
    assert r0[2:4] == [0, 0.0] and r1[2:4] == [0, 0.0]
    assert r0[4:] == [0, 0.0] and r1[4:] == [0, 0.0]


# ---- record-parallel learner updates (sharding.bidder_update_record_parallel: the path taken
# at N > 1 when the learners are fewer than the ranks) -- the CPU restatement run on every rank's
# own records with each epoch's exact sums all-reduced over gloo (oracle.set_reduce) equals the
# single-process fit bit for bit: the decomposition the device's per-epoch launches use.

def _rp_shard(n, rank, world):
    from auctiongym_amd.sharding import shard_range
    return shard_range(n, rank, world)


def _rp_cases(O):
    """(name, fn(lo, hi) -> flat result) of the fits the record-parallel test runs on records
    [lo, hi): a DoublyRobustBidder's DR policy fit (FP_DR_TS KAT agent 0 from its initialised
    policy and the win-rate model as given: 2650 epochs), a ValueLearningBidder's win-rate fit
    (FP_DM_TS KAT agent 2, its first 400 records) and an LR-TS allocator (SP_Truthful_TS KAT
    agent 2); the DR fit's noise columns are the records' global indices."""
    dr = np.load(os.path.join(ROOT, "tests", "golden", "dr_update_kat.npz"))
    kd = lambda s: dr[f"a0_{s}"]  # noqa: E731
    zd = O.fit_noise(3, 0, 3000, len(kd("est_ctr")))
    dm = np.load(os.path.join(ROOT, "tests", "golden", "dm_update_kat.npz"))
    km = lambda s: dm[f"a2_{s}"][:400]  # noqa: E731
    ts = np.load(os.path.join(ROOT, "tests", "golden", "sp_ts_update_kat.npz"))

    def f_dr(lo, hi):
        r = O.dr_update(*(kd(f)[lo:hi] for f in ("est_ctr", "value", "gamma", "propensity", "won", "util")),
                        kd("wr0_0").ravel().tolist() + kd("wr0_1").ravel().tolist(),
                        np.concatenate([kd(f"pol0_{i}").ravel() for i in range(6)]), True,
                        np.ascontiguousarray(zd[:, lo:hi]), trace=False, skip_winrate=True)
        return np.concatenate([r["pol"], r["epochs"].astype(np.float32)])

    def f_vl(lo, hi):
        r = O.vl_update(*(km(f)[lo:hi] for f in ("est_ctr", "value", "gamma", "won")),
                        np.concatenate([dm["a2_wr0_0"].ravel(), dm["a2_wr0_1"].ravel()]),
                        np.concatenate([dm[f"a2_pol0_{i}"].ravel() for i in (0, 1, 4, 5, 8, 9)]), False, None,
                        trace=False)
        return np.concatenate([r["wr"], r["epochs"].astype(np.float32)])

    def f_ts(lo, hi):
        m, pm, q, ep, _ = O.lrts_update(ts["a2_X"][lo:hi], ts["a2_A"][lo:hi], ts["a2_y"][lo:hi], ts["a2_m0"],
                                        ts["a2_prevm0"], ts["a2_q0"], trace=False)
        return np.concatenate([m.ravel(), q.ravel(), [ep]])
    return [("dr", len(kd("est_ctr")), f_dr), ("vl", 400, f_vl), ("lrts", len(ts["a2_y"]), f_ts)]


def _rp_oracle_worker(rank, world, port, cases, out_path):
    import sys
    for p in (os.path.join(ROOT, "auction-gym_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import oracle as O
    torch.set_num_threads(1)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allreduce(w):
        t = torch.from_numpy(w.copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        w[:] = t.numpy()
    res = []
    for name, n, fn in _rp_cases(O):
        if name not in cases:
            continue
        lo, hi = _rp_shard(n, rank, world)  # a contiguous shard of the records in log order
        O.set_reduce(allreduce, n)
        res.append(fn(lo, hi))
        O.set_reduce(None)
    np.save(out_path + f".{rank}.npy", np.concatenate(res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,cases", [(2, ("dr", "vl", "lrts")), (3, ("dr", "lrts"))])
def test_record_parallel_fits_equal_single_process(tmp_path, oracle, world, cases):
    """Record-parallel learner updates on gloo: every rank fits on its own
    records, each epoch's exact fixed-point sums all-reduced, and ends with the single process's
    models and epochs bit for bit (DoublyRobustBidder policy fit, ValueLearningBidder win-rate
    fit, LR-TS allocator)."""
    out = str(tmp_path / "rp")
    mp.spawn(_rp_oracle_worker, args=(world, _free_port(), cases, out), nprocs=world, join=True)
    got = [np.load(out + f".{r}.npy") for r in range(world)]
    want = np.concatenate([fn(0, n) for name, n, fn in _rp_cases(oracle) if name in cases])
    for g in got:
        assert np.array_equal(g, want)


def test_record_parallel_cost_model():
    """sharding.record_parallel_pays: record-parallel for FP_DR_TS's 3
    learners on 8 GPUs (agent-parallel would give each owner 8/3 of one GPU's work), not on 2
    or 4 GPUs, nor when every rank owns a learner."""
    from auctiongym_amd.sharding import record_parallel_pays
    assert record_parallel_pays(3, 8) and record_parallel_pays(1, 2) and record_parallel_pays(2, 8)
    assert not record_parallel_pays(3, 4) and not record_parallel_pays(3, 2) and not record_parallel_pays(21, 8)
    assert not record_parallel_pays(8, 8) and not record_parallel_pays(3, 1)
