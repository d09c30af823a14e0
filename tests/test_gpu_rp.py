"""The resumable, record-parallel learning-bidder update (ag_bidder_rp_*: one launch per epoch,
the training state in HBM) against the persistent trainer (ag_bidder_update), which the other
GPU tests pin to the oracle bit for bit. src/Bidder.py:204-325 (ValueLearningBidder), :473-615
(DoublyRobustBidder)."""
import numpy as np
import pytest

from test_gpu_parity import _dr_noise, _kat_learners, _learner_store

pytestmark = pytest.mark.gpu

SPECS = [("dm", "dm_update_kat.npz", 0), ("dr", "dr_update_kat.npz", 0), ("dm", "dm_update_kat.npz", 2),
         ("dr", "dr_update_kat.npz", 1)]


def _engine(bk, modes, state0):
    from auctiongym_amd.engine import AuctionEngine
    N = len(bk)
    eng = AuctionEngine(N, min(2, N), 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), bk, np.ones(N), np.full(N, 0.02))
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    eng.set_bidder_modes(modes)
    eng.set_fit_noise_seed(5)
    return eng


def _rp_run(engines, stores, mask, totals=None, bases=None, poll=64):
    """The record-parallel loop over `engines` (ranks) in ONE process: after each epoch launch
    the ranks' int64 totals are summed (what sharding.bidder_update_record_parallel's
    all-reduce does across processes)."""
    import torch
    tots = [eng.bidder_rp_begin(st, agents=mask, records_total=totals,
                                records_base=None if bases is None else bases[r])
            for r, (eng, st) in enumerate(zip(engines, stores))]
    sel = mask.astype(bool)
    while True:
        for _ in range(poll):
            ks = [eng.bidder_rp_epoch(1) for eng in engines]
            if len(engines) > 1:
                s = sum(t[k & 1] for t, k in zip(tots, ks))
                for t, k in zip(tots, ks):
                    t[k & 1].copy_(s)
        torch.cuda.synchronize()
        fits = [eng.bidder_rp_poll()[0] for eng in engines]
        for f in fits[1:]:
            assert np.array_equal(f, fits[0])
        if (fits[0][sel] < 0).all():
            break
    return [eng.bidder_rp_end() for eng in engines]


def test_rp_update_equals_persistent_trainer(gpu):
    """One process: the per-epoch-launch update (synthetic rsample draws) gives the persistent
    trainer's epochs, status and models bit for bit, for ValueLearningBidder 'policy' and
    DoublyRobustBidder agents trained together."""
    bk, modes, state0, recs, _ = _kat_learners(SPECS)
    N = len(SPECS)
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    ep, stat = eng.bidder_update(st, None, np.zeros(N, np.int64), 0)
    state, init = eng.dr_state()
    assert (stat == 0).all() and (ep[:, 2] > 0).all()
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    (ep2, stat2), = _rp_run([eng], [st], np.ones(N, np.int32))
    state2, init2 = eng.dr_state()
    assert np.array_equal(ep2, ep) and np.array_equal(stat2, stat)
    assert np.array_equal(state2, state) and np.array_equal(init2, init)
    eng.close()


@pytest.mark.parametrize("shards", [2, 3])
def test_rp_sharded_records_equal_one_process(gpu, shards):
    """`shards` ranks (engines on the one GPU, each holding a contiguous part of every agent's
    records in log order) whose per-epoch totals are summed: every rank ends with the model the
    persistent trainer fits on all the records in one process -- the record-parallel multi-GPU
    update (sharding.bidder_update_record_parallel) without the processes. A rank may hold no
    record of an agent."""
    bk, modes, state0, recs, _ = _kat_learners(SPECS)
    N = len(SPECS)
    ref = _engine(bk, modes, state0)
    ep, stat = ref.bidder_update(_learner_store(ref, recs), None, np.zeros(N, np.int64), 0)
    state, init = ref.dr_state()
    ref.close()
    # split every agent's records (log order) into `shards` contiguous parts; the last rank gets
    # none of agent 0's
    engines, stores, counts = [], [], np.zeros((shards, N), np.int64)
    for r in range(shards):
        part = {f: [] for f in recs}
        for a in range(N):
            n = len(recs["agent"][a])
            cut = [0] + [n * (j + 1) // shards for j in range(shards)]
            if a == 0:
                cut = [0] + [n * (j + 1) // (shards - 1) for j in range(shards - 1)] + [n]
            lo, hi = cut[r], cut[r + 1]
            for f in recs:
                part[f].append(recs[f][a][lo:hi])
            counts[r, a] = hi - lo
        eng = _engine(bk, modes, state0)
        engines.append(eng)
        stores.append(_learner_store(eng, part))
    assert counts[-1, 0] == 0
    res = _rp_run(engines, stores, np.ones(N, np.int32), totals=counts.sum(0),
                  bases=[counts[:r].sum(0) for r in range(shards)])
    for r, eng in enumerate(engines):
        s2, i2 = eng.dr_state()
        assert np.array_equal(res[r][0], ep) and np.array_equal(res[r][1], stat), r
        assert np.array_equal(s2, state) and np.array_equal(i2, init), r
        eng.close()


def test_rp_host_noise_windows_equal_one_shot(gpu, oracle):
    """A policy fit fed its rsample noise window by window (ag_bidder_rp_noise: it waits at a
    window's end with its state kept) equals the persistent trainer given all the epochs' noise
    at once, and the oracle -- the drop-in update's single pass (no fit is re-run)."""
    import torch
    specs = [("dr", "dr_update_kat.npz", 0)]
    bk, modes, state0, recs, data = _kat_learners(specs)
    k = data[0]
    n = len(k("est_ctr"))
    E = 6000
    z = _dr_noise(k("dr_rng_state"), n, E)
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    ep, stat = eng.bidder_update(st, torch.from_numpy(z.ravel()).to(eng.device), np.zeros(1, np.int64), E)
    state, _ = eng.dr_state()
    assert stat[0] == 0 and ep[0, 2] < E
    r = oracle.dr_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("won"), k("util"),
                         state0[0, :4], state0[0, 4:], False, z)
    assert list(ep[0]) == list(r["epochs"]) and np.array_equal(state[0, 4:], r["pol"])
    eng.set_dr_state(state0, np.zeros(1, np.int32))
    eng.bidder_rp_begin(st, agents=np.ones(1, np.int32))
    W, w0, waits = 333, 0, 0
    eng.bidder_rp_noise(torch.from_numpy(z[:W].ravel()).to(eng.device), n, 0, W)
    while True:
        eng.bidder_rp_epoch(200)
        fit, epoch, need = eng.bidder_rp_poll()
        if fit[0] < 0:
            break
        if need[0] >= 0:
            assert need[0] == w0 + W and fit[0] == 4
            w0 = int(need[0])
            waits += 1
            eng.bidder_rp_noise(torch.from_numpy(z[w0:w0 + W].ravel()).to(eng.device), n, w0, W)
    ep2, stat2 = eng.bidder_rp_end()
    state2, _ = eng.dr_state()
    assert waits >= ep[0, 2] // W - 1
    assert np.array_equal(ep2, ep) and np.array_equal(stat2, stat) and np.array_equal(state2, state)
    eng.close()


def test_rp_fallback_and_errors(gpu):
    """A ValueLearningBidder without a won record falls back (status 1, nothing trained, bids
    stay Gaussian) as in ag_bidder_update; a PolicyLearningBidder is refused (float sums in a
    fixed order cannot be split over ranks); ending while an agent still trains is an error."""
    from auctiongym_amd import _lib
    bk, modes, state0, recs, _ = _kat_learners([("dm", "dm_update_kat.npz", 1), ("dm", "dm_update_kat.npz", 2)])
    recs["won"][0] = np.zeros_like(recs["won"][0])
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    (ep, stat), = _rp_run([eng], [st], np.ones(2, np.int32))
    state, init = eng.dr_state()
    assert stat[0] == 1 and list(ep[0]) == [0, 0, 0] and init[0] == _lib.LEARNER_UNINITIALISED
    assert np.array_equal(state[0], state0[0]) and stat[1] == 0 and init[1] == _lib.LEARNER_POLICY
    eng.bidder_rp_begin(st, agents=np.ones(2, np.int32))
    eng.bidder_rp_epoch(3)
    with pytest.raises(_lib.AgError, match="still training"):
        eng.bidder_rp_end()
    eng.close()
    bk3, modes3, s3, recs3, _ = _kat_learners([("ips", "ips_update_kat.npz", 0)])
    eng = _engine(bk3, modes3, s3)
    with pytest.raises(NotImplementedError, match="PolicyLearningBidder"):
        eng.bidder_rp_begin(_learner_store(eng, recs3), agents=np.ones(1, np.int32))
    eng.close()


# ---- LR-TS allocators (ag_lrts_rp_*: src/BidderAllocation.py:29-65) ----
def _lrts_setup(shards):
    """The SP_Truthful_TS KAT population (6 LR-TS agents, the reference's own update samples):
    a reference engine, and `shards` engines each holding a slice of every agent's samples."""
    from test_gpu_parity import _fill_store, _kat_population, _lrts_engine
    kat, m0, q0, pm0 = _kat_population()
    per = {a: (kat[f"a{a}_X"], kat[f"a{a}_A"], kat[f"a{a}_y"]) for a in range(6)}

    def engine():
        eng = _lrts_engine()
        eng.load_lrts(m0, q0, pm0)
        return eng
    ref = engine()
    ref_st = _fill_store(ref, per)
    parts = []
    for r in range(shards):
        sub = {}
        for a, (X, A, y) in per.items():
            n = len(y)
            lo, hi = n * r // shards, n * (r + 1) // shards
            if shards > 1 and a == 1 and r == shards - 1:  # this rank holds none of agent 1's samples
                lo = hi
            if shards > 1 and a == 1 and r == shards - 2:
                hi = n
            sub[a] = (X[lo:hi], A[lo:hi], y[lo:hi])
        eng = engine()
        parts.append((eng, _fill_store(eng, sub, seed=r + 1)))
    return ref, ref_st, parts


@pytest.mark.parametrize("shards", [1, 2, 3])
def test_lrts_rp_equals_persistent_trainer(gpu, shards):
    """The per-epoch-launch LR-TS update over `shards` ranks (engines on the one GPU whose
    per-epoch totals are summed, as the multi-GPU all-reduce does; shards = 1: one process)
    ends, on every rank, with the persistent trainer's m, q, prev_m and epochs bit for bit."""
    import torch
    ref, ref_st, parts = _lrts_setup(shards)
    ep = ref.lrts_update(ref_st)
    want = ref.lrts_state()
    ref.close()
    counts = np.zeros(6, np.int64)
    for eng, st in parts:
        key = st["key"][:int(st["count"][0])].cpu().numpy().view(np.uint32)
        counts += np.bincount(key >> 16, minlength=6)[:6]
    tots = [eng.lrts_rp_begin(st, samples_total=counts) for eng, st in parts]
    while True:
        for _ in range(64):
            ks = [eng.lrts_rp_epoch(1) for eng, _ in parts]
            if shards > 1:
                s = sum(t[k & 1] for t, k in zip(tots, ks))
                for t, k in zip(tots, ks):
                    t[k & 1].copy_(s)
        torch.cuda.synchronize()
        left = [eng.lrts_rp_poll() for eng, _ in parts]
        assert len(set(left)) == 1
        if left[0] == 0:
            break
    for eng, _ in parts:
        assert np.array_equal(eng.lrts_rp_end(), ep)
        for x, y in zip(eng.lrts_state(), want):
            assert np.array_equal(x, y)
        eng.close()


@pytest.mark.parametrize("agent,first", [(2, 3), (4, 37)])
def test_lrts_rp_odd_polls_one_agent_mask(gpu, agent, first):
    """One agent in the mask, polled after an odd number of launches (`first`, then 37 at a
    time): ag_lrts_rp_poll reads the state of the launch parity it is at (k_lrts_rp_init writes
    both parities, so a poll before the first even launch sees a started fit), the update
    terminates, and the agent ends with the persistent trainer's m, q, prev_m and epochs bit for
    bit; the agents outside the mask are left as they were."""
    ref, ref_st, parts = _lrts_setup(1)
    ep = ref.lrts_update(ref_st)
    want = ref.lrts_state()
    ref.close()
    (eng, st), = parts
    before = eng.lrts_state()
    mask = np.zeros(6, np.int32)
    mask[agent] = 1
    eng.lrts_rp_begin(st, agents=mask)
    launches, polls = 0, 0
    n = first
    while True:
        eng.lrts_rp_epoch(n)
        launches += n
        polls += 1
        left = eng.lrts_rp_poll()
        assert left in (0, 1)
        if left == 0:
            break
        assert launches < 20000, "the masked fit never finished"
        n = 37
    assert polls >= 2  # polled at odd launch counts (first, first + 74, ...) while the fit ran
    ep2 = eng.lrts_rp_end()
    assert ep2[agent] == ep[agent]
    got = eng.lrts_state()
    for x, y, b in zip(got, want, before):
        assert np.array_equal(x[agent], y[agent])
        others = np.arange(6) != agent
        assert np.array_equal(x[others], b[others])
    eng.close()


def test_rp_graph_block_equals_eager(gpu):
    """sharding.rp_epoch_blocks with graph=True (each block of launches + exchanges captured once
    in a hipGraph and replayed) against the eager loop and the launches issued from C, with a
    same-size device copy standing in for the all-reduce (one process): the same epochs and
    the same posteriors, bit for bit (LR-TS), and the same models (learning bidders)."""
    import torch
    from auctiongym_amd.sharding import bidder_update_record_parallel, lrts_update_record_parallel
    runs = []
    for mode in ("c", "eager", "graph"):
        ref, ref_st, parts = _lrts_setup(1)
        ref.close()
        (eng, st), = parts
        if mode == "c":
            ep = lrts_update_record_parallel(eng, st, range(6))
        else:
            ep = lrts_update_record_parallel(eng, st, range(6), poll=16, exchange=lambda t: t.copy_(t.clone()),
                                             graph=(mode == "graph"))
        torch.cuda.synchronize()
        runs.append((ep,) + tuple(eng.lrts_state()))
        eng.close()
    for r in runs[1:]:
        for x, y in zip(r, runs[0]):
            assert np.array_equal(x, y)
    bk, modes, state0, recs, _ = _kat_learners(SPECS)
    res = []
    for mode in ("eager", "graph"):
        eng = _engine(bk, modes, state0)
        st = _learner_store(eng, recs)
        ep, stat = bidder_update_record_parallel(eng, st, range(len(SPECS)), poll=16,
                                                 exchange=lambda t: t.copy_(t.clone()), graph=(mode == "graph"))
        res.append((ep, stat) + tuple(eng.dr_state()))
        eng.close()
    for x, y in zip(*res):
        assert np.array_equal(x, y)


# ---- the pipelined persistent launches (k_bidder_pipe: ag_bidder_update's exact-sum
# learners, ag_bidder_rp_run) ----
def _trained(eng):
    state, init = eng.dr_state()
    return state, init


@pytest.mark.parametrize("host_noise", [False, True], ids=["synthetic", "host_noise"])
def test_pipe_equals_persistent_trainer(gpu, monkeypatch, host_noise):
    """ag_bidder_update's pipelined launches (AG_BIDDER_PIPE=1: every ValueLearning /
    DoublyRobust learner in the same persistent launches, each one's per-epoch sum overlapped
    with the others' epochs) against k_bidder_train (the default): epochs, status and models bit for bit -- DM and
    DR learners (DR imitating on its first update) trained together, a PPO PolicyLearningBidder
    beside them (k_bidder_train either way). host_noise: the caller's draws with 600 policy
    epochs, too few for some fits (status -3, model not applied, in both)."""
    import torch
    specs = SPECS + [("ips", "ips_update_kat.npz", 0)]
    bk, modes, state0, recs, _ = _kat_learners(specs)
    N = len(specs)
    E = 600 if host_noise else 0
    ns = [len(r) for r in recs["agent"]]
    noff = np.concatenate([[0], np.cumsum([n * E for n in ns])[:-1]]).astype(np.int64)
    z = np.random.default_rng(3).standard_normal(sum(ns) * E).astype(np.float32) if host_noise else None
    runs = []
    for pipe in ("0", "1"):
        monkeypatch.setenv("AG_BIDDER_PIPE", pipe)
        eng = _engine(bk, modes, state0)
        st = _learner_store(eng, recs)
        noise = torch.from_numpy(z).to(eng.device) if host_noise else None
        ep, stat = eng.bidder_update(st, noise, noff, E)
        runs.append((ep, stat) + _trained(eng))
        eng.close()
    ep, stat = runs[0][:2]
    assert (ep[:4, 0] > 0).all()
    assert np.isin(stat, [0, -3] if host_noise else [0]).all()
    for x, y in zip(*runs):
        assert np.array_equal(x, y)


def test_rp_run_windows_equal_one_shot(gpu, oracle):
    """ag_bidder_rp_run fed the rsample noise window by window (it stops at a window's end, the
    state kept) equals the persistent trainer given every epoch's draws at once, and the
    oracle: the drop-in update's path (Auction._fit_with_torch_noise)."""
    import torch
    specs = [("dr", "dr_update_kat.npz", 0)]
    bk, modes, state0, recs, data = _kat_learners(specs)
    k = data[0]
    n = len(k("est_ctr"))
    E = 6000
    z = _dr_noise(k("dr_rng_state"), n, E)
    r = oracle.dr_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("won"), k("util"),
                         state0[0, :4], state0[0, 4:], False, z)
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    eng.bidder_rp_begin(st, agents=np.ones(1, np.int32))
    W, w0, waits = 333, 0, 0
    eng.bidder_rp_noise(torch.from_numpy(z[:W].ravel()).to(eng.device), n, 0, W)
    while True:
        eng.bidder_rp_run()
        fit, epoch, need = eng.bidder_rp_poll()
        if fit[0] < 0:
            break
        assert need[0] == w0 + W and fit[0] == 4
        w0 = int(need[0])
        waits += 1
        eng.bidder_rp_noise(torch.from_numpy(z[w0:w0 + W].ravel()).to(eng.device), n, w0, W)
    ep, stat = eng.bidder_rp_end()
    state, _ = eng.dr_state()
    assert stat[0] == 0 and waits >= ep[0, 2] // W - 1
    assert list(ep[0]) == list(r["epochs"]) and np.array_equal(state[0, 4:], r["pol"])
    eng.close()


def test_rp_run_after_epoch_launches(gpu, monkeypatch):
    """Per-epoch launches (ag_bidder_rp_epoch, their last totals pending) then ag_bidder_rp_run
    to the end: the persistent trainer's epochs, status and models bit for bit."""
    bk, modes, state0, recs, _ = _kat_learners(SPECS)
    N = len(SPECS)
    monkeypatch.setenv("AG_BIDDER_PIPE", "0")
    ref = _engine(bk, modes, state0)
    ep, stat = ref.bidder_update(_learner_store(ref, recs), None, np.zeros(N, np.int64), 0)
    want = (ep, stat) + _trained(ref)
    ref.close()
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    eng.bidder_rp_begin(st, agents=np.ones(N, np.int32))
    eng.bidder_rp_epoch(37)
    eng.bidder_rp_run()
    fit, _, _ = eng.bidder_rp_poll()
    assert (fit < 0).all()
    got = eng.bidder_rp_end() + _trained(eng)
    for x, y in zip(got, want):
        assert np.array_equal(x, y)
    eng.close()


def test_rp_run_refuses_a_shard(gpu):
    """A rank holding part of the records steps per epoch with the other ranks: rp_run refuses."""
    bk, modes, state0, recs, _ = _kat_learners(SPECS[:1])
    eng = _engine(bk, modes, state0)
    st = _learner_store(eng, recs)
    n = len(recs["agent"][0])
    eng.bidder_rp_begin(st, agents=np.ones(1, np.int32), records_total=np.array([2 * n]),
                        records_base=np.array([0]))
    with pytest.raises(NotImplementedError, match="ag_bidder_rp_epoch"):
        eng.bidder_rp_run()
    eng.close()
