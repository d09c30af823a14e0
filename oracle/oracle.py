"""ctypes binding of the CPU restatement (oracle/ag_oracle.c) -- TEST INFRASTRUCTURE ONLY.

The oracle is the checker: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module. The product path (auction-gym_amd/) never does.

Arrays follow the fixtures' row-major layout: per-round [B], per-(round, slot) [B][P].
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# AG_ORACLE_LIB selects another build of the checker, e.g. the sanitizer build
# (make -C oracle sanitize; tools/sanitize_oracle.sh runs the oracle tests under it)
_SO = os.environ.get("AG_ORACLE_LIB") or os.path.join(_HERE, "libag_oracle.so")

FIRST_PRICE, SECOND_PRICE = 0, 1
COUNTERS = ("net", "gross", "allocation_regret", "estimation_regret", "overbid_regret",
            "underbid_regret", "ctr_sqerr", "ctr_bias_sum", "best_ev_sum", "n_logs", "n_won",
            "paid")
NUM_COUNTERS = len(COUNTERS)

_lib = None


class _Shape(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("P", ctypes.c_int32), ("K", ctypes.c_int32),
                ("E", ctypes.c_int32), ("mech", ctypes.c_int32)]


class _Pop(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("P", ctypes.c_int32), ("K", ctypes.c_int32),
                ("E", ctypes.c_int32), ("OE", ctypes.c_int32), ("mech", ctypes.c_int32),
                ("alloc_kind", ctypes.c_void_p), ("bid_kind", ctypes.c_void_p),
                ("prev_gamma", ctypes.c_void_p), ("gamma_sigma", ctypes.c_void_p),
                ("ts_m", ctypes.c_void_p), ("ts_sample", ctypes.c_int32),
                ("dr_state", ctypes.c_void_p), ("dr_init", ctypes.c_void_p), ("num_items", ctypes.c_void_p)]


class _In(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("ctx", "part", "u", "gamma_raw", "ts_noise", "policy_eps",
                                              "gamma_grid")]


class _Out(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("winner", "price", "second_price", "outcome",
                                              "item", "value", "bid", "est_ctr", "true_ctr",
                                              "best_ev", "gamma", "propensity")]


def build():
    if not os.environ.get("AG_ORACLE_LIB"):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        d, i32, i64, u64 = ctypes.c_double, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
        vp = ctypes.c_void_p
        L.ora_set_reduce.restype = None
        L.ora_set_reduce.argtypes = [ctypes.c_void_p, i64]
        L.ora_sigmoid.restype = d
        L.ora_sigmoid.argtypes = [d]
        L.ora_dot.restype = d
        L.ora_dot.argtypes = [vp, vp, i32]
        L.ora_bernoulli.restype = i32
        L.ora_bernoulli.argtypes = [d, d]
        L.ora_allocate.restype = None
        L.ora_allocate.argtypes = [i32, vp, i64, i32, vp, vp, vp]
        L.ora_simulate.restype = None
        L.ora_simulate.argtypes = [ctypes.POINTER(_Shape), vp, vp, i64, vp, vp, vp] + [vp] * 12 + [i32]
        L.ora_simulate_pop.restype = None
        L.ora_simulate_pop.argtypes = [ctypes.POINTER(_Pop), vp, vp, i64, ctypes.POINTER(_In),
                                       ctypes.POINTER(_Out), vp, vp, i32]
        L.ora_ts_ctr.restype = ctypes.c_float
        L.ora_ts_ctr.argtypes = [vp, vp, i32, i32, i32]
        L.ora_ts_logit.restype = ctypes.c_float
        L.ora_ts_logit.argtypes = [vp, vp, i32, i32, i32]
        L.ora_ts_sigmoid.restype = ctypes.c_float
        L.ora_ts_sigmoid.argtypes = [ctypes.c_float, i32, i32]
        L.ora_to_fx.restype = i64
        L.ora_to_fx.argtypes = [d]
        L.ora_gen_uniform.restype = d
        L.ora_gen_uniform.argtypes = [u64, u64]
        L.ora_gen_participants.restype = None
        L.ora_gen_participants.argtypes = [u64, u64, i32, i32, vp]
        L.ora_philox4x32_10.restype = None
        L.ora_philox4x32_10.argtypes = [vp, vp, vp]
        L.ora_lrts_loss_grad.restype = ctypes.c_float
        L.ora_lrts_loss_grad.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp, vp, vp]
        L.ora_empirical_update.restype = i32
        L.ora_empirical_update.argtypes = [i64, vp, vp, vp]
        L.ora_dr_update.restype = i32
        L.ora_dr_update.argtypes = [i64] + [vp] * 8 + [i32, vp, i64] + [vp] * 5
        L.ora_vl_update.restype = i32
        L.ora_vl_update.argtypes = [i64] + [vp] * 6 + [i32, vp, i64] + [vp] * 3
        L.ora_pl_update.restype = i32
        L.ora_pl_update.argtypes = [i64] + [vp] * 6 + [i32, i32, i32] + [vp] * 3
        L.ora_fit_noise.restype = None
        L.ora_fit_noise.argtypes = [u64, ctypes.c_uint32, i32, i64, vp]
        L.ora_pl_loss_grad.restype = ctypes.c_float
        L.ora_pl_loss_grad.argtypes = [i64] + [vp] * 6 + [i32, vp]
        L.ora_search_gamma.restype = d
        L.ora_search_gamma.argtypes = [vp, d, d, vp, i64]
        L.ora_log1p_restated.restype = d
        L.ora_log1p_restated.argtypes = [d]
        L.ora_torch_sigmoidf.restype = ctypes.c_float
        L.ora_torch_sigmoidf.argtypes = [ctypes.c_float]
        L.ora_lrts_update.restype = i32
        L.ora_lrts_update.argtypes = [i64, i32, i32, vp, vp, vp, vp, vp, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def sigmoid(z):
    L = lib()
    return np.array([L.ora_sigmoid(float(v)) for v in np.ravel(z)]).reshape(np.shape(z))


def allocate(mech, bids):
    bids = np.ascontiguousarray(bids, np.float64)
    B, P = bids.shape
    w = np.empty(B, np.int32)
    pr = np.empty(B)
    sp = np.empty(B)
    lib().ora_allocate(int(mech), _p(bids), B, P, _p(w), _p(pr), _p(sp))
    return w, pr, sp


def simulate(mech, items, values, ctx, part, u, nthreads=1):
    """Replay B rounds of Oracle+Truthful agents; returns dict of outputs + counters [N][C]."""
    items = np.ascontiguousarray(items, np.float64)
    values = np.ascontiguousarray(values, np.float64)
    ctx = np.ascontiguousarray(ctx, np.float64)
    part = np.ascontiguousarray(part, np.int32)
    u = np.ascontiguousarray(u, np.float64)
    N, K, D = items.shape
    B, P = part.shape
    E = ctx.shape[1]
    assert D == E + 1 and values.shape == (N, K) and u.shape == (B,)
    sh = _Shape(N, P, K, E, int(mech))
    out = dict(winner=np.empty(B, np.int32), price=np.empty(B), second_price=np.empty(B),
               outcome=np.empty(B, np.uint8), item=np.empty((B, P), np.int32),
               value=np.empty((B, P)), bid=np.empty((B, P)), est_ctr=np.empty((B, P)),
               true_ctr=np.empty((B, P)), best_ev=np.empty((B, P)),
               counters=np.zeros((N, NUM_COUNTERS)),
               counters_fx=np.zeros((N, NUM_COUNTERS, 3), np.int64))
    lib().ora_simulate(ctypes.byref(sh), _p(items), _p(values), B, _p(ctx), _p(part), _p(u),
                       _p(out["winner"]), _p(out["price"]), _p(out["second_price"]),
                       _p(out["outcome"]), _p(out["item"]), _p(out["value"]), _p(out["bid"]),
                       _p(out["est_ctr"]), _p(out["true_ctr"]), _p(out["best_ev"]),
                       _p(out["counters"]), _p(out["counters_fx"]), int(nthreads))
    return out


def simulate_pop(mech, items, values, ctx, part, u, alloc_kind, bid_kind, prev_gamma=None,
                 gamma_sigma=None, OE=None, ts_m=None, ts_noise=None, gamma_raw=None,
                 ts_sample=True, dr_state=None, dr_init=None, policy_eps=None, gamma_grid=None, nthreads=1,
                 num_items=None):
    """General population (OracleAllocator / LR-TS allocators; truthful / shading bidders in
    their first iteration). Row-major replay inputs; returns outputs + counters. num_items [N]:
    each agent's own item count (catalogues padded to K with value-0 rows), None: all K."""
    items = np.ascontiguousarray(items, np.float64)
    values = np.ascontiguousarray(values, np.float64)
    ctx = np.ascontiguousarray(ctx, np.float64)
    part = np.ascontiguousarray(part, np.int32)
    u = np.ascontiguousarray(u, np.float64)
    N, K, D = items.shape
    B, P = part.shape
    E = ctx.shape[1]
    OE = E if OE is None else OE
    keep = []

    def arr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dt)
        keep.append(a)
        return a

    ak, bk = arr(alloc_kind, np.int32), arr(bid_kind, np.int32)
    pg = arr(prev_gamma if prev_gamma is not None else np.ones(N), np.float64)
    gs = arr(gamma_sigma if gamma_sigma is not None else np.ones(N), np.float64)
    tm = arr(ts_m if ts_m is not None else np.zeros((N, K, OE + 1)), np.float32)
    gr = arr(gamma_raw if gamma_raw is not None else np.full((B, P), np.nan), np.float64)
    tn = arr(ts_noise if ts_noise is not None else np.zeros((B, P, K, OE + 1)), np.float32)
    ds = arr(dr_state if dr_state is not None else np.zeros((N, 16)), np.float32)
    di = arr(dr_init if dr_init is not None else np.zeros(N), np.int32)
    pe = arr(policy_eps if policy_eps is not None else np.zeros((B, P)), np.float32)
    gg = arr(gamma_grid if gamma_grid is not None else np.zeros((1, 1, 128)), np.float64)
    ni = arr(num_items, np.int32)
    pop = _Pop(N, P, K, E, OE, int(mech), ak.ctypes.data, bk.ctypes.data, pg.ctypes.data,
               gs.ctypes.data, tm.ctypes.data, int(bool(ts_sample)), ds.ctypes.data, di.ctypes.data,
               None if ni is None else ni.ctypes.data)
    out = dict(winner=np.empty(B, np.int32), price=np.empty(B), second_price=np.empty(B),
               outcome=np.empty(B, np.uint8), item=np.empty((B, P), np.int32),
               value=np.empty((B, P)), bid=np.empty((B, P)), est_ctr=np.empty((B, P)),
               true_ctr=np.empty((B, P)), best_ev=np.empty((B, P)), gamma=np.empty((B, P)),
               propensity=np.empty((B, P)), counters=np.zeros((N, NUM_COUNTERS)),
               counters_fx=np.zeros((N, NUM_COUNTERS, 3), np.int64))
    cin = _In(ctx.ctypes.data, part.ctypes.data, u.ctypes.data, gr.ctypes.data, tn.ctypes.data,
              pe.ctypes.data, gg.ctypes.data)
    cout = _Out(*[out[k].ctypes.data for k in ("winner", "price", "second_price", "outcome", "item",
                                               "value", "bid", "est_ctr", "true_ctr", "best_ev",
                                               "gamma", "propensity")])
    lib().ora_simulate_pop(ctypes.byref(pop), _p(items), _p(values), B, ctypes.byref(cin),
                           ctypes.byref(cout), _p(out["counters"]), _p(out["counters_fx"]),
                           int(nthreads))
    return out


def fx_limbs_to_int(limbs):
    """[..., 3] normalised limbs -> Python ints (exact), units of 2^-36."""
    limbs = np.asarray(limbs)
    flat = limbs.reshape(-1, 3)
    vals = [int(a) + (int(b) << 42) + (int(c) << 84) for a, b, c in flat]
    return np.array(vals, dtype=object).reshape(limbs.shape[:-1])


def gen_uniform(seed, idx):
    return lib().ora_gen_uniform(seed, idx)


def gen_participants(seed, idx, N, P):
    out = np.empty(P, np.int32)
    lib().ora_gen_participants(seed, idx, N, P, _p(out))
    return out


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    o = np.empty(4, np.uint32)
    lib().ora_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def lrts_update(X, A, y, m, prev_m, q, trace=True):
    """PyTorchLogisticRegressionAllocator.update (src/BidderAllocation.py:29-65) of one
    agent on its won samples X [n][Do], A [n], y [n]; returns (m, prev_m, q, epochs,
    losses) after the update (inputs are not modified)."""
    X = np.ascontiguousarray(X, np.float32)
    A = np.ascontiguousarray(A, np.int32)
    y = np.ascontiguousarray(np.asarray(y) != 0, np.uint8)
    m = np.array(m, np.float32, order="C")
    pm = np.array(prev_m, np.float32, order="C")
    q = np.array(q, np.float32, order="C")
    K, Do = m.shape
    tr = np.zeros(16384, np.float32)
    ep = lib().ora_lrts_update(len(y), K, Do, _p(X), _p(A), _p(y), _p(m), _p(pm), _p(q),
                               _p(tr) if trace else None)
    return m, pm, q, int(ep), tr[:ep].astype(np.float64)


def lrts_loss_grad(X, A, y, m, prev_m, q):
    """Loss and float32 gradient of one epoch of the LR-TS update at m."""
    X = np.ascontiguousarray(X, np.float32)
    A = np.ascontiguousarray(A, np.int32)
    y = np.ascontiguousarray(np.asarray(y) != 0, np.uint8)
    m = np.ascontiguousarray(m, np.float32)
    pm = np.ascontiguousarray(prev_m, np.float32)
    q = np.ascontiguousarray(q, np.float32)
    g = np.empty_like(m)
    loss = lib().ora_lrts_loss_grad(len(y), m.shape[0], m.shape[1], _p(X), _p(A), _p(y), _p(m),
                                    _p(pm), _p(q), _p(g))
    return float(loss), g


EMPIRICAL_ERRORS = {-1: "zero-size array to reduction operation minimum which has no identity",
                    -2: "attempt to get argmax of an empty sequence",
                    -3: "All-NaN slice encountered"}


def empirical_update(gammas, utilities):
    """EmpiricalShadedBidder.update (src/Bidder.py:60-147) -> new prev_gamma; raises
    ValueError where the reference does."""
    g = np.ascontiguousarray(gammas, np.float64)
    u = np.ascontiguousarray(utilities, np.float64)
    out = np.zeros(1)
    rc = lib().ora_empirical_update(len(g), _p(g), _p(u), _p(out))
    if rc:
        raise ValueError(EMPIRICAL_ERRORS[rc])
    return float(out[0])


def dr_update(ctr, value, gamma, prop, won, util, wr, pol, initialised, noise, trace=True, skip_winrate=False):
    """DoublyRobustBidder.update (src/Bidder.py:473-615) of one agent; noise [E][n] float32
    per-epoch rsample draws of the DR fit. skip_winrate: wr is an already fitted win-rate
    model (test hook: the later fits from the reference's own fitted model). Returns dict(wr,
    pol, epochs, wr_losses, init_losses, dr_losses, est_util)."""
    n = len(ctr)
    a = [np.ascontiguousarray(v, np.float64) for v in (ctr, value, gamma, prop)]
    w = np.ascontiguousarray(np.asarray(won) != 0, np.uint8)
    u = np.ascontiguousarray(util, np.float64)
    wr = np.array(wr, np.float32).ravel().copy()
    pol = np.array(pol, np.float32).ravel().copy()
    noise = np.ascontiguousarray(noise, np.float32)
    E = noise.shape[0] if noise.size else 0
    ep = np.zeros(3, np.int32)
    tr = [np.zeros(32768, np.float32), np.zeros(16384, np.float32), np.zeros(32768, np.float32)]
    eu = np.zeros(n)
    rc = lib().ora_dr_update(n, *[_p(v) for v in a], _p(w), _p(u), _p(wr), _p(pol),
                             int(bool(initialised)) | (2 if skip_winrate else 0),
                             _p(noise), E, _p(ep), *[(_p(t) if trace else None) for t in tr], _p(eu))
    if rc:
        raise ValueError("DoublyRobustBidder.update without logs")
    return {"wr": wr, "pol": pol, "epochs": ep.copy(), "wr_losses": tr[0][:ep[0]].astype(np.float64),
            "init_losses": tr[1][:ep[1]].astype(np.float64), "dr_losses": tr[2][:ep[2]].astype(np.float64),
            "est_util": eu}


PL_LOSSES = {"REINFORCE": 0, "REINFORCE_offpolicy": 1, "TRPO": 2, "PPO": 3}


def vl_update(ctr, value, gamma, won, wr, pol, policy, noise, trace=True):
    """ValueLearningBidder.update (src/Bidder.py:204-325) of one agent; noise [E][n] float32
    per-epoch rsample draws of the policy fit (policy=True). Returns dict(wr, pol, epochs,
    wr_losses, pol_losses, fallback)."""
    n = len(ctr)
    a = [np.ascontiguousarray(v, np.float64) for v in (ctr, value, gamma)]
    w = np.ascontiguousarray(np.asarray(won) != 0, np.uint8)
    wr = np.array(wr, np.float32).ravel().copy()
    pol = np.array(pol, np.float32).ravel().copy()
    noise = np.ascontiguousarray(noise if noise is not None else np.zeros((0, n)), np.float32)
    E = noise.shape[0] if noise.size else 0
    ep = np.zeros(3, np.int32)
    tr = [np.zeros(32768, np.float32), np.zeros(16384, np.float32)]
    rc = lib().ora_vl_update(n, *[_p(v) for v in a], _p(w), _p(wr), _p(pol), int(bool(policy)), _p(noise), E,
                             _p(ep), *[(_p(t) if trace else None) for t in tr])
    if rc < 0:
        raise ValueError("ValueLearningBidder.update without logs")
    return {"wr": wr, "pol": pol, "epochs": ep.copy(), "fallback": rc == 1,
            "wr_losses": tr[0][:ep[0]].astype(np.float64), "pol_losses": tr[1][:ep[2]].astype(np.float64)}


def pl_update(ctr, value, gamma, prop, util, pol, initialised, loss="PPO", trace=True, nblk=1):
    """PolicyLearningBidder.update (src/Bidder.py:364-431) of one agent, its policy-fit sums in
    the order of `nblk` device workgroups. Returns dict(pol, epochs, init_losses, pl_losses,
    nan)."""
    n = len(ctr)
    a = [np.ascontiguousarray(v, np.float64) for v in (ctr, value, gamma, prop, util)]
    pol = np.array(pol, np.float32).ravel().copy()
    ep = np.zeros(3, np.int32)
    tr = [np.zeros(16384, np.float32), np.zeros(16384, np.float32)]
    rc = lib().ora_pl_update(n, *[_p(v) for v in a], _p(pol), int(bool(initialised)), PL_LOSSES[loss], int(nblk),
                             _p(ep),
                             *[(_p(t) if trace else None) for t in tr])
    if rc == -1:
        raise ValueError("PolicyLearningBidder.update without logs")
    return {"pol": pol, "epochs": ep.copy(), "nan": rc == -2,
            "init_losses": tr[0][:ep[1]].astype(np.float64), "pl_losses": tr[1][:ep[2]].astype(np.float64)}


def pl_loss_grad(ctr, value, gamma, prop, util, pol, loss="PPO"):
    """One epoch of a PolicyLearningBidder loss (src/Models.py:174-199) at pol: (loss, grad[12])."""
    n = len(ctr)
    a = [np.ascontiguousarray(v, np.float64) for v in (ctr, value, gamma, prop, util)]
    pol = np.ascontiguousarray(pol, np.float32).ravel()
    g = np.zeros(12, np.float32)
    loss_v = lib().ora_pl_loss_grad(n, *[_p(v) for v in a], _p(pol), PL_LOSSES[loss], _p(g))
    return float(loss_v), g


def search_gamma(wr, ctr, value, grid):
    """ValueLearningBidder 'search' (src/Bidder.py:180-196) for one bid over grid [128]."""
    wr = np.ascontiguousarray(wr, np.float32)
    grid = np.ascontiguousarray(grid, np.float64)
    return float(lib().ora_search_gamma(_p(wr), float(ctr), float(value), _p(grid), 1))


REDUCE_FN = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32)
_reduce_cb = None


def set_reduce(fn, n_total=0):
    """Record-parallel fits (oracle/ag_oracle.h ora_set_reduce): fn(words) sums an int64 numpy
    array in place over the ranks (e.g. a torch.distributed all-reduce); the updates then run
    on this process's records with every exact per-epoch sum taken over all ranks, and means
    over n_total records. fn None: back to single-process fits."""
    global _reduce_cb
    if fn is None:
        _reduce_cb = None
        lib().ora_set_reduce(None, 0)
        return

    def cb(ptr, n):
        w = np.ctypeslib.as_array(ptr, shape=(n,))
        fn(w)
    _reduce_cb = REDUCE_FN(cb)
    lib().ora_set_reduce(ctypes.cast(_reduce_cb, ctypes.c_void_p), int(n_total))


def fit_noise(seed, agent, epochs, n):
    """The synthetic rsample noise of ag_bidder_update(noise=NULL): float32 [epochs][n]."""
    out = np.zeros((epochs, n), np.float32)
    lib().ora_fit_noise(int(seed), int(agent), int(epochs), int(n), _p(out))
    return out
