"""HIP path vs the oracle and the golden vectors (needs an MI355X; `-m gpu`).

Everything goes through the C-ABI (libauctiongym_hip.so) via auctiongym_amd.engine.
Bar: bit-exact for items, bids, CTRs, winners, prices, outcomes and the fixed-point
counters; 1e-9 relative for the float counters against the reference aggregates
(north star: 1e-5).
"""
import json
import os

import numpy as np
import pytest

from conftest import CAPTURES, GOLDEN, load_capture, mech_code

pytestmark = pytest.mark.gpu


def _engine(meta, gpu):
    from auctiongym_amd.engine import AuctionEngine
    return AuctionEngine(meta["N"], meta["P"], meta["K"], meta["E"], meta["OE"], mech_code(meta),
                         meta["var"])


def _run(eng, ctx, part, u):
    """ctx [B][E], part [B][P], u [B] host -> outputs as host arrays in [B]/[B][P] layout."""
    import torch
    d = eng.device
    inp = {"ctx": torch.from_numpy(np.ascontiguousarray(ctx.T)).to(d),
           "part": torch.from_numpy(np.ascontiguousarray(part.T.astype(np.int32))).to(d),
           "u": torch.from_numpy(np.ascontiguousarray(u)).to(d)}
    out = eng.alloc_outputs(len(u))
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev"):
        o[k] = np.ascontiguousarray(o[k].T)
    o["counters_fx"] = cnt.cpu().numpy()
    return o


def test_device_sigmoid_kat(gpu):
    import torch
    from auctiongym_amd.engine import device_exp
    kat = np.load(os.path.join(GOLDEN, "sigmoid_kat.npz"))
    z = torch.from_numpy(kat["z"]).to(gpu)
    assert np.array_equal(device_exp(z, sigmoid=True).cpu().numpy(), kat["sigmoid"])


def _libm_exp(x):
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    libm.exp.restype = ctypes.c_double
    libm.exp.argtypes = [ctypes.c_double]
    return np.array([libm.exp(float(v)) for v in x])


def test_device_exp_matches_glibc_exactly(gpu):
    import torch
    from auctiongym_amd.engine import device_exp
    g = np.random.default_rng(6)
    x = np.concatenate([g.uniform(-40, 40, 200000), g.uniform(-745.2, 709.8, 100000),
                        np.array([0.0, -0.0, 1e-300, -1e-310, 709.78, -708.4, -745.13, 0.5, -0.5])])
    y = device_exp(torch.from_numpy(x).to(gpu)).cpu().numpy()
    ref = _libm_exp(x)
    bad = np.flatnonzero(y.view(np.int64) != ref.view(np.int64))
    assert bad.size == 0, (x[bad[:5]], y[bad[:5]], ref[bad[:5]])


def test_allocate_kat(gpu, oracle):
    import torch
    from auctiongym_amd.engine import AuctionEngine
    kat = np.load(os.path.join(GOLDEN, "alloc_kat.npz"))
    for P in (1, 2, 3, 4, 8, 32, 64, 100):
        bids = kat[f"P{P}_bids"]
        for mech_name, mech in (("FirstPrice", 0), ("SecondPrice", 1)):
            eng = AuctionEngine(P, P, 1, 1, 0, mech)
            w, pr, sp = eng.allocate(torch.from_numpy(np.ascontiguousarray(bids.T)).to(gpu))
            w, pr, sp = w.cpu().numpy(), pr.cpu().numpy(), sp.cpu().numpy()
            ow, opr, osp = oracle.allocate(mech, bids)
            assert np.array_equal(w, ow), (P, mech_name)
            np.testing.assert_array_equal(pr, opr)
            np.testing.assert_array_equal(sp, osp)
            np.testing.assert_array_equal(pr, kat[f"{mech_name}_P{P}_price"])
            np.testing.assert_array_equal(sp, kat[f"{mech_name}_P{P}_second_price"])
            eng.close()


def test_allocate_ragged_and_large(gpu, oracle):
    import torch
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(3)
    for P, B in ((2, 1), (2, 255), (3, 70001), (8, 1 << 20), (33, 5000), (200, 777)):
        bids = g.random((B, P)) * (g.random((B, P)) < 0.7)
        for mech in (0, 1):
            eng = AuctionEngine(P, P, 1, 1, 0, mech)
            w, pr, sp = eng.allocate(torch.from_numpy(np.ascontiguousarray(bids.T)).to(gpu))
            ow, opr, osp = oracle.allocate(mech, bids)
            assert np.array_equal(w.cpu().numpy(), ow)
            np.testing.assert_array_equal(pr.cpu().numpy(), opr)
            np.testing.assert_array_equal(sp.cpu().numpy(), osp)
            eng.close()


# test_simulate_replay_matches_reference: tests/test_00_configs_gpu.py (first in the suite)


def test_generator_matches_oracle(gpu, oracle):
    from auctiongym_amd.engine import AuctionEngine
    eng = AuctionEngine(32, 8, 12, 5, 4, 1, 1.0)
    inp = eng.alloc_inputs(100003)
    eng.generate(1234, 5_000_000_000, inp)
    part = inp["part"].cpu().numpy()
    u = inp["u"].cpu().numpy()
    ctx = inp["ctx"].cpu().numpy()
    for i in list(range(0, 100003, 997)) + [100002]:
        idx = 5_000_000_000 + i
        assert u[i] == oracle.gen_uniform(1234, idx)
        assert np.array_equal(part[:, i], oracle.gen_participants(1234, idx, 32, 8))
    assert abs(ctx.mean()) < 0.01 and abs(ctx.std() - 1.0) < 0.01
    assert (np.sort(part, axis=0)[1:] != np.sort(part, axis=0)[:-1]).all()
    # the contexts' distribution (float32 Box-Muller from 32-bit uniforms, round 5): N(0, 1) by a
    # Kolmogorov-Smirnov test over 500k draws, and the tails' frequencies
    from scipy import stats
    z = ctx.ravel()
    assert stats.kstest(z, "norm").pvalue > 1e-4
    for t, p in ((2.0, 0.0455), (3.0, 0.0027), (4.0, 6.33e-5)):
        f = float(np.mean(np.abs(z) > t))
        assert abs(f - p) < 5 * np.sqrt(p / z.size) + 1e-6, (t, f, p)
    eng.close()


def test_full_size_synthetic_batch_bit_exact(gpu, oracle):
    """The bench workload shape (SP_Oracle: N=6, P=2, K=12, E=5) at 4M auctions, Philox
    inputs generated on the GPU, every output compared with the oracle on the same inputs."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    import auctiongym_amd.main as M
    with open(os.path.join(GOLDEN, "sp_oracle_full_run.json")) as f:
        cfg = json.load(f)["config"]
    B = 1 << 22
    g = np.random.default_rng(0)
    items = np.concatenate([g.normal(0, 1, (6, 12, 5)), -3.0 - g.random((6, 12, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (6, 12))
    eng = AuctionEngine(6, 2, 12, 5, 4, 1, cfg["embedding_var"])
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    eng.generate(0, 0, inp)
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    ctx = np.ascontiguousarray(inp["ctx"].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"].cpu().numpy().T)
    u = inp["u"].cpu().numpy()
    orc = oracle.simulate(1, items, values, ctx, part, u, nthreads=16)
    assert np.array_equal(out["winner"].cpu().numpy(), orc["winner"])
    assert np.array_equal(out["price"].cpu().numpy(), orc["price"])
    assert np.array_equal(out["bid"].cpu().numpy().T, orc["bid"])
    assert np.array_equal(out["item"].cpu().numpy().T, orc["item"])
    assert np.array_equal(out["best_ev"].cpu().numpy().T, orc["best_ev"])
    assert np.array_equal(out["outcome"].cpu().numpy(), orc["outcome"])
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    # the exact item scan, two auctions per lane, and a batch run as several launches
    # (odd-sized auction ranges) give the same bits
    # (the default is the dedicated Oracle kernel, k_oracle; the general kernel must agree)
    for exact, lanes, cap, generic in ((True, 1, 0, False), (False, 2, 0, False), (False, 1, 1000002, False),
                                       (False, 2, 777778, False), (False, 1, 0, True), (False, 1, 777777, True),
                                       (False, 1, 333333, False)):
        eng.set_item_search(exact)
        eng.set_lane_auctions(lanes)
        eng.set_launch_auctions(cap)
        eng.set_simulate_kernel(generic)
        out_x = eng.alloc_outputs(B)
        cnt_x = eng.new_counters()
        eng.simulate(inp, out_x, cnt_x)
        for k in out:
            assert torch.equal(out[k], out_x[k]), (k, exact, lanes, cap, generic)
        assert torch.equal(cnt, cnt_x)
    eng.set_item_search(False)
    eng.set_lane_auctions(1)
    eng.set_launch_auctions(0)
    eng.set_simulate_kernel(False)
    # the bench's output set (no second_price) and no counters: same arrays
    sub = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    out_s = eng.alloc_outputs(B, sub)
    eng.simulate(inp, out_s, None)
    for k in sub:
        assert torch.equal(out[k], out_s[k]), k
    # batch split invariance: two halves accumulate to the same exact counters
    cnt2 = eng.new_counters()
    for lo, hi in ((0, B // 3), (B // 3, B)):
        sub_in = {"ctx": inp["ctx"][:, lo:hi].contiguous(), "part": inp["part"][:, lo:hi].contiguous(),
                  "u": inp["u"][lo:hi].contiguous()}
        eng.simulate(sub_in, eng.alloc_outputs(hi - lo, ("winner",)), cnt2)
    assert torch.equal(cnt, cnt2)
    eng.close()


def test_driver_sp_oracle_matches_reference_full_run(gpu, tmp_path):
    """auctiongym_amd.main on SP_Oracle.json as shipped (3 x 20 x 10k rounds) vs the
    reference's per-iteration revenue / net / gross (SURVEY §4 known answers)."""
    import auctiongym_amd.main as M
    with open(os.path.join(GOLDEN, "sp_oracle_full_run.json")) as f:
        ref = json.load(f)
    cfg = dict(ref["config"], output_dir=str(tmp_path / "out"))
    p = tmp_path / "SP_Oracle.json"
    p.write_text(json.dumps(cfg))
    run2stats, run2rev = M.main([str(p), "--quiet"])
    rows = iter(ref["iterations"])
    total = 0.0
    for run in range(cfg["num_runs"]):
        stats = run2stats[run]
        names = list(stats["net_utility"].keys())
        for it in range(cfg["num_iter"]):
            row = next(rows)
            np.testing.assert_allclose(run2rev[run][it], row["revenue"], rtol=1e-12)
            np.testing.assert_allclose([stats["net_utility"][n][it] for n in names], row["net"], rtol=1e-11)
            np.testing.assert_allclose([stats["gross_utility"][n][it] for n in names], row["gross"],
                                       rtol=1e-11)
            np.testing.assert_allclose([stats["best_expected_value"][n][it] for n in names],
                                       row["mean_best_ev"], rtol=1e-11)
            assert all(stats["allocation_regret"][n][it] == 0.0 for n in names)
            total += run2rev[run][it]
    np.testing.assert_allclose(total, 247455.77552418958, rtol=1e-12)
    assert (tmp_path / "out").is_dir()


def test_notebook_call_pattern(gpu, tmp_path):
    """The reference notebooks' loop: simulate_opportunity() per round, then read
    net/gross/revenue, update, clear (src/*.ipynb cell 4)."""
    import auctiongym_amd.main as M
    d, meta, agg = load_capture("sp_oracle_r4096")
    with open(os.path.join(GOLDEN, "sp_oracle_full_run.json")) as f:
        cfg = json.load(f)["config"]
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for _ in range(4096):
        auction.simulate_opportunity()
    np.testing.assert_allclose([a.net_utility for a in agents], agg["net_utility"], rtol=1e-11)
    np.testing.assert_allclose(auction.revenue, agg["revenue"], rtol=1e-12)
    logs = agents[0].logs
    assert len(logs) == agg["n_logs"][0]
    for a in agents:
        a.update(iteration=0)
        a.clear_utility()
        a.clear_logs()
    auction.clear_revenue()
    assert auction.revenue == 0.0 and agents[0].net_utility == 0.0 and agents[0].logs == []


def test_errors_are_loud(gpu):
    from auctiongym_amd.engine import AuctionEngine
    with pytest.raises(ValueError):
        AuctionEngine(3, 4, 12, 5, 4, 1)  # P > N: rng.choice raises ValueError too
    eng = AuctionEngine(4, 2, 12, 5, 4, 1)
    inp = eng.alloc_inputs(8)
    with pytest.raises(RuntimeError):
        eng.simulate(inp, eng.alloc_outputs(8))  # catalogue not loaded
    with pytest.raises(NotImplementedError):
        eng.set_agent_kinds([7, 0, 0, 0], [0, 0, 0, 0])  # no such allocator kind
    with pytest.raises(ValueError):
        eng.set_agent_params([0] * 4, [1, 0, 0, 0])  # shading bidder without its parameters
    eng.set_agent_params([1, 0, 0, 0], [0] * 4)
    g = np.random.default_rng(1)
    eng.load_catalog(g.normal(size=(4, 12, 6)), g.random((4, 12)))
    with pytest.raises(RuntimeError):
        eng.simulate(eng.alloc_inputs(8), eng.alloc_outputs(8))  # LR-TS posterior not loaded
    eng.close()


def test_empty_batch(gpu):
    import torch
    from auctiongym_amd.engine import AuctionEngine
    eng = AuctionEngine(4, 2, 12, 5, 4, 0)
    g = np.random.default_rng(1)
    eng.load_catalog(g.normal(size=(4, 12, 6)), g.random((4, 12)))
    cnt = eng.new_counters()
    eng.simulate(eng.alloc_inputs(0), eng.alloc_outputs(0), cnt)
    assert int(cnt.abs().sum()) == 0
    w, p, s = eng.allocate(torch.empty((2, 0), dtype=torch.float64, device=gpu))
    assert w.numel() == 0
    eng.close()


def test_generate_mode_equals_hbm_inputs(gpu):
    """ag_simulate_generated (inputs drawn inside k_oracle) == ag_generate + ag_simulate, bit
    for bit: every output and the exact counters, for a batch run as several launches with a
    nonzero first auction index, P in {1, 2, 5}, both mechanisms."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(5)
    for N, P, mech, B, cap in ((6, 2, 1, 1 << 20, 0), (6, 2, 0, 300001, 65537), (9, 5, 0, 100000, 0),
                               (3, 1, 1, 50000, 7777)):
        items = np.concatenate([g.normal(0, 1, (N, 12, 5)), -3.0 - g.random((N, 12, 1))], axis=2)
        values = g.lognormal(0.1, 0.2, (N, 12))
        eng = AuctionEngine(N, P, 12, 5, 4, mech, 1.3)
        eng.load_catalog(items, values)
        eng.set_launch_auctions(cap)
        first = 123456789012
        inp = eng.alloc_inputs(B)
        eng.generate(42, first, inp)
        out, cnt = eng.alloc_outputs(B), eng.new_counters()
        eng.simulate(inp, out, cnt)
        out_g, cnt_g = eng.alloc_outputs(B), eng.new_counters()
        eng.simulate_generated(42, first, out_g, cnt_g)
        torch.cuda.synchronize()
        for k in out:
            assert torch.equal(out[k], out_g[k]) or (torch.isnan(out[k]).all() and torch.isnan(out_g[k]).all()), k
        assert torch.equal(cnt, cnt_g)
        eng.close()
    eng = AuctionEngine(4, 2, 12, 5, 4, 1)  # outside k_oracle's bounds: refused, loudly
    items = np.concatenate([g.normal(0, 1, (4, 12, 5)), -3.0 - g.random((4, 12, 1))], axis=2)
    eng.load_catalog(items, np.full((4, 12), 5000.0))
    with pytest.raises(NotImplementedError, match="ag_simulate_generated"):
        eng.simulate_generated(0, 0, eng.alloc_outputs(64))
    eng.close()


_GEN_POPS = {
    # name: (N, mechanism, allocator kinds, bidder kinds, fitted policies)
    "sp_truthful_ts": (8, 1, [1] * 8, [0] * 8, [0] * 8),                      # configs[1]
    "fp_dr_ts": (3, 0, [1] * 3, [4] * 3, [1] * 3),                            # configs[3], fitted
    "fp_dm_ts": (3, 0, [1] * 3, [2] * 3, [1] * 3),                            # configs[2], fitted
    # 32 agents: Oracle / LR-TS allocators x Truthful, EmpiricalShaded, uninitialised and fitted
    # learners (Gaussian shading draws, rsample draws)
    "mix": (32, 0, [i % 2 for i in range(32)], [(0, 1, 2, 4, 4, 3, 0, 2)[i % 8] for i in range(32)],
            [1 if i % 8 in (3, 5) else 0 for i in range(32)]),
}


@pytest.mark.parametrize("pop,P,B,cap", [("sp_truthful_ts", 2, (1 << 18) + 37, 0), ("sp_truthful_ts", 8, 70001, 0),
                                         ("fp_dr_ts", 2, (1 << 18) + 3, 65536), ("fp_dm_ts", 2, 50000, 0),
                                         ("mix", 2, (1 << 17) + 11, 0), ("mix", 8, 40000, 9000)])
def test_generate_mode_general_equals_hbm_inputs(gpu, pop, P, B, cap):
    """Generate mode for general populations (ag_simulate_generated ->
    k_simulate<..., GEN>): contexts, participants, uniforms, the LR-TS agents' Thompson noise
    (torch.normal(0, 1/sqrt(q)), src/Models.py:31), the fitted policies' rsample draws and the
    shading draws made inside the kernel equal ag_generate + ag_generate_noise + ag_simulate bit
    for bit -- every output and the exact counters -- for the TruthfulBidder build (P = 2 and the
    streamed P = 8), the full build in 256-, 1024- and (P = 8) 768-lane workgroups, ragged
    batches, several launches per batch, a nonzero first auction index."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N, mech, ak, bk, init = _GEN_POPS[pop]
    K, E, OE = 12, 5, 4
    ak, bk, init = (np.asarray(v, np.int32) for v in (ak, bk, init))
    g = np.random.default_rng(71 + P)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    eng = AuctionEngine(N, P, K, E, OE, mech, 1.0)
    eng.set_agent_params(ak, bk, 0.5 + 0.5 * g.random(N), 0.01 + 0.05 * g.random(N))
    eng.load_catalog(items, values)
    eng.load_lrts(g.normal(0, 1, (N, K, OE + 1)).astype(np.float32),
                  (0.5 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32), thompson_sampling=True)
    if (bk >= 2).any():
        eng.set_dr_state(g.normal(0, 0.7, (N, 16)).astype(np.float32), init)
    eng.set_launch_auctions(cap)
    first = 98765432109
    inp = eng.alloc_inputs(B)
    eng.generate(11, first, inp)
    eng.generate_noise(11, first, inp)
    out, cnt = eng.alloc_outputs(B), eng.new_counters()
    eng.simulate(inp, out, cnt)
    out_g, cnt_g = eng.alloc_outputs(B), eng.new_counters()
    eng.simulate_generated(11, first, out_g, cnt_g)
    torch.cuda.synchronize()
    for k in out:
        assert np.array_equal(out[k].cpu().numpy(), out_g[k].cpu().numpy(), equal_nan=True), k
    assert torch.equal(cnt, cnt_g)
    if pop == "mix":  # the generated draws are the stored ones: N(0, 1/q) noise, N(pg, sigma) shading
        assert np.isfinite(out_g["gamma"].cpu().numpy()[:, :1000][bk[inp["part"][:, :1000].cpu().numpy()] != 0]).all()
    eng.close()


def test_generate_mode_general_refusals(gpu):
    """Generate mode refuses, loudly, what it does not draw: ValueLearningBidder 'search' grids,
    and general populations outside the shipped shape (E = 5, OE = 4)."""
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(3)
    eng = AuctionEngine(3, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(3, np.int32), np.full(3, 2, np.int32), np.ones(3), np.full(3, 0.02))
    eng.load_catalog(np.concatenate([g.normal(0, 1, (3, 12, 5)), -3.0 - g.random((3, 12, 1))], axis=2),
                     g.lognormal(0.1, 0.2, (3, 12)))
    eng.load_lrts(g.normal(0, 1, (3, 12, 5)).astype(np.float32), np.ones((3, 12, 5), np.float32))
    eng.set_dr_state(g.normal(0, 0.7, (3, 16)).astype(np.float32), np.full(3, _lib.LEARNER_SEARCH, np.int32))
    eng.set_bidder_modes(np.full(3, _lib.VL_SEARCH, np.int32))
    with pytest.raises(NotImplementedError, match="search"):
        eng.simulate_generated(0, 0, eng.alloc_outputs(64))
    eng.close()
    eng = AuctionEngine(4, 2, 12, 3, 2, 0, 1.0)  # E = 3: no shipped-shape build
    eng.set_agent_params(np.ones(4, np.int32), np.zeros(4, np.int32))
    eng.load_catalog(np.concatenate([g.normal(0, 1, (4, 12, 3)), -3.0 - g.random((4, 12, 1))], axis=2),
                     g.lognormal(0.1, 0.2, (4, 12)))
    eng.load_lrts(g.normal(0, 1, (4, 12, 3)).astype(np.float32), np.ones((4, 12, 3), np.float32))
    with pytest.raises(NotImplementedError, match="shipped shape"):
        eng.simulate_generated(0, 0, eng.alloc_outputs(64))
    eng.close()


def test_stale_binding_is_refused(gpu):
    """A caller compiled against another layout of the ABI structs (here the 3-field
    ag_batch_in of ABI 14) is refused with AG_ERR_INVALID before any field is used."""
    import ctypes
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    eng = AuctionEngine(6, 2, 12, 5, 4, 1)
    g = np.random.default_rng(0)
    eng.load_catalog(np.concatenate([g.normal(0, 1, (6, 12, 5)), -3.0 - g.random((6, 12, 1))], axis=2),
                     g.lognormal(0.1, 0.2, (6, 12)))

    class OldIn(ctypes.Structure):
        _fields_ = [("ctx", ctypes.c_void_p), ("part", ctypes.c_void_p), ("u", ctypes.c_void_p)]
    inp = eng.alloc_inputs(64)
    eng.generate(0, 0, inp)
    out = eng.alloc_outputs(64)
    old = OldIn(inp["ctx"].data_ptr(), inp["part"].data_ptr(), inp["u"].data_ptr())
    bo = _lib.AgBatchOut(*[out[k].data_ptr() if k in out else None for k in
                           ("winner", "price", "second_price", "outcome", "item", "bid", "est_ctr",
                            "true_ctr", "best_ev", "gamma", "propensity")])
    L = eng.L
    rc = L.ag_simulate(eng._h, 64, ctypes.cast(ctypes.pointer(old), ctypes.POINTER(_lib.AgBatchIn)),
                       ctypes.byref(bo), None, None)
    assert rc == _lib.AG_ERR_INVALID
    assert b"struct_size" in L.ag_last_error()
    bo.struct_size = 12345
    rc = L.ag_simulate(eng._h, 64, ctypes.byref(_lib.AgBatchIn(inp["ctx"].data_ptr(), inp["part"].data_ptr(),
                                                                inp["u"].data_ptr())), ctypes.byref(bo), None, None)
    assert rc == _lib.AG_ERR_INVALID
    torch.cuda.synchronize()
    eng.close()


def _integration_block():
    """The python block of INTEGRATION.md section 2 (the reference-side ctypes stub)."""
    text = open(os.path.join(os.path.dirname(GOLDEN), "..", "INTEGRATION.md")).read()
    sec = text[text.index("## 2. Raw C-ABI"):text.index("## 3. ")]
    return sec[sec.index("```python") + len("```python"):sec.index("```", sec.index("```python") + 9)]


def test_integration_stub_runs_verbatim(gpu):
    """INTEGRATION.md's ctypes stub, executed as published, on a stand-in for the reference's
    Auction built exactly as src/main.py builds SP_Oracle (seed 0): the draws it makes are the
    reference's, so its winners, prices, utilities and revenue equal the reference's own
    capture (sp_oracle_r4096)."""
    import ctypes
    import types
    import auctiongym_amd.main as M
    from auctiongym_amd import _lib
    d, meta, agg = load_capture("sp_oracle_r4096")
    ns = {"AG_LIB": _lib.LIB_PATH, "__name__": "integration_stub"}
    exec(compile(_integration_block(), "INTEGRATION.md#2", "exec"), ns)
    with open(os.path.join(GOLDEN, "sp_oracle_full_run.json")) as f:
        cfg = json.load(f)["config"]
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "ag_integration_sp_oracle.json")
    with open(path, "w") as f:
        json.dump(cfg, f)
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(path)
    SecondPrice = type("SecondPrice", (), {})
    auction = types.SimpleNamespace(
        rng=rng, agents=[types.SimpleNamespace(name=c["name"], net_utility=0.0, gross_utility=0.0)
                         for c in agent_configs],
        num_participants_per_round=config["num_participants_per_round"], agents2item_values=a2v,
        agent2items=a2i, embedding_size=E, obs_embedding_size=OE, embedding_var=var,
        allocation=SecondPrice(), max_slots=max_slots, revenue=0.0)
    path_ = ns["GPUAuctionPath"](auction)
    B = 4096
    path_.run_rounds(B)
    w = np.empty(B, np.int32)
    pr = np.empty(B)
    ns["d2h"](w, ctypes.c_void_p(path_.last["winner"]))
    ns["d2h"](pr, ctypes.c_void_p(path_.last["price"]))
    assert np.array_equal(w, d["winner"])
    assert np.array_equal(pr, d["price"])
    np.testing.assert_allclose([a.net_utility for a in auction.agents], agg["net_utility"], rtol=1e-9)
    np.testing.assert_allclose(auction.revenue, agg["revenue"], rtol=1e-9)
    # the buffers are allocated once per batch size and reused; close() frees them with the ctx
    bufs = list(path_.bufs)
    path_.run_rounds(B)
    assert [p.value for p in path_.bufs] == [p.value for p in bufs]
    path_.close()
    assert path_.bufs == [] and path_.ctx is None


def test_screened_search_adversarial_catalogues(gpu, oracle):
    """Catalogues built to stress the f32 screen: exact duplicate items (ties -> first max),
    near-ties 1 ulp apart, huge embeddings (guard -> exact scan), intercepts so negative
    that f32 exp overflows, and values differing in the last bits."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(11)
    N, K, E, P, B = 8, 12, 5, 3, 1 << 18
    base = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    cats = []
    c = base.copy(); v = values.copy()
    c[:, 5] = c[:, 2]; v[:, 5] = v[:, 2]                        # exact duplicates
    c[:, 7] = c[:, 1]; v[:, 7] = np.nextafter(v[:, 1], 10)      # 1-ulp value near-ties
    cats.append((c, v))
    c = base.copy(); c[:4] *= 40.0                               # |a| large: guard path
    cats.append((c, values))
    c = base.copy(); c[:, :, -1] = -150.0 - g.random((N, K))     # sigmoid ~ e^-150
    cats.append((c, values))
    c = base.copy(); c[:, :, :E] *= 1e-9                         # all items ~ equal z
    cats.append((c, values * (1 + 1e-15 * g.random((N, K)))))
    c = base.copy(); v = values.copy(); v[0, 3] = 2000.0            # a value beyond k_oracle's
    cats.append((c, v))                                              # bound: general kernel
    c = base.copy(); v = values.copy(); v[1, 4] = -0.5               # negative value: general kernel
    cats.append((c, v))
    for items, vals in cats:
        for generic in (False, True):  # the dedicated Oracle kernel and the general one
            eng = AuctionEngine(N, P, K, E, 4, 0, 1.0)
            eng.load_catalog(items, vals)
            eng.set_simulate_kernel(generic)
            inp = eng.alloc_inputs(B)
            eng.generate(7, 0, inp)
            out = eng.alloc_outputs(B)
            cnt = eng.new_counters()
            eng.simulate(inp, out, cnt)
            ctx = np.ascontiguousarray(inp["ctx"].cpu().numpy().T)
            part = np.ascontiguousarray(inp["part"].cpu().numpy().T)
            u = inp["u"].cpu().numpy()
            orc = oracle.simulate(0, items, vals, ctx, part, u, nthreads=16)
            assert np.array_equal(out["item"].cpu().numpy().T, orc["item"])
            assert np.array_equal(out["bid"].cpu().numpy().T, orc["bid"])
            assert np.array_equal(out["best_ev"].cpu().numpy().T, orc["best_ev"])
            assert np.array_equal(out["price"].cpu().numpy(), orc["price"])
            assert np.array_equal(out["second_price"].cpu().numpy(), orc["second_price"])
            assert np.array_equal(out["outcome"].cpu().numpy(), orc["outcome"])
            assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
            eng.close()


# ---- general populations: LR-TS allocators, shading bidders (first iteration) ----
from conftest import POP_CAPTURES, pop_args  # noqa: E402


def _pop_engine(meta, d, gpu):
    from auctiongym_amd.engine import AuctionEngine
    args = pop_args(d, meta)
    eng = AuctionEngine(meta["N"], meta["P"], meta["K"], meta["E"], meta["OE"], mech_code(meta),
                        meta["var"])
    eng.set_agent_params(args["alloc_kind"], args["bid_kind"], args["prev_gamma"], args["gamma_sigma"])
    if meta.get("num_items") and min(meta["num_items"]) < meta["K"]:
        eng.set_agent_items(meta["num_items"])  # per-agent item counts (catalogue rows padded)
    eng.load_catalog(d["items"], d["values"])
    if args["ts_m"] is not None:
        eng.load_lrts(args["ts_m"], np.ones_like(args["ts_m"]), thompson_sampling=True)
    return eng, args


def _pop_run(eng, ctx, part, u, gamma_raw=None, ts_noise=None):
    """Row-major host replay inputs -> outputs in row-major host layout + fx counters."""
    import torch
    d = eng.device
    B = len(u)
    inp = {"ctx": torch.from_numpy(np.ascontiguousarray(ctx.T)).to(d),
           "part": torch.from_numpy(np.ascontiguousarray(part.T.astype(np.int32))).to(d),
           "u": torch.from_numpy(np.ascontiguousarray(u)).to(d)}
    if gamma_raw is not None:
        inp["gamma_raw"] = torch.from_numpy(np.ascontiguousarray(gamma_raw.T)).to(d)
    if ts_noise is not None:
        inp["ts_noise"] = torch.from_numpy(eng.tile_ts_noise(ts_noise)).to(d)
    out = eng.alloc_outputs(B, ("winner", "price", "second_price", "outcome", "item", "bid",
                                "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"))
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
        o[k] = np.ascontiguousarray(o[k].T)
    o["counters_fx"] = cnt.cpu().numpy()
    return o


@pytest.mark.parametrize("name", POP_CAPTURES)
def test_population_replay_matches_oracle_and_reference(gpu, oracle, name):
    d, meta, agg = load_capture(name)
    eng, args = _pop_engine(meta, d, gpu)
    o = _pop_run(eng, d["ctx"], d["part"], d["u"], d["gamma_raw"], d.get("ts_noise"))
    orc = oracle.simulate_pop(mech_code(meta), d["items"], d["values"], d["ctx"], d["part"], d["u"],
                              **args)
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "winner", "price", "second_price",
              "outcome"):
        assert np.array_equal(o[k], orc[k], equal_nan=True), k
    sh = ~np.isnan(orc["gamma"])
    assert np.array_equal(o["gamma"][sh], orc["gamma"][sh])
    pr = ~np.isnan(orc["propensity"])
    assert np.array_equal(o["propensity"][pr], orc["propensity"][pr])
    assert np.array_equal(o["counters_fx"], orc["counters_fx"])
    # and the reference itself (the oracle's own pinning), LR-TS float32 CTRs included
    assert np.array_equal(o["item"], d["item"]) and np.array_equal(o["winner"], d["winner"])
    assert np.array_equal(o["true_ctr"], d["slot_true_ctr"])
    assert np.array_equal(o["est_ctr"], d["slot_est_ctr"])
    assert np.array_equal(o["bid"], d["slot_bid"])
    assert np.array_equal(o["price"], d["price"], equal_nan=True)
    eng.close()


def test_mixed_population_full_size(gpu, oracle):
    """Mixed population (Oracle / LR-TS allocators x truthful / shading bidders), 32 agents,
    P = 8, FirstPrice: synthetic inputs and noise generated on the GPU, every output
    compared with the oracle on the same inputs (2^20 auctions)."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N, P, K, E, OE, B = 32, 8, 12, 5, 4, 1 << 20
    g = np.random.default_rng(21)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.array([i % 2 for i in range(N)], np.int32)             # Oracle / LR-TS
    bk = np.array([(i // 2) % 5 for i in range(N)], np.int32)      # all five bidder kinds
    pg = 0.5 + 0.5 * g.random(N)
    gs = 0.01 + 0.05 * g.random(N)
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = (1.0 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32)
    eng = AuctionEngine(N, P, K, E, OE, 0, 1.0)
    eng.set_agent_params(ak, bk, pg, gs)
    eng.load_catalog(items, values)
    eng.load_lrts(m, q, thompson_sampling=True)
    inp = eng.alloc_inputs(B)
    eng.generate(5, 0, inp)
    eng.generate_noise(5, 0, inp)
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    ctx = np.ascontiguousarray(inp["ctx"].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"].cpu().numpy().T)
    u = inp["u"].cpu().numpy()
    gr = np.ascontiguousarray(inp["gamma_raw"].cpu().numpy().T)
    tn = eng.untile_ts_noise(inp["ts_noise"], B).reshape(B, P, K, OE + 1)
    # generator sanity: shading draws ~ N(prev_gamma, sigma), LR-TS noise ~ N(0, 1/q)
    a0 = part[:, 0]
    zs = (gr[:, 0] - pg[a0]) / gs[a0]
    zs = zs[bk[a0] != 0]
    assert abs(zs.mean()) < 0.01 and abs(zs.std() - 1) < 0.01
    orc = oracle.simulate_pop(0, items, values, ctx, part, u, ak, bk, pg, gs, OE=OE, ts_m=m,
                              ts_noise=tn, gamma_raw=gr, nthreads=16)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
        assert np.array_equal(np.ascontiguousarray(got[k].T), orc[k], equal_nan=True), k
    for k in ("winner", "price", "second_price", "outcome"):
        assert np.array_equal(got[k], orc[k], equal_nan=True), k
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    eng.close()


@pytest.mark.parametrize("P,B,block", [(2, (1 << 20) + 37, 0), (2, 4099, 1024), (8, 1 << 18, 0), (12, 1 << 14, 0)])
def test_compact_ts_noise_equals_dense(gpu, P, B, block):
    """The compact Thompson-noise layout (ag_batch_in.ts_noise_index, ag_ts_noise_index,
    ag_generate_ts_noise_compact): the index is numpy's exclusive cumsum of the LR-TS flags in
    (slot, auction) order, the compact draws are the dense generator's values of the LR-TS
    pairs, and every output and exact counter of ag_simulate is the same bit for bit as with
    the dense tiles (register-array and runtime-P kernels, both block sizes, ragged B)."""
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    N, K, E, OE = 32, 12, 5, 4
    g = np.random.default_rng(77 + P)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.array([1 if i % 3 else 0 for i in range(N)], np.int32)   # 2/3 LR-TS
    bk = np.array([4 if i % 3 == 2 else 0 for i in range(N)], np.int32)
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = (1.0 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32)
    eng = AuctionEngine(N, P, K, E, OE, 0, 1.0)
    eng.set_agent_params(ak, bk, np.ones(N), np.full(N, 0.02))
    eng.load_catalog(items, values)
    eng.load_lrts(m, q, thompson_sampling=True)
    if block:
        eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_BLOCK_THREADS, block), "ag_set_option")
    inp = eng.alloc_inputs(B)
    eng.generate(9, 1000, inp)
    eng.generate_noise(9, 1000, inp)
    out_d, cnt_d = eng.alloc_outputs(B), eng.new_counters()
    eng.simulate(inp, out_d, cnt_d)
    dense = inp["ts_noise"].cpu().numpy()
    cin = {k: v for k, v in inp.items() if k != "ts_noise"}
    n = eng.compact_ts_noise(9, 1000, cin)
    flags = ak[inp["part"].cpu().numpy()] == 1
    want = np.where(flags, np.cumsum(flags.ravel()).reshape(flags.shape) - 1, -1)
    assert n == int(flags.sum())
    assert np.array_equal(cin["ts_noise_index"].cpu().numpy(), want)
    back = eng.compact_to_dense_ts_noise(cin["ts_noise"], cin["ts_noise_index"], P, B)
    mask = np.broadcast_to(flags[:, :, None], (P, B, K * (OE + 1)))
    dn = eng.untile_ts_noise(dense, B).transpose(1, 0, 2)
    bk_ = eng.untile_ts_noise(back, B).transpose(1, 0, 2)
    assert np.array_equal(dn[mask], bk_[mask])
    out_c, cnt_c = eng.alloc_outputs(B), eng.new_counters()
    eng.simulate(cin, out_c, cnt_c)
    torch.cuda.synchronize()
    for k in out_d:
        assert torch.equal(out_d[k], out_c[k]) or np.array_equal(out_d[k].cpu().numpy(), out_c[k].cpu().numpy(),
                                                                   equal_nan=True), k
    assert torch.equal(cnt_d, cnt_c)
    eng.close()


@pytest.mark.parametrize("P,mech,mixed", [(9, 1, False), (16, 0, True), (40, 1, True), (12, 0, False)])
def test_wide_participants_match_oracle(gpu, oracle, P, mech, mixed):
    """More than 8 participants per round (src/Auction.py:42 has no bound): the runtime-P
    simulate kernel, every output and the exact counters equal to the oracle (Oracle-only
    and mixed populations, both mechanisms, P up to N)."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N, K, E, OE = 40, 12, 5, 4
    B = 1 << 16 if P < 32 else 1 << 14
    g = np.random.default_rng(100 + P)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.array([i % 2 for i in range(N)] if mixed else [0] * N, np.int32)
    bk = np.array([(i // 2) % 5 for i in range(N)] if mixed else [0] * N, np.int32)
    pg = 0.5 + 0.5 * g.random(N)
    gs = 0.01 + 0.05 * g.random(N)
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = (1.0 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32)
    eng = AuctionEngine(N, P, K, E, OE, mech, 1.0)
    eng.set_agent_params(ak, bk, pg, gs)
    eng.load_catalog(items, values)
    if mixed:
        eng.load_lrts(m, q, thompson_sampling=True)
    inp = eng.alloc_inputs(B)
    eng.generate(7, 0, inp)
    if mixed:
        eng.generate_noise(7, 0, inp)
    out = eng.alloc_outputs(B, ("winner", "price", "second_price", "outcome", "item", "bid", "est_ctr",
                                "true_ctr", "best_ev", "gamma", "propensity"))
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    ctx = np.ascontiguousarray(inp["ctx"].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"].cpu().numpy().T)
    assert all(len(set(r)) == P for r in part[:100])  # distinct participants per round
    u = inp["u"].cpu().numpy()
    kw = {}
    if mixed:
        kw = dict(OE=OE, ts_m=m, ts_noise=eng.untile_ts_noise(inp["ts_noise"], B).reshape(B, P, K, OE + 1),
                  gamma_raw=np.ascontiguousarray(inp["gamma_raw"].cpu().numpy().T))
    orc = oracle.simulate_pop(mech, items, values, ctx, part, u, ak, bk, pg, gs, nthreads=16, **kw)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
        assert np.array_equal(np.ascontiguousarray(got[k].T), orc[k], equal_nan=True), k
    for k in ("winner", "price", "second_price", "outcome"):
        assert np.array_equal(got[k], orc[k], equal_nan=True), k
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    eng.close()


@pytest.mark.parametrize("case", ["ties", "large_logits", "tiny_values"])
def test_thompson_screen_adversarial(gpu, oracle, case):
    """The screened Thompson item choice (hardware exp2 / rcp estimates, exact scores of the
    near-best items) against the oracle's plain loop: exactly tied items (duplicate model rows
    and values, noise ~1e-15 so the tie survives: first argmax), values 1 ulp apart, logits
    beyond the screen's |z| < 64 bound, and values spanning 1e-30..1e30."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N, P, K, E, OE, B = 8, 2, 12, 5, 4, 1 << 18
    g = np.random.default_rng(31)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = np.ones_like(m)
    if case == "ties":
        m[:, 5] = m[:, 2]; values[:, 5] = values[:, 2]
        m[:, 7] = m[:, 1]; values[:, 7] = np.nextafter(values[:, 1], 10)
        m[:, 9] = m[:, 3]; values[:, 9] = np.nextafter(values[:, 3], -10)
        q[:] = 1e30
    elif case == "large_logits":
        m *= 40.0
    else:
        values = values * 10.0 ** g.integers(-30, 31, (N, K))
    eng = AuctionEngine(N, P, K, E, OE, 1, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), np.zeros(N, np.int32))
    eng.load_catalog(items, values)
    eng.load_lrts(m, q, thompson_sampling=True)
    inp = eng.alloc_inputs(B)
    eng.generate(3, 0, inp)
    eng.generate_noise(3, 0, inp)
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    ctx = np.ascontiguousarray(inp["ctx"].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"].cpu().numpy().T)
    u = inp["u"].cpu().numpy()
    tn = eng.untile_ts_noise(inp["ts_noise"], B).reshape(B, P, K, OE + 1)
    orc = oracle.simulate_pop(1, items, values, ctx, part, u, np.ones(N, np.int32), np.zeros(N, np.int32),
                              np.ones(N), np.full(N, 0.02), OE=OE, ts_m=m, ts_noise=tn, nthreads=16)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev"):
        assert np.array_equal(np.ascontiguousarray(got[k].T), orc[k], equal_nan=True), k
    for k in ("winner", "price", "second_price", "outcome"):
        assert np.array_equal(got[k], orc[k], equal_nan=True), k
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    if case == "ties":  # the tie is real: item 5 never beats item 2 for the same draw
        assert (got["item"] != 5).any()
    eng.close()


@pytest.mark.parametrize("P,B,block,compact", [(4, 1 << 18, 0, False), (2, (1 << 17) + 45, 1024, True),
                                               (2, 777, 0, False), (8, (1 << 16) + 3, 1024, False),
                                               (12, 5000, 0, False)])
def test_fitted_policy_bids_match_oracle(gpu, oracle, P, B, block, compact):
    """Learning bidders bidding from a fitted policy (src/Bidder.py:198-203 ValueLearningBidder
    'policy', :358-362 PolicyLearningBidder, :466-470 DoublyRobustBidder): the gamma is the
    policy's rsample on (estimated CTR, value), the propensity its Normal density. Mixed
    population where half of the learning bidders bid from random fitted policies; every
    output compared with the oracle on the same inputs and the same generated draws. The
    kernel compacts a wave's fitted-policy bids across its slots (ragged last tiles: fewer
    active lanes than tasks; P = 12: the runtime-P kernel, not compacted), both workgroup
    sizes, dense and compact Thompson-noise layouts."""
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    N, K, E, OE = 20, 12, 5, 4
    g = np.random.default_rng(33)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.array([i % 2 for i in range(N)], np.int32)
    bk = np.array([4 if i % 3 else (i // 3) % 4 for i in range(N)], np.int32)
    pg = 0.5 + 0.5 * g.random(N)
    gs = 0.01 + 0.05 * g.random(N)
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = (1.0 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32)
    state = g.normal(0, 0.7, (N, 16)).astype(np.float32)
    init = np.array([1 if (bk[a] >= 2 and (a % 2 == 0 or a == 9)) else 0 for a in range(N)], np.int32)
    assert init.sum() >= 4 and ((bk >= 2) & (init == 0)).sum() >= 4
    assert {2, 3, 4} <= set(bk[init == 1].tolist())
    eng = AuctionEngine(N, P, K, E, OE, 1, 1.0)
    eng.set_agent_params(ak, bk, pg, gs)
    eng.load_catalog(items, values)
    eng.load_lrts(m, q, thompson_sampling=True)
    eng.set_dr_state(state, init)
    if block:
        eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_BLOCK_THREADS, block), "ag_set_option")
    inp = eng.alloc_inputs(B)
    assert "policy_eps" in inp
    eng.generate(9, 0, inp)
    eng.generate_noise(9, 0, inp, compact=compact)
    tn = (eng.compact_to_dense_ts_noise(inp["ts_noise"], inp["ts_noise_index"], P, B) if compact
          else inp["ts_noise"])
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    T = lambda t: np.ascontiguousarray(t.cpu().numpy().T)  # noqa: E731
    pe = T(inp["policy_eps"])
    if B >= 1 << 16:
        assert abs(pe.mean()) < 0.01 and abs(pe.std() - 1) < 0.01
    orc = oracle.simulate_pop(1, items, values, T(inp["ctx"]), T(inp["part"]), inp["u"].cpu().numpy(),
                              ak, bk, pg, gs, OE=OE, ts_m=m,
                              ts_noise=eng.untile_ts_noise(tn, B).reshape(B, P, K, OE + 1),
                              gamma_raw=T(inp["gamma_raw"]), dr_state=state, dr_init=init,
                              policy_eps=pe, nthreads=16)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
        assert np.array_equal(np.ascontiguousarray(got[k].T), orc[k], equal_nan=True), k
    for k in ("winner", "price", "second_price", "outcome"):
        assert np.array_equal(got[k], orc[k], equal_nan=True), k
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    # fitted agents' gammas are clipped policy draws, not N(prev_gamma, sigma) draws
    part = T(inp["part"])
    fitted = init[part] == 1
    gam = np.ascontiguousarray(got["gamma"].T)
    assert fitted.any() and (gam[fitted] >= 0).all() and (gam[fitted] <= 1).all()
    # without policy_eps the launch is refused
    del inp["policy_eps"]
    with pytest.raises(ValueError, match="policy_eps"):
        eng.simulate(inp, out, eng.new_counters())
    eng.close()


# ---- LR-TS allocator update (Agent.update -> PyTorchLogisticRegressionAllocator.update) ----
def _kat_population():
    kat = np.load(os.path.join(GOLDEN, "sp_ts_update_kat.npz"))
    stack = lambda n: np.stack([kat[f"a{a}_{n}"] for a in range(6)]).astype(np.float32)  # noqa: E731
    return kat, stack("m0"), stack("q0"), stack("prevm0")


def _fill_store(eng, per_agent, capacity=None, seed=0):
    """Caller-owned sample store holding `per_agent` {agent: (X, A, y)}, shuffled."""
    import torch
    keys, xs = [], []
    for a, (X, A, y) in per_agent.items():
        keys.append((np.int64(a) << 16) | (np.asarray(A, np.int64) << 1) | (np.asarray(y) != 0))
        xs.append(np.asarray(X, np.float32))
    key = np.concatenate(keys).astype(np.uint32)
    x = np.concatenate(xs)
    perm = np.random.default_rng(seed).permutation(len(key))
    key, x = key[perm], x[perm]
    cap = capacity or len(key)
    st = eng.new_lrts_samples(cap)
    n = min(len(key), cap)
    st["key"][:n] = torch.from_numpy(key[:n].view(np.int32)).to(eng.device)
    st["x"][:, :n] = torch.from_numpy(np.ascontiguousarray(x[:n].T)).to(eng.device)
    st["count"][0] = len(key)
    return st


def _lrts_engine(N=6, P=2, K=12, E=5, OE=4, lrts=None):
    from auctiongym_amd.engine import AuctionEngine
    d, meta, _ = load_capture("sp_ts_r2048")
    eng = AuctionEngine(N, P, K, E, OE, 1, 1.0)
    ak = np.ones(N, np.int32) if lrts is None else np.asarray(lrts, np.int32)
    eng.set_agent_params(ak, np.zeros(N, np.int32))
    if N == 6:
        eng.load_catalog(d["items"], d["values"])
    return eng


def test_lrts_update_matches_oracle_and_reference(gpu, oracle):
    """The six SP_Truthful_TS agents' iteration-0 updates on the GPU (all six at once) vs
    the oracle, bit for bit: epochs run, every epoch's loss, m, q and prev_m; and vs the
    reference within the oracle's pinned tolerances."""
    import torch
    kat, m0, q0, pm0 = _kat_population()
    eng = _lrts_engine()
    eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
    st = _fill_store(eng, {a: (kat[f"a{a}_X"], kat[f"a{a}_A"], kat[f"a{a}_y"]) for a in range(6)})
    ep, tr = eng.lrts_update(st, trace=True)
    m, q, pm = eng.lrts_state()
    tr = tr.cpu().numpy()
    # the same update spread over several cooperating workgroups per agent (64 or 100
    # samples each: 3-8 workgroups, one barrier per epoch): bit-identical
    for chunk in (64, 100):
        eng.set_lrts_block_samples(chunk)
        eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
        ep2, tr2 = eng.lrts_update(st, trace=True)
        m2, q2, pm2 = eng.lrts_state()
        assert np.array_equal(ep2, ep) and torch.equal(tr2.cpu(), torch.from_numpy(tr))
        assert np.array_equal(m2, m) and np.array_equal(q2, q) and np.array_equal(pm2, pm)
    eng.set_lrts_block_samples(0)
    for a in range(6):
        k = lambda n: kat[f"a{a}_{n}"]  # noqa: E731
        om, opm, oq, oep, oL = oracle.lrts_update(k("X"), k("A"), k("y"), k("m0"), k("prevm0"), k("q0"))
        assert ep[a] == oep
        assert np.array_equal(tr[a, :oep], oL.astype(np.float32))
        assert np.array_equal(m[a], om) and np.array_equal(q[a], oq) and np.array_equal(pm[a], opm)
        np.testing.assert_allclose(m[a], k("m1"), atol=2e-2)
        np.testing.assert_allclose(q[a], k("q1"), rtol=2e-3)
    eng.close()


def test_lrts_collect_from_replay_and_update(gpu, oracle):
    """Replay the SP_Truthful_TS capture, collect the won samples on the GPU: the store holds
    exactly the reference's Agent.update samples (as a multiset; float32 contexts); the
    update from that store equals the update from the reference's own samples."""
    import torch
    d, meta, _ = load_capture("sp_ts_r2048")
    kat, m0, q0, pm0 = _kat_population()
    eng, args = _pop_engine(meta, d, gpu)
    eng.load_lrts(np.asarray(d["ts_m"], np.float32), q0, pm0, thompson_sampling=True)
    B, P, Do = len(d["u"]), meta["P"], meta["OE"] + 1
    dev = eng.device
    inp = {"ctx": torch.from_numpy(np.ascontiguousarray(d["ctx"].T)).to(dev),
           "part": torch.from_numpy(np.ascontiguousarray(d["part"].T.astype(np.int32))).to(dev),
           "u": torch.from_numpy(np.ascontiguousarray(d["u"])).to(dev),
           "gamma_raw": torch.from_numpy(np.ascontiguousarray(d["gamma_raw"].T)).to(dev),
           "ts_noise": torch.from_numpy(eng.tile_ts_noise(d["ts_noise"])).to(dev)}
    out = eng.alloc_outputs(B)
    st = eng.new_lrts_samples(B)
    half = B // 2  # two batches, as two flushes of one iteration
    for lo, hi in ((0, half), (half, B)):
        bi = {k: (v[..., lo:hi] if k != "ts_noise" else v[:, lo // 64:hi // 64]).contiguous()
              for k, v in inp.items()}
        bo = eng.alloc_outputs(hi - lo)
        eng.simulate(bi, bo)
        eng.lrts_collect(bi, bo, st)
    torch.cuda.synchronize()
    n = int(st["count"][0])
    key = st["key"][:n].cpu().numpy().view(np.uint32)
    x = st["x"][:, :n].cpu().numpy().T
    got = sorted(zip(key.tolist(), map(tuple, x.tolist())))
    want = []
    for a in range(6):
        X, A, y = kat[f"a{a}_X"], kat[f"a{a}_A"], kat[f"a{a}_y"]
        Xf = X.astype(np.float32)
        for j in range(len(y)):
            want.append(((a << 16) | (int(A[j]) << 1) | int(y[j]), tuple(Xf[j].tolist())))
    assert got == sorted(want)
    # the update from the collected store == the update from the reference's samples
    eng.load_lrts(m0, q0, pm0, thompson_sampling=True)
    ep = eng.lrts_update(st)
    m, q, pm = eng.lrts_state()
    for a in range(6):
        k = lambda n: kat[f"a{a}_{n}"]  # noqa: E731
        om, opm, oq, oep, _ = oracle.lrts_update(k("X"), k("A"), k("y"), k("m0"), k("prevm0"), k("q0"))
        assert ep[a] == oep and np.array_equal(m[a], om) and np.array_equal(q[a], oq)
    eng.close()


def test_lrts_update_edge_cases(gpu, oracle):
    """< 2 samples: unchanged (src/BidderAllocation.py:33-34); non-LR-TS agents untouched;
    an overflowed store is an error, not a silent truncation."""
    g = np.random.default_rng(3)
    N, K, Do = 4, 12, 5
    eng = _lrts_engine(N=N, lrts=[1, 1, 0, 1])
    m0 = g.normal(0, 1, (N, K, Do)).astype(np.float32)
    q0 = (1 + g.random((N, K, Do))).astype(np.float32)
    pm0 = (m0 + 0.5).astype(np.float32)
    eng.load_lrts(m0, q0, pm0)
    X = np.concatenate([g.normal(0, 1, (200, Do - 1)), np.ones((200, 1))], axis=1)
    A, y = g.integers(0, K, 200), g.random(200) < 0.3
    st = _fill_store(eng, {0: (X[:1], A[:1], y[:1]), 3: (X, A, y)})
    ep = eng.lrts_update(st)
    m, q, pm = eng.lrts_state()
    assert ep[0] == 0 and ep[1] == 0 and ep[2] == 0 and ep[3] > 0
    for a in (0, 1, 2):
        assert np.array_equal(m[a], m0[a]) and np.array_equal(q[a], q0[a]) and np.array_equal(pm[a], pm0[a])
    om, opm, oq, oep, _ = oracle.lrts_update(X, A, y, m0[3], pm0[3], q0[3])
    assert ep[3] == oep and np.array_equal(m[3], om) and np.array_equal(q[3], oq)
    over = _fill_store(eng, {3: (X, A, y)}, capacity=100)
    with pytest.raises(ValueError, match="overflow"):
        eng.lrts_update(over)
    eng.close()


def test_lrts_update_at_scale(gpu, oracle):
    """A mixed 32-agent population simulated on 2^16 synthetic auctions, collected and
    trained on the GPU (16 LR-TS agents, ~1.4k samples each); four agents re-trained by the
    oracle on the collected samples, bit for bit."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N, P, K, E, OE, B = 32, 8, 12, 5, 4, 1 << 16
    g = np.random.default_rng(22)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.array([i % 2 for i in range(N)], np.int32)
    bk = np.zeros(N, np.int32)
    m0 = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q0 = np.ones((N, K, OE + 1), np.float32)
    eng = AuctionEngine(N, P, K, E, OE, 0, 1.0)
    eng.set_agent_params(ak, bk)
    eng.load_catalog(items, values)
    eng.load_lrts(m0, q0)
    inp = eng.alloc_inputs(B)
    eng.generate(9, 0, inp)
    eng.generate_noise(9, 0, inp)
    out = eng.alloc_outputs(B)
    eng.simulate(inp, out)
    st = eng.new_lrts_samples(B)
    eng.lrts_collect(inp, out, st)
    torch.cuda.synchronize()
    n = int(st["count"][0])
    key = st["key"][:n].cpu().numpy().view(np.uint32)
    x = np.ascontiguousarray(st["x"][:, :n].cpu().numpy().T)
    ep = eng.lrts_update(st)
    m, q, pm = eng.lrts_state()
    assert (ep[ak == 1] > 0).all() and (ep[ak == 0] == 0).all()
    for a in (1, 7, 21, 31):
        sel = (key >> 16) == a
        om, opm, oq, oep, _ = oracle.lrts_update(x[sel], (key[sel] >> 1) & 0x7FFF, key[sel] & 1,
                                                 m0[a], m0[a], q0[a])
        assert ep[a] == oep and np.array_equal(m[a], om) and np.array_equal(q[a], oq)
    eng.close()


SP_TRUTHFUL_TS = {  # config/SP_Truthful_TS.json as shipped
    "random_seed": 0, "num_runs": 3, "num_iter": 20, "rounds_per_iter": 10000,
    "num_participants_per_round": 2, "embedding_size": 5, "embedding_var": 1.0,
    "obs_embedding_size": 4, "allocation": "SecondPrice",
    "agents": [{"name": "Truthful Learnt", "num_copies": 6, "num_items": 12,
                "allocator": {"type": "PyTorchLogisticRegressionAllocator",
                              "kwargs": {"embedding_size": 4, "num_items": 12}},
                "bidder": {"type": "TruthfulBidder", "kwargs": {}}}],
    "output_dir": "results/SP_Truthful_TS/"}


@pytest.mark.parametrize("path", ["per_round", "batch"])
@pytest.mark.parametrize("name", ["sp_ts_mixed_flags_r2048", "ragged_items_r2048"])
def test_dropin_surface_captures(gpu, tmp_path, path, name):
    """Two surfaces the reference allows, through the drop-in classes against the reference's
    own runs, per round (simulate_opportunity) and as one batch (simulate_batch:
    ag_replay_draw_population): thompson_sampling set per allocator (src/BidderAllocation.py:
    24-26; sp_ts_mixed_flags_r2048: 4 LR-TS agents sample, 4 bid from their MAP estimates), and
    per-agent num_items (src/main.py:61,66; ragged_items_r2048: Oracle agents with 12 items,
    LR-TS agents with 9, 6 and 13 -- catalogues padded, each LR-TS choice over the agent's own
    rows, its torch draws of its own K*Do). The reference's items and estimated CTRs per agent,
    utilities and revenue to the exact sums' 1e-11, and torch's generator left where the
    reference's calls leave it."""
    import torch

    import auctiongym_amd.main as M
    d, meta, agg = load_capture(name)
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(meta["config"]))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(meta["torch_seed"])
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    if name.startswith("sp_ts_mixed"):
        assert [a.allocator.thompson_sampling for a in agents] == [True] * 4 + [False] * 4
    auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    if path == "per_round":
        for _ in range(meta["rounds"]):
            auction.simulate_opportunity()
    else:
        auction.simulate_batch(meta["rounds"])
    rt = dict(rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose([a.net_utility for a in agents], agg["net_utility"], **rt)
    np.testing.assert_allclose([a.gross_utility for a in agents], agg["gross_utility"], **rt)
    np.testing.assert_allclose(auction.revenue, agg["revenue"], **rt)
    assert [a.num_logs() for a in agents] == list(agg["n_logs"])
    for i, a in enumerate(agents):
        rows, slots = np.nonzero(d["part"] == i)
        assert [o.item for o in a.logs] == list(d["item"][rows, slots])
        np.testing.assert_array_equal([o.estimated_CTR for o in a.logs], d["slot_est_ctr"][rows, slots])
    # the generator: the LR-TS agents' initial m (torch.nn.init.normal_ of [K_a][OE+1], agent
    # order), then K_a*(OE+1) torch.normal values per sampling participation, in round order
    ref = torch.Generator().manual_seed(meta["torch_seed"])
    kdo = [a.allocator.response_model.q.numel() if hasattr(a.allocator, "response_model") else 0 for a in agents]
    for k in kdo:
        if k:
            torch.empty(k).normal_(generator=ref)
    samp = [bool(k) and a.allocator.thompson_sampling for k, a in zip(kdo, agents)]
    for a in d["part"].ravel():
        if samp[a]:
            torch.empty(kdo[a]).normal_(generator=ref)
    assert torch.equal(torch.get_rng_state(), ref.get_state())


def test_dropin_batch_small_thompson_model(gpu, tmp_path):
    """a sampling LR-TS agent whose K*(OE+1) < 16 (num_items = 3, OE = 4: 15 draws per
    participation, torch's scalar normal path, which ag_replay_draw_population does not restate)
    -- simulate_batch takes the per-round loop and gives exactly the per-round run's results and
    torch / numpy generator states, instead of raising."""
    import torch

    import auctiongym_amd.main as M
    cfg = dict(SP_TRUTHFUL_TS, agents=[
        {"name": "Small TS", "num_copies": 3, "num_items": 3,
         "allocator": {"type": "PyTorchLogisticRegressionAllocator", "kwargs": {"embedding_size": 4, "num_items": 3}},
         "bidder": {"type": "TruthfulBidder", "kwargs": {}}},
        {"name": "Oracle", "num_copies": 2, "num_items": 12,
         "allocator": {"type": "OracleAllocator", "kwargs": {}}, "bidder": {"type": "TruthfulBidder", "kwargs": {}}}])
    p = tmp_path / "small.json"
    p.write_text(json.dumps(cfg))
    res = {}
    for path in ("per_round", "batch"):
        rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
        torch.manual_seed(5)
        agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
        auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
        assert not auction._native_draws()
        if path == "per_round":
            for _ in range(700):
                auction.simulate_opportunity()
        else:
            auction.simulate_batch(700)
        res[path] = ([a.net_utility for a in agents], auction.revenue, torch.get_rng_state(),
                     rng.bit_generator.state["state"]["state"], [[o.item for o in a.logs] for a in agents])
    a, b = res["per_round"], res["batch"]
    assert a[0] == b[0] and a[1] == b[1] and torch.equal(a[2], b[2]) and a[3] == b[3] and a[4] == b[4]


def test_driver_sp_truthful_ts_iteration(gpu, oracle, tmp_path):
    """SP_Truthful_TS.json through the drop-in classes with torch seeded as the capture was:
    the same LR-TS initial models (torch.nn.init.normal_), the same Thompson draws
    (torch.normal in slot order), the reference's rounds (capture sp_ts_r2048: winners,
    items and the float32 CTRs exact, so utilities and revenue to the exact sums' 1e-11); then Agent.update trains all six
    LR-TS agents on the GPU (== the oracle on the reference's own update samples); the next
    iteration samples with the updated posterior."""
    import torch

    import auctiongym_amd.main as M
    d, meta, agg = load_capture("sp_ts_r2048")
    kat = np.load(os.path.join(GOLDEN, "sp_ts_update_kat.npz"))
    p = tmp_path / "SP_Truthful_TS.json"
    p.write_text(json.dumps(SP_TRUTHFUL_TS))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(meta["torch_seed"])
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    for i, a in enumerate(agents):
        assert np.array_equal(a.allocator.response_model.m.numpy(), d["ts_m"][i])
    auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for _ in range(meta["rounds"]):
        auction.simulate_opportunity()
    rt = dict(rtol=1e-11, atol=1e-12)
    np.testing.assert_allclose([a.net_utility for a in agents], agg["net_utility"], **rt)
    np.testing.assert_allclose([a.gross_utility for a in agents], agg["gross_utility"], **rt)
    np.testing.assert_allclose(auction.revenue, agg["revenue"], **rt)
    assert [a.num_logs() for a in agents] == list(agg["n_logs"])
    items = [[o.item for o in a.logs] for a in agents]
    for i in range(6):
        rows, slots = np.nonzero(d["part"] == i)
        assert items[i] == list(d["item"][rows, slots])
    for a in agents:
        a.update(iteration=0)
        a.clear_utility()
        a.clear_logs()
    auction.clear_revenue()
    for i, a in enumerate(agents):
        k = lambda n: kat[f"a{i}_{n}"]  # noqa: E731
        om, opm, oq, oep, _ = oracle.lrts_update(k("X"), k("A"), k("y"), k("m0"), k("prevm0"), k("q0"))
        rm = a.allocator.response_model
        assert a.allocator.epochs == oep
        assert np.array_equal(rm.m.numpy(), om) and np.array_equal(rm.q.numpy(), oq)
        assert np.array_equal(rm.prev_iter_m.numpy(), opm)
        np.testing.assert_allclose(rm.m.numpy(), k("m1"), atol=2e-2)
    # iteration 1: Thompson draws now use the updated q (std = 1/sqrt(q))
    auction.simulate_batch(1024)
    assert sum(a.num_logs() for a in agents) == 2 * 1024
    assert auction.revenue > 0
    for a in agents:
        a.update(iteration=1)
        a.clear_utility()
        a.clear_logs()
    assert all(a.allocator.epochs > 0 for a in agents)


@pytest.mark.parametrize("case", ["empirical", "lrts"])
def test_driver_memory_matches_reference(gpu, tmp_path, case):
    """Agent(memory=M) (src/Agent.py:124-129, config key 'memory', src/main.py:87) through the
    reference's driver loop: after clear_logs an agent keeps its last M records, in its
    metrics and in the records its next update trains on. Fixture: the reference's own run
    (tests/golden/make_golden.py --only memory). EmpiricalShaded (FirstPrice, M = 300):
    every iteration's revenue, utilities, metrics and new prev_gamma to 1e-9; LR-TS
    (SP_Truthful_TS, M = 150): log counts exact, iteration 0 metrics and utilities to 1e-9
    (the float32 CTRs are the reference's bit for bit), the later iterations (after float32 torch fits: parity unpinned beyond
    that) within 2 %."""
    import torch

    import auctiongym_amd.main as M
    kat = np.load(os.path.join(GOLDEN, "memory_driver_kat.npz"))
    cfg = json.loads(str(kat[f"{case}_cfg"]))
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    assert all(a.memory == cfg["agents"][0]["memory"] for a in agents)
    auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for it in range(cfg["num_iter"]):
        auction.simulate_batch(cfg["rounds_per_iter"])
        k = f"{case}_it{it}"
        tight = case == "empirical" or it == 0
        rt = dict(rtol=1e-9, atol=1e-9) if tight else dict(rtol=2e-2, atol=2e-2)
        np.testing.assert_allclose(auction.revenue, kat[k + "_revenue"], **rt)
        np.testing.assert_allclose([a.net_utility for a in agents], kat[k + "_net"], **rt)
        np.testing.assert_allclose([a.gross_utility for a in agents], kat[k + "_gross"], **rt)
        met = []
        for i, a in enumerate(agents):
            assert len(a.logs) == int(kat[k + f"_a{i}_nlogs"])  # participation: numpy draws only
            a.update(iteration=it)
            met.append([a.get_allocation_regret(), a.get_estimation_regret(), a.get_overbid_regret(),
                        a.get_underbid_regret(), a.get_CTR_RMSE(), a.get_CTR_bias(),
                        a.get_mean_best_expected_value()])
            if case == "empirical":
                assert a.bidder.prev_gamma == float(kat[k + f"_a{i}_pg"])
            elif it == 0:
                np.testing.assert_allclose(a.allocator.response_model.m.numpy(), kat[k + f"_a{i}_m"], atol=2e-2)
            a.clear_utility()
            a.clear_logs()
        np.testing.assert_allclose(np.array(met), kat[k + "_metrics"], **rt)
        auction.clear_revenue()


# ---- EmpiricalShadedBidder.update (src/Bidder.py:60-147) ----
def _empirical_engine(N=6):
    from auctiongym_amd.engine import AuctionEngine
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.zeros(N, np.int32), np.ones(N, np.int32), np.full(N, 0.9), np.full(N, 0.05))
    g = np.random.default_rng(0)
    eng.load_catalog(g.normal(size=(N, 12, 6)), g.random((N, 12)))
    return eng


def _fill_shading(eng, per_agent, seed=0):
    import torch
    ag = np.concatenate([np.full(len(gm), a, np.int32) for a, (gm, _) in per_agent.items()])
    gm = np.concatenate([np.asarray(gm, np.float64) for gm, _ in per_agent.values()])
    ut = np.concatenate([np.asarray(u, np.float64) for _, u in per_agent.values()])
    perm = np.random.default_rng(seed).permutation(len(ag))
    st = eng.new_shading_samples(max(len(ag), 1))
    if len(ag):
        st["agent"][:len(ag)] = torch.from_numpy(ag[perm]).to(eng.device)
        st["gamma"][:len(ag)] = torch.from_numpy(gm[perm]).to(eng.device)
        st["utility"][:len(ag)] = torch.from_numpy(ut[perm]).to(eng.device)
    st["count"][0] = len(ag)
    return st


def test_empirical_update_matches_oracle_and_reference(gpu, oracle):
    """Every (population, iteration) of empirical_update_kat.npz: the six agents' updates in
    one launch == the oracle == the reference's prev_gamma, bit for bit."""
    k = np.load(os.path.join(GOLDEN, "empirical_update_kat.npz"))
    eng = _empirical_engine()
    for ci in range(3):
        for it in range(3):
            per = {a: (k[f"c{ci}_it{it}_a{a}_gammas"], k[f"c{ci}_it{it}_a{a}_util"]) for a in range(6)}
            pg = eng.empirical_update(_fill_shading(eng, per, seed=ci * 3 + it))
            for a in range(6):
                want = float(k[f"c{ci}_it{it}_a{a}_pg1"])
                assert pg[a] == want == oracle.empirical_update(*per[a]), (ci, it, a)
    eng.close()


def test_empirical_update_errors(gpu):
    eng = _empirical_engine(N=2)
    g = np.random.default_rng(1)
    ok = (0.5 + 0.05 * g.standard_normal(500), g.normal(0, 0.1, 500))
    with pytest.raises(ValueError, match="All-NaN"):
        eng.empirical_update(_fill_shading(eng, {0: ok, 1: ([0.1, 0.2, 0.3], [0.0, 1.0, 0.0])}))
    with pytest.raises(ValueError, match="empty sequence"):
        eng.empirical_update(_fill_shading(eng, {0: ok, 1: ([0.5, 0.501], [0.1, 0.2])}))
    with pytest.raises(ValueError, match="zero-size"):
        eng.empirical_update(_fill_shading(eng, {0: ok}))
    eng.close()


@pytest.mark.parametrize("case", range(3))
def test_driver_empirical_three_iterations(gpu, tmp_path, case):
    """The reference's driver loop on an EmpiricalShadedBidder population for three
    iterations through the drop-in classes: each iteration's revenue and net utilities, and
    every agent's prev_gamma after each GPU update, equal the reference's."""
    import auctiongym_amd.main as M
    k = np.load(os.path.join(GOLDEN, "empirical_update_kat.npz"))
    cfg = json.loads(str(k[f"c{case}_cfg"]))
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, num_iter, rounds, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for it in range(num_iter):
        auction.simulate_batch(rounds)
        np.testing.assert_allclose(auction.revenue, float(k[f"c{case}_it{it}_revenue"]), rtol=1e-9)
        # reference: sequential float64 sums; here exact sums (north star: 1e-5 relative)
        np.testing.assert_allclose([a.net_utility for a in agents], k[f"c{case}_it{it}_net"], rtol=1e-9)
        for i, a in enumerate(agents):
            assert a.bidder.prev_gamma == float(k[f"c{case}_it{it}_a{i}_pg0"])
            a.update(iteration=it)
            assert a.bidder.prev_gamma == float(k[f"c{case}_it{it}_a{i}_pg1"]), (it, i)
            a.clear_utility()
            a.clear_logs()
        auction.clear_revenue()


@pytest.mark.parametrize("case", ["sp_oracle", "fp_empirical"])
def test_main_csv_outputs_match_reference(gpu, tmp_path, case):
    """auctiongym_amd.main writes the reference's CSV files (src/main.py:270-345): same file
    names, columns, row order and keys; every value within 1e-9 relative of the reference's
    own output (tests/golden/csv/<case>, produced by the reference's __main__; its sums are
    sequential float64, ours exact)."""
    import pandas as pd

    import auctiongym_amd.main as M
    src = os.path.join(GOLDEN, "csv", case)
    with open(os.path.join(src, "config.json")) as f:
        cfg = json.load(f)
    cfg["output_dir"] = str(tmp_path / "out")
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    M.main([str(p), "--quiet"])
    want = sorted(f for f in os.listdir(src) if f.endswith(".csv"))
    assert sorted(os.listdir(tmp_path / "out")) == want
    for fname in want:
        ref = pd.read_csv(os.path.join(src, fname))
        got = pd.read_csv(tmp_path / "out" / fname)
        assert list(got.columns) == list(ref.columns), fname
        assert len(got) == len(ref), fname
        for col in ref.columns:
            if ref[col].dtype == object:
                assert list(got[col]) == list(ref[col]), (fname, col)
            elif col in ("Run", "Iteration"):
                assert np.array_equal(got[col].to_numpy(), ref[col].to_numpy()), (fname, col)
            else:
                np.testing.assert_allclose(got[col].to_numpy(), ref[col].to_numpy(), rtol=1e-9,
                                           atol=1e-12, err_msg=f"{fname}:{col}")


# ---- DoublyRobustBidder.update (src/Bidder.py:473-615) ----
def _dr_noise(state, n, epochs):
    import torch
    saved = torch.get_rng_state()
    torch.set_rng_state(torch.from_numpy(np.asarray(state)))
    z = np.stack([torch.empty(n).normal_().numpy() for _ in range(epochs)])
    torch.set_rng_state(saved)
    return z


def test_dr_update_matches_oracle(gpu, oracle):
    """The three FP_DR_TS agents' first DoublyRobustBidder.update on the GPU (one launch, a
    workgroup per agent, three fits each) vs the oracle on the same records and noise, bit
    for bit: epochs of every fit, every epoch's loss, the final models."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    kat = np.load(os.path.join(GOLDEN, "dr_update_kat.npz"))
    N = 3
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), np.full(N, 4, np.int32), np.ones(N), np.full(N, 0.02))
    state0 = np.zeros((N, 16), np.float32)
    recs = {f: [] for f in ("agent", "gamma", "utility", "ctr", "value", "propensity", "won", "order")}
    noises, offs, E, orc = [], [], 0, []
    off = 0
    for a in range(N):
        k = lambda s: kat[f"a{a}_{s}"]  # noqa: E731
        n = len(k("est_ctr"))
        state0[a, :4] = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
        state0[a, 4:] = np.concatenate([k(f"pol0_{j}").ravel() for j in range(6)])
        for f, v in (("agent", np.full(n, a)), ("gamma", k("gamma")), ("utility", k("util")),
                     ("ctr", k("est_ctr")), ("value", k("value")), ("propensity", k("propensity")),
                     ("won", k("won")), ("order", 7 * np.arange(n) + a)):  # the agent's log order
            recs[f].append(v)
        Ea = len(k("dr_losses")) + 600
        z = _dr_noise(k("dr_rng_state"), n, 10300)  # every agent gets the same epoch budget
        noises.append(z.ravel())
        offs.append(off)
        off += z.size
        orc.append(oracle.dr_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("won"),
                                    k("util"), state0[a, :4], state0[a, 4:], False, z))
        E = 10300
        assert Ea <= E
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    n_tot = sum(len(v) for v in recs["agent"])
    st = eng.new_shading_samples(n_tot, learning=True)
    perm = np.random.default_rng(5).permutation(n_tot)
    dt = {"agent": np.int32, "won": np.uint8, "order": np.int64}
    for f, parts in recs.items():
        v = np.concatenate(parts).astype(dt.get(f, np.float64))[perm]
        st[f][:n_tot] = torch.from_numpy(v).to(eng.device)
    st["count"][0] = n_tot
    noise = torch.from_numpy(np.concatenate(noises)).to(eng.device)
    ep, tr = eng.dr_update(st, noise, offs, E, trace=True)
    state, ini = eng.dr_state()
    tr = tr.cpu().numpy()
    assert (ini == 1).all()
    for a in range(N):
        r = orc[a]
        assert list(ep[a]) == list(r["epochs"]), (a, ep[a], r["epochs"])
        assert np.array_equal(tr[a, 0, :ep[a, 0]], r["wr_losses"].astype(np.float32))
        assert np.array_equal(tr[a, 1, :ep[a, 1]], r["init_losses"].astype(np.float32))
        assert np.array_equal(tr[a, 2, :ep[a, 2]], r["dr_losses"].astype(np.float32))
        assert np.array_equal(state[a, :4], r["wr"]) and np.array_equal(state[a, 4:], r["pol"])
        # and the reference's own update (the oracle's pinned tolerances)
        k = lambda s: kat[f"a{a}_{s}"]  # noqa: E731
        assert ep[a, 2] == len(k("dr_losses"))
        pol1 = np.concatenate([k(f"pol1_{j}").ravel() for j in range(6)])
        np.testing.assert_allclose(state[a, 4:], pol1, atol=2e-6)
    eng.close()


# ---- ValueLearningBidder / PolicyLearningBidder updates (src/Bidder.py:204-325, :364-431) ----
def test_vl_pl_update_matches_oracle(gpu, oracle):
    """One ag_bidder_update launch over a population of FP_DM_TS's three ValueLearningBidders
    ('policy'), FP_IPS_TS's three PolicyLearningBidders ('PPO') and a ValueLearningBidder that
    won nothing (the reference's fallback), on the reference's own logs (tests/golden/
    dm_update_kat.npz, ips_update_kat.npz), records shuffled: every fit's epochs and
    per-epoch losses and the final models equal the oracle's bit for bit; the fallback
    agent trains nothing and reverts to Gaussian shading; the fitted agents bid from their
    policies afterwards. Against the reference: the pinned tolerances of
    tests/test_oracle_golden.py (DM agent 2: same epochs, losses within 1e-7)."""
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    dm = np.load(os.path.join(GOLDEN, "dm_update_kat.npz"))
    ips = np.load(os.path.join(GOLDEN, "ips_update_kat.npz"))
    N = 7
    bk = np.array([2, 2, 2, 3, 3, 3, 2], np.int32)
    modes = np.array([_lib.VL_POLICY] * 3 + [_lib.PL_LOSSES["PPO"]] * 3 + [_lib.VL_POLICY], np.int32)
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), bk, np.ones(N), np.full(N, 0.02))
    state0 = np.zeros((N, 16), np.float32)
    recs = {f: [] for f in ("agent", "gamma", "utility", "ctr", "value", "propensity", "won", "order")}
    noises, offs, off, orc = [], [], 0, []
    E = 0
    for a in range(N):
        kat, j = (dm, a) if a < 3 else ((ips, a - 3) if a < 6 else (dm, 1))
        k = lambda s: kat[f"a{j}_{s}"]  # noqa: E731
        n = len(k("est_ctr"))
        won = k("won") if a < 6 else np.zeros(n, np.int8)
        if a < 3 or a == 6:
            state0[a, :4] = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
            state0[a, 4:] = np.concatenate([k(f"pol0_{i}").ravel() for i in (0, 1, 4, 5, 8, 9)])
            Ea = len(k("fit1_losses")) + 300
            z = _dr_noise(k("fit1_rng"), n, 3800)
            assert Ea <= 3800
            E = 3800
            orc.append(oracle.vl_update(k("est_ctr"), k("value"), k("gamma"), won, state0[a, :4], state0[a, 4:],
                                        True, z))
        else:
            state0[a, 4:] = np.concatenate([k(f"pol0_{i}").ravel() for i in range(6)])
            z = np.zeros((0, n), np.float32)
            orc.append(oracle.pl_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("util"),
                                        state0[a, 4:], False, "PPO"))
        noises.append(z.ravel())
        offs.append(off)
        off += z.size
        for f, v in (("agent", np.full(n, a)), ("gamma", k("gamma")), ("utility", k("util")),
                     ("ctr", k("est_ctr")), ("value", k("value")), ("propensity", k("propensity")),
                     ("won", won), ("order", 5 * np.arange(n) + a)):
            recs[f].append(v)
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    eng.set_bidder_modes(modes)
    n_tot = sum(len(v) for v in recs["agent"])
    st = eng.new_shading_samples(n_tot, learning=True)
    perm = np.random.default_rng(6).permutation(n_tot)
    dt = {"agent": np.int32, "won": np.uint8, "order": np.int64}
    for f, parts in recs.items():
        v = np.concatenate(parts).astype(dt.get(f, np.float64))[perm]
        st[f][:n_tot] = torch.from_numpy(v).to(eng.device)
    st["count"][0] = n_tot
    noise = torch.from_numpy(np.concatenate(noises)).to(eng.device)
    ep, stat, tr = eng.bidder_update(st, noise, offs, E, trace=True)
    state, ini = eng.dr_state()
    tr = tr.cpu().numpy()
    assert list(stat) == [0, 0, 0, 0, 0, 0, 1]
    assert list(ini) == [1, 1, 1, 1, 1, 1, 0]
    for a in range(6):
        r = orc[a]
        assert list(ep[a]) == list(r["epochs"]), (a, ep[a], r["epochs"])
        if a < 3:
            assert np.array_equal(tr[a, 0, :ep[a, 0]], r["wr_losses"].astype(np.float32))
            assert np.array_equal(tr[a, 2, :ep[a, 2]], r["pol_losses"].astype(np.float32))
            assert np.array_equal(state[a, :4], r["wr"])
        else:
            assert np.array_equal(tr[a, 1, :ep[a, 1]], r["init_losses"].astype(np.float32))
            assert np.array_equal(tr[a, 2, :ep[a, 2]], r["pl_losses"].astype(np.float32))
        assert np.array_equal(state[a, 4:], r["pol"]), a
    assert list(ep[6]) == [0, 0, 0] and np.array_equal(state[6], state0[6])
    k = lambda s: dm[f"a2_{s}"]  # noqa: E731  the reference, DM agent 2
    assert ep[2, 0] == len(k("fit0_losses")) and ep[2, 2] == len(k("fit1_losses"))
    np.testing.assert_allclose(tr[2, 2, :ep[2, 2]], k("fit1_losses"), atol=1e-7)
    eng.close()


def test_bidder_update_errors(gpu):
    """Loud failures where the reference fails: a learning bidder without logs, an unknown
    PolicyLearningBidder loss, a ValueLearningBidder inference that is neither mode."""
    import torch
    from auctiongym_amd.engine import AuctionEngine
    N = 3
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.zeros(N, np.int32), np.array([2, 3, 0], np.int32), np.ones(N), np.full(N, 0.02))
    eng.set_dr_state(np.zeros((N, 16), np.float32), np.zeros(N, np.int32))
    with pytest.raises(NotImplementedError, match="PolicyLearningBidder loss"):
        eng.set_bidder_modes([0, 7, 0])
    with pytest.raises(ValueError, match="inference"):
        eng.set_bidder_modes([5, 3, 0])
    st = eng.new_shading_samples(16, learning=True)
    with pytest.raises(ValueError, match="without logs"):
        eng.bidder_update(st, torch.zeros(1, device=eng.device), [0, 0, 0], 0)
    eng.close()


# ---- drop-in driver on the learning-bidder configs (FP_DR_TS, FP_DM_TS, FP_IPS_TS) ----
def _run_driver_learners(tag, tmp_path, check):
    import torch
    import auctiongym_amd.main as M
    k = np.load(os.path.join(GOLDEN, f"{tag}_driver_kat.npz"))
    cfg = json.loads(str(k["cfg"]))
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, num_iter, rounds, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    for it in range(num_iter):
        auction.simulate_batch(rounds)
        check(k, it, auction, agents, rng, None)
        for i, a in enumerate(agents):
            a.update(iteration=it)
            check(k, it, auction, agents, rng, i)
            a.clear_utility()
            a.clear_logs()
        auction.clear_revenue()


def test_driver_fp_dr_ts(gpu, tmp_path):
    """FP_DR_TS (3 LR-TS allocators + DoublyRobustBidders, FirstPrice) through the drop-in
    driver for 3 iterations x 1000 rounds vs the reference's own run (tests/golden/
    dr_driver_kat.npz): the numpy draw order stays aligned every iteration; iteration 0
    (Gaussian shading) matches to 1e-8; every agent's first update runs the reference's
    number of DR-fit epochs on the same torch draws and leaves torch's generator where the
    reference's is; iteration 1 (bids from the fitted policies) within 1e-4. Later updates'
    stopping epochs are chaotic in float32 (a 1e-6 improvement rule) and drift apart
    (measured: iteration 2 revenue within 2.6e-3)."""
    import torch

    def check(k, it, auction, agents, rng, i):
        if i is None:
            assert json.dumps(rng.bit_generator.state) == str(k[f"it{it}_np_state"])
            tol = {0: 1e-8, 1: 1e-4, 2: 2e-2}[it]
            np.testing.assert_allclose(auction.revenue, float(k[f"it{it}_revenue"]), rtol=tol)
            if it == 0:
                np.testing.assert_allclose([a.net_utility for a in agents], k["it0_net"], rtol=1e-8)
        elif it == 0:
            b = agents[i].bidder
            assert b.model_initialised and b.epochs[2] == k[f"it0_a{i}_fits"][1]
            assert np.array_equal(torch.get_rng_state().numpy(), k[f"it0_a{i}_torch_state"])
    _run_driver_learners("dr", tmp_path, check)


def test_driver_fp_dm_ts(gpu, tmp_path):
    """FP_DM_TS (ValueLearningBidder 'policy') through the drop-in driver vs the reference's own
    run, 3 iterations x 1000 rounds: the numpy and torch generators stay aligned through
    every round and every update (each policy fit runs the reference's epoch count on the
    same draws); revenue within 1e-8 in iteration 0 and 1e-4 afterwards (measured 7e-6)."""
    import torch

    def check(k, it, auction, agents, rng, i):
        if i is None:
            assert json.dumps(rng.bit_generator.state) == str(k[f"it{it}_np_state"])
            np.testing.assert_allclose(auction.revenue, float(k[f"it{it}_revenue"]), rtol=1e-8 if it == 0 else 1e-4)
        else:
            b = agents[i].bidder
            assert b.model_initialised and b.epochs[2] == k[f"it{it}_a{i}_fits"][1]
            assert np.array_equal(torch.get_rng_state().numpy(), k[f"it{it}_a{i}_torch_state"])
    _run_driver_learners("dm", tmp_path, check)


def test_driver_fp_ips_ts(gpu, tmp_path):
    """FP_IPS_TS (PolicyLearningBidder, PPO) through the drop-in driver vs the reference's own
    run, 3 iterations x 1000 rounds: both generators stay aligned throughout (the PPO fit
    draws nothing; the post-fit rsample of every record is replayed); revenue within 1e-8
    in iteration 0 and 1e-3 afterwards (measured 7.7e-5)."""
    import torch

    def check(k, it, auction, agents, rng, i):
        if i is None:
            assert json.dumps(rng.bit_generator.state) == str(k[f"it{it}_np_state"])
            np.testing.assert_allclose(auction.revenue, float(k[f"it{it}_revenue"]), rtol=1e-8 if it == 0 else 1e-3)
        else:
            assert agents[i].bidder.model_initialised
            assert np.array_equal(torch.get_rng_state().numpy(), k[f"it{it}_a{i}_torch_state"])
            if it == 0:
                assert agents[i].bidder.epochs[1] == int(k[f"it0_a{i}_imitation"])
    _run_driver_learners("ips", tmp_path, check)


def test_search_bids_match_oracle(gpu, oracle):
    """ValueLearningBidder 'search' bids (src/Bidder.py:180-196): the gamma maximising the
    win-rate model's utility over the 128-point grid. Population of OracleAllocator +
    ValueLearningBidders, half bidding by search (random win-rate models), the rest with
    Gaussian shading; synthetic contexts, draws and (unsorted) grids; every output equal to
    the oracle's on the same inputs."""
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    N, P, K, E, OE, B = 8, 3, 12, 5, 4, 1 << 16
    g = np.random.default_rng(44)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    ak = np.zeros(N, np.int32)
    bk = np.full(N, 2, np.int32)
    pg, gs = np.ones(N), np.full(N, 0.02)
    state = g.normal(0, 2.0, (N, 16)).astype(np.float32)
    init = np.array([2 if a % 2 == 0 else 0 for a in range(N)], np.int32)
    eng = AuctionEngine(N, P, K, E, OE, 0, 1.0)
    eng.set_agent_params(ak, bk, pg, gs)
    eng.load_catalog(items, values)
    eng.set_dr_state(state, init)
    eng.set_bidder_modes(np.full(N, _lib.VL_SEARCH, np.int32))
    inp = eng.alloc_inputs(B)
    assert "gamma_grid" in inp
    eng.generate(3, 0, inp)
    eng.generate_noise(3, 0, inp)
    eng.generate_search_grid(3, 0, inp)
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    T = lambda t: np.ascontiguousarray(t.cpu().numpy().T)  # noqa: E731
    grid = np.ascontiguousarray(inp["gamma_grid"].cpu().numpy().transpose(2, 0, 1))  # [B][P][128]
    assert grid.min() >= 0.1 and grid.max() < 1.0
    orc = oracle.simulate_pop(0, items, values, T(inp["ctx"]), T(inp["part"]), inp["u"].cpu().numpy(),
                              ak, bk, pg, gs, OE=OE, gamma_raw=T(inp["gamma_raw"]), dr_state=state,
                              dr_init=init, gamma_grid=grid, nthreads=16)
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
        assert np.array_equal(np.ascontiguousarray(got[k].T), orc[k], equal_nan=True), k
    for k in ("winner", "price", "second_price", "outcome"):
        assert np.array_equal(got[k], orc[k], equal_nan=True), k
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"])
    part = T(inp["part"])
    searched = init[part] == 2
    gam = np.ascontiguousarray(got["gamma"].T)
    prop = np.ascontiguousarray(got["propensity"].T)
    assert searched.any() and (prop[searched] == 1.0).all()
    assert (gam[searched][:, None] == grid[searched]).any(axis=1).all()  # one of its grid points
    # without a grid the launch is refused
    del inp["gamma_grid"]
    with pytest.raises(ValueError, match="gamma_grid"):
        eng.simulate(inp, out, eng.new_counters())
    eng.close()


def test_driver_fp_dm_oracle(gpu, tmp_path):
    """FP_DM_Oracle (OracleAllocator + ValueLearningBidder 'search') through the drop-in driver
    vs the reference's own run, 3 iterations x 1000 rounds: the numpy draw order (128 grid
    draws per searching participant) stays aligned; revenue within 1e-8 in iteration 0 and
    1e-3 afterwards (measured 2.4e-5); the win-rate models after each update within 5e-2
    (their fits stop by the chaotic 1e-6 rule: measured up to 4.7e-2 apart in iteration 2)."""
    def check(k, it, auction, agents, rng, i):
        if i is None:
            assert json.dumps(rng.bit_generator.state) == str(k[f"it{it}_np_state"])
            np.testing.assert_allclose(auction.revenue, float(k[f"it{it}_revenue"]), rtol=1e-8 if it == 0 else 1e-3)
        else:
            b = agents[i].bidder
            assert b.model_initialised == bool(k[f"it{it}_a{i}_init"])
            np.testing.assert_allclose(b._state16()[:4], k[f"it{it}_a{i}_winrate_model"], atol=5e-2)
    _run_driver_learners("dmo", tmp_path, check)


def _learner_store(eng, recs):
    import torch
    n_tot = sum(len(v) for v in recs["agent"])
    st = eng.new_shading_samples(n_tot, learning=True)
    perm = np.random.default_rng(9).permutation(n_tot)
    dt = {"agent": np.int32, "won": np.uint8, "order": np.int64}
    for f, parts in recs.items():
        v = np.concatenate(parts).astype(dt.get(f, np.float64))[perm]
        st[f][:n_tot] = torch.from_numpy(v).to(eng.device)
    st["count"][0] = n_tot
    return st


def _kat_learners(specs):
    """specs: [(kind, kat file, kat agent)] -> engine inputs: bidder kinds, modes, state0 [N][16],
    records {field: [per agent]}, per-agent data dicts."""
    from auctiongym_amd import _lib
    N = len(specs)
    bk = np.array([{"dm": 2, "ips": 3, "dr": 4}[s[0]] for s in specs], np.int32)
    modes = np.array([_lib.VL_POLICY if s[0] == "dm" else (_lib.PL_LOSSES["PPO"] if s[0] == "ips" else 0)
                      for s in specs], np.int32)
    state0 = np.zeros((N, 16), np.float32)
    recs = {f: [] for f in ("agent", "gamma", "utility", "ctr", "value", "propensity", "won", "order")}
    data = []
    for a, (kind, fname, j) in enumerate(specs):
        kat = np.load(os.path.join(GOLDEN, fname))
        k = lambda s, kat=kat, j=j: kat[f"a{j}_{s}"]  # noqa: E731
        n = len(k("est_ctr"))
        if kind == "ips":
            state0[a, 4:] = np.concatenate([k(f"pol0_{i}").ravel() for i in range(6)])
        else:
            state0[a, :4] = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
            idx = (0, 1, 4, 5, 8, 9) if kind == "dm" else range(6)
            state0[a, 4:] = np.concatenate([k(f"pol0_{i}").ravel() for i in idx])
        for f, v in (("agent", np.full(n, a)), ("gamma", k("gamma")), ("utility", k("util")),
                     ("ctr", k("est_ctr")), ("value", k("value")), ("propensity", k("propensity")),
                     ("won", k("won")), ("order", N * np.arange(n) + a)):
            recs[f].append(v)
        data.append(k)
    return bk, modes, state0, recs, data


def test_bidder_update_multi_workgroup(gpu, oracle):
    """The learning bidders' trainer with every agent split over several cooperating
    workgroups (200 records each): DM and DR fits (exact sums) give the single-workgroup
    oracle's results bit for bit; the PPO fit's fixed-order sums follow the split, equal to
    the oracle run with the same number of workgroups."""
    _learners_vs_oracle(oracle, 200, -1)


@pytest.mark.parametrize("cache", [0, 512])
def test_bidder_update_record_cache(gpu, oracle, cache):
    """One workgroup per learning bidder with its record cache in LDS capped (512 records:
    the rest of each epoch read from the store; 0: every record from the store): the same
    bits as the oracle."""
    _learners_vs_oracle(oracle, 1 << 30, cache)


def _learners_vs_oracle(oracle, block, cache):
    import torch
    from auctiongym_amd.engine import AuctionEngine
    specs = [("dm", "dm_update_kat.npz", 2), ("ips", "ips_update_kat.npz", 0), ("ips", "ips_update_kat.npz", 1),
             ("dr", "dr_update_kat.npz", 0)]
    bk, modes, state0, recs, data = _kat_learners(specs)
    N = len(specs)
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), bk, np.ones(N), np.full(N, 0.02))
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    eng.set_bidder_modes(modes)
    eng.set_bidder_block_samples(block)
    eng.set_bidder_record_cache(cache)
    E = 10300
    noises, offs, off, orc = [], [], 0, []
    for a, (kind, _, _) in enumerate(specs):
        k = data[a]
        n = len(k("est_ctr"))
        nblk = (n + block - 1) // block
        if kind == "dm":
            z = _dr_noise(k("fit1_rng"), n, E)
            orc.append(oracle.vl_update(k("est_ctr"), k("value"), k("gamma"), k("won"), state0[a, :4], state0[a, 4:],
                                        True, z[:3800]))
        elif kind == "dr":
            z = _dr_noise(k("dr_rng_state"), n, E)
            orc.append(oracle.dr_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("won"), k("util"),
                                        state0[a, :4], state0[a, 4:], False, z))
        else:
            z = np.zeros((0, n), np.float32)
            orc.append(oracle.pl_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("util"),
                                        state0[a, 4:], False, "PPO", nblk=nblk))
        noises.append(z.ravel())
        offs.append(off)
        off += z.size
    st = _learner_store(eng, recs)
    noise = torch.from_numpy(np.concatenate(noises)).to(eng.device)
    ep, stat, tr = eng.bidder_update(st, noise, offs, E, trace=True)
    state, ini = eng.dr_state()
    tr = tr.cpu().numpy()
    assert list(stat) == [0] * N and list(ini) == [1] * N
    for a, (kind, _, _) in enumerate(specs):
        r = orc[a]
        assert list(ep[a]) == list(r["epochs"]), (a, ep[a], r["epochs"])
        for slot, key in ((0, "wr_losses"), (1, "init_losses"), (2, {"dm": "pol_losses", "dr": "dr_losses",
                                                                    "ips": "pl_losses"}[kind])):
            if key in r:
                assert np.array_equal(tr[a, slot, :ep[a, slot]], r[key].astype(np.float32)), (a, key)
        assert np.array_equal(state[a, 4:], r["pol"]), a
        if kind != "ips":
            assert np.array_equal(state[a, :4], r["wr"]), a
    eng.close()


def test_bidder_update_synthetic_noise(gpu, oracle):
    """ag_bidder_update without caller noise: the DR and DM fits draw their rsample noise on
    the device (Philox4x32-10 + polar method, keyed by the fit-noise seed); equal bit for bit
    to the oracle fed ora_fit_noise's draws of the same seed."""
    from auctiongym_amd.engine import AuctionEngine
    specs = [("dm", "dm_update_kat.npz", 1), ("dr", "dr_update_kat.npz", 1)]
    bk, modes, state0, recs, data = _kat_learners(specs)
    N = len(specs)
    eng = AuctionEngine(N, 2, 12, 5, 4, 0, 1.0)
    eng.set_agent_params(np.ones(N, np.int32), bk, np.ones(N), np.full(N, 0.02))
    eng.set_dr_state(state0, np.zeros(N, np.int32))
    eng.set_bidder_modes(modes)
    eng.set_fit_noise_seed(77)
    st = _learner_store(eng, recs)
    ep, stat, tr = eng.bidder_update(st, None, np.zeros(N, np.int64), 0, trace=True)
    state, _ = eng.dr_state()
    tr = tr.cpu().numpy()
    assert list(stat) == [0, 0]
    k0, k1 = data
    n0, n1 = len(k0("est_ctr")), len(k1("est_ctr"))
    r0 = oracle.vl_update(k0("est_ctr"), k0("value"), k0("gamma"), k0("won"), state0[0, :4], state0[0, 4:], True,
                          oracle.fit_noise(77, 0, int(ep[0, 2]) + 1, n0))
    r1 = oracle.dr_update(k1("est_ctr"), k1("value"), k1("gamma"), k1("propensity"), k1("won"), k1("util"),
                          state0[1, :4], state0[1, 4:], False, oracle.fit_noise(77, 1, int(ep[1, 2]) + 1, n1))
    assert list(ep[0]) == list(r0["epochs"]) and list(ep[1]) == list(r1["epochs"])
    assert np.array_equal(tr[0, 2, :ep[0, 2]], r0["pol_losses"].astype(np.float32))
    assert np.array_equal(tr[1, 2, :ep[1, 2]], r1["dr_losses"].astype(np.float32))
    assert np.array_equal(state[0, 4:], r0["pol"]) and np.array_equal(state[1, 4:], r1["pol"])
    z = oracle.fit_noise(77, 0, 3, n0)
    assert abs(z.mean()) < 0.05 and abs(z.std() - 1) < 0.05
    eng.close()


# ---- the per-call plugin surface (src/BidderAllocation.py:67-82, src/Bidder.py bid / update,
# src/Agent.py:29-68), outside a batched Auction ----
def test_per_call_estimate_and_bid_match_reference(gpu, oracle):
    """OracleAllocator.estimate_CTR, Agent.select_item and Agent.bid called one request at a
    time (B = 1 calls into the kernels) reproduce the reference's own capture bit for bit:
    items, estimated CTRs and bids of SP_Oracle's first 300 rounds; the shading bidders'
    Gaussian-shading bids (the rng.normal draw patched to the recorded one) equal the
    reference's bids, and their propensities the oracle's."""
    import types
    from auctiongym_amd.Agent import Agent
    from auctiongym_amd.Bidder import DoublyRobustBidder, TruthfulBidder
    from auctiongym_amd.BidderAllocation import OracleAllocator
    d, meta, _ = load_capture("sp_oracle_r4096")
    agents = []
    for a in range(meta["N"]):
        al = OracleAllocator(None)
        al.update_item_embeddings(d["items"][a])
        agents.append(Agent(None, f"A{a}", meta["K"], d["values"][a], al, TruthfulBidder(None)))
    for r in range(300):
        x = np.concatenate([d["ctx"][r], [1.0]])
        for s_ in range(meta["P"]):
            ag = agents[d["part"][r, s_]]
            ctr = ag.allocator.estimate_CTR(x)
            item, est = ag.select_item(x)
            assert item == d["item"][r, s_] and est == d["slot_est_ctr"][r, s_] == ctr[item]
            b, it2 = ag.bid(x)
            assert it2 == item and b == d["slot_bid"][r, s_]
    assert len(agents[0].logs) == sum((d["part"][:300] == 0).ravel())  # per-call records are logged
    # Gaussian shading of an uninitialised DoublyRobustBidder (FP_DR_TS capture)
    d, meta, _ = load_capture("fp_dr_ts_r1024")
    kw = meta["bidder_kwargs"][0]
    args = pop_args(d, meta)
    orc = oracle.simulate_pop(0, d["items"], d["values"], d["ctx"], d["part"], d["u"], **args)
    for r in range(200):
        for s_ in range(meta["P"]):
            bd = DoublyRobustBidder(None, **kw)
            bd.rng = types.SimpleNamespace(normal=lambda loc, sc, g=d["gamma_raw"][r, s_]: g)
            b = bd.bid(d["slot_value"][r, s_], None, d["slot_est_ctr"][r, s_])
            assert b == d["slot_bid"][r, s_]
            assert bd.gammas == [d["gamma_raw"][r, s_]]
            assert bd.propensities[0] == orc["propensity"][r, s_]


def test_per_call_lrts_estimate_matches_oracle_forward(gpu, oracle):
    """PyTorchLogisticRegressionAllocator.estimate_CTR on the GPU against ora_ts_ctr -- the
    reference's forward `torch.sigmoid(F.linear(x32, m [+ normal(0, 1/sqrt(q))]))`
    (src/BidderAllocation.py:67-68, src/Models.py:28-33) as torch computes it on the golden
    fixtures' machine (tests/test_oracle_golden.py::test_ts_forward_matches_torch pins it
    there) -- bit for bit: item counts with and without a remainder after the sgemv's 4-row
    blocks, the Thompson draw and the MAP forward, posteriors of several widths (q). Not
    compared with the box's own torch: MKL's sgemv summation order depends on the host CPU
    (this box's AMD EPYC sums in order; the Intel host that ran the reference here does not)."""
    import torch
    from auctiongym_amd.BidderAllocation import PyTorchLogisticRegressionAllocator
    L = oracle.lib()
    g = np.random.default_rng(8)
    for K in (1, 2, 3, 5, 7, 11, 12):
        torch.manual_seed(K)
        al = PyTorchLogisticRegressionAllocator(None, 4, K)
        rm = al.response_model
        rm.q = torch.from_numpy(g.uniform(1.0, 400.0, (K, 5)).astype(np.float32))
        for r in range(40):
            x = np.concatenate([g.normal(0, 1, 4), [1.0]])
            x32 = x.astype(np.float32)
            for sample in (True, False):
                state = torch.get_rng_state()
                got = al.estimate_CTR(x, sample=sample)
                torch.set_rng_state(state)
                w = rm.m + torch.normal(mean=0.0, std=1.0 / torch.sqrt(rm.q)) if sample else rm.m
                W = np.ascontiguousarray(w.numpy(), np.float32)
                want = np.array([L.ora_ts_ctr(W[k].ctypes.data, x32.ctypes.data, 5, k, K) for k in range(K)],
                                np.float32)
                assert got.dtype == np.float32 and np.array_equal(got, want), (K, r, sample)


def test_per_call_lrts_estimate_matches_simulate(gpu, oracle):
    """PyTorchLogisticRegressionAllocator.estimate_CTR (Thompson draw patched to the recorded
    torch.normal noise) and Agent.select_item on SP_Truthful_TS's capture: the items the
    reference chose and the MAP CTRs the oracle computes, bit for bit."""
    from auctiongym_amd.Agent import Agent
    from auctiongym_amd.Bidder import TruthfulBidder
    from auctiongym_amd.BidderAllocation import PyTorchLogisticRegressionAllocator
    import torch
    d, meta, _ = load_capture("sp_ts_r2048")
    args = pop_args(d, meta)
    orc = oracle.simulate_pop(mech_code(meta), d["items"], d["values"], d["ctx"], d["part"], d["u"], **args)
    OE, K = meta["OE"], meta["K"]
    agents = []
    for a in range(meta["N"]):
        al = PyTorchLogisticRegressionAllocator(None, OE, K)
        al.response_model.m = torch.from_numpy(np.ascontiguousarray(args["ts_m"][a], np.float32))
        al.response_model.prev_iter_m = al.response_model.m.clone()
        al.response_model.q = torch.ones(K, OE + 1)
        agents.append(Agent(None, f"TS{a}", K, d["values"][a], al, TruthfulBidder(None)))
    for r in range(200):
        x = np.concatenate([d["ctx"][r, :OE], [1.0]])
        for s_ in range(meta["P"]):
            ag = agents[d["part"][r, s_]]
            z = torch.from_numpy(np.ascontiguousarray(d["ts_noise"][r, s_].reshape(K, OE + 1), np.float32))
            ag.allocator.response_model.sample_noise = lambda z=z: z
            item, est = ag.select_item(x)
            assert item == d["item"][r, s_] == orc["item"][r, s_]
            assert est == np.float32(orc["est_ctr"][r, s_])


def test_plugin_level_updates_match_oracle(gpu, oracle):
    """The reference's plugin-level update(...) calls, made directly on a plugin: the LR-TS
    allocator (sp_ts_update_kat), EmpiricalShadedBidder (empirical_update_kat) and a
    DoublyRobustBidder (dr_update_kat, its torch rsample noise drawn from the recorded
    generator state) train on the GPU and equal the oracle / the reference bit for bit."""
    import torch
    from auctiongym_amd.Bidder import DoublyRobustBidder, EmpiricalShadedBidder
    from auctiongym_amd.BidderAllocation import PyTorchLogisticRegressionAllocator
    kat = np.load(os.path.join(GOLDEN, "sp_ts_update_kat.npz"))
    X, A, y = kat["a0_X"], kat["a0_A"], kat["a0_y"]
    K, Do = kat["a0_m0"].shape
    al = PyTorchLogisticRegressionAllocator(None, Do - 1, K)
    rm = al.response_model
    rm.m = torch.from_numpy(kat["a0_m0"].copy())
    rm.prev_iter_m = torch.from_numpy(kat["a0_prevm0"].copy())
    rm.q = torch.from_numpy(kat["a0_q0"].copy())
    al.update(X, A, y, 0)
    om, opm, oq, oep, _ = oracle.lrts_update(X, A, y, kat["a0_m0"], kat["a0_prevm0"], kat["a0_q0"])
    assert al.epochs == oep
    assert np.array_equal(rm.m.numpy(), om) and np.array_equal(rm.q.numpy(), oq)
    assert np.array_equal(rm.prev_iter_m.numpy(), opm)
    # EmpiricalShadedBidder
    ek = np.load(os.path.join(GOLDEN, "empirical_update_kat.npz"))
    for a in range(3):
        g, u = ek[f"c0_it0_a{a}_gammas"], ek[f"c0_it0_a{a}_util"]
        b = EmpiricalShadedBidder(None, gamma_sigma=0.05, init_gamma=float(ek[f"c0_it0_a{a}_pg0"]))
        b.gammas = list(g)
        n = len(g)  # utility = value * outcome - price on won records: value = u, outcome 1, price 0
        b.update(None, u, None, np.zeros(n), np.ones(n), None, np.ones(n, bool), 0)
        assert b.prev_gamma == float(ek[f"c0_it0_a{a}_pg1"])
    # DoublyRobustBidder
    dk = np.load(os.path.join(GOLDEN, "dr_update_kat.npz"))
    k = lambda s: dk[f"a0_{s}"]  # noqa: E731
    b = DoublyRobustBidder(None, gamma_sigma=0.02, init_gamma=1.0)
    st0 = np.zeros(16, np.float32)
    st0[:4] = np.concatenate([k("wr0_0").ravel(), k("wr0_1").ravel()])
    st0[4:] = np.concatenate([k(f"pol0_{j}").ravel() for j in range(6)])
    b._load_state16(st0)
    b.gammas, b.propensities = list(k("gamma")), list(k("propensity"))
    n = len(b.gammas)
    torch.set_rng_state(torch.from_numpy(np.asarray(k("dr_rng_state"))))
    b.update(None, k("value"), None, k("price"), k("outcome"), k("est_ctr"), k("won").astype(bool), 0)
    after = torch.get_rng_state()
    z = _dr_noise(k("dr_rng_state"), n, int(b.epochs[2]) + 1)
    orc = oracle.dr_update(k("est_ctr"), k("value"), k("gamma"), k("propensity"), k("won"), k("util"),
                           st0[:4], st0[4:], False, z[:-1])
    assert list(b.epochs) == list(orc["epochs"])
    assert np.array_equal(b._state16()[:4], orc["wr"]) and np.array_equal(b._state16()[4:], orc["pol"])
    assert b.model_initialised
    # the generator is where the reference leaves it: the fit's draws + one rsample of every record
    torch.set_rng_state(torch.from_numpy(np.asarray(k("dr_rng_state"))))
    for _ in range(int(b.epochs[2]) + 1):
        torch.empty(n).normal_()
    assert torch.equal(torch.get_rng_state(), after)


POP_CASES = [  # (P, mech, ts_sample, compact, block, B, launch cap, counters, population)
    (2, 1, True, False, 0, (1 << 18) + 37, 0, True, "ts"),          # SP_Truthful_TS shape
    (2, 0, True, False, 0, 70001, 0, True, "dm"),                   # FP_DM_TS, fitted policies
    (2, 0, True, True, 1024, 70001, 25000, True, "mix"),            # the mixed population
    (8, 0, True, True, 0, 40003, 0, True, "mix"),
    (3, 1, False, False, 256, 30011, 7777, True, "mix"),            # MAP item choice (no sampling)
    (1, 0, True, False, 0, 20000, 0, True, "mix"),                  # P = 1: nobody charged
    (2, 0, True, False, 0, 30000, 0, False, "search"),              # 'search' bids, no counters
    (5, 1, True, True, 1024, 50000, 0, True, "all"),                # every bidder kind / state
    (8, 1, True, False, 0, (1 << 17) + 5, 0, True, "ts"),           # configs_1 at P = 8 (streamed slots)
    (8, 0, True, True, 1024, 33333, 11111, True, "all"),
]


@pytest.mark.parametrize("case", POP_CASES)
def test_general_kernel_builds_agree(gpu, oracle, case):
    """k_simulate's builds for general populations of the shipped catalogue shape (K = 12,
    E = 5, OE = 4): the AUTO choice and AG_SIM_KERNEL_GENERIC (the compile-time LR-TS width
    build, DOS = 5; streamed slots for TruthfulBidder-only populations at P >= 3) against the
    runtime-width build on the same inputs: every output and the exact counter limbs bit for bit -- LR-TS + truthful, fitted-policy and search
    bidders, Gaussian shading, Oracle agents among them, 1..8 participants, both mechanisms,
    with and without Thompson sampling, dense and compact noise, both workgroup sizes, ragged B,
    batches split over several launches, with and without counters. k_simulate is pinned to the
    oracle by the tests above; one case is also compared with the oracle directly."""
    import torch
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    P, mech, sample, compact, block, B, cap, counters, pop = case
    N, K, E, OE = {"ts": 8, "dm": 3, "mix": 32, "search": 6, "all": 20}[pop], 12, 5, 4
    g = np.random.default_rng(1000 + P * 7 + B % 97)
    items = np.concatenate([g.normal(0, 1, (N, K, E)), -3.0 - g.random((N, K, 1))], axis=2)
    values = g.lognormal(0.1, 0.2, (N, K))
    if pop == "ts":
        ak, bk = np.ones(N, np.int32), np.zeros(N, np.int32)
    elif pop == "dm":
        ak, bk = np.ones(N, np.int32), np.full(N, 2, np.int32)
    elif pop == "search":
        ak, bk = np.array([i % 2 for i in range(N)], np.int32), np.full(N, 2, np.int32)
    elif pop == "mix":
        ak = np.array([0 if i < 11 else 1 for i in range(N)], np.int32)
        bk = np.array([4 if i >= 22 else 0 for i in range(N)], np.int32)
    else:
        ak = np.array([i % 2 for i in range(N)], np.int32)
        bk = np.array([(i // 2) % 5 for i in range(N)], np.int32)
    pg = 0.5 + 0.5 * g.random(N)
    gs = 0.01 + 0.05 * g.random(N)
    m = g.normal(0, 1, (N, K, OE + 1)).astype(np.float32)
    q = (1.0 + 3.0 * g.random((N, K, OE + 1))).astype(np.float32)
    state = g.normal(0, 0.7, (N, 16)).astype(np.float32)
    if pop == "search":
        init = np.full(N, _lib.LEARNER_SEARCH, np.int32)
        modes = np.full(N, _lib.VL_SEARCH, np.int32)
    else:
        init = np.array([1 if bk[a] >= 2 and (pop == "dm" or a % 3 != 1) else 0 for a in range(N)], np.int32)
        modes = np.full(N, _lib.VL_POLICY, np.int32)
    runs = []
    for generic in (False, True, "noship"):
        eng = AuctionEngine(N, P, K, E, OE, mech, 1.0)
        if generic == "noship":  # k_simulate's runtime-width build (AUTO / GENERIC: the DOS = 5 one)
            eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_SHIPPED_SHAPE, 0), "ag_set_option")
            generic = True
        eng.set_agent_params(ak, bk, pg, gs)
        eng.load_catalog(items, values)
        if ak.any():
            eng.load_lrts(m, q, thompson_sampling=sample)
        if (bk >= 2).any():
            eng.set_dr_state(state, init)
            eng.set_bidder_modes(modes)
        eng.set_simulate_kernel(generic)
        if block:
            eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_BLOCK_THREADS, block), "ag_set_option")
        eng.set_launch_auctions(cap)
        inp = eng.alloc_inputs(B)
        eng.generate(17, 5, inp)
        eng.generate_noise(17, 5, inp, compact=compact and "ts_noise" in inp)
        if "gamma_grid" in inp:
            eng.generate_search_grid(17, 5, inp)
        out = eng.alloc_outputs(B)
        cnt = eng.new_counters() if counters else None
        eng.simulate(inp, out, cnt)
        torch.cuda.synchronize()
        runs.append((eng, inp, out, cnt))
    (e0, i0, o0, c0) = runs[0]
    for _, _, o1, c1 in runs[1:]:  # GENERIC; the runtime-width build
        for k in o0:
            assert np.array_equal(o0[k].cpu().numpy(), o1[k].cpu().numpy(), equal_nan=True), (k, case)
        if counters:
            assert torch.equal(c0, c1)
    if case == POP_CASES[2]:  # the mixed population directly against the oracle too
        T = lambda t: np.ascontiguousarray(t.cpu().numpy().T)  # noqa: E731
        tn = e0.compact_to_dense_ts_noise(i0["ts_noise"], i0["ts_noise_index"], P, B)
        orc = oracle.simulate_pop(mech, items, values, T(i0["ctx"]), T(i0["part"]), i0["u"].cpu().numpy(),
                                  ak, bk, pg, gs, OE=OE, ts_m=m,
                                  ts_noise=e0.untile_ts_noise(tn, B).reshape(B, P, K, OE + 1),
                                  gamma_raw=T(i0["gamma_raw"]), dr_state=state, dr_init=init,
                                  policy_eps=T(i0["policy_eps"]), nthreads=16)
        for k in ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity"):
            assert np.array_equal(T(o0[k]), orc[k], equal_nan=True), k
        for k in ("winner", "price", "second_price", "outcome"):
            assert np.array_equal(o0[k].cpu().numpy(), orc[k], equal_nan=True), k
        assert np.array_equal(c0.cpu().numpy(), orc["counters_fx"])
    for e, *_ in runs:
        e.close()


def test_agent_items_validation(gpu):
    """ag_set_agent_items refuses counts outside [1, K] loudly (ValueError) and accepts NULL
    (every agent has K); a padded catalogue with per-agent counts equal to K runs the plain path."""
    from auctiongym_amd.engine import AuctionEngine
    eng = AuctionEngine(4, 2, 12, 5, 4, 1)
    with pytest.raises(ValueError):
        eng.set_agent_items([12, 0, 5, 7])
    with pytest.raises(ValueError):
        eng.set_agent_items([12, 13, 5, 7])
    eng.set_agent_items([12, 3, 5, 7])
    eng.set_agent_items(None)
    eng.close()


@pytest.mark.parametrize("pop", ["empirical", "lrts"])
def test_interleaved_updates_match_reference(gpu, tmp_path, pop):
    """Notebook-style use of the per-agent surface against the reference's own run
    (tests/golden/interleave_kat.npz, make_golden.py --only interleave): rounds simulated
    between one agent's update() and the others', a second update() of an agent's grown logs,
    clear_logs() of some agents only (src/Agent.py:79-94, :124-129). After every step: the log
    counts exactly; EmpiricalShadedBidders (exact arithmetic): every prev_gamma bit for bit and
    revenue / utilities to 1e-9; LR-TS allocators (the reference's float32 torch fits, whose
    stopping epoch is chaotic): m and q to the update KATs' tolerances,
    revenue / utilities to 1e-9 until a fitted model has bid, 3 % after."""
    import torch

    import auctiongym_amd.main as M
    k = np.load(os.path.join(GOLDEN, "interleave_kat.npz"))
    steps = json.loads(str(k["steps"]))
    cfg = json.loads(str(k[f"{pop}_cfg"]))
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, agent_configs, a2i, a2v, _, max_slots, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, agent_configs, a2v, a2i)
    auction, _, _, _ = M.instantiate_auction(rng, config, a2i, a2v, agents, max_slots, E, var, OE)
    fitted_bid = False
    for j, (op, arg) in enumerate(steps):
        if op == "sim":
            auction.simulate_batch(arg)
            fitted_bid |= any(getattr(a.allocator, "epochs", 0) for a in agents)
        elif op == "upd":
            agents[arg].update(iteration=j)
        else:
            agents[arg].clear_logs()
        key = f"{pop}_s{j}"
        assert [a.num_logs() for a in agents] == list(k[key + "_nlogs"]), (j, op, arg)
        rt = dict(rtol=3e-2, atol=1e-6) if (pop == "lrts" and fitted_bid) else dict(rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(auction.revenue, k[key + "_revenue"], **rt, err_msg=str(j))
        np.testing.assert_allclose([a.net_utility for a in agents], k[key + "_net"], **rt, err_msg=str(j))
        if pop == "empirical":
            assert [a.bidder.prev_gamma for a in agents] == list(k[key + "_pg"]), j
        else:
            m = np.stack([a.allocator.response_model.m.numpy() for a in agents])
            q = np.stack([a.allocator.response_model.q.numpy() for a in agents])
            np.testing.assert_allclose(m, k[key + "_m"], rtol=3e-2, atol=3e-2, err_msg=str(j))
            np.testing.assert_allclose(q, k[key + "_q"], rtol=5e-3, atol=1e-3, err_msg=str(j))
