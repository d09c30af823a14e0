"""First in the GPU suite: every BASELINE config's exact bench population at its full per-GPU
size, every output and the exact counter limbs compared bit for bit with the oracle
(oracle.simulate_pop, the C restatement of src/Auction.py:28-74 and src/Agent.py:29-68), plus
the reference captures replayed through the Oracle kernels.

The populations, catalogues, models and inputs are bench.py's own (build_sp_ts,
population_first_iteration, population_update, population_fitted_inputs), so a kernel
change that breaks a bench line breaks these tests first. Bar: bit-exact for items, bids,
estimated / true CTRs, best EV, gamma, propensity, winners, prices, second prices, outcomes
and the fixed-point counters (north star: allocation indices and second-price charges
bit-identical; the float counters within 1e-5 -- exact here).
"""
import numpy as np
import pytest

from conftest import CAPTURES, load_capture, mech_code

pytestmark = pytest.mark.gpu

_FIELDS = ("item", "bid", "est_ctr", "true_ctr", "best_ev", "gamma", "propensity")
_ROUND = ("winner", "price", "second_price", "outcome")


def _compare(out, cnt, orc, what):
    """Device outputs ([P][B] / [B]) and counters against the oracle's ([B][P] / [B]); a
    winner_outcome word (the bench lines' ABI 17 output) is checked as its winner and outcome."""
    from auctiongym_amd.engine import unpack_outputs
    out = unpack_outputs(out)
    for k in _FIELDS:
        if k in out:
            got = np.ascontiguousarray(out[k].cpu().numpy().T)
            bad = ~((got == orc[k]) | (np.isnan(got) & np.isnan(orc[k])))
            assert not bad.any(), (what, k, int(bad.sum()), np.argwhere(bad)[:3].tolist())
    for k in _ROUND:
        if k in out:
            got = out[k].cpu().numpy()
            bad = ~((got == orc[k]) | (np.isnan(got.astype(np.float64)) & np.isnan(orc[k].astype(np.float64))))
            assert not bad.any(), (what, k, int(bad.sum()), np.flatnonzero(bad)[:3].tolist())
    assert np.array_equal(cnt.cpu().numpy(), orc["counters_fx"]), (what, "counters")


def _oracle_on(eng, dims, inp, st16, init, B):
    import bench
    O, args, kw = bench.oracle_population_args(eng, dims["items"], dims["values"], inp, dims["ak"], dims["bk"],
                                               st16, init, B, 16)
    return O.simulate_pop(*args, **kw)


@pytest.mark.parametrize("P", [2, 8])
def test_configs_1_sp_truthful_ts_full_size(gpu, oracle, P):
    """configs[1] (SP_Truthful_TS: 8 LR-TS Thompson-sampling truthful bidders, SecondPrice) at
    the bench's 2^20 auctions, P = 2 and P = 8 (k_simulate's TruthfulBidder build; streamed
    slots at P = 8), inputs and Thompson noise as the bench generates them."""
    import torch
    import bench
    B = 1 << 20
    eng, inp, out, cnt, dims = bench.build_sp_ts(B, 0, P)
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    orc = _oracle_on(eng, dims, inp, None, None, B)
    _compare(out, cnt, orc, f"configs_1 P={P}")
    # the bench's timed loop re-runs the same step: same bits every launch
    out2, cnt2 = eng.alloc_outputs(B, packed=True), eng.new_counters()
    eng.simulate(inp, out2, cnt2)
    for k in out:
        assert torch.equal(out[k], out2[k]), k
    assert torch.equal(cnt, cnt2)
    # the bench's generate-mode line: every draw inside the kernel, the same bits
    _same_generated(eng, 0, dims["lo"], out, cnt, B)
    eng.close()


def _same_generated(eng, seed, first, out, cnt, B):
    """ag_simulate_generated(seed, first) == the HBM-resident batch's outputs and counters."""
    import torch
    out_g, cnt_g = eng.alloc_outputs(B, packed=True), eng.new_counters()
    eng.simulate_generated(seed, first, out_g, cnt_g)
    torch.cuda.synchronize()
    from auctiongym_amd.engine import unpack_outputs
    a, b = unpack_outputs(out), unpack_outputs(out_g)
    for k in b:
        if k in a:
            assert np.array_equal(a[k].cpu().numpy(), b[k].cpu().numpy(), equal_nan=True), ("generated", k)
    assert torch.equal(cnt, cnt_g), ("generated", "counters")


@pytest.mark.parametrize("key,P,update", [("configs_2", 2, True), ("configs_3", 2, True),
                                          ("configs_4", 2, True), ("configs_4", 8, False)],
                         ids=["configs_2", "configs_3", "configs_4", "configs_4_p8"])
def test_population_configs_full_size(gpu, oracle, key, P, update):
    """configs[2..4] (FP_DM_TS 2^20, FP_DR_TS 2^19 per GPU, the 32-bidder mix 2^21 per GPU;
    FirstPrice) exactly as bench.run_population runs them: iteration 0 with Gaussian shading,
    checked; the update of every learner on its records (P = 2 lines, as the bench times it);
    then the timed step's batch with bids from the fitted policies (compact Thompson noise for
    the mix), checked -- every output and the counter limbs against the oracle on the same
    inputs and models. configs_4 at P = 8 takes the bench's P = 8 line (constructor policies,
    no update)."""
    import torch
    import bench
    eng, what, B, ak, bk, st16, dims, lo, inp, out, cnt = bench.population_first_iteration(key, 0, P)
    orc = _oracle_on(eng, dims, inp, st16, np.zeros(eng.N, np.int32), B)
    _compare(out, cnt, orc, f"{key} P={P} iteration 0")
    del orc
    if update:
        ms, lep, ep, lst, sst, m_pre = bench.population_update(eng, inp, out, B, lo, ak, bk, 1)
        st_fit, init = eng.dr_state()
        learners = bk >= 2
        assert (init[learners] != 0).all(), "every learner fitted a policy"
    else:
        init = np.where(bk >= 2, 1, 0).astype(np.int32)
        eng.set_dr_state(st16, init)
        st_fit = st16
    del inp
    inp, compact = bench.population_fitted_inputs(eng, B, lo, ak)
    assert compact == (key == "configs_4")
    out, cnt = eng.alloc_outputs(B), eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    orc = _oracle_on(eng, dims, inp, st_fit, init, B)
    _compare(out, cnt, orc, f"{key} P={P} fitted")
    # the bench's generate-mode line (population_fitted_inputs draws with seed 1)
    _same_generated(eng, 1, lo, out, cnt, B)
    eng.close()


# ---- the reference's own captures through the Oracle kernels (moved first in the suite) ----
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


@pytest.mark.parametrize("exact", [False, True], ids=["screened", "exact"])
@pytest.mark.parametrize("name", CAPTURES)
def test_simulate_replay_matches_reference(gpu, oracle, name, exact):
    """The reference's SP_Oracle-family captures (tests/golden/make_golden.py): every output
    equal to the reference's, the counters to the oracle's, the aggregates to 1e-9."""
    from auctiongym_amd.engine import AuctionEngine
    d, meta, agg = load_capture(name)
    eng = AuctionEngine(meta["N"], meta["P"], meta["K"], meta["E"], meta["OE"], mech_code(meta), meta["var"])
    eng.set_item_search(exact)
    eng.load_catalog(d["items"], d["values"])
    o = _run(eng, d["ctx"], d["part"], d["u"])
    for mine, ref in (("item", "item"), ("bid", "slot_bid"), ("est_ctr", "slot_est_ctr"),
                      ("true_ctr", "slot_true_ctr"), ("best_ev", "slot_best_ev")):
        assert np.array_equal(o[mine], d[ref]), mine
    assert np.array_equal(o["winner"], d["winner"])
    if meta["P"] >= 2:
        assert np.array_equal(o["price"], d["price"])
        assert np.array_equal(o["second_price"], d["second_price"])
        assert np.array_equal(o["outcome"], d["outcome"])
    else:
        assert np.isnan(o["price"]).all()
    orc = oracle.simulate(mech_code(meta), d["items"], d["values"], d["ctx"], d["part"], d["u"])
    assert np.array_equal(o["counters_fx"], orc["counters_fx"])
    cnt = AuctionEngine.counters_to_numpy(o["counters_fx"])
    C = {n: i for i, n in enumerate(oracle.COUNTERS)}
    rt = dict(rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(cnt[:, C["net"]], agg["net_utility"], **rt)
    np.testing.assert_allclose(cnt[:, C["gross"]], agg["gross_utility"], **rt)
    np.testing.assert_allclose(cnt[:, C["paid"]].sum(), agg["revenue"], **rt)
    np.testing.assert_allclose(cnt[:, C["underbid_regret"]], agg["underbid_regret"], **rt)
    np.testing.assert_allclose(cnt[:, C["overbid_regret"]], agg["overbid_regret"], **rt)
    eng.close()
