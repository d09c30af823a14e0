"""Host-side logic and the C-ABI library, without a GPU."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, load_capture

LIB = os.path.join(ROOT, "auction-gym_amd", "auctiongym_amd", "libauctiongym_hip.so")
HDR = os.path.join(ROOT, "include", "auctiongym.h")


def _declared_symbols():
    import re
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^(?:int|int32_t|const char\s*\*)\s*(ag_\w+)\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from auctiongym_amd import _lib
    assert os.path.exists(LIB), "build with `make -C auction-gym_amd`"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    declared = _declared_symbols()
    assert declared and set(declared) <= exported, set(declared) - exported
    assert set(declared) == set(_lib.EXPORTS)


def test_library_loads_without_gpu_and_reports_abi():
    from auctiongym_amd import _lib
    L = _lib.load()
    assert L.ag_abi_version() == _lib.ABI_VERSION == 17


def test_ctypes_structs_match_the_c_header(tmp_path):
    """The ctypes mirrors of the ABI structs (auctiongym_amd/_lib.py) have the sizes and
    field offsets a C compiler gives include/auctiongym.h, and set struct_size themselves."""
    import ctypes
    from auctiongym_amd import _lib
    structs = {"ag_shape": _lib.AgShape, "ag_batch_in": _lib.AgBatchIn, "ag_batch_out": _lib.AgBatchOut,
               "ag_lrts_samples": _lib.AgLrtsSamples, "ag_shading_samples": _lib.AgShadingSamples,
               "ag_pcg64_state": _lib.AgPcg64State}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "auctiongym.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                        check=True).stdout.splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)
    for cls in list(structs.values())[1:]:
        assert cls().struct_size == ctypes.sizeof(cls)


def test_counters_to_double_host_helper():
    from auctiongym_amd import _lib
    L = _lib.load()
    vals = [0, 1, -1, (1 << 36) * 3, -((1 << 90) + 12345), (1 << 100) + 7]
    limbs = []
    for v in vals:
        m = (1 << 42) - 1
        limbs.append([v & m, (v >> 42) & m, v >> 84])
    fx = np.array(limbs, np.int64)
    out = np.empty(len(vals))
    assert L.ag_counters_to_double(fx.ctypes.data, len(vals), out.ctypes.data) == 0
    np.testing.assert_array_equal(out, [float(v) * 2.0 ** -36 for v in vals])


def test_ctx_creation_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from auctiongym_amd.engine import AuctionEngine
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        AuctionEngine(6, 2, 12, 5, 4, 1)


def _sp_config(tmp_path):
    with open(os.path.join(GOLDEN, "sp_oracle_full_run.json")) as f:
        cfg = json.load(f)["config"]
    p = tmp_path / "SP_Oracle.json"
    p.write_text(json.dumps(cfg))
    return str(p)


def test_parse_config_reproduces_reference_catalogue(tmp_path):
    import auctiongym_amd.main as M
    d, meta, _ = load_capture("sp_oracle_r4096")
    rng, config, agent_configs, a2i, a2v, num_runs, max_slots, E, var, OE = M.parse_config(
        _sp_config(tmp_path))
    names = [c["name"] for c in agent_configs]
    assert names == [f"Truthful Oracle {i}" for i in range(1, 7)]
    assert np.array_equal(np.stack([a2i[n] for n in names]), d["items"])
    assert np.array_equal(np.stack([a2v[n] for n in names]), d["values"])
    assert (num_runs, max_slots, E, var, OE) == (3, 1, 5, 1.0, 4)


def test_replay_draws_reproduce_reference_inputs(tmp_path):
    import auctiongym_amd.main as M
    from auctiongym_amd.replay import draw_rounds
    d, meta, _ = load_capture("sp_oracle_r4096")
    rng, config, agent_configs, *_ = M.parse_config(_sp_config(tmp_path))
    ctx, part, u = draw_rounds(rng, 4096, meta["N"], meta["P"], meta["E"], meta["var"])
    assert np.array_equal(ctx.T, d["ctx"]) and np.array_equal(part.T, d["part"])
    assert np.array_equal(u, d["u"])


def test_replay_draws_native_reproduce_reference_inputs(tmp_path):
    """ag_replay_draw (C: PCG64 restated, numpy's own distributions) gives the reference's
    captured SP_Oracle inputs and leaves the generator where the Python loop leaves it."""
    import auctiongym_amd.main as M
    from auctiongym_amd.replay import draw_rounds, draw_rounds_native
    d, meta, _ = load_capture("sp_oracle_r4096")
    rng, *_ = M.parse_config(_sp_config(tmp_path))
    rng2, *_ = M.parse_config(_sp_config(tmp_path))
    ctx, part, u, g = draw_rounds_native(rng, 4096, meta["N"], meta["P"], meta["E"], meta["var"])
    assert g is None
    assert np.array_equal(ctx.T, d["ctx"]) and np.array_equal(part.T, d["part"]) and np.array_equal(u, d["u"])
    draw_rounds(rng2, 4096, meta["N"], meta["P"], meta["E"], meta["var"])
    assert rng.bit_generator.state == rng2.bit_generator.state


@pytest.mark.parametrize("N,P,E,var,slots,seed", [
    (6, 2, 5, 1.0, 1, 0), (1, 1, 3, 0.5, 1, 1), (8, 8, 5, 2.0, 3, 2), (40, 7, 0, 1.0, 2, 3),
    (33, 32, 6, 1.0, 1, 4), (3, 3, 5, 1.0, 5, 5),
    (20000, 500, 2, 1.0, 1, 6),   # numpy's tail-shuffle choice branch (N > 10000, P > N // 50)
    (20000, 3, 2, 1.0, 1, 7)])    # Floyd's branch at a large population
def test_replay_draws_native_match_numpy(N, P, E, var, slots, seed):
    """Round for round and state for state equal to the Python loop over numpy's Generator
    (the reference's draws), including multi-slot integers draws, P == N, the 32-bit half
    buffer the choice leaves behind, and a generator that starts with a buffered half."""
    from auctiongym_amd.replay import draw_rounds, draw_rounds_native
    B = 3000 if N < 10000 else 40
    a, b = np.random.default_rng(seed), np.random.default_rng(seed)
    a.integers(0, 5), b.integers(0, 5)      # a 32-bit draw: has_uint32 set on entry
    a.random(), b.random()
    x = draw_rounds_native(a, B, N, P, E, var, slots)
    y = draw_rounds(b, B, N, P, E, var, slots)
    for u, v in zip(x[:3], y):
        assert np.array_equal(u, v)
    assert a.bit_generator.state == b.bit_generator.state
    assert a.random() == b.random()


class _TsModel:
    """The LR-TS model's Thompson draw as src/Models.py:31 makes it (the same torch call)."""

    def __init__(self, q):
        self.q = q

    def sample_noise(self):
        return torch.normal(mean=0.0, std=1.0 / torch.sqrt(self.q))


@pytest.mark.parametrize("case", ["ts", "ts_policy", "mixed", "search", "ts_kdo_mult16", "ts_threads", "ragged"])
def test_replay_population_draws_match_python(case):
    """ag_replay_draw_population (C: torch's mt19937 CPU generator and its normal kernels
    restated, numpy's PCG64 and distributions) against the Python loop that makes the
    reference's own calls (draw_round_population: torch.normal(0, 1/sqrt(q)),
    torch.empty(1).normal_(), rng.uniform(0.1, 1, 128) sorted, rng.normal): every number and
    both generators' states afterwards. The rsample's cached second normal is carried across
    rounds (odd draw counts); the Thompson draws of K*Do = 60 take normal_fill's recomputed
    last block, K*Do = 64 does not."""

    from auctiongym_amd.engine import AuctionEngine
    from auctiongym_amd.replay import draw_round_population, draw_rounds_native_population
    N, P, E, B = 9, 3, 5, (6000 if case == "ts_threads" else 700)  # >= 2048 rounds: threaded transforms
    KDo = 64 if case == "ts_kdo_mult16" else 60
    gen = torch.Generator().manual_seed(5)
    qs = [torch.rand(KDo // 5 if KDo == 60 else 16, 5 if KDo == 60 else 4, generator=gen) * 3 + 0.05 for _ in range(N)]
    kdo_max = None
    if case == "ragged":  # per-agent num_items (src/main.py:61,66): models of 12, 9, 6, 13 rows
        qs = [torch.rand((12, 9, 6, 13)[a % 4], 5, generator=gen) * 3 + 0.05 for a in range(N)]
        kdo_max = KDo = 13 * 5
    ts = [_TsModel(qs[a]) if case != "search" and a % 3 != 1 else None for a in range(N)]
    policy = search = None
    shading = [None] * N
    if case in ("ts_policy", "mixed"):
        policy = [a % 2 == 0 for a in range(N)]
    if case in ("mixed", "search"):
        search = [a % 4 == 3 for a in range(N)]
        shading = [(1.0 + 0.1 * a, 0.05) if a % 4 == 1 else None for a in range(N)]
    a_rng, b_rng = np.random.default_rng(21), np.random.default_rng(21)
    torch.manual_seed(99)
    torch.empty(1).normal_()  # a cached second normal on entry
    t0 = torch.get_rng_state()
    ctx, part, g, u, noise, eps, grid = draw_rounds_native_population(a_rng, B, N, P, E, 1.0, shading, ts, 1,
                                                                      policy, search, kdo_max=kdo_max)
    t_native = torch.get_rng_state()
    torch.set_rng_state(t0)
    rows = [draw_round_population(b_rng, N, P, E, 1.0, shading, ts, 1, policy, search, kdo_max=kdo_max)
            for _ in range(B)]
    assert torch.equal(torch.get_rng_state(), t_native)
    assert a_rng.bit_generator.state == b_rng.bit_generator.state
    z = np.zeros((B, P, KDo), np.float32)
    for r, (c, p, gr, uu, nz, ee, gg) in enumerate(rows):
        assert np.array_equal(ctx[:, r], c) and np.array_equal(part[:, r], p) and uu == u[r]
        if g is not None:
            assert np.array_equal(g[:, r], gr, equal_nan=True)
        if nz is not None:
            z[r] = nz
        if eps is not None:
            assert np.array_equal(eps[:, r], ee if ee is not None else np.zeros(P, np.float32))
        if grid is not None:
            assert np.array_equal(grid[:, :, r], gg if gg is not None else np.zeros((P, 128)))
    if noise is not None:
        assert np.array_equal(noise, AuctionEngine.tile_ts_noise(z))
    assert (noise is not None) == (case != "search") and (eps is not None) == (policy is not None)


def test_torch_normal_fill_restatement():
    """The Box-Muller block of torch's float normal kernel (normal_fill_16_AVX2 with avx_mathfun's
    Cephes log / sincos, restated in ag_replay.cpp) on torch's own uniforms equals
    torch.empty(n).normal_() for 400 seeds, n = 16 and 60 (the recomputed last block). The same
    block is checked on all 2^24 uniforms by tools/torch_normal_probe.sh."""
    L = ctypes.CDLL(os.path.join(ROOT, "auction-gym_amd", "auctiongym_amd", "libauctiongym_hip.so"))
    for seed in range(400):
        for n in (16, 60):
            torch.manual_seed(seed)
            s0 = torch.get_rng_state()
            want = torch.empty(n).normal_().numpy()
            torch.set_rng_state(s0)
            u = torch.empty(n + (16 if n % 16 else 0)).uniform_().numpy().copy()
            x = u[:n].copy()
            for i in range(0, n - 15, 16):
                b = np.ascontiguousarray(x[i:i + 16])
                L.ag_torch_normal_block16(ctypes.c_void_p(b.ctypes.data))
                x[i:i + 16] = b
            if n % 16:
                b = np.ascontiguousarray(u[n:n + 16])
                L.ag_torch_normal_block16(ctypes.c_void_p(b.ctypes.data))
                x[n - 16:] = b
            assert np.array_equal(x.view(np.uint32), want.view(np.uint32)), (seed, n)


def test_replay_draws_native_shading_match_numpy():
    """With shading bidders (Gaussian gammas, src/Bidder.py:51, 177, 354, 461) in slot order:
    the same as draw_round_population with no torch draws."""
    from auctiongym_amd.replay import draw_round_population, draw_rounds_native
    N, P, E, B = 7, 3, 5, 2000
    shading = [(1.0, 0.02), None, (0.7, 0.1), None, None, (0.9, 0.05), (1.2, 0.3)]
    a, b = np.random.default_rng(11), np.random.default_rng(11)
    ctx, part, u, g = draw_rounds_native(a, B, N, P, E, 1.0, 1, shading=shading)
    for r in range(B):
        c, p, gr, uu, *_ = draw_round_population(b, N, P, E, 1.0, shading, [None] * N)
        assert np.array_equal(ctx[:, r], c) and np.array_equal(part[:, r], p) and uu == u[r]
        assert np.array_equal(g[:, r], gr, equal_nan=True)
    assert a.bit_generator.state == b.bit_generator.state


def test_replay_draws_native_errors():
    from auctiongym_amd.replay import draw_rounds_native
    with pytest.raises(ValueError, match="larger sample than population"):
        draw_rounds_native(np.random.default_rng(0), 4, 3, 4, 5, 1.0)
    with pytest.raises(NotImplementedError):
        draw_rounds_native(np.random.Generator(np.random.MT19937(0)), 4, 6, 2, 5, 1.0)


def test_plugin_factory_semantics(tmp_path):
    import auctiongym_amd.main as M
    from auctiongym_amd.Bidder import TruthfulBidder, ValueLearningBidder
    rng = np.random.default_rng(0)
    b = M.make_plugin("ValueLearningBidder", rng,
                      {"gamma_sigma": 0.02, "init_gamma": 1.0, "inference": '"policy"'})
    assert isinstance(b, ValueLearningBidder) and b.kwargs["inference"] == "policy"
    assert isinstance(M.make_plugin("TruthfulBidder", rng, {}), TruthfulBidder)
    with pytest.raises(ValueError):
        M.make_plugin("os.system", rng, {})
    mech = M.make_plugin("SecondPrice", rng, {}, pass_rng=False)
    assert mech.code == 1


def test_plugins_parse_and_no_cpu_fallback(tmp_path):
    """Learning plugins parse with the reference's kwargs and carry their kernel kinds;
    without a GPU the auction refuses to run (no silent CPU path)."""
    import torch

    import auctiongym_amd.main as M
    from auctiongym_amd import _lib
    from auctiongym_amd.Auction import Auction
    from auctiongym_amd.AuctionAllocation import FirstPrice
    cfg = {"random_seed": 0, "num_runs": 1, "num_iter": 1, "rounds_per_iter": 10,
           "num_participants_per_round": 2, "embedding_size": 5, "embedding_var": 1.0,
           "obs_embedding_size": 4, "allocation": "FirstPrice", "output_dir": str(tmp_path),
           "agents": [{"name": "DR", "num_copies": 3, "num_items": 12,
                       "allocator": {"type": "PyTorchLogisticRegressionAllocator",
                                     "kwargs": {"embedding_size": 4, "num_items": 12}},
                       "bidder": {"type": "DoublyRobustBidder",
                                  "kwargs": {"gamma_sigma": 0.02, "init_gamma": 1.0}}}]}
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    rng, config, ac, a2i, a2v, _, ms, E, var, OE = M.parse_config(str(p))
    torch.manual_seed(0)
    agents = M.instantiate_agents(rng, ac, a2v, a2i)
    assert all(a.allocator.kind == _lib.ALLOCATOR_LRTS for a in agents)
    assert all(a.bidder.kind == _lib.BIDDER_DOUBLY_ROBUST for a in agents)
    # the LR-TS model draws m from torch's global generator as src/Models.py:21-22 does
    torch.manual_seed(0)
    ref = torch.empty(12, 5)
    torch.nn.init.normal_(ref, mean=0.0, std=1.0)
    assert torch.equal(agents[0].allocator.response_model.m, ref)
    assert torch.equal(agents[0].allocator.response_model.prev_iter_m, ref)
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            Auction(rng, FirstPrice(), agents, a2i, a2v, ms, E, var, OE, 2)


def test_graft_entry_build_is_idempotent():
    import __graft_entry__ as G
    G.build()
    assert os.path.exists(LIB)


def test_ts_noise_tiling_roundtrip():
    """The 64-auction tile layout of ag_batch_in.ts_noise (include/auctiongym.h)."""
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(0)
    for B in (1, 63, 64, 65, 200):
        z = g.normal(size=(B, 2, 12, 5)).astype(np.float32)
        t = AuctionEngine.tile_ts_noise(z)
        T = (B + 63) // 64
        assert t.shape == (2, T, 60, 64)
        flat = t.ravel()
        for i in (0, B // 2, B - 1):
            for s in (0, 1):
                for c in (0, 17, 59):
                    assert flat[((s * T + i // 64) * 60 + c) * 64 + i % 64] == z[i, s].ravel()[c]
        assert np.array_equal(AuctionEngine.untile_ts_noise(t, B), z.reshape(B, 2, 60))


def test_compact_ts_noise_layout_host():
    """The compact Thompson-noise layout (ag_batch_in.ts_noise_index, ABI 16): pair j = the
    rank of an LR-TS pair in (slot, auction) order, coefficient c at ((j/64)*KDo + c)*64 + j%64;
    compact_to_dense_ts_noise puts every pair's coefficients back at its dense tile place
    (zeros for other agents' pairs), as the GPU test compares against the dense generator."""
    from auctiongym_amd.engine import AuctionEngine
    g = np.random.default_rng(1)
    P, KDo = 3, 60
    for B in (1, 64, 65, 300):
        flags = g.random((P, B)) < 0.6
        idx = np.where(flags, np.cumsum(flags.ravel()).reshape(P, B) - 1, -1).astype(np.int32)
        n = int(flags.sum())
        z = g.normal(size=(B, P, KDo)).astype(np.float32)  # dense draws per (auction, slot)
        comp = np.zeros(((n + 63) // 64 * 64 * KDo,), np.float32)
        for s in range(P):
            for i in range(B):
                j = idx[s, i]
                if j >= 0:
                    for c in range(KDo):
                        comp[((j // 64) * KDo + c) * 64 + j % 64] = z[i, s, c]
        comp = comp.reshape(-1, KDo, 64)
        dense = AuctionEngine.compact_to_dense_ts_noise(comp, idx, P, B)
        assert dense.shape == (P, (B + 63) // 64, KDo, 64)
        back = AuctionEngine.untile_ts_noise(dense, B)  # [B][P][KDo]
        want = np.where(flags.T[:, :, None], z, 0.0)
        assert np.array_equal(back, want)


@pytest.mark.parametrize("n", [1, 5, 15, 16, 17, 48, 1000, 6001])
def test_torch_normal_epochs_restatement(n):
    """ag_torch_normal_epochs (the drop-in learner update's rsample draws, host C): `epochs` x
    torch.empty(n).normal_() -- the same float32 numbers as torch's own calls (its scalar kernel
    below 16 elements, normal_fill_AVX2 from 16 on) and the generator blob left where torch's
    is, so a fit fed window by window leaves torch's global generator as the reference's."""
    from auctiongym_amd.engine import torch_normal_epochs
    torch.manual_seed(11 + n)
    torch.empty(3).normal_()  # a cached second Box-Muller value in the generator
    state = torch.get_rng_state().numpy().copy()
    ref = torch.stack([torch.empty(n).normal_() for _ in range(9)]).numpy()
    got = np.concatenate([torch_normal_epochs(state, n, 4), torch_normal_epochs(state, n, 5)])
    assert np.array_equal(got, ref)
    assert np.array_equal(state, torch.get_rng_state().numpy())


def test_per_call_agent_charge_metrics_and_update():
    """The per-call Agent surface outside an Auction: Agent.bid records completed by
    the reference's own loop calls (logs[-1].set_true_CTR, charge, set_price; src/Auction.py:
    48-73), utilities and every getter equal the reference's formulas over those records
    (src/Agent.py:70-122), Agent.update trains the plugins on exactly the reference's arrays
    (src/Agent.py:79-94), clear_logs(memory=M) keeps the last M records."""
    from auctiongym_amd.Agent import Agent

    class StubAllocator:  # estimate_CTR from a fixed table (the GPU plugins need a device)
        def __init__(self, ctr):
            self.ctr, self.calls = ctr, []

        def estimate_CTR(self, context):
            return self.ctr[int(abs(context[0]) * 7) % len(self.ctr)]

        def update(self, *a):
            self.calls.append(a)

    class StubBidder:
        def __init__(self):
            self.calls = []

        def bid(self, value, context, estimated_CTR):
            return value * estimated_CTR * 0.9

        def update(self, *a):
            self.calls.append(a)

        def clear_logs(self, memory):
            pass

    rng = np.random.default_rng(3)
    K = 5
    agents = [Agent(rng, f"a{i}", K, rng.uniform(0.5, 2.0, K), StubAllocator(rng.uniform(0.01, 0.2, (9, K))),
                    StubBidder(), memory=4) for i in range(3)]
    ref = {a.name: dict(net=0.0, gross=0.0, logs=[]) for a in agents}
    for r in range(40):
        ctx = np.concatenate([rng.normal(size=4), [1.0]])
        part = rng.choice(3, 2, replace=False)
        bids = []
        for idx in part:
            ag = agents[idx]
            b, it = ag.bid(ctx)
            bids.append(b)
            tc = rng.uniform(0.01, 0.3, K)
            ag.logs[-1].set_true_CTR(float(np.max(tc * ag.item_values)), float(tc[it]))
            ref[ag.name]["logs"].append(dict(value=ag.item_values[it], bid=b, bev=float(np.max(tc * ag.item_values)),
                                             tru=float(tc[it]), est=ag.logs[-1].estimated_CTR, price=0.0,
                                             second=0.0, won=False, outcome=False, item=it, ctx=ctx))
        w = int(np.argmax(bids))
        price, second = float(sorted(bids)[-1]), float(sorted(bids)[-2])
        oc = bool(rng.integers(0, 2))
        for k, idx in enumerate(part):
            ag, lg = agents[idx], ref[agents[idx].name]["logs"][-1]
            if k == w:
                ag.charge(price, second, oc)
                lg.update(price=price, second=second, won=True, outcome=oc)
                ref[ag.name]["net"] += lg["value"] * oc - price
                ref[ag.name]["gross"] += lg["value"] * oc
            else:
                ag.set_price(price)
                lg["price"] = price
    for ag in agents:
        R, L = ref[ag.name], ref[ag.name]["logs"]
        close = lambda a, b: abs(a - b) <= 1e-9 * max(1.0, abs(b))  # noqa: E731
        assert close(ag.net_utility, R["net"]) and close(ag.gross_utility, R["gross"])
        assert ag.num_logs() == len(L)
        assert close(ag.get_allocation_regret(), sum(o["bev"] - o["tru"] * o["value"] for o in L))
        assert close(ag.get_estimation_regret(), sum(o["est"] * o["value"] - o["tru"] * o["value"] for o in L))
        assert close(ag.get_overbid_regret(), sum((o["price"] - o["second"]) * o["won"] for o in L))
        assert close(ag.get_underbid_regret(), sum((o["price"] - o["bid"]) * (not o["won"]) *
                                                   (o["price"] < o["tru"] * o["value"]) for o in L))
        assert close(ag.get_CTR_RMSE(), float(np.sqrt(np.mean([(o["tru"] - o["est"]) ** 2 for o in L]))))
        assert close(ag.get_CTR_bias(), float(np.mean([o["est"] / o["tru"] for o in L if o["won"]])))
        ag.update(0)
        (ca,), (cb,) = ag.allocator.calls, ag.bidder.calls
        won = np.array([o["won"] for o in L])
        assert np.array_equal(ca[0], np.array([o["ctx"] for o in L])[won])
        assert np.array_equal(ca[1], np.array([o["item"] for o in L])[won])
        assert np.array_equal(cb[2], np.array([o["bid"] for o in L])) and np.array_equal(cb[6], won)
        assert np.array_equal(cb[3], np.array([o["price"] for o in L]))
        ag.clear_logs()
        assert len(ag.logs) == 4 and [o.bid for o in ag.logs] == [o["bid"] for o in L[-4:]]
        assert ag.num_logs() == 4
        assert close(ag.get_allocation_regret(), sum(o["bev"] - o["tru"] * o["value"] for o in L[-4:]))
        # a second clear_logs with no new records keeps the same M records in the metrics
        # (src/Agent.py:124-129 keeps logs[-M:] of the kept ones), and update() still trains on them
        ag.clear_logs()
        assert len(ag.logs) == 4 and ag.num_logs() == 4
        assert close(ag.get_allocation_regret(), sum(o["bev"] - o["tru"] * o["value"] for o in L[-4:]))
        ag.update(1)
        assert len(ag.allocator.calls) == 2 and len(ag.bidder.calls) == 2
        assert np.array_equal(ag.bidder.calls[1][2], np.array([o["bid"] for o in L[-4:]]))


def test_native_draws_gate():
    """Auction._native_draws: the C restatement of torch's normal_ covers the
    >= 16-element vectorised kernel of AVX2 / AVX512 builds; a sampling LR-TS agent with
    K*(OE+1) < 16, or a torch build on its DEFAULT kernels, keeps the per-round loop (which makes
    the reference's own torch calls) instead of raising in ag_replay_draw_population."""
    from types import SimpleNamespace
    from unittest import mock

    from auctiongym_amd.Auction import Auction

    def ns(K, OE, ts=True, lrts=True, rng=None):
        return SimpleNamespace(rng=rng or np.random.default_rng(0), _lrts=np.array([lrts, False]), _ts=ts,
                               _num_items=np.array([K, 12]), obs_embedding_size=OE,
                               _ts_agent=np.array([ts and lrts, False]),
                               _TORCH_NORMAL_AVX2=Auction._TORCH_NORMAL_AVX2)
    cap = torch.backends.cpu.get_cpu_capability()
    native = cap in Auction._TORCH_NORMAL_AVX2
    assert Auction._native_draws(ns(12, 4)) == native
    assert not Auction._native_draws(ns(3, 4))             # 3 * 5 = 15 draws: torch's scalar path
    assert Auction._native_draws(ns(3, 4, ts=False))       # no Thompson draws at all
    assert Auction._native_draws(ns(4, 3)) == native       # 4 * 4 = 16
    assert not Auction._native_draws(ns(12, 4, rng=np.random.Generator(np.random.MT19937(0))))
    with mock.patch("torch.backends.cpu.get_cpu_capability", return_value="DEFAULT"):
        assert not Auction._native_draws(ns(12, 4))
        assert Auction._native_draws(ns(12, 4, ts=False))


def test_fit_noise_draws_gate_on_torch_build():
    """The learner fits' rsample windows (engine.torch_normal_epochs): with torch's vectorised
    normal kernel the C restatement equals torch's own calls number for number and state for
    state; on a torch build without it (mocked DEFAULT capability) the windows are torch's own
    calls from the given state, the caller's generator untouched (the restatement
    must not be used where it does not hold)."""
    from unittest import mock

    import torch
    from auctiongym_amd.engine import TORCH_NORMAL_AVX2, torch_normal_epochs
    torch.manual_seed(123)
    start = torch.get_rng_state().numpy().copy()
    n, epochs = 37, 5

    def via_torch():
        torch.set_rng_state(torch.from_numpy(start.copy()))
        out = np.stack([torch.empty(n).normal_().numpy() for _ in range(epochs)])
        return out, torch.get_rng_state().numpy().copy()
    want, want_state = via_torch()
    if torch.backends.cpu.get_cpu_capability() in TORCH_NORMAL_AVX2:
        st = start.copy()
        got = torch_normal_epochs(st, n, epochs)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)) and np.array_equal(st, want_state)
    torch.manual_seed(7)
    caller = torch.get_rng_state().clone()
    with mock.patch("torch.backends.cpu.get_cpu_capability", return_value="DEFAULT"):
        st = start.copy()
        got = torch_normal_epochs(st, n, epochs)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)) and np.array_equal(st, want_state)
    assert torch.equal(torch.get_rng_state(), caller)
