#!/usr/bin/env python3
"""A/B timing of library builds (make variant NAME=... VFLAGS=...) on a population line of
bench.py (configs_2..4, bids from the constructors' policies as bench's --no-update path),
interleaved in ONE process; outputs and counters checked equal across builds.

    python tools/ab_pop.py configs_4 early [more variants...]
    AG_AB_DENSE=1: the dense Thompson-noise layout instead of the compact one.
    AG_AB_NOCHECK=1: no output comparison (diagnostic ablation builds, make variant-p AG_ABLATE).
    A variant named "generic" is the base library with AG_SIM_KERNEL_GENERIC (k_simulate
    instead of the dedicated kernels), "<variant>+generic" that variant with it; "bt256" /
    "bt1024" force the workgroup size; "grouporder" is the base library reading the compact
    Thompson noise with its pairs ranked in (64-auction group, slot, auction) order instead of
    ag_ts_noise_index's (slot, auction) order (one contiguous run per wave over all its slots);
    "packed" is the base library writing the ABI 17 word winner | outcome << 31 instead of the
    winner and outcome arrays.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "auction-gym_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from auctiongym_amd import _lib  # noqa: E402


def main():
    key = sys.argv[1]
    P = 2
    if ":" in key:  # configs_1:8 -> P = 8 participants per auction
        key, P = key.split(":")[0], int(key.split(":")[1])
    vdir = os.path.join(ROOT, "auction-gym_amd", "build", "variants")
    paths = {"base": _lib.LIB_PATH}
    special = {"generic", "wide", "bt256", "bt1024", "nocnt", "noship", "grouporder", "packed",
               "bpc1", "bpc2", "bpc3"}
    for n in sys.argv[2:]:  # "<variant>+generic": that build with k_simulate forced
        v = n[:-len("+generic")] if n.endswith("+generic") else n
        paths[n] = _lib.LIB_PATH if v in special else os.path.join(vdir, f"libauctiongym_hip_{v}.so")
    base_path = _lib.LIB_PATH
    runs = {}
    for n, p in paths.items():
        _lib.LIB_PATH = p
        if key == "configs_1":  # SP_Truthful_TS as bench.run_sp_ts
            from auctiongym_amd.engine import AuctionEngine
            items, values = bench.catalogue(bench.SP_TS)
            N, K, D = items.shape
            OE = bench.SP_TS["obs_embedding_size"]
            eng = AuctionEngine(N, P, K, D - 1, OE, _lib.SECOND_PRICE, bench.SP_TS["embedding_var"], device=0)
            eng.set_agent_params(np.ones(N, np.int32), np.zeros(N, np.int32))
            eng.load_catalog(items, values)
            g = torch.Generator().manual_seed(0)
            m = torch.empty(N, K, OE + 1)
            for a in range(N):
                m[a].normal_(0.0, 1.0, generator=g)
            eng.load_lrts(m.numpy(), np.ones((N, K, OE + 1), np.float32), thompson_sampling=True)
            B, ak = 1 << 20, np.ones(N, np.int32)
        else:
            eng, what, B, ak, bk, st16, dims = bench.build_population(key, 0, P=P)
            eng.set_dr_state(st16, np.where(bk >= 2, 1, 0).astype(np.int32))
        if n in ("generic", "wide"):
            eng.set_simulate_kernel(True if n == "generic" else n)
        elif n.endswith("+generic"):
            eng.set_simulate_kernel(True)
        if n == "noship":  # k_simulate's runtime-shape build
            eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_SHIPPED_SHAPE, 0), "ag_set_option")
        if n in ("bpc1", "bpc2", "bpc3"):  # the grid capped at that many workgroups per CU
            eng.set_blocks_per_cu(int(n[3:]))
        if n in ("bt256", "bt1024"):
            eng._check(eng.L.ag_set_option(eng._h, _lib.OPT_SIM_BLOCK_THREADS, int(n[2:])), "ag_set_option")
        inp = eng.alloc_inputs(B)
        eng.generate(1, 0, inp)
        compact = not os.environ.get("AG_AB_DENSE") and bool((ak == 1).any() and (ak != 1).any())
        eng.generate_noise(1, 0, inp, compact=compact)
        if n == "grouporder" and compact:  # the same draws, pairs ranked in (i / 64, slot, i) order
            from auctiongym_amd.engine import _ptr, _stream
            fl = torch.from_numpy(ak).to(inp["part"].device)[inp["part"].long()] == 1
            Pn, Bn = fl.shape
            T = (Bn + 63) // 64
            fp = torch.zeros((Pn, T * 64), dtype=torch.int64, device=fl.device)
            fp[:, :Bn] = fl
            r = torch.cumsum(fp.view(Pn, T, 64).transpose(0, 1).flatten(), 0) - 1
            r = r.view(T, Pn, 64).transpose(0, 1).reshape(Pn, T * 64)[:, :Bn]
            inp["ts_noise_index"] = torch.where(fl, r, -1).to(torch.int32).contiguous()
            eng._check(eng.L.ag_generate_ts_noise_compact(eng._h, 1, 0, B, _ptr(inp["part"]),
                                                          _ptr(inp["ts_noise_index"]), _ptr(inp["ts_noise"]),
                                                          _stream()), "ag_generate_ts_noise_compact")
        if n == "packed":  # the ABI 17 word winner | outcome << 31 instead of the two arrays
            from auctiongym_amd.engine import _CORE_FIELDS, _OUT_FIELDS
            fields = [f for f in (_OUT_FIELDS[:11] if getattr(eng, "shading", False) else _CORE_FIELDS)
                      if f not in ("winner", "outcome")] + ["winner_outcome"]
            out = eng.alloc_outputs(B, fields)
        else:
            out = eng.alloc_outputs(B)
        cnt = None if n == "nocnt" else eng.new_counters()
        runs[n] = (eng, inp, out, cnt)
    _lib.LIB_PATH = base_path
    for n, (eng, inp, out, cnt) in runs.items():  # warm-up
        for _ in range(20):
            if cnt is not None:
                cnt.zero_()
            eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    ref = runs["base"]
    for n, (eng, inp, out, cnt) in ([] if os.environ.get("AG_AB_NOCHECK") else runs.items()):  # ablations differ
        for k in out:
            if k == "winner_outcome":
                wo = out[k].cpu().numpy().view(np.uint32)
                assert np.array_equal((wo & 0x7FFFFFFF).astype(np.int32), ref[2]["winner"].cpu().numpy()), n
                assert np.array_equal((wo >> 31).astype(np.uint8), ref[2]["outcome"].cpu().numpy()), n
                continue
            a, b = out[k].cpu().numpy(), ref[2][k].cpu().numpy()
            assert np.array_equal(a, b, equal_nan=True), (n, k)
        assert cnt is None or torch.equal(cnt, ref[3]), n
    times = {n: [] for n in runs}
    for rep in range(30):
        for n, (eng, inp, out, cnt) in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if cnt is not None:
                cnt.zero_()
            e0.record()
            eng.simulate(inp, out, cnt)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1))
    for n, t in times.items():
        print(f"{key} {n}: median {np.median(t):.4f} ms  min {np.min(t):.4f} ms  (B = {runs[n][1]['u'].shape[0]}, "
              f"outputs equal to base)", flush=True)


if __name__ == "__main__":
    main()
