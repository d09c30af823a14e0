#!/usr/bin/env python3
"""Throughput of the AuctionGym hot path on MI355X: auctions resolved per second.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N ... bench.py --gpus N     (one process per GPU)

Workload (north star "SP_Oracle-shaped batches"): the SP_Oracle.json
population -- 6 agents with OracleAllocator + TruthfulBidder, 12 items, E = 5, P = 2
participants per auction, SecondPrice -- with the catalogue drawn exactly as
src/main.py:60-72 does from seed 0. Each GPU owns a contiguous shard of B auctions
(weak scaling); inputs are synthetic (Philox4x32-10 keyed by seed 0 and the GLOBAL
auction index) and resident in HBM before timing. One step = one fused pass
(ag_simulate: k_simulate + the exact counter reduction) over the shard, writing every
per-auction / per-participant output in SoA form; with N > 1 the per-agent counters are
then summed across GPUs (int64 all-reduce over RCCL: the only collective of the path).

Printed: one JSON line (rank 0). `roofline.achieved` = algorithmic bytes per launch
(141 B per auction) / average ag_simulate duration from HIP events on the
launch stream. `cpu_baseline` = the oracle (the C restatement of the reference path,
kind "port") timed on host cores on a bounded sample of the same inputs.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "auction-gym_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# SP_Oracle.json as shipped (reference config/SP_Oracle.json)
SP_ORACLE = {"random_seed": 0, "num_runs": 3, "num_iter": 20, "rounds_per_iter": 10000,
             "num_participants_per_round": 2, "embedding_size": 5, "embedding_var": 1.0,
             "obs_embedding_size": 4, "allocation": "SecondPrice",
             "agents": [{"name": "Truthful Oracle", "num_copies": 6, "num_items": 12,
                         "allocator": {"type": "OracleAllocator", "kwargs": {}},
                         "bidder": {"type": "TruthfulBidder", "kwargs": {}}}],
             "output_dir": "results/SP_Oracle/"}

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); measured copy ~6290


def algorithmic_bytes_per_auction(E, P, first_price):
    reads = 8 * E + 4 * P + 8                       # ctx, part, u
    writes = 4 + 8 + 1 + P * (4 + 8 + 8 + 8 + 8)    # winner, price, outcome; per slot
    if first_price:
        writes += 8                                 # second price (== price under SP)
    return reads + writes


def catalogue(cfg=None):
    import tempfile

    import auctiongym_amd.main as M
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(cfg or SP_ORACLE, f)
    try:
        rng, config, agent_configs, a2i, a2v, *_ = M.parse_config(f.name)
    finally:
        os.unlink(f.name)
    names = [c["name"] for c in agent_configs]
    return np.stack([a2i[n] for n in names]), np.stack([a2v[n] for n in names])


def cpu_baseline(items, values, inp, sample, threads):
    """Time the oracle (C restatement of the reference path) on `sample` auctions of the
    same inputs; also check its outputs equal the GPU's on that sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    ctx = np.ascontiguousarray(inp["ctx"][:, :sample].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"][:, :sample].cpu().numpy().T)
    u = inp["u"][:sample].cpu().numpy()
    O.simulate(1, items, values, ctx[:1000], part[:1000], u[:1000], nthreads=threads)  # warm
    t0 = time.perf_counter()
    o = O.simulate(1, items, values, ctx, part, u, nthreads=threads)
    dt = time.perf_counter() - t0
    return sample / dt, dt, o


SP_TS = dict(SP_ORACLE, agents=[{"name": "Truthful TS", "num_copies": 8, "num_items": 12,
                                  "allocator": {"type": "PyTorchLogisticRegressionAllocator",
                                                "kwargs": {"embedding_size": 4, "num_items": 12}},
                                  "bidder": {"type": "TruthfulBidder", "kwargs": {}}}],
             output_dir="results/SP_Truthful_TS/")


def algorithmic_bytes_ts(E, P, K, Do):
    """SP_Truthful_TS replay: the Thompson noise of both participants is read from HBM."""
    return algorithmic_bytes_per_auction(E, P, first_price=False) + P * K * Do * 4


def timed_steps(step, steps, warmup, world, stream):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(ev[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=stream.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def run_sp_ts(B, steps, warmup, world, rank, local, with_update=True):
    """configs[1]: SP_Truthful_TS, 8 LR-TS truthful bidders, 1M auctions per GPU, SecondPrice.
    Inputs (contexts, participants, uniforms AND the Thompson noise z / sqrt(q) of both
    participants) generated on the GPU and resident in HBM; initial models as
    src/Models.py:21-24 (m ~ N(0,1) from torch seeded 0, q = 1). One step = ag_simulate.
    Then one Agent.update of all 8 agents on the last batch's won samples (collect + the
    GPU training loop), timed separately (the reference: 14.3 s per 10k-round iteration)."""
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    from auctiongym_amd.sharding import allreduce_counters, shard_range
    items, values = catalogue(SP_TS)
    N, K, D = items.shape
    E, P, OE = D - 1, SP_TS["num_participants_per_round"], SP_TS["obs_embedding_size"]
    Do = OE + 1
    dev = torch.device("cuda", local)
    eng = AuctionEngine(N, P, K, E, OE, _lib.SECOND_PRICE, SP_TS["embedding_var"], device=local)
    eng.set_agent_params(np.ones(N, np.int32), np.zeros(N, np.int32))
    eng.load_catalog(items, values)
    g = torch.Generator().manual_seed(0)
    m = torch.empty(N, K, Do)
    for a in range(N):
        m[a].normal_(0.0, 1.0, generator=g)
    eng.load_lrts(m.numpy(), np.ones((N, K, Do), np.float32), thompson_sampling=True)
    inp = eng.alloc_inputs(B)
    lo, hi = shard_range(B * world, rank, world)
    eng.generate(0, lo, inp)
    eng.generate_noise(0, lo, inp)
    out = eng.alloc_outputs(B)
    cnt = eng.new_counters()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()

    def step(ev):
        cnt.zero_()
        if ev is not None:
            ev[0].record(stream)
        eng.simulate(inp, out, cnt)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            allreduce_counters(cnt)

    elapsed, kern_ms = timed_steps(step, steps, warmup, world, stream)
    bpa = algorithmic_bytes_ts(E, P, K, Do)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f).get("configs_1", {})
        if tj.get("batch") == B:
            traffic = tj.get("hbm_bytes_per_launch")
    res = {"workload": "SP_Truthful_TS (configs[1]): 8 LR-TS Thompson-sampling truthful bidders, "
                       "K=12, E=5, OE=4, P=2, SecondPrice",
           "value": B * world * steps / elapsed, "unit": "auctions/s", "ms_per_step": elapsed / steps * 1e3,
           "auctions_per_gpu_per_step": B, "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": bpa,
           "roofline": {"bound": "hbm", "achieved": bpa * B / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": bpa * B / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "traffic": traffic}}
    if with_update:
        from auctiongym_amd.sharding import gather_records
        st = eng.new_lrts_samples(B)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        eng.lrts_collect(inp, out, st)
        if world > 1:  # every rank trains on all ranks' samples: identical models everywhere
            st = gather_records(st)
        ep = eng.lrts_update(st)  # synchronises
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        if world > 1:
            t = torch.tensor([ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t[0])
        res["agent_update"] = {"ms": ms, "won_samples": int(st["count"][0]),
                               "epochs": [int(e) for e in ep],
                               "what": "Agent.update of all 8 LR-TS agents (ag_lrts_collect"
                                       + (" + all-gather of the won samples over RCCL" if world > 1 else "")
                                       + " + ag_lrts_update: Adam, ReduceLROnPlateau, early stop, Laplace q)"}
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=60,
                    help="untimed steps first (lets the clocks settle under sustained load)")
    ap.add_argument("--batch", type=int, default=1 << 24, help="auctions per GPU per step")
    ap.add_argument("--cpu-sample", type=int, default=1 << 23)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, cpu_count)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ts-batch", type=int, default=1 << 20, help="SP_Truthful_TS auctions per GPU per step")
    ap.add_argument("--no-ts", action="store_true", help="skip the SP_Truthful_TS (configs[1]) line")
    ap.add_argument("--no-update", action="store_true", help="skip timing the LR-TS Agent.update")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    from auctiongym_amd.sharding import allreduce_counters, shard_range

    items, values = catalogue()
    N, K, D = items.shape
    E, P = D - 1, SP_ORACLE["num_participants_per_round"]
    B = int(args.batch)
    eng = AuctionEngine(N, P, K, E, SP_ORACLE["obs_embedding_size"], _lib.SECOND_PRICE,
                        SP_ORACLE["embedding_var"], device=local)
    eng.load_catalog(items, values)
    inp = eng.alloc_inputs(B)
    lo, hi = shard_range(B * world, rank, world)  # global auction indices of this rank
    eng.generate(0, lo, inp)
    fields = ("winner", "price", "outcome", "item", "bid", "est_ctr", "true_ctr", "best_ev")
    out = eng.alloc_outputs(B, fields)
    cnt = eng.new_counters()
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    nev = args.steps
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(nev)]

    def step(i=None):
        cnt.zero_()
        if i is not None:
            ev[i][0].record(stream)
        eng.simulate(inp, out, cnt)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1:
            allreduce_counters(cnt)  # exact int64 limb sums across shards (RCCL)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    total_auctions = B * world * args.steps
    value = total_auctions / elapsed
    bpa = algorithmic_bytes_per_auction(E, P, first_price=False)
    achieved = bpa * B / (kern_ms * 1e-3) / 1e9

    traffic = None
    traffic_src = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f)
        if tj.get("batch") == B:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = tj.get("source")

    result = {
        "metric": "auctions resolved/sec (SP_Oracle-shaped batches)",
        "value": value,
        "unit": "auctions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Philox4x32-10 contexts/participants/uniforms resident in HBM; "
                "catalogue drawn as src/main.py:60-72 with seed 0)",
        "config": {"workload": "SP_Oracle-shaped: 6 agents OracleAllocator+TruthfulBidder, "
                               "K=12 items, E=5, P=2, SecondPrice (config/SP_Oracle.json)",
                   "auctions_per_gpu_per_step": B, "global_batch": B * world,
                   "parallelism": f"dp{world} (independent auction shards; int64 counter all-reduce)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "kernel": "ag_simulate (k_simulate + k_reduce_counters)",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": bpa},
    }

    if not args.no_ts:
        result["configs_1"] = run_sp_ts(args.ts_batch, args.steps, args.warmup, world, rank, local,
                                        with_update=not args.no_update)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        sample = min(args.cpu_sample, B)
        cps, dt, o = cpu_baseline(items, values, inp, sample, threads)
        gpu_bid = out["bid"][:, :sample].cpu().numpy().T
        same = bool(np.array_equal(gpu_bid, o["bid"]) and
                    np.array_equal(out["winner"][:sample].cpu().numpy(), o["winner"]))
        result["cpu_baseline"] = {
            "value": cps, "unit": "auctions/s", "cores": threads, "kind": "port",
            "sample": f"{sample} auctions of the same synthetic batch, oracle/ag_oracle.c "
                      f"(OpenMP, {threads} threads), {dt:.2f} s; outputs identical to GPU: {same}"}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
