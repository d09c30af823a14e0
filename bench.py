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
(140 B per auction: SURVEY §8d's 141 with winner and outcome as one 4-B word) / average ag_simulate duration from HIP events on the
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); the measured copy peak is
#                        measured live (measured_copy_peak) and reported beside it


def all_reduce_max(t):
    """MAX over ranks in place (RCCL on the device; a gloo rehearsal goes through host memory)."""
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def algorithmic_bytes_per_auction(E, P, first_price, packed_winner=False):
    """packed_winner: winner and outcome as the one ABI 17 word winner | outcome << 31 (4 B)
    instead of the int32 winner and the byte outcome (5 B)."""
    reads = 8 * E + 4 * P + 8                       # ctx, part, u
    writes = (4 if packed_winner else 4 + 1) + 8 + P * (4 + 8 + 8 + 8 + 8)  # winner(+outcome), price; per slot
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """(threads the process may run on, CPU quota of its cgroup in CPUs or None)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return n, quota


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    return O


def timed(fn, min_seconds, max_passes=40):
    """Run fn() until min_seconds have passed (at least once); returns (passes, seconds, last)."""
    t0 = time.perf_counter()
    out = fn()
    n = 1
    while time.perf_counter() - t0 < min_seconds and n < max_passes:
        out = fn()
        n += 1
    return n, time.perf_counter() - t0, out


def oracle_population_args(eng, items, values, inp, ak, bk, st16, init, sample, threads):
    """The oracle's (oracle.simulate_pop) arguments for the first `sample` auctions of a
    population batch resident on the GPU: the same inputs, LR-TS posteriors, Thompson noise
    (compact layouts expanded to dense), shading / rsample draws and fitted models. Returns
    (O, args, kwargs)."""
    O = _oracle()
    T = lambda t: np.ascontiguousarray(t[..., :sample].cpu().numpy().T)  # noqa: E731
    B = inp["u"].shape[0]
    N, P, K, OE = eng.N, eng.P, eng.K, eng.OE
    m, q, _ = eng.lrts_state()
    kw = dict(OE=OE, ts_m=m, nthreads=threads)
    if "ts_noise" in inp:
        tn = (eng.compact_to_dense_ts_noise(inp["ts_noise"], inp["ts_noise_index"], P, B)
              if "ts_noise_index" in inp else inp["ts_noise"])
        kw["ts_noise"] = np.ascontiguousarray(eng.untile_ts_noise(tn, B)[:sample].reshape(sample, P, K, OE + 1))
        del tn
    if "gamma_raw" in inp:
        kw["gamma_raw"] = T(inp["gamma_raw"])
    if "policy_eps" in inp:
        kw.update(policy_eps=T(inp["policy_eps"]), dr_state=st16, dr_init=init)
    ctx, part, u = T(inp["ctx"]), T(inp["part"]), inp["u"][:sample].cpu().numpy()
    pg, gs = np.ones(N), np.full(N, 0.02)
    return O, (eng.mechanism, items, values, ctx, part, u, ak, bk, pg, gs), kw


def cpu_baseline_population(eng, items, values, inp, out, ak, bk, st16, init, sample, threads, min_seconds=3.0):
    """The oracle's restatement of the general-population round (oracle.simulate_pop, the C
    build of the reference path; OpenMP over `threads`) on the first `sample` auctions of the
    GPU's own inputs: auctions/s, and whether its outputs equal the GPU's on that sample."""
    O, args, kw = oracle_population_args(eng, items, values, inp, ak, bk, st16, init, sample, threads)
    fn = lambda: O.simulate_pop(*args, **kw)  # noqa: E731
    fn()  # warm
    passes, dt, o = timed(fn, min_seconds)
    from auctiongym_amd.engine import unpack_outputs
    out = unpack_outputs(out)
    same = all(np.array_equal(out[k][..., :sample].cpu().numpy().T if out[k].dim() == 2 else
                              out[k][:sample].cpu().numpy(), o[k], equal_nan=True)
               for k in ("item", "bid", "winner", "price"))
    return sample * passes / dt, dt, passes, same


def cpu_baseline_lrts(state, store, agent, n_max=20000):
    """The oracle's LR-TS update restatement (oracle/ag_oracle.c ora_lrts_update: Adam,
    ReduceLROnPlateau, early stop, Laplace q; one thread) on up to n_max of `agent`'s won
    samples from the GPU's own store: sample-epochs per second."""
    O = _oracle()
    n = int(store["count"][0])
    key = store["key"][:n].cpu().numpy().view(np.uint32)
    sel = np.nonzero((key >> 16) == agent)[0][:n_max]
    X = store["x"][:, :n].cpu().numpy().T[sel]
    A, y = (key[sel] >> 1) & 0x7FFF, key[sel] & 1
    m, q, pm = state  # the posteriors the update started from
    t0 = time.perf_counter()
    _, _, _, ep, _ = O.lrts_update(X, A, y, m[agent], pm[agent], q[agent], trace=False)
    dt = time.perf_counter() - t0
    return len(sel) * ep / dt, dt, len(sel), ep


def cpu_baseline_bidder(store, agent, st16, kind, n_max=512):
    """The oracle's learning-bidder update restatement (oracle/ag_oracle_dr.c: ValueLearningBidder
    'policy' = win-rate fit + policy fit; DoublyRobustBidder = win-rate fit + imitation + DR
    policy fit; one thread) on up to n_max of `agent`'s records from the GPU's own store:
    record-epochs per second (epochs of every fit summed, as the GPU's figure counts them)."""
    O = _oracle()
    n = int(store["count"][0])
    ag = store["agent"][:n].cpu().numpy()
    sel = np.nonzero(ag == agent)[0][:n_max]
    col = {k: store[k][:n].cpu().numpy()[sel] for k in ("ctr", "value", "gamma", "won", "propensity", "utility")}
    wr, pol = st16[agent][:4], st16[agent][4:]
    noise = O.fit_noise(0, agent, 16384, len(sel))
    t0 = time.perf_counter()
    if kind == "dr":
        r = O.dr_update(col["ctr"], col["value"], col["gamma"], col["propensity"], col["won"], col["utility"],
                        wr, pol, False, noise, trace=False)
    else:
        r = O.vl_update(col["ctr"], col["value"], col["gamma"], col["won"], wr, pol, True, noise, trace=False)
    dt = time.perf_counter() - t0
    ep = int(np.sum(r["epochs"]))
    return len(sel) * ep / dt, dt, len(sel), [int(e) for e in r["epochs"]]


def measured_copy_peak(nbytes=1 << 32, reps=20):
    """HBM bandwidth of a 16-B non-temporal streaming copy (ag_stream_copy) of nbytes:
    (read + write bytes) / time, HIP events on the launch stream."""
    from auctiongym_amd.engine import stream_copy
    src = torch.empty(nbytes // 8, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    src.fill_(1.0)
    for _ in range(10):
        stream_copy(src, dst)
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        stream_copy(src, dst)
    b.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    del src, dst
    return 2 * nbytes / (ms * 1e-3) / 1e9


def cpu_baseline(items, values, inp, sample, threads, min_seconds=10.0, max_passes=40):
    """Time the oracle (C restatement of the reference path) on `sample` auctions of the
    same inputs, repeated until at least `min_seconds` of CPU work; also check its outputs
    equal the GPU's on that sample. Returns (auctions/s, seconds, passes, outputs)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    O.build()
    ctx = np.ascontiguousarray(inp["ctx"][:, :sample].cpu().numpy().T)
    part = np.ascontiguousarray(inp["part"][:, :sample].cpu().numpy().T)
    u = inp["u"][:sample].cpu().numpy()
    O.simulate(1, items, values, ctx[:1000], part[:1000], u[:1000], nthreads=threads)  # warm
    t0 = time.perf_counter()
    o = O.simulate(1, items, values, ctx, part, u, nthreads=threads)
    passes = 1
    while time.perf_counter() - t0 < min_seconds and passes < max_passes:
        O.simulate(1, items, values, ctx, part, u, nthreads=threads)
        passes += 1
    dt = time.perf_counter() - t0
    return sample * passes / dt, dt, passes, o


SP_TS = dict(SP_ORACLE, agents=[{"name": "Truthful TS", "num_copies": 8, "num_items": 12,
                                  "allocator": {"type": "PyTorchLogisticRegressionAllocator",
                                                "kwargs": {"embedding_size": 4, "num_items": 12}},
                                  "bidder": {"type": "TruthfulBidder", "kwargs": {}}}],
             output_dir="results/SP_Truthful_TS/")


def algorithmic_bytes_ts(E, P, K, Do):
    """SP_Truthful_TS replay: the Thompson noise of both participants is read from HBM; winner
    and outcome written as the one ABI 17 word."""
    return algorithmic_bytes_per_auction(E, P, first_price=False, packed_winner=True) + P * K * Do * 4


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
        all_reduce_max(t)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def generate_mode_line(eng, seed, lo, out, cnt, B, steps, warmup, world, stream, write_bytes, what):
    """SURVEY 8d's generate mode for a population line: the same step with every input drawn
    inside the kernel (ag_simulate_generated -> k_simulate<..., GEN>: contexts, participants,
    uniforms, the LR-TS agents' Thompson noise, the fitted policies' rsample draws -- the bits
    ag_generate + ag_generate_noise store for the HBM-resident line, so the outputs are
    identical); only the outputs touch HBM. Roofline: the writes against the HBM peak."""
    from auctiongym_amd.sharding import allreduce_counters

    def gstep(ev):
        cnt.zero_()
        if ev is not None:
            ev[0].record(stream)
        eng.simulate_generated(seed, lo, out, cnt)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            allreduce_counters(cnt)

    elapsed, kern_ms = timed_steps(gstep, steps, warmup, world, stream)
    ach = write_bytes * B / (kern_ms * 1e-3) / 1e9
    return {"workload": what + " in generate mode: every input drawn on the chip (Philox4x32-10; the bits the "
                               "HBM-resident line reads, outputs identical)",
            "value": B * world * steps / elapsed, "unit": "auctions/s", "ms_per_step": elapsed / steps * 1e3,
            "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": write_bytes,
            "roofline": {"bound": "VALU (Philox4x32-10: 15 calls per LR-TS participant for its 60 Thompson "
                                  "normals) -- the writes' HBM roofline below",
                         "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS}}


def gpu_record_epochs(counts, epochs, ms):
    """Records x epochs (every fit's epochs summed) per second of a GPU update."""
    work = sum(int(n) * int(np.sum(e)) for n, e in zip(counts, epochs))
    return work / (ms * 1e-3)


def build_sp_ts(B, local, P=None, world=1, rank=0):
    """configs[1]'s engine and resident inputs (what run_sp_ts times and what the configs tests
    check against the oracle): SP_Truthful_TS, 8 LR-TS truthful bidders, SecondPrice; initial
    models as src/Models.py:21-24 (m ~ N(0,1) from torch seeded 0, q = 1); contexts,
    participants, uniforms and the Thompson noise of every participant generated on the GPU
    for this rank's shard. Returns (eng, inp, out, cnt, dims)."""
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    from auctiongym_amd.sharding import shard_range
    items, values = catalogue(SP_TS)
    N, K, D = items.shape
    E, OE = D - 1, SP_TS["obs_embedding_size"]
    P = P or SP_TS["num_participants_per_round"]
    Do = OE + 1
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
    out = eng.alloc_outputs(B, packed=True)  # winner | outcome << 31 (ABI 17), as the headline
    cnt = eng.new_counters()
    torch.cuda.synchronize()
    dims = dict(N=N, K=K, E=E, P=P, OE=OE, Do=Do, items=items, values=values, lo=lo,
                ak=np.ones(N, np.int32), bk=np.zeros(N, np.int32))
    return eng, inp, out, cnt, dims


def run_sp_ts(B, steps, warmup, world, rank, local, with_update=True, cpu_threads=0, P=None):
    """configs[1]: SP_Truthful_TS, 8 LR-TS truthful bidders, 1M auctions per GPU, SecondPrice.
    Inputs (contexts, participants, uniforms AND the Thompson noise z / sqrt(q) of both
    participants) generated on the GPU and resident in HBM (build_sp_ts). One step =
    ag_simulate. Then one Agent.update of all 8 agents on the last batch's won samples
    (collect + the GPU training loop), timed separately (the reference: 14.3 s per 10k-round
    iteration)."""
    from auctiongym_amd.sharding import allreduce_counters
    eng, inp, out, cnt, dims = build_sp_ts(B, local, P, world, rank)
    N, K, E, P, OE, Do = (dims[k] for k in ("N", "K", "E", "P", "OE", "Do"))
    items, values = dims["items"], dims["values"]
    dev = torch.device("cuda", local)
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
    gen = None
    if GENERATE_LINES:
        wb = bpa - (8 * E + 4 * P + 8) - P * K * Do * 4  # the writes alone
        gen = generate_mode_line(eng, 0, dims["lo"], out, cnt, B, steps, warmup, world, stream, wb,
                                 f"SP_Truthful_TS (configs[1]), P={P}")
    traffic = traffic_src = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f).get("configs_1" if P == 2 else f"configs_1_p{P}", {})
        if tj.get("batch") == B:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = tj.get("source")
    res = {"workload": "SP_Truthful_TS (configs[1]): 8 LR-TS Thompson-sampling truthful bidders, "
                       f"K=12, E=5, OE=4, P={P}, SecondPrice",
           "value": B * world * steps / elapsed, "unit": "auctions/s", "ms_per_step": elapsed / steps * 1e3,
           "auctions_per_gpu_per_step": B, "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": bpa,
           "roofline": {"bound": "hbm", "achieved": bpa * B / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": bpa * B / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "traffic": traffic, "traffic_source": traffic_src}}
    if gen is not None:
        res["generate_mode"] = gen
    if cpu_threads:
        rate, dt, passes, same = cpu_baseline_population(eng, items, values, inp, out, np.ones(N, np.int32),
                                                         np.zeros(N, np.int32), None, None, 1 << 15, cpu_threads)
        res["cpu_baseline"] = {"value": rate, "unit": "auctions/s", "cores": cpu_threads, "kind": "port",
                               "what": "build restatement: oracle.simulate_pop (oracle/ag_oracle.c, the reference "
                                       "path's round restated in C, OpenMP) on the same inputs",
                               "sample": f"{passes} passes over the first 32768 auctions of the step's inputs, "
                                         f"{dt:.1f} s; outputs identical to GPU: {same}"}
    if with_update:
        from auctiongym_amd.sharding import lrts_update_agent_parallel
        m_pre = eng.lrts_state()
        st = eng.new_lrts_samples(B)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        eng.lrts_collect(inp, out, st)
        # agent-parallel at N > 1: samples routed to their agent's owner rank, owners train,
        # posteriors exchanged (sharding.lrts_update_agent_parallel)
        ep = lrts_update_agent_parallel(eng, st, list(range(N)))  # synchronises
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        if world > 1:
            t = torch.tensor([ms], dtype=torch.float64, device=dev)
            all_reduce_max(t)
            ms = float(t[0])
        res["agent_update"] = {"ms": ms, "won_samples_rank0": int(st["count"][0]),
                               "epochs": [int(e) for e in ep],
                               "what": "Agent.update of all 8 LR-TS agents (ag_lrts_collect"
                                       + (" + won samples routed to their agent's owner rank, posteriors "
                                          "exchanged over RCCL" if world > 1 else "")
                                       + " + ag_lrts_update: Adam, ReduceLROnPlateau, early stop, Laplace q)"}
        n_all = int(st["count"][0])
        counts = np.bincount(st["key"][:n_all].cpu().numpy().view(np.uint32) >> 16, minlength=N)
        res["agent_update"]["sample_epochs_per_s"] = gpu_record_epochs(counts, ep, ms)
        if cpu_threads:
            rate, dt, n_s, ep_s = cpu_baseline_lrts(m_pre, st, 0)
            res["agent_update"]["cpu_baseline"] = {
                "value": rate, "unit": "sample-epochs/s", "cores": 1, "kind": "port",
                "what": "build restatement: oracle.lrts_update (oracle/ag_oracle.c ora_lrts_update) of agent 0",
                "sample": f"{n_s} of agent 0's won samples from the same store, {ep_s} epochs, {dt:.1f} s",
                "gpu_value": res["agent_update"]["sample_epochs_per_s"]}
    eng.close()
    return res


def _agents_cfg(groups, base):
    """A config dict whose agents are `groups`: [(name, copies, allocator type, bidder type,
    bidder kwargs)] (the reference config schema)."""
    ag = []
    for name, copies, alloc, bidder, kw in groups:
        akw = {"embedding_size": 4, "num_items": 12} if alloc == "PyTorchLogisticRegressionAllocator" else {}
        ag.append({"name": name, "num_copies": copies, "num_items": 12,
                   "allocator": {"type": alloc, "kwargs": akw}, "bidder": {"type": bidder, "kwargs": kw}})
    return dict(base, agents=ag)


LRTS, ORACLE_A = "PyTorchLogisticRegressionAllocator", "OracleAllocator"
POPULATIONS = {
    # BASELINE.json configs[2..4]
    "configs_2": ("FP_DM_TS (configs[2]): 3 LR-TS allocators + ValueLearningBidder('policy'), FirstPrice",
                  [("DM (policy)", 3, LRTS, "ValueLearningBidder",
                    {"gamma_sigma": 0.02, "init_gamma": 1.0, "inference": "policy"})], 1 << 20, "dm"),
    "configs_3": ("FP_DR_TS (configs[3]): 3 LR-TS allocators + DoublyRobustBidder, FirstPrice; 4M auctions "
                  "over 8 GPUs = 512k per GPU",
                  [("DR", 3, LRTS, "DoublyRobustBidder", {"gamma_sigma": 0.02, "init_gamma": 1.0})], 1 << 19, "dr"),
    "configs_4": ("Mixed population (configs[4]): 32 bidders = 11 Oracle+Truthful, 11 LR-TS+Truthful, "
                  "10 LR-TS+DoublyRobust, FirstPrice; 16M auctions over 8 GPUs = 2M per GPU",
                  [("Oracle", 11, ORACLE_A, "TruthfulBidder", {}), ("TS", 11, LRTS, "TruthfulBidder", {}),
                   ("DR", 10, LRTS, "DoublyRobustBidder", {"gamma_sigma": 0.02, "init_gamma": 1.0})],
                  1 << 21, "mixed"),
    # not a BASELINE config (run with --populations fp_ips_ts): FP_IPS_TS.json's population, whose
    # PolicyLearningBidder (PPO) fits stay agent-parallel over ranks
    "fp_ips_ts": ("FP_IPS_TS (config/FP_IPS_TS.json): 3 LR-TS allocators + PolicyLearningBidder(PPO), FirstPrice; "
                  "512k auctions per GPU",
                  [("IPS", 3, LRTS, "PolicyLearningBidder", {"gamma_sigma": 0.02, "init_gamma": 1.0, "loss": "PPO"})],
                  1 << 19, "ips"),
}
DEFAULT_POPULATIONS = "configs_2,configs_3,configs_4"


def algorithmic_bytes_population(E, P, K, Do, ak, bk, init, compact=False):
    """Expected bytes per auction of a general population with bids from fitted policies:
    reads ctx, part, u and, per participant (uniform over agents), its Thompson noise (LR-TS),
    its rsample draw (fitted policy) or shading draw (uninitialised shading); writes winner,
    price, second price, outcome and per participant item, bid, est / true CTR, best EV,
    gamma, propensity (winner and outcome as the one ABI 17 word). compact: the Thompson noise
    in the compact layout, located through ts_noise_index (4 B per LR-TS slot)."""
    per_slot = []
    for a in range(len(ak)):
        b = K * Do * 4 + (4 if compact else 0) if ak[a] == 1 else 0  # + its ts_noise_index entry
        if bk[a] != 0:
            b += 4 if init[a] == 1 else 8
        per_slot.append(b)
    reads = 8 * E + 4 * P + 8 + P * float(np.mean(per_slot))
    writes = 4 + 8 + 8 + P * (4 + 8 * 6)  # winner_outcome, price, second price; per slot
    return reads + writes


def build_population(key, local, P=2):
    """Engine for a BASELINE config population: catalogue as src/main.py:60-72, LR-TS posteriors
    and learning bidders' models as the reference constructors draw them (seeded torch)."""
    from auctiongym_amd import _lib
    from auctiongym_amd.engine import AuctionEngine
    what, groups, B0, tag = POPULATIONS[key]
    cfg = _agents_cfg(groups, dict(SP_ORACLE, allocation="FirstPrice"))
    items, values = catalogue(cfg)
    N, K, D = items.shape
    E, OE = D - 1, 4
    Do = OE + 1
    ak, bk, modes = [], [], []
    kinds = {"TruthfulBidder": 0, "ValueLearningBidder": 2, "PolicyLearningBidder": 3, "DoublyRobustBidder": 4}
    for _, copies, alloc, bidder, kw in groups:
        for _ in range(copies):
            ak.append(1 if alloc == LRTS else 0)
            bk.append(kinds[bidder])
            modes.append(_lib.VL_POLICY if kw.get("inference") == "policy" else _lib.PL_LOSSES.get(kw.get("loss"), 0))
    ak, bk, modes = np.array(ak, np.int32), np.array(bk, np.int32), np.array(modes, np.int32)
    eng = AuctionEngine(N, P, K, E, OE, _lib.FIRST_PRICE, 1.0, device=local)
    eng.set_agent_params(ak, bk, np.ones(N), np.full(N, 0.02))
    eng.load_catalog(items, values)
    g = torch.Generator().manual_seed(0)
    m = torch.empty(N, K, Do)
    for a in range(N):
        m[a].normal_(0.0, 1.0, generator=g)
    eng.load_lrts(m.numpy(), np.ones((N, K, Do), np.float32), thompson_sampling=True)
    st16 = np.zeros((N, 16), np.float32)
    torch.manual_seed(0)
    for a in range(N):  # win-rate models and policies as the constructors draw them (torch.nn.Linear)
        lins = [torch.nn.Linear(3, 1), torch.nn.Linear(2, 2), torch.nn.Linear(2, 1), torch.nn.Linear(2, 1)]
        st16[a] = np.concatenate([p.detach().numpy().ravel() for lin in lins for p in lin.parameters()])
    eng.set_dr_state(st16, np.zeros(N, np.int32))
    eng.set_bidder_modes(modes)
    dims = dict(N=N, K=K, E=E, P=P, Do=Do, items=items, values=values)
    return eng, what, B0, ak, bk, st16, dims


def _record_parallel(bk, world):
    from auctiongym_amd.sharding import record_parallel_pays
    learners = [a for a in range(len(bk)) if bk[a] >= 2]
    if LEARNER_PARALLEL != "auto":  # (forced "record" at N = 1: the per-epoch launches, no exchange)
        return LEARNER_PARALLEL == "record"
    return all(bk[a] in (2, 4) for a in learners) and record_parallel_pays(len(learners), world)


def population_first_iteration(key, local, P=2, batch=None, world=1, rank=0):
    """A BASELINE config population (build_population) at its per-GPU shard size, its
    iteration 0 simulated once: Gaussian shading (uninitialised learners), Philox inputs for
    this rank's shard resident in HBM. Returns (eng, what, B, ak, bk, st16, dims, lo, inp,
    out, cnt)."""
    from auctiongym_amd.sharding import shard_range
    eng, what, B0, ak, bk, st16, dims = build_population(key, local, P)
    B = int(batch or B0)
    lo, _ = shard_range(B * world, rank, world)
    inp = eng.alloc_inputs(B)
    eng.generate(0, lo, inp)
    eng.generate_noise(0, lo, inp)
    out = eng.alloc_outputs(B, packed=True)  # winner | outcome << 31 (ABI 17), as the headline
    cnt = eng.new_counters()
    eng.simulate(inp, out, cnt)
    torch.cuda.synchronize()
    dims = dict(dims, lo=lo, ak=ak, bk=bk)
    return eng, what, B, ak, bk, st16, dims, lo, inp, out, cnt


LEARNER_PARALLEL = "auto"  # --learner-parallel: multi-GPU learning-bidder updates
GENERATE_LINES = True  # --no-generate: no generate-mode lines


def population_update(eng, inp, out, B, lo, ak, bk, world):
    """The update of every learner on iteration 0's records (LR-TS allocators: won samples;
    learning bidders: every record; synthetic on-device rsample noise); at N > 1 LR-TS
    agent-parallel and the learning bidders agent- or record-parallel (sharding.bidder_update's
    cost model, or --learner-parallel). Returns (ms [lrts, bidders] max over ranks, LR-TS
    epochs, bidder epochs, LR-TS store, shading store, the LR-TS state before the update)."""
    from auctiongym_amd.sharding import (bidder_update, bidder_update_agent_parallel,
                                         bidder_update_record_parallel, lrts_update_agent_parallel)
    from auctiongym_amd.sharding import lrts_update, lrts_update_record_parallel
    bidder_fn = {"auto": bidder_update, "agent": bidder_update_agent_parallel,
                 "record": bidder_update_record_parallel}[LEARNER_PARALLEL]
    lrts_fn = {"auto": lrts_update, "agent": lrts_update_agent_parallel,
               "record": lrts_update_record_parallel}[LEARNER_PARALLEL]
    N = eng.N
    P = eng.P
    m_pre = eng.lrts_state()
    lst = eng.new_lrts_samples(B)
    sst = eng.new_shading_samples(B * P, learning=True)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    eng.lrts_collect(inp, out, lst)
    eng.shading_collect(inp, out, sst, first_auction=lo)
    # agent-parallel at N > 1 (each learner trained by one owner rank on every rank's
    # records of it; sharding.*_agent_parallel); identical to one process
    lep = lrts_fn(eng, lst, [a for a in range(N) if ak[a] == 1])
    t1 = time.perf_counter()
    ep, stat = bidder_fn(eng, sst, [a for a in range(N) if bk[a] >= 2])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    ms = [(t1 - t0) * 1e3, (t2 - t1) * 1e3]
    if world > 1:
        t = torch.tensor(ms, dtype=torch.float64, device=eng.device)
        all_reduce_max(t)
        ms = [float(x) for x in t]
    return ms, lep, ep, lst, sst, m_pre


def population_fitted_inputs(eng, B, lo, ak):
    """The timed steps' inputs: the fitted policies' rsample draws now; for mixed allocators
    the Thompson noise in the compact layout (LR-TS pairs only, located through
    ts_noise_index); all-LR-TS populations keep the dense tiles (nothing to drop)."""
    inp = eng.alloc_inputs(B)
    eng.generate(1, lo, inp)
    compact = bool((ak == 1).any() and (ak != 1).any())
    eng.generate_noise(1, lo, inp, compact=compact)
    return inp, compact


def run_population(key, steps, warmup, world, rank, local, batch=None, with_update=True, cpu_threads=0, P=2):
    """A BASELINE config population on the GPU at its per-GPU shard size: iteration 0 with
    Gaussian shading (uninitialised learners), the update of every learner (LR-TS allocators
    and learning bidders, on the GPU, synthetic rsample noise; records routed agent-parallel
    when N > 1) timed, then the timed steps with bids from the fitted policies. Inputs
    Philox-generated and resident in HBM."""
    from auctiongym_amd.sharding import allreduce_counters
    eng, what, B, ak, bk, st16, dims, lo, inp, out, cnt = population_first_iteration(key, local, P, batch,
                                                                                      world, rank)
    if P != 2:
        what = what.replace('FirstPrice', f'FirstPrice, P={P}')
    N, K, E, P, Do = (dims[k] for k in ("N", "K", "E", "P", "Do"))
    res = {"workload": what, "auctions_per_gpu_per_step": B,
           "parity": "simulate: bit-exact vs the oracle; learner updates: bit-exact vs the oracle, which tracks "
                     "the reference's float32 torch fits -- after the first update their stopping epochs are "
                     "chaotic, so later iterations match the reference within 7e-6 (FP_DM_TS) .. 2.6e-3 "
                     "(FP_DR_TS) of revenue, not bit for bit (DESIGN.md section 5)"}
    if with_update:
        ms, lep, ep, lst, sst, m_pre = population_update(eng, inp, out, B, lo, ak, bk, world)
        learners = np.nonzero(bk >= 2)[0]
        res["agent_update"] = {
            "ms": ms[0] + ms[1], "lrts_ms": ms[0], "bidders_ms": ms[1],
            "records_per_bidder": int(sst["count"][0]) // max(1, N),
            "bidder_epochs": [[int(x) for x in ep[a]] for a in learners[:4]],
            "what": "Agent.update of every learner: LR-TS allocators (ag_lrts_update) + learning bidders "
                    "(ag_bidder_update: win-rate fit, imitation, policy fit; synthetic on-device rsample noise)"
                    + (f"; over {world} ranks: "
                       + ("record-parallel (every rank its own records, each epoch's exact partials all-reduced)"
                          if _record_parallel(bk, world) else
                          "agent-parallel (records routed to their agent's owner, owners train, models exchanged)")
                       if world > 1 else "")}
        tp = os.path.join(ROOT, "profiles", "trainer_pmc.json")
        if key == "configs_2" and os.path.exists(tp):  # PMC passes of this same update (tools/trainer_pmc.py)
            pm = json.load(open(tp))
            vr = {k: {"frac": round(v["valu_roofline_frac"], 3), "valu_issue_ms": round(v["valu_issue_ms"], 1),
                      "kernel_ms": round(v["ms_mean_over_passes"], 1), "clock_ghz": round(v["clock_ghz"], 2)}
                  for k, v in pm.items() if isinstance(v, dict) and "valu_roofline_frac" in v}
            vr["what"] = ("VALU-issue roofline: wave-level VALU instructions x 4 cycles over 1024 SIMDs at the "
                          "measured clock, / the dispatch time")
            vr["source"] = "profiles/trainer_pmc.json (rocprofv3 --pmc passes of this update)"
            res["agent_update"]["valu_roofline"] = vr
        n_sh = int(sst["count"][0])
        rec_counts = np.bincount(sst["agent"][:n_sh].cpu().numpy(), minlength=N)
        res["agent_update"]["bidder_record_epochs_per_s"] = gpu_record_epochs(rec_counts[learners], ep[learners], ms[1])
        kind = {4: "dr", 2: "vl"}.get(int(bk[learners[0]])) if len(learners) else None
        if cpu_threads and kind:
            rate, dt, n_s, ep_s = cpu_baseline_bidder(sst, int(learners[0]), st16, kind)
            res["agent_update"]["cpu_baseline"] = {
                "value": rate, "unit": "record-epochs/s", "cores": 1, "kind": "port",
                "what": f"build restatement: oracle.{kind}_update (oracle/ag_oracle_dr.c) of learner {learners[0]}",
                "sample": f"{n_s} of its records from the same store, epochs {ep_s} (win-rate, imitation, policy), "
                          f"{dt:.1f} s",
                "gpu_value": res["agent_update"]["bidder_record_epochs_per_s"]}
            lts = [a for a in range(N) if ak[a] == 1]
            if lts:
                rate, dt, n_s, ep_s = cpu_baseline_lrts(m_pre, lst, lts[0])
                n_l = int(lst["count"][0])
                lc = np.bincount(lst["key"][:n_l].cpu().numpy().view(np.uint32) >> 16, minlength=N)
                res["agent_update"]["lrts_cpu_baseline"] = {
                    "value": rate, "unit": "sample-epochs/s", "cores": 1, "kind": "port",
                    "what": f"build restatement: oracle.lrts_update of agent {lts[0]}",
                    "sample": f"{n_s} of its won samples, {ep_s} epochs, {dt:.1f} s",
                    "gpu_value": gpu_record_epochs(lc, lep, ms[0])}
        st_fit, init = eng.dr_state()
    else:
        init = np.where(bk >= 2, 1, 0).astype(np.int32)
        eng.set_dr_state(st16, init)
        st_fit = st16
    inp, compact = population_fitted_inputs(eng, B, lo, ak)
    res["ts_noise_layout"] = "compact (ts_noise_index)" if compact else "dense"
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
    bpa = algorithmic_bytes_population(E, P, K, Do, ak, bk, init, compact)
    if GENERATE_LINES:
        wb = 4 + 8 + 8 + P * (4 + 8 * 6)  # the writes alone (algorithmic_bytes_population's)
        res["generate_mode"] = generate_mode_line(eng, 1, lo, out, cnt, B, steps, warmup, world, stream, wb,
                                                  what.split(":")[0])
    traffic = traffic_src = None
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):
        with open(tfile) as f:
            tj = json.load(f).get(key if P == 2 else f"{key}_p{P}", {})
        if tj.get("batch") == B:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = tj.get("source")
    if cpu_threads:
        rate, dt, passes, same = cpu_baseline_population(eng, dims["items"], dims["values"], inp, out, ak, bk, st_fit,
                                                         init, 1 << 14, cpu_threads)
        res["cpu_baseline"] = {"value": rate, "unit": "auctions/s", "cores": cpu_threads, "kind": "port",
                               "what": "build restatement: oracle.simulate_pop (oracle/ag_oracle.c) on the same inputs "
                                       "and fitted models",
                               "sample": f"{passes} passes over the first 16384 auctions of the step's inputs, "
                                         f"{dt:.1f} s; outputs identical to GPU: {same}"}
    res.update({"value": B * world * steps / elapsed, "unit": "auctions/s", "ms_per_step": elapsed / steps * 1e3,
                "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": bpa,
                "roofline": {"bound": "hbm", "achieved": bpa * B / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": bpa * B / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "traffic": traffic, "traffic_source": traffic_src}})
    eng.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=60,
                    help="untimed steps first (lets the clocks settle under sustained load)")
    ap.add_argument("--batch", type=int, default=1 << 27,
                    help="auctions per GPU per step (2^27: 19 GB of inputs + outputs resident in HBM; a "
                         "step of ~3.5 ms keeps the driver's few warm-up steps past the clock ramp of a "
                         "fresh process, DESIGN.md section 6)")
    ap.add_argument("--no-generate", action="store_true", help="skip the generate-mode lines")
    ap.add_argument("--peak-last", action="store_true",
                    help="measure the copy peak after the timed steps (A/B of the clock warm-up; default: before)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 24)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: every CPU the process may use (affinity mask capped by the cgroup CPU quota)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ts-batch", type=int, default=1 << 20, help="SP_Truthful_TS auctions per GPU per step")
    ap.add_argument("--no-ts", action="store_true", help="skip the SP_Truthful_TS (configs[1]) line")
    ap.add_argument("--no-update", action="store_true", help="skip timing the Agent.update of learners")
    ap.add_argument("--no-p8", action="store_true", help="skip the P = 8 variants of configs_1 and configs_4")
    ap.add_argument("--p8-only", action="store_true",
                    help="of configs_1 / the populations, only the P = 8 lines (profiling passes)")
    ap.add_argument("--no-populations", action="store_true",
                    help="skip the configs[2..4] lines (FP_DM_TS, FP_DR_TS, mixed population)")
    ap.add_argument("--populations", default=DEFAULT_POPULATIONS,
                    help="comma-separated subset of the configs[2..4] lines to run")
    ap.add_argument("--learner-parallel", choices=("auto", "agent", "record"), default="auto",
                    help="N > 1: learning-bidder updates agent-parallel, record-parallel, or by the cost model "
                         "(sharding.record_parallel_pays: record-parallel when the learners are few for the ranks)")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="N > 1 ranks sharing the visible GPU(s) over gloo: exercises the multi-GPU code path "
                         "(shards, counter all-reduce, agent-parallel updates) where only one GPU is at hand; "
                         "its timings mean nothing")
    args = ap.parse_args()
    global LEARNER_PARALLEL, GENERATE_LINES
    LEARNER_PARALLEL = args.learner_parallel
    GENERATE_LINES = not args.no_generate

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    if args.rehearse_on_one_gpu:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.rehearse_on_one_gpu:
            dist.init_process_group("gloo")
        else:
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
    # every output of the round: winner and outcome as the ABI 17 packed word (the byte-wide
    # outcome stream cost 6 % of the kernel's time, profiles/r05c_ab_packed.log), the rest per field
    from auctiongym_amd.engine import HEADLINE_FIELDS, unpack_outputs
    out = eng.alloc_outputs(B, HEADLINE_FIELDS)
    cnt = eng.new_counters()
    torch.cuda.synchronize()

    # the measured HBM peak (ag_stream_copy, ~40 ms of streaming) before the timed steps: it is
    # part of the line, and it brings a fresh process's clocks up before the W warm-up steps
    # (a cold process ran the first 2^27-auction steps up to 10 % slower, tools/archive/warm_probe.py)
    peak_meas = None if args.peak_last else measured_copy_peak()
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
        all_reduce_max(t)
        elapsed, kern_ms = float(t[0]), float(t[1])

    total_auctions = B * world * args.steps
    value = total_auctions / elapsed
    bpa = algorithmic_bytes_per_auction(E, P, first_price=False, packed_winner=True)
    achieved = bpa * B / (kern_ms * 1e-3) / 1e9

    gen = None
    if not args.no_generate:
        # generate mode: the same workload with the inputs drawn inside the
        # kernel (ag_simulate_generated: the bits ag_generate wrote), writes only
        def gstep(i=None):
            cnt.zero_()
            if i is not None:
                ev[i][0].record(stream)
            eng.simulate_generated(0, lo, out, cnt)
            if i is not None:
                ev[i][1].record(stream)
            if world > 1:
                allreduce_counters(cnt)
        for _ in range(args.warmup):
            gstep()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for i in range(args.steps):
            gstep(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        gel = time.perf_counter() - g0
        gk = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        if world > 1:
            t = torch.tensor([gel, gk], dtype=torch.float64, device=dev)
            all_reduce_max(t)
            gel, gk = float(t[0]), float(t[1])
        wb = bpa - (8 * E + 4 * P + 8)  # the writes alone
        gen = {"workload": "the headline workload in generate mode: contexts, participants and uniforms "
                           "drawn on the chip (Philox4x32-10, the bits ag_generate writes); outputs identical",
               "value": B * world * args.steps / gel, "unit": "auctions/s", "ms_per_step": gel / args.steps * 1e3,
               "kernel_ms": gk, "algorithmic_bytes_per_auction": wb,
               "roofline": {"bound": "hbm (writes) / FP64 VALU (Philox + Box-Muller)",
                            "achieved": wb * B / (gk * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": wb * B / (gk * 1e-3) / 1e9 / HBM_PEAK_GBS}}
    if peak_meas is None:
        peak_meas = measured_copy_peak()

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
                     "frac": achieved / HBM_PEAK_GBS,
                     "peak_measured": peak_meas, "frac_of_measured": achieved / peak_meas,
                     "peak_measured_what": "ag_stream_copy: 4 GiB -> 4 GiB, 16-B non-temporal loads/stores, "
                                           "(read + write bytes) / time",
                     "traffic": traffic,
                     "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
                     "traffic_source": traffic_src,
                     "kernel": "ag_simulate (k_oracle + k_reduce_counters)",
                     "kernel_ms": kern_ms, "algorithmic_bytes_per_auction": bpa,
                     "bytes_what": "56 read (ctx 40, part 8, u 8) + 84 written (winner | outcome << 31 4, "
                                   "price 8, per slot item 4 + bid, est_ctr, true_ctr, best_ev 8 each)"},
    }

    if gen is not None:
        result["generate_mode"] = gen

    n_threads, quota = host_threads()
    # every CPU this process may use: its affinity mask, capped by its cgroup's CPU quota (the
    # GPU box: 256 threads, quota 16 CPUs -- 256 OpenMP threads there are throttled to 16 CPUs'
    # worth and measured 4.8 M auctions/s against 19-22 M/s on 16, profiles/r03h_bench.log)
    usable = min(n_threads, int(np.ceil(quota))) if quota else n_threads
    threads = args.cpu_threads or usable
    cpu_lines = threads if (rank == 0 and world == 1 and not args.no_cpu_baseline) else 0
    if not args.no_ts and not args.p8_only:
        result["configs_1"] = run_sp_ts(args.ts_batch, args.steps, args.warmup, world, rank, local,
                                        with_update=not args.no_update, cpu_threads=cpu_lines)

    if not args.no_populations and not args.p8_only:
        for key in [k for k in args.populations.split(",") if k]:
            result[key] = run_population(key, max(5, args.steps // 5), max(5, args.warmup // 5), world, rank, local,
                                         with_update=not args.no_update, cpu_threads=cpu_lines)

    if not args.no_p8:
        # configs_1 and configs_4 also at P = 8 participants per round (simulate only:
        # the learners' updates are timed on the P = 2 lines)
        if not args.no_ts:
            result["configs_1_p8"] = run_sp_ts(args.ts_batch, args.steps, args.warmup, world, rank, local,
                                               with_update=False, P=8)
        if not args.no_populations and "configs_4" in args.populations.split(","):
            result["configs_4_p8"] = run_population("configs_4", max(5, args.steps // 5), max(5, args.warmup // 5),
                                                    world, rank, local, with_update=False, P=8)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample = min(args.cpu_sample, B)
        cps, dt, passes, o = cpu_baseline(items, values, inp, sample, threads)
        gpu_bid = out["bid"][:, :sample].cpu().numpy().T
        same = bool(np.array_equal(gpu_bid, o["bid"]) and
                    np.array_equal(unpack_outputs(out)["winner"][:sample].cpu().numpy(), o["winner"]))
        s1 = min(1 << 22, sample)
        cps1, dt1, passes1, _ = cpu_baseline(items, values, inp, s1, 1, min_seconds=5.0)
        result["cpu_baseline"] = {
            "value": cps, "unit": "auctions/s", "cores": threads, "kind": "port",
            "sample": f"{passes} passes over {sample} auctions of the same synthetic batch, "
                      f"oracle/ag_oracle.c (OpenMP, {threads} threads), {dt:.1f} s; "
                      f"outputs identical to GPU: {same}",
            "one_core": {"value": cps1, "unit": "auctions/s", "cores": 1,
                         "sample": f"{passes1} passes over {s1} auctions, 1 thread, {dt1:.1f} s"},
            "nproc": os.cpu_count(), "threads_available": n_threads, "cgroup_cpu_quota": quota,
            "threads_used": f"{threads}: every CPU the process may use (affinity mask capped by the cgroup quota)",
            "cpu_model": cpu_model(),
            "reference_itself": "12.8k auctions/s on one core of the survey container (the reference's "
                                "Python/numpy path, BASELINE.md section 2; it cannot run on the GPU box)"}
    if rank == 0:
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
