"""Multi-GPU: independent auction shards, one process per GPU, one tiny collective.

Auctions are independent given agent state, so a batch of B auctions
is split into contiguous shards of global auction indices, one per rank; synthetic
inputs are keyed by the global index (ag_generate), so every per-auction output is the
same whatever the number of GPUs. The only exchange of the simulation is the per-agent
counter sums: exact int64 fixed-point limbs (include/auctiongym.h AG_FX_*), summed with an
int64 all-reduce (RCCL over xGMI with backend "nccl", gloo on CPU) -- integer addition, so
the totals are bit-identical for any world size and any reduction order.

Learner updates (Agent.update, src/Agent.py:79-94, called per agent by src/main.py:127-128)
are agent-parallel: each learning agent has an owner rank (round robin over the learners,
`owners`), every record travels once to its agent's owner (`route_records`, one
all-to-all), the owner trains its agents alone, and the trained states are exchanged
(`take_owned_rows`, one all-gather of a few KB). A rank's update work is its own agents'
records only -- not every agent's, as training on all-gathered records would be.

With fewer learners than ranks (A < G: FP_DR_TS's 3 learners on 8 GPUs) agent-parallel leaves
ranks idle and gives each owner G/A times one GPU's records; the exact-sum learning bidders
then train record-parallel (`bidder_update_record_parallel`): every rank keeps its own
records, the fits run as one launch per epoch (ag_bidder_rp_*), and each epoch's exact int64
partial sums are all-reduced, so every rank steps to the same model -- the model one process
fits on all the records. `bidder_update` picks the mode by the cost model of DESIGN.md
section 7.
"""
import numpy as np
import torch
import torch.distributed as dist

LIMB_BITS = 42
LIMB_MASK = (1 << LIMB_BITS) - 1


def shard_range(total, rank, world):
    """Contiguous [lo, hi) of `total` global auction indices owned by `rank`."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def allreduce_counters(limbs, group=None):
    """Sum [.., 3] int64 limb tensors across ranks in place (exact)."""
    if limbs.dtype != torch.int64:
        raise TypeError("counter limbs are int64")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if limbs.is_cuda and dist.get_backend(group) == "gloo":  # gloo rehearsal: via host memory
            h = limbs.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            limbs.copy_(h)
        else:
            dist.all_reduce(limbs, op=dist.ReduceOp.SUM, group=group)
    return limbs


def normalize_limbs(limbs):
    """Carry-normalise [.., 3] limbs (each limb sum of <= 2^21 normalised limb arrays fits
    int64) so limb0, limb1 are in [0, 2^42)."""
    L = np.array(limbs, dtype=object)
    flat = L.reshape(-1, 3)
    out = np.empty(flat.shape, dtype=np.int64)
    for i, (a, b, c) in enumerate(flat):
        v = int(a) + (int(b) << LIMB_BITS) + (int(c) << (2 * LIMB_BITS))
        out[i, 0] = v & LIMB_MASK
        out[i, 1] = (v >> LIMB_BITS) & LIMB_MASK
        out[i, 2] = v >> (2 * LIMB_BITS)
    return out.reshape(np.shape(limbs))


def _world(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _store_shape(store):
    """(count, capacity) of a record store (count read back from the device)."""
    fields = [k for k in store if k != "count"]
    return int(store["count"][0].item()), int(store[fields[0]].shape[-1])


def _check_all(store, group=None):
    """All ranks' (count, capacity), all-gathered; raises on EVERY rank if any rank's store
    overflowed (count > capacity: records were dropped, the update would be wrong) -- so no
    rank is left waiting in the next collective."""
    n, cap = _store_shape(store)
    dev = store["count"].device
    mine = torch.tensor([n, cap], dtype=torch.int64, device=dev)
    allc = [torch.zeros_like(mine) for _ in range(_world(group))]
    dist.all_gather(allc, mine, group=group)
    allc = [(int(t[0]), int(t[1])) for t in allc]
    bad = [r for r, (c, k) in enumerate(allc) if c > k]
    if bad:
        raise ValueError(f"record store overflow on rank(s) {bad}: count > capacity {allc}")
    return allc


def _host_staged(store, group, fn):
    """gloo has no device all-to-all: under gloo, device stores are staged through host
    memory (the multi-process GPU tests run ranks that share one GPU over gloo); under RCCL
    the collectives run on the device buffers directly."""
    dev = store["count"].device
    if _world(group) > 1 and dev.type == "cuda" and dist.get_backend(group) == "gloo":
        out = fn({k: v.cpu() for k, v in store.items()})
        return {k: v.to(dev) for k, v in out.items()}
    return fn(store)


def gather_records(store, group=None):
    """All-gather a record store across ranks (LR-TS won samples: key [cap], x [Do][cap],
    count [1]; or shading records: agent / gamma / utility [cap], count [1]) into one store
    holding every rank's records, on every rank. The updates' sums are exact, so training on
    the gathered records gives bit-identical results on every rank and equals a single
    process training on the whole batch -- the update needs no per-epoch collective.
    One all-gather of the counts, one of each record array (padded to the largest count)."""
    if _world(group) == 1:
        return store
    return _host_staged(store, group, lambda st: _gather(st, group))


def _gather(store, group):
    world = _world(group)
    counts = [c for c, _ in _check_all(store, group)]
    mx = max(max(counts), 1)
    total = sum(counts)
    fields = [k for k in store if k != "count"]
    out = {}
    for k in fields:
        v = store[k]
        lead = v.shape[:-1]
        if v.shape[-1] >= mx:
            part = v[..., :mx].contiguous()
        else:  # this rank's store is smaller than the largest count: pad (never read)
            part = torch.zeros(lead + (mx,), dtype=v.dtype, device=v.device)
            part[..., :v.shape[-1]] = v
        bufs = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(bufs, part, group=group)
        merged = torch.empty(lead + (max(total, 1),), dtype=v.dtype, device=v.device)
        off = 0
        for c, b in zip(counts, bufs):
            merged[..., off:off + c] = b[..., :c]
            off += c
        out[k] = merged
    out["count"] = torch.tensor([total], dtype=store["count"].dtype, device=store["count"].device)
    return out


def owners(agents, world):
    """Owner rank of each agent in `agents` (round robin in the given order), as a dict."""
    return {int(a): i % world for i, a in enumerate(agents)}


def record_agents(store):
    """Agent of every record of a store ([count] int64, device): LR-TS won samples carry it
    in key >> 16 (ag_lrts_samples), shading / learning-bidder records in `agent`."""
    n = int(store["count"][0].item())
    if "key" in store:
        return (store["key"][:n].to(torch.int64) >> 16) & 0xFFFF
    return store["agent"][:n].to(torch.int64)


def route_records(store, owner, group=None):
    """Send every record of a store to the rank that owns its agent (`owner`: agent ->
    rank; records of agents without an owner are dropped). One all-to-all of the counts,
    one per field. The result is a store (same fields) holding, on each rank, every rank's
    records of the agents it owns. Record order within the store is not meaningful: the
    updates' sums are exact (LR-TS) or the records carry their log order (learning
    bidders, ag_shading_samples.order), so training on the routed store equals training on
    all records."""
    if _world(group) == 1:
        return store
    return _host_staged(store, group, lambda st: _route(st, owner, group))


def _route(store, owner, group):
    world = _world(group)
    _check_all(store, group)
    dev = store["count"].device
    agent = record_agents(store)
    N = int(max(owner) + 1) if owner else 1
    if agent.numel():
        N = max(N, int(agent.max().item()) + 1)
    table = torch.full((N,), -1, dtype=torch.int64, device=dev)
    for a, r in owner.items():
        table[a] = r
    dest = table[agent] if agent.numel() else agent
    keep = dest >= 0
    idx = torch.nonzero(keep).flatten()
    dest = dest[idx]
    order = torch.argsort(dest, stable=True)
    idx = idx[order]
    send = torch.bincount(dest, minlength=world).to(torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    sl, rl = [int(x) for x in send.tolist()], [int(x) for x in recv.tolist()]
    total = sum(rl)
    out = {}
    for k, v in store.items():
        if k == "count":
            continue
        lead = v.shape[:-1]
        width = int(np.prod(lead)) if len(lead) else 1       # explicit: m may be 0
        rows = v[..., idx].movedim(-1, 0).reshape(idx.numel(), width).contiguous()  # [m][fields]
        dst = torch.empty((total, width), dtype=v.dtype, device=dev)
        dist.all_to_all_single(dst, rows, output_split_sizes=rl, input_split_sizes=sl, group=group)
        merged = torch.zeros(lead + (max(total, 1),), dtype=v.dtype, device=dev)
        merged[..., :total] = dst.t().reshape(lead + (total,))
        out[k] = merged
    out["count"] = torch.tensor([total], dtype=store["count"].dtype, device=dev)
    return out


def take_owned_rows(local, owner, group=None, device=None):
    """Per-agent state rows (array [N, ...]) trained by their owners: every rank sends its
    whole array (one all-gather of a few KB) and takes agent a's row from rank owner[a]
    (agents without an owner keep the local row). Returns a numpy array like `local`."""
    world = _world(group)
    if world == 1:
        return np.array(local)
    arr = np.ascontiguousarray(local)
    t = torch.from_numpy(arr.copy())
    if device is not None:
        t = t.to(device)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t, group=group)
    bufs = [b.cpu().numpy() for b in bufs]
    out = arr.copy()
    for a, r in owner.items():
        out[a] = bufs[r][a]
    return out


def _gather_device(eng, group=None):
    """Where take_owned_rows' all-gather runs: the GPU under RCCL ("nccl"), host under gloo."""
    return eng.device if dist.get_backend(group) == "nccl" else None


def lrts_update_agent_parallel(eng, store, lrts_agents, group=None):
    """Agent.update of every LR-TS allocator (src/Agent.py:79-91) across ranks: samples
    routed to their agent's owner, each owner trains its agents (ag_lrts_update; agents
    with < 2 samples -- here every agent it does not own -- are left unchanged), then every
    rank loads the owners' posteriors. Bit-identical to one process training on all
    samples (exact sums). Returns the epochs [N] (owners' values)."""
    if _world(group) == 1:
        return eng.lrts_update(store)
    own = owners(lrts_agents, _world(group))
    st = route_records(store, own, group)
    ep = eng.lrts_update(st)
    dev = _gather_device(eng, group)
    m, q, pm = (take_owned_rows(x, own, group, dev) for x in eng.lrts_state())
    eng.load_lrts(m, q, pm, thompson_sampling=eng.ts_sample)
    return take_owned_rows(ep, own, group, dev)


def bidder_update_agent_parallel(eng, store, learners, group=None):
    """Agent.update of every learning bidder (src/Agent.py:79-94 -> Bidder.update) across
    ranks: records routed to their agent's owner (they carry their log order, which the
    trainer restores), each owner trains its own agents (ag_bidder_update with an agent
    mask; synthetic rsample noise keyed by agent and log position, so the fit does not
    depend on the rank), then every rank takes the owners' models. Returns (epochs [N][3],
    status [N])."""
    world = _world(group)
    N = eng.N
    if world == 1:
        return eng.bidder_update(store, None, np.zeros(N, np.int64), 0)
    rank = dist.get_rank(group)
    own = owners(learners, world)
    st = route_records(store, own, group)
    mask = np.zeros(N, np.int32)
    for a, r in own.items():
        if r == rank:
            mask[a] = 1
    ep = np.zeros((N, 3), np.int32)
    stat = np.zeros(N, np.int32)
    if mask.any():
        ep, stat = eng.bidder_update(st, None, np.zeros(N, np.int64), 0, agents=mask)
    dev = _gather_device(eng, group)
    state, init = eng.dr_state()
    state, init = take_owned_rows(state, own, group, dev), take_owned_rows(init, own, group, dev)
    eng.set_dr_state(state, init)
    return take_owned_rows(ep, own, group, dev), take_owned_rows(stat, own, group, dev)


def _allreduce_sum(t, group=None):
    """In-place int64 SUM over the ranks (RCCL on the device; gloo through host memory)."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def record_counts_over_ranks(eng, store, group=None):
    """(records_total [N], records_base [N]) of a shading store over the ranks: every agent's
    records on all ranks, and the global log-order index of this rank's first one (the ranks
    hold contiguous auction shards in rank order, so a rank's records follow every lower
    rank's). One all-gather of N counts."""
    world = _world(group)
    cnt = np.asarray(eng.shading_counts(store), np.int64)
    if world == 1:
        return cnt, np.zeros_like(cnt)
    dev = _gather_device(eng, group)
    t = torch.from_numpy(cnt.copy())
    if dev is not None:
        t = t.to(dev)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t, group=group)
    allc = np.stack([b.cpu().numpy() for b in bufs])
    rank = dist.get_rank(group)
    return allc.sum(0), allc[:rank].sum(0)


RP_POLL_LAUNCHES = 64  # epoch launches between two polls of the learners' progress (even)
# record-parallel epochs: each block of launches + exchanges captured in a hipGraph. Off by
# default: measured in one process (tools/rp_issue.py, profiles/r05s_rp_issue.log) the eager
# per-epoch loop costs 2-3 us per epoch over the launches issued back to back from C, against
# 33-38 us of kernel per epoch -- the host already runs ahead -- and the graph saved nothing
# there; an untested RCCL-in-graph capture is not worth the 8-GPU run's risk
RP_GRAPH = False


def _capturable(group, exchange):
    """The block can be captured: the exchange runs on the device stream (RCCL, or a
    stand-in device copy); gloo goes through host memory and is issued eagerly."""
    if exchange is not None:
        return True
    return dist.is_initialized() and dist.get_backend(group) == "nccl"


def rp_epoch_blocks(epoch, tot, done, poll=RP_POLL_LAUNCHES, exchange=None, group=None, graph=None):
    """Run the record-parallel epochs until done(): blocks of `poll` (even) iterations of
    [one epoch launch -> exchange of its int64 totals tot[k & 1]], done() polled between blocks.
    The exchange is the SUM over the ranks (_allreduce_sum; `exchange` replaces it, e.g. a
    same-size device copy standing in for it in one process). With graph (default RP_GRAPH)
    and a device-side exchange the first block is captured into a hipGraph (torch.cuda.CUDAGraph)
    and replayed: one host call per block instead of two per epoch. The launches' arguments
    depend only on the launch parity (ag_*_rp_epoch), so an even-length block replays exactly:
    the same launches, in the same order, as the eager loop. Returns the blocks run."""
    if poll % 2:
        raise ValueError("poll must be even (a block must end on the parity it starts with)")
    ex = exchange or (lambda t: _allreduce_sum(t, group))
    graph = RP_GRAPH if graph is None else graph

    def block():
        for _ in range(poll):
            k = epoch()
            ex(tot[k & 1])

    if graph and _capturable(group, exchange):
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):  # recorded, not run: no launch happens here
            block()
        # (rp.k advanced by the even block on the host, no launch ran: the parity is unchanged)
        n = 0
        while True:
            g.replay()
            n += 1
            if done():
                return n
    n = 0
    while True:
        block()
        n += 1
        if done():
            return n


def bidder_update_record_parallel(eng, store, learners, group=None, poll=RP_POLL_LAUNCHES, exchange=None,
                                  graph=None):
    """Agent.update of the exact-sum learning bidders (ValueLearningBidder, DoublyRobustBidder;
    src/Bidder.py:204-325, :473-615) record-parallel: every rank trains every learner on its own
    records, one launch per epoch (ag_bidder_rp_epoch), each epoch's exact int64 partial sums
    all-reduced (SUM) before the next launch -- every rank steps to the same model, bit for bit
    the model one process fits on all the records (synthetic rsample draws keyed by the
    records' global log-order index). Returns (epochs [N][3], status [N])."""
    N = eng.N
    world = _world(group)
    mask = np.zeros(N, np.int32)
    mask[list(learners)] = 1
    total, base = record_counts_over_ranks(eng, store, group)
    tot = eng.bidder_rp_begin(store, agents=mask, records_total=total, records_base=base)
    sel = mask.astype(bool)

    def done():
        fit, ep, _ = eng.bidder_rp_poll()
        return bool((fit[sel] < 0).all())
    if world > 1 or exchange is not None:
        rp_epoch_blocks(lambda: eng.bidder_rp_epoch(1), tot, done, poll, exchange, group, graph)
    else:  # one process, nothing to exchange: the launches back to back from C
        while True:
            eng.bidder_rp_epoch(4 * poll)
            if done():
                break
    return eng.bidder_rp_end()


def record_parallel_pays(num_learners, world):
    """DESIGN.md section 7's cost model: agent-parallel gives each owner ceil(A / G) agents of
    G times one GPU's records, i.e. ceil(A / G) * G / A of one GPU's update work; record-parallel
    keeps one GPU's work plus one small all-reduce per epoch. The threshold is a cost model, not
    a measurement: no 8-GPU run of the update exists here (the per-epoch issue cost at world 1
    is measured, tools/rp_issue.py)."""
    A = int(num_learners)
    if world <= 1 or A == 0:
        return False
    return -(-A // world) * world / A > 1.6


def bidder_update(eng, store, learners, group=None):
    """Agent.update of every learning bidder across ranks: record-parallel where it pays
    (exact-sum learners only, A < G per record_parallel_pays), else agent-parallel."""
    learners = [int(a) for a in learners]
    exact = all(int(eng._bkind[a]) in (2, 4) for a in learners)  # ValueLearning, DoublyRobust
    if exact and record_parallel_pays(len(learners), _world(group)):
        return bidder_update_record_parallel(eng, store, learners, group)
    return bidder_update_agent_parallel(eng, store, learners, group)


def lrts_update_record_parallel(eng, store, lrts_agents, group=None, poll=RP_POLL_LAUNCHES, exchange=None,
                                graph=None):
    """Agent.update of the LR-TS allocators (src/BidderAllocation.py:29-65) record-parallel:
    every rank keeps its own won samples, the fit runs one launch per epoch (ag_lrts_rp_epoch)
    with each epoch's exact partials (and the Laplace terms) all-reduced -- every rank ends
    with the posterior one process computes from all samples. Returns the epochs [N]."""
    N = eng.N
    world = _world(group)
    mask = np.zeros(N, np.int32)
    mask[list(lrts_agents)] = 1
    n = int(store["count"][0].item())
    key = store["key"][:n]
    cnt = torch.bincount((key.to(torch.int64) >> 16) & 0xFFFF, minlength=N)[:N].to(torch.int64)
    if world > 1:
        dev = _gather_device(eng, group)
        t = cnt.to(dev) if dev is not None else cnt.cpu()
        _allreduce_sum(t, group)
        cnt = t
    tot = eng.lrts_rp_begin(store, agents=mask, samples_total=cnt.cpu().numpy())
    if world > 1 or exchange is not None:
        rp_epoch_blocks(lambda: eng.lrts_rp_epoch(1), tot, lambda: eng.lrts_rp_poll() == 0, poll, exchange, group,
                        graph)
    else:
        while True:
            eng.lrts_rp_epoch(4 * poll)
            if eng.lrts_rp_poll() == 0:
                break
    return eng.lrts_rp_end()


def lrts_update(eng, store, lrts_agents, group=None):
    """Agent.update of every LR-TS allocator across ranks: record-parallel where it pays (few
    allocators for the ranks, record_parallel_pays), else agent-parallel."""
    lrts_agents = [int(a) for a in lrts_agents]
    if record_parallel_pays(len(lrts_agents), _world(group)):
        return lrts_update_record_parallel(eng, store, lrts_agents, group)
    return lrts_update_agent_parallel(eng, store, lrts_agents, group)
