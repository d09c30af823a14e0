"""Multi-GPU: independent auction shards, one process per GPU, one tiny collective.

Auctions are independent given agent state, so a batch of B auctions
is split into contiguous shards of global auction indices, one per rank; synthetic
inputs are keyed by the global index (ag_generate), so every per-auction output is the
same whatever the number of GPUs. The only exchange is the per-agent counter sums: exact
int64 fixed-point limbs (include/auctiongym.h AG_FX_*), summed with an int64 all-reduce
(RCCL over xGMI with backend "nccl", gloo on CPU) -- integer addition, so the totals are
bit-identical for any world size and any reduction order.
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


def gather_records(store, group=None):
    """All-gather a record store across ranks (LR-TS won samples: key [cap], x [Do][cap],
    count [1]; or shading records: agent / gamma / utility [cap], count [1]) into one store
    holding every rank's records, on every rank. The updates' sums are exact, so training on
    the gathered records gives bit-identical results on every rank and equals a single
    process training on the whole batch -- the update needs no per-epoch collective.
    One all-gather of the counts, one of each record array (padded to the largest count)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return store
    world = dist.get_world_size(group)
    n = store["count"].clone()
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    mx = max(max(counts), 1)
    total = sum(counts)
    fields = [k for k in store if k != "count"]
    out = {}
    for k in fields:
        v = store[k]
        lead = v.shape[:-1]
        if v.shape[-1] < mx:
            raise ValueError(f"store field {k} holds {v.shape[-1]} < {mx} records")
        part = v[..., :mx].contiguous()
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
