"""nsd_dist.py - multi-GPU plumbing of the dissection path.

One process per GPU.  Packets are independent, so a batch shards into
contiguous packet ranges with no data-path collective; the only exchange is
the per-protocol counter vector (NSD_NCOUNTERS x u64, 512 B), summed with one
all-reduce (RCCL over xGMI on MI355X, gloo in the CPU tests)."""
import torch


def shard_range(total, rank, world):
    """Contiguous [lo, hi) of `total` packets for `rank` (strong scaling)."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi


def weak_shard(per_rank, rank):
    """Weak scaling: every rank owns its own `per_rank` packets."""
    return rank * per_rank, (rank + 1) * per_rank


def reduce_counters(counters, group=None):
    """Sum the counter vectors of all ranks in place (int64 tensor)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def max_over_ranks(values, device, group=None):
    """Max of a list of floats over ranks (bench timing)."""
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(x) for x in t]
