"""Column sharding across GPUs (one process per GPU, torch.distributed: RCCL on GPUs, gloo on CPU).

Columns are independent in every hot-path routine (no reference routine couples columns), so a
contiguous column range per rank is the whole decomposition.  The only exchange is the final
all-gather of broadband flux slabs (north star), done once per job, not per step.
"""
import torch
import torch.distributed as dist


def column_range(ncol, rank, world):
    """Contiguous [lo, hi) column range of `rank`; the first ncol % world ranks get one extra column."""
    base, extra = divmod(ncol, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_columns(local, ncol, world):
    """All-gather per-rank (ncol_local, ...) slabs into the full (ncol, ...) array on every rank.
    Shards may differ by one column; they are padded to equal size for the collective."""
    per = -(-ncol // world)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    parts = []
    for r in range(world):
        lo, hi = column_range(ncol, r, world)
        parts.append(outs[r][:hi - lo])
    return torch.cat(parts, dim=0)
