"""Channel sharding across GPUs (one process per GPU, torch.distributed).

25 kHz channels are independent: rank r of W owns a contiguous block of channels and
runs the whole chain on them with no data-path collective.  The only collective is the timing
reduction (max elapsed over ranks) the benchmark contract asks for.
"""


def rank_channels(total, world, rank):
    """Contiguous block of channels for `rank`: (first, count); blocks differ by at most one."""
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def rank_seed(base_seed, rank):
    return base_seed + 1000 * rank


def max_over_ranks(value, device=None, force=False):
    """max of a float over all ranks (identity when torch.distributed is not initialised).  With a
    `device` the reduction runs on a device tensor (RCCL); `force` runs it even in a one-rank group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size() == 1 and not force):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_msps(samples_per_rank, world, steps, elapsed_s):
    """Whole-job throughput: samples processed by all ranks / slowest rank's time."""
    return samples_per_rank * world * steps / elapsed_s / 1e6
