"""N>1 path on CPU: world_size-2 gloo processes shard channels and reduce timing like bench.py.

Each rank runs its channel block through the CPU oracle (no GPU here); the gathered results must
equal a single-process run over all channels, and max-over-ranks must be the slowest rank's time."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "tetraear-bladerf_amd"), os.path.join(repo, "oracle")]
    import torch.distributed as dist
    from tetraear.shard import rank_channels, max_over_ranks, aggregate_msps
    import compat as oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = rank_channels(total, world, rank)
    out = {}
    for ch in range(first, first + count):
        rng = np.random.default_rng(100 + ch)
        x = (0.3 * (rng.standard_normal(4000) + 1j * rng.standard_normal(4000))).astype(np.complex64)
        out[ch] = oracle.SignalProcessor(2.4e6).process(x, 0).tolist()
    elapsed = 1.0 + rank            # rank 1 is the slowest
    mx = max_over_ranks(elapsed)
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        q.put((merged, mx, aggregate_msps(count * 4000, world, 1, mx)))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_channels_partition():
    from tetraear.shard import rank_channels
    for total in (1, 7, 8, 65536, 65537):
        for world in (1, 2, 4, 8):
            blocks = [rank_channels(total, world, r) for r in range(world)]
            assert sum(c for _, c in blocks) == total
            assert all(blocks[r][0] + blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    assert rank_channels(65536, 8, 3) == (3 * 8192, 8192)


def test_two_rank_gloo_matches_single_process():
    import sys
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    total = 6
    ps = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in ps:
        p.start()
    merged, mx, agg = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert mx == 2.0
    import compat as oracle
    for ch in range(total):
        rng = np.random.default_rng(100 + ch)
        x = (0.3 * (rng.standard_normal(4000) + 1j * rng.standard_normal(4000))).astype(np.complex64)
        assert merged[ch] == oracle.SignalProcessor(2.4e6).process(x, 0).tolist()
    assert abs(agg - 3 * 4000 * 2 / 2.0 / 1e6) < 1e-12
