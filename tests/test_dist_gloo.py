"""N>1 path on CPU: world_size-2 gloo processes run bench.py's own distributed code.

Each rank imports bench.py and uses its seeding (rank_seed), its timing (time_steps: warm-up,
barrier-bracketed timed steps), its max-over-ranks reduction and its whole-job aggregate, with a
CPU step in place of the GPU chain (no GPU here).  A second test shards channels (rank_channels)
through the oracle and checks the gathered results against a single-process run."""
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


def _bench_worker(rank, world, port, q):
    import sys
    import time
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "tetraear-bladerf_amd"), os.path.join(repo, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import bench
    import compat as oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seed = bench.rank_seed(1000, rank)            # the bench's per-rank data seed
    rng = np.random.default_rng(seed)
    x = (0.3 * (rng.standard_normal(8000) + 1j * rng.standard_normal(8000))).astype(np.complex64)
    done = []

    def step():                                   # one "step": this rank's batch through the chain
        done.append(oracle.SignalProcessor(2.4e6).process(x, 0))
        time.sleep(0.05 * (rank + 1))             # rank 1 is the slower one

    elapsed = bench.time_steps(step, 3, 2, world, lambda: None)
    mx = bench.max_over_ranks(elapsed)            # bench's reduction (host tensor on gloo)
    value = bench.aggregate_msps(8000, world, 3, mx)
    allv = [None] * world
    dist.all_gather_object(allv, (seed, elapsed, len(done), done[-1].tolist()))
    if rank == 0:
        q.put((allv, mx, value))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_runs_bench_timing_and_aggregate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    allv, mx, value = q.get(timeout=180)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (s0, e0, n0, h0), (s1, e1, n1, h1) = allv
    assert s0 != s1 and h0 != h1                  # each rank works on its own data
    assert n0 == n1 == 5                          # warm-up 2 + timed 3 steps on every rank
    assert mx == max(e0, e1) and e1 >= 3 * 0.1    # the slowest rank's time
    assert abs(value - 2 * 3 * 8000 / mx / 1e6) < 1e-12   # whole-job: both ranks' samples / max time


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


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    import subprocess
    import sys
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=e,
                          capture_output=True, text=True, timeout=120)


def test_gpus_must_equal_launcher_world():
    """A launcher that started 1 rank for --gpus 2 is refused before any GPU work (rc 2)."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2" in r.stderr and "WORLD_SIZE=1" in r.stderr
    assert '{"metric"' not in r.stdout


def test_gpus_over_visible_devices_refused_on_rccl():
    """Bare --gpus 2 with RCCL needs two visible GPUs (none here): refused, nothing launched."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], TETRA_BENCH_DIST="nccl")
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "visible" in r.stderr


def test_bare_gpus_n_starts_n_ranks_as_a_child(monkeypatch):
    """Bare --gpus 2 starts torch.distributed.run --nproc-per-node 2 on bench.py with the same
    arguments, as a child process, and returns its exit code (the GPU run: tests/test_gpu_dist.py)."""
    import subprocess
    import sys
    sys.path.insert(0, REPO)
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("TETRA_BENCH_DIST", "gloo")
    argv = ["bench.py", "--gpus", "2", "--channels", "256", "--steps", "3"]
    monkeypatch.setattr(sys, "argv", argv)
    a = bench.parse()
    assert bench.launch_ranks(a) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert os.path.samefile(cmd[cmd.index("--master-port") + 2], os.path.join(REPO, "bench.py"))
    assert cmd[-len(argv) + 1:] == argv[1:]
    # one rank, or a launcher-started rank, runs in this process
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "1"])
    assert bench.launch_ranks(bench.parse()) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.launch_ranks(bench.parse()) is None
