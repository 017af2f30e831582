"""bench.py's N>1 path on the GPU box, launched the way the driver launches it (torchrun, one rank
per GPU), as a fresh child process.  A one-GPU box runs both ranks on its card with
TETRA_BENCH_DIST=gloo (rank -> LOCAL_RANK mod device count, the timing reduction on a host tensor);
the driver's 8-GPU run takes the same code path with RCCL.  SURVEY.md §8e: channels are independent
shards, weak scaling, no data-path collective."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torchrun_two_ranks_bench():
    C, N, steps = 256, 131072, 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--channels", str(C), "--samples", str(N),
           "--steps", str(steps), "--warmup", "1", "--no-cpu", "--cells", "given"]
    env = dict(os.environ, TETRA_BENCH_DIST="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one line
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == steps and d["scaling"] == "weak"
    assert d["config"]["channels_per_gpu"] == C
    q = d["decoded_last_step"]
    assert q["blocks"] >= 3 * C and q["crc_ok"] == q["blocks"], q   # every decoded block CRC-good
    # whole-job aggregate = both ranks' samples / the slowest rank's time
    elapsed = d["ms_per_step"] * steps / 1e3
    want = 2 * C * N * steps / elapsed / 1e6
    assert abs(d["value"] - want) <= 1e-3 * want, (d["value"], want)


def test_torchrun_one_rank_rccl():
    """bench.py's RCCL branch on the box's one GPU: torchrun --nproc-per-node 1 with the nccl (= RCCL)
    backend, and TETRA_BENCH_FORCE_DIST=1 so the process group is joined and the timing all_reduce(MAX)
    runs on a device tensor even at world size 1 (bench.py main, shard.max_over_ranks)."""
    C, N, steps = 256, 131072, 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "1", "--channels", str(C), "--samples", str(N),
           "--steps", str(steps), "--warmup", "1", "--no-cpu", "--cells", "given"]
    env = dict(os.environ, TETRA_BENCH_DIST="nccl", TETRA_BENCH_FORCE_DIST="1", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["dist"] == {"backend": "nccl", "world": 1, "reduce_tensor": "cuda"}, d["dist"]
    assert d["n_gpus"] == 1 and d["steps"] == steps
    q = d["decoded_last_step"]
    assert q["blocks"] >= 3 * C and q["crc_ok"] == q["blocks"], q


def test_bare_gpus2_self_launches_two_ranks():
    """`python3 bench.py --gpus 2` with no launcher: bench starts torch.distributed.run
    --nproc-per-node 2 on itself as a child; both ranks share the box's one GPU over gloo and rank 0
    prints the one line, with n_gpus 2 and a world-2 process group."""
    C, N, steps = 256, 131072, 3
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--channels", str(C),
           "--samples", str(N), "--steps", str(steps), "--warmup", "1", "--no-cpu", "--cells", "given"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(TETRA_BENCH_DIST="gloo", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 2 and d["dist"]["world"] == 2 and d["dist"]["backend"] == "gloo", d["dist"]
    q = d["decoded_last_step"]
    assert q["blocks"] >= 3 * C and q["crc_ok"] == q["blocks"], q


def test_one_rank_launcher_given_gpus2_fails_loudly():
    """torchrun --nproc-per-node 1 ... bench.py --gpus 2: refused with a message, no JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--channels", "256", "--steps", "1", "--warmup", "0",
           "--no-cpu"]
    r = subprocess.run(cmd, cwd=REPO, env=dict(os.environ, OMP_NUM_THREADS="4"), capture_output=True, text=True,
                       timeout=110)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
    assert '{"metric"' not in r.stdout
