#!/usr/bin/env python3
"""bench.py's CPU baseline legs (TEST INFRASTRUCTURE: the checker timed on the host, never the product).

BASELINE.md §3: the baseline on the GPU box is the build's CPU restatement of the reference's
compat path (oracle/compat.py + liboracle.so -- process() + decode() through the MAC PDU stage,
/root/reference/tetraear/signal/processor.py:221-273 and core/decoder.py:835-1100), verified equal
to the reference in the build container through tests/golden.  It is timed single-core and on all
cores the box grants, in worker PROCESSES (the restatement's Python holds the GIL; threads do not
scale), each a fresh interpreter started as a child (never a fork of the GPU-initialised bench
process).  Beside it, the ETSI chain's C oracle (oracle/etsi_oracle.c: channel filter, timing,
sync, Viterbi), whose C calls release the GIL, in a thread pool.

    python tools/cpu_baseline.py --compat-worker SECONDS   # one worker: prints its chunk count
"""
import argparse
import concurrent.futures
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
FS = 2.4e6


def _paths():
    for p in (os.path.join(REPO, "oracle"), os.path.join(REPO, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _compat_chunks(N, k=4, seed=0):
    import numpy as np
    _paths()
    import _signals
    rng = np.random.default_rng(seed)
    return [_signals.family("tetra", rng, N, FS)[0] for _ in range(k)]


def compat_loop(chunks, seconds):
    """process() + decode() of the compat restatement, chunk after chunk, for `seconds`."""
    _paths()
    import compat as oracle
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        h = oracle.SignalProcessor(FS).process(chunks[n % len(chunks)], 0)
        oracle.decode_with_mac(h)
        n += 1
    return n, time.perf_counter() - t0


def host_cores():
    """Cores this process may use: the affinity set, capped by OMP_NUM_THREADS (16 on a one-GPU box)."""
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", str(n)))))


def compat_rate(N, single_s, all_s, procs=None):
    """Compat restatement: single-core Msamples/s in this process, then all-core over `procs`
    child processes running concurrently for all_s seconds."""
    chunks = _compat_chunks(N)
    compat_loop(chunks, 0.2)   # warm (library load, first-call costs)
    n1, dt1 = compat_loop(chunks, single_s)
    procs = procs or host_cores()
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1",
               HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.abspath(__file__), "--compat-worker", str(all_s), "--samples", str(N)]
    t0 = time.perf_counter()
    ps = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, env=env) for _ in range(procs)]
    outs = [json.loads(p.communicate(timeout=all_s + 120)[0]) for p in ps]
    wall = time.perf_counter() - t0
    total = sum(o["chunks"] for o in outs)
    # each worker times its own loop (interpreter start excluded); the pool rate is the sum of the
    # workers' rates, all running at once
    vall = sum(o["chunks"] * N / o["seconds"] for o in outs) / 1e6
    return dict(value=vall, unit="Msamples/s", cores=procs, kind="port", single_thread_value=n1 * N / dt1 / 1e6,
                sample=f"compat restatement (oracle/compat.py: process() + decode() with the MAC PDU stage) on "
                       f"{N}-sample cf32 chunks @2.4 MSps: 1 core {n1} chunks in {dt1:.1f} s; {procs} worker "
                       f"processes {total} chunks in {all_s:.0f} s each ({wall:.1f} s wall)")


def etsi_rate(x, cells, seconds, threads=None):
    """ETSI chain C oracle: one thread for a third of `seconds`, then a thread pool for the rest."""
    import numpy as np
    _paths()
    import etsi as oracle
    N = x.shape[1]

    def worker(deadline, k0):
        rx = oracle.Receiver(FS)
        n = 0
        while time.perf_counter() < deadline:
            sym, soft, hard, _ = rx.demod(x[(k0 + n) % len(x)])
            rx.lower_mac(soft, hard, int(cells[(k0 + n) % len(x)]))
            n += 1
        return n

    t0 = time.perf_counter()
    n1 = worker(t0 + seconds / 3, 0)
    v1 = n1 * N / (time.perf_counter() - t0) / 1e6
    threads = threads or host_cores()
    t1 = time.perf_counter()
    deadline = t1 + 2 * seconds / 3
    with concurrent.futures.ThreadPoolExecutor(threads) as ex:
        counts = list(ex.map(lambda k: worker(deadline, k), range(threads)))
    vt = sum(counts) * N / (time.perf_counter() - t1) / 1e6
    return dict(value=vt, unit="Msamples/s", cores=threads, single_thread_value=v1,
                sample=f"{sum(counts)} channel chunks x {N} cf32 @2.4 MSps through the ETSI C oracle "
                       f"(chanfilt+timing+sync+Viterbi) on {threads} threads in {2 * seconds / 3:.0f} s; "
                       f"single thread: {n1} chunks")


def wideband_rate(step, seconds):
    """C3 (wideband) on the host: the float64 channeliser restatement (oracle/wideband.py) over one
    timing chunk per carrier (the GPU's chunk length: stride m2 plus the overlap two chunks share),
    then the ETSI C oracle's timing + lower MAC per carrier (a sample of carriers, extrapolated to
    all), one thread.  Rated per stride: the channeliser's time scaled to m2 of the chunk's samples
    (a host chain channelises each sample once), the timing's whole (it re-reads the overlap as the
    GPU does)."""
    import numpy as np
    _paths()
    import etsi as E
    import wideband as W
    from tetraear.signal.wideband import DOWN, P_WB, UP
    d = W.design(step.fs, step.plan.M)
    L, m2 = step.ck.length, step.m2
    nw = (L * DOWN) // UP * step.plan.D + step.plan.M * P_WB + 64 * step.plan.D   # one chunk per carrier
    x = step.x[:nw].cpu().numpy().view(np.complex64)[:, 0]
    t0 = time.perf_counter()
    y = W.channelize(x.astype(np.complex128), d, L).astype(np.complex64)
    t_ch = time.perf_counter() - t0
    cells = step.cells[::step.nchunk].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
    rx = E.Receiver()
    t1 = time.perf_counter()
    k = 0
    while k < step.plan.M and (k < 8 or time.perf_counter() - t0 < seconds):
        sym, soft, hard, _ = rx.timing(y[k])
        rx.lower_mac(soft, hard, int(cells[k]))
        k += 1
    t_c = (time.perf_counter() - t1) / k
    total = t_ch * m2 / L + step.plan.M * t_c
    ns = m2 * step.fs / 72000.0   # wideband samples per stride
    return dict(value=ns / total / 1e6, unit="Msamples/s", cores=1, kind="port",
                sample=f"{nw} samples @{step.fs / 1e6:g} MSps: numpy float64 channeliser ({t_ch:.2f} s, rated for "
                       f"{m2} of {L} samples) + C oracle timing+lower MAC on chunks of {L} samples on {k} of "
                       f"{step.plan.M} carriers (x{step.plan.M / k:.1f} extrapolated), rated per {m2}-sample "
                       f"stride, 1 thread")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compat-worker", type=float, default=None)
    ap.add_argument("--samples", type=int, default=131072)
    a = ap.parse_args()
    if a.compat_worker is not None:
        chunks = _compat_chunks(a.samples, seed=os.getpid())
        compat_loop(chunks, 0.2)
        n, dt = compat_loop(chunks, a.compat_worker)
        print(json.dumps({"chunks": n, "seconds": dt}))
        return
    print(json.dumps(compat_rate(a.samples, 3.0, 6.0)))


if __name__ == "__main__":
    main()
