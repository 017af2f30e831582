#!/usr/bin/env python3
"""Where the fused ETSI demod's workgroups spend their time (GPU box): TETRA_TIMING_PROBE=1 makes each
channel's diag entry hold four wall-clock stamps -- the workgroup's start, the end of its channel-filter
stream (the tail's start), the end of its Gardner tracking, and its end.  Prints the per-workgroup
stream and tail durations, and over the launch how many workgroups are streaming and how many are in
their tail (the tail runs one tracking wave while the rest wait: the CU's other workgroup streams).
usage: python tools/probe_demod_tail.py [C] [N] [cf32|sc16]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))
import torch  # noqa: E402

from tetraear import _hip  # noqa: E402
from tetraear.signal.etsi import BenchStep  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
    fmt = sys.argv[3] if len(sys.argv) > 3 else "cf32"
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    st = BenchStep(c, C, N, 2.4e6, seed=1000, device=dev, iq_format=fmt, cells="given")
    diag = torch.zeros((C, 4), dtype=torch.float32, device=dev)
    f = _hip.TETRA_SC16 if fmt == "sc16" else _hip.TETRA_CF32

    def run():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        c.check(c.lib.tetra_demod_etsi_fmt(c.handle, st.plan, _hip.ptr(st.iq), f, C, N, _hip.ptr(st.sym),
                                           _hip.ptr(st.soft), _hip.ptr(st.hard), _hip.ptr(st.nsym), st.smax,
                                           _hip.ptr(diag)), "demod")
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1)

    for probe in ("0", "1", "0", "1"):
        os.environ["TETRA_TIMING_PROBE"] = probe
        ms = run()
        if probe == "0":
            print(f"plain launch {ms:.4f} ms")
            continue
        t = diag.cpu().numpy().view(np.uint32).astype(np.int64)
        t = (t - t[:, 0].min()) % (1 << 32)
        span = t[:, 3].max()
        tick = ms * 1e3 / span   # µs per tick
        stream, tail, track = (t[:, 1] - t[:, 0]) * tick, (t[:, 3] - t[:, 1]) * tick, (t[:, 2] - t[:, 1]) * tick
        q = lambda a: f"{np.median(a):6.1f} / {np.percentile(a, 90):6.1f}"
        print(f"probed launch {ms:.4f} ms, tick {tick * 1e3:.2f} ns; per workgroup (median / p90 µs): "
              f"stream {q(stream)}  tail {q(tail)}  (tracking {q(track)})")
        # occupancy over time: workgroups streaming / in their tail, in 20 bins
        bins = np.linspace(0, span, 21)
        row = []
        for a, b in zip(bins[:-1], bins[1:]):
            mid = (a + b) / 2
            s = int(((t[:, 0] <= mid) & (t[:, 1] > mid)).sum())
            tl = int(((t[:, 1] <= mid) & (t[:, 3] > mid)).sum())
            row.append(f"{s}/{tl}")
        print("   streaming/tail workgroups over the launch:", " ".join(row))
        print(f"   tail-only time (no stream left on the CU's partner) ~ launch end - last stream end: "
              f"{(span - t[:, 1].max()) * tick:.1f} µs")
    os.environ["TETRA_TIMING_PROBE"] = "0"


if __name__ == "__main__":
    main()
