"""Latency probe of k_timing on the wideband bench's carrier chunks (run on the GPU box).

TETRA_TIMING_PROBE=1 makes each chunk's diag entry hold four wall-clock stamps: the wave's start, the
end of its Oerder-Meyr pass, the end of its Gardner loop, and its end.  This prints, per k_timing form,
the kernel span, the spread of wave start times, and the per-phase durations (median / p90) in µs; the
wall-clock rate is calibrated against the launch's HIP-event time.
usage: python tools/probe_timing.py [NW]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tetraear-bladerf_amd"))
from tetraear import _hip  # noqa: E402
from tetraear.signal.wideband import BenchStep  # noqa: E402


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    dev = torch.device("cuda", 0)
    c = _hip.ctx()
    c.check(c.lib.tetra_set_stream(c.handle, None), "set_stream")
    st = BenchStep(c, nw, seed=1, device=dev)
    st._front(c, st.y, None)   # waterfall + channeliser: y for every carrier chunk (plain k_timing forms: no om)
    torch.cuda.synchronize(dev)
    C, m2, sm = st.C, st.m2, st.sm
    diag = torch.zeros((C, 4), dtype=torch.float32, device=dev)
    forms = [(f"RING={r} LEAN={l}", {"TETRA_TIMING_RING": r, "TETRA_TIMING_LEAN": l})
             for r, l in (("0", "1"), ("1", "1"), ("2", "1"), ("0", "0"))]
    for name, env in forms:
        os.environ.update(env)
        for probe in ("0", "1", "0", "1"):
            os.environ["TETRA_TIMING_PROBE"] = probe
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            c.check(c.lib.tetra_etsi_timing(c.handle, st.etsi, _hip.ptr(st.y), C, m2, _hip.ptr(st.sym),
                                            _hip.ptr(st.soft), _hip.ptr(st.hard), _hip.ptr(st.nsym), sm,
                                            _hip.ptr(diag)), "etsi_timing")
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1)
            if probe == "0":
                ms_plain = ms
                continue
            t = diag.cpu().numpy().view(np.uint32).astype(np.int64)
            t = (t - t[:, :1].min()) % (1 << 32)
            span = t[:, 3].max() - t[:, 0].min()
            tick_us = ms * 1e3 / span          # calibrated: µs per wall-clock tick
            om, gard, dec, tot = (t[:, 1] - t[:, 0]), (t[:, 2] - t[:, 1]), (t[:, 3] - t[:, 2]), (t[:, 3] - t[:, 0])
            q = lambda a: f"{np.median(a) * tick_us:6.1f} / {np.percentile(a, 90) * tick_us:6.1f}"
            print(f"{name}: launch {ms_plain:.4f} ms plain, {ms:.4f} ms probed; tick {tick_us * 1e3:.2f} ns; "
                  f"start spread med/p90/max {np.median(t[:, 0]) * tick_us:.1f} / "
                  f"{np.percentile(t[:, 0], 90) * tick_us:.1f} / {t[:, 0].max() * tick_us:.1f} us")
            print(f"   per chunk (median / p90 us): OM {q(om)}  Gardner {q(gard)}  decide {q(dec)}  total {q(tot)}")
    os.environ["TETRA_TIMING_PROBE"] = "0"


if __name__ == "__main__":
    main()
