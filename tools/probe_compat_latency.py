"""Where one compat process() call's time goes (C2, one 131072-sample chunk from host memory):
per-stage device times from the library's HIP-event profile (tetra_profile) for the time-blocked and
the sequential decimator, and the host wall time of the call.  usage: python tools/probe_compat_latency.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))


def stages(c):
    names = ctypes.create_string_buffer(4096)
    ms = (ctypes.c_double * 64)()
    cnt = (ctypes.c_int64 * 64)()
    n = ctypes.c_int(0)
    c.check(c.lib.tetra_profile_read(c.handle, names, 4096, ms, cnt, 64, ctypes.byref(n)), "profile_read")
    raw = names.raw.split(b"\0")
    return {raw[i].decode(): (round(ms[i] / max(1, cnt[i]), 4), int(cnt[i])) for i in range(n.value)}


def main():
    from tetraear import _hip
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import synth
    iq = synth(1, 131072, seed=7, snr_db=18.0)[0]
    x = np.ascontiguousarray(iq[0])
    c = _hip.ctx()
    out = {}
    for dec in ("auto", "sequential"):
        p = SignalProcessor(2.4e6, decimator=dec)
        for _ in range(3):
            p.process(x, 1171.875)
        t = []
        for _ in range(20):
            t0 = time.perf_counter()
            p.process(x, 1171.875)
            t.append(time.perf_counter() - t0)
        c.check(c.lib.tetra_profile(c.handle, 1), "profile")
        stages(c)
        for _ in range(10):
            p.process(x, 1171.875)
        st = stages(c)
        c.check(c.lib.tetra_profile(c.handle, 0), "profile")
        out[dec] = {"wall_ms_median": round(1e3 * float(np.median(t)), 3), "stages_ms": st}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
