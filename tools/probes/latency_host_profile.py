"""Host-side cost of one-chunk compat process() calls (C2, the reference's call pattern): cProfile
of 200 calls after warm-up, top entries by own time.  usage: python tools/probes/latency_host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))


def main():
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import synth
    x = np.ascontiguousarray(synth(1, 131072, seed=7, snr_db=18.0)[0][0])
    p = SignalProcessor(2.4e6)
    for _ in range(20):
        p.process(x, 1171.875)
    t0 = time.perf_counter()
    for _ in range(200):
        p.process(x, 1171.875)
    print("wall per call ms", round((time.perf_counter() - t0) / 200 * 1e3, 4))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        p.process(x, 1171.875)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
