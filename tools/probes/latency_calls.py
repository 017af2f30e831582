"""Diagnostic: 40 one-chunk compat process() calls (latency mode) for a HIP API trace
(rocprofv3 --hip-trace --kernel-trace --stats -- python tools/probes/latency_calls.py)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))
from tetraear.signal import SignalProcessor  # noqa: E402
from tetraear.signal.etsi import synth  # noqa: E402

x = np.ascontiguousarray(synth(1, 131072, seed=7, snr_db=18.0)[0][0])
p = SignalProcessor(2.4e6)
for _ in range(5):
    p.process(x, 1171.875)
t = []
for _ in range(40):
    t0 = time.perf_counter()
    p.process(x, 1171.875)
    t.append(time.perf_counter() - t0)
print("median ms", round(1e3 * float(np.median(t)), 4))
