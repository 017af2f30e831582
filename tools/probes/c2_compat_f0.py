"""C2 compat process() latency with and without an AFC offset (one 131072-sample chunk from host
memory, median of 30 calls): what the filtfilt's mixer-free path costs against the pre-mixed one.
Round 6, final library: 7.010 ms at offset 0, 6.988 ms at 2343.75 Hz -- the same."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "tetraear-bladerf_amd"))
from tetraear.signal import SignalProcessor   # noqa: E402
from tetraear.signal.etsi import synth   # noqa: E402

iq = synth(1, 131072, seed=7, snr_db=18.0, cfo_max=600.0)[0][0]
p = SignalProcessor(2.4e6)
for f in (0.0, 2343.75):
    for _ in range(3):
        p.process(iq, f)
    t = []
    for _ in range(30):
        t0 = time.perf_counter()
        p.process(iq, f)
        t.append(time.perf_counter() - t0)
    print(f"freq_offset {f}: {1e3 * np.median(t):.3f} ms", flush=True)
