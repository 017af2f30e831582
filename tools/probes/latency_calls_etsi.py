"""Diagnostic: 40 one-chunk ETSI process() + decode() calls for a HIP API trace
(rocprofv3 --hip-trace --kernel-trace --stats -- python tools/probes/latency_calls_etsi.py)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))
from tetraear.signal import SignalProcessor  # noqa: E402
from tetraear.core import TetraDecoder  # noqa: E402
from tetraear.signal.etsi import synth  # noqa: E402

iq, cells = synth(1, 131072, seed=7, snr_db=18.0)[:2]
x = np.ascontiguousarray(iq[0])
p = SignalProcessor(2.4e6, mode="etsi")
d = TetraDecoder(mode="etsi")
d._etsi_rx().cell_state = np.array([cells[0]], np.uint32)
for _ in range(5):
    d.decode(p.process(x))
tp, td = [], []
for _ in range(40):
    t0 = time.perf_counter()
    h = p.process(x)
    t1 = time.perf_counter()
    d.decode(h)
    t2 = time.perf_counter()
    tp.append(t1 - t0)
    td.append(t2 - t1)
print("median ms process", round(1e3 * float(np.median(tp)), 4), "decode", round(1e3 * float(np.median(td)), 4))
