"""Kernel trace target: the default compat process() on one 131072-sample chunk (C2), 30 calls, with
and without an AFC offset -- run under rocprofv3 --kernel-trace --stats to split the 8.5 ms by kernel."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "tetraear-bladerf_amd"))
from tetraear.signal import SignalProcessor   # noqa: E402
from tetraear.signal.etsi import synth   # noqa: E402

iq = synth(1, 131072, seed=7, snr_db=18.0, cfo_max=600.0)[0][0]
p = SignalProcessor(2.4e6)
f = float(os.environ.get("C2_OFFSET", "2343.75"))
for _ in range(30):
    p.process(iq, f)
print("ok", len(p.symbols))
