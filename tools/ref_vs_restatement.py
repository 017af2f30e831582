#!/usr/bin/env python3
"""Reference vs. compat restatement on the same chunks, single core (BUILD CONTAINER ONLY).

BASELINE.md §3 / SURVEY.md §8d: the GPU box times the build's CPU restatement of the compat path
(tools/cpu_baseline.py), because the reference cannot travel.  This script relates that number back
to the reference: it imports the reference from /root/reference (with the oracle's bitstring shim,
as tests/golden/make_golden.py does) and times its SignalProcessor.process + TetraDecoder.decode
(auto_decrypt=False, /root/reference/tetraear/signal/processor.py:221 and core/decoder.py:835)
next to the restatement (oracle/compat.py process + decode_with_mac) on the same seeded 131072-sample
chunks, one core each, and checks that both decode the same frames.

    python tools/ref_vs_restatement.py > profiles/r03_cpu_ref_vs_restatement.json
"""
import json
import logging
import os
import platform
import sys
import time
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("TETRA_REFERENCE", "/root/reference")
sys.path[:0] = [os.path.join(REPO, "oracle", "shim"), REF, os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tests", "golden")]

import numpy as np  # noqa: E402

warnings.simplefilter("ignore")
logging.disable(logging.CRITICAL)
FS, N = 2.4e6, 131072


def timed(fn, chunks, seconds):
    fn(chunks[0])
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds:
        fn(chunks[n % len(chunks)])
        n += 1
    dt = time.perf_counter() - t0
    return n, dt, n * N / dt / 1e6


def main():
    os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})   # one core
    import _signals
    import compat as O
    from tetraear.signal.processor import SignalProcessor as RefProcessor   # the reference
    from tetraear.core.decoder import TetraDecoder as RefDecoder
    rng = np.random.default_rng(20260130)
    chunks = [_signals.family("tetra", rng, N, FS)[0] for _ in range(4)]

    def ref(x):
        h = RefProcessor(FS).process(x, 0)
        return RefDecoder(auto_decrypt=False).decode(h)

    def port(x):
        return O.decode_with_mac(O.SignalProcessor(FS).process(x, 0))

    same = all([(f["number"], f["header"], f.get("burst_crc")) for f in ref(x)] ==
               [(f["number"], f["header"], f["burst_crc"]) for f in port(x)] for x in chunks)
    nr, dr, vr = timed(ref, chunks, 15.0)
    npt, dp, vp = timed(port, chunks, 15.0)
    print(json.dumps({
        "what": "single-core Msamples/s of process()+decode() on the same 4 seeded 131072-sample cf32 "
                "chunks @2.4 MSps: the reference (/root/reference, bitstring shim) vs the compat "
                "restatement the GPU box times as cpu_baseline (oracle/compat.py + liboracle.so)",
        "host": platform.processor() or platform.machine(), "cpus_visible": os.cpu_count(),
        "reference": {"chunks": nr, "seconds": round(dr, 2), "msps": round(vr, 3)},
        "restatement": {"chunks": npt, "seconds": round(dp, 2), "msps": round(vp, 3)},
        "restatement_over_reference": round(vp / vr, 3),
        "same_frames": bool(same),
        "note": "box cpu_baseline / this ratio = the reference's expected rate on the box's cores",
    }, indent=1))


if __name__ == "__main__":
    main()
