"""C2 (BASELINE.json configs[1]): one 25 kHz channel on one MI355X, called the way the reference's
CaptureThread calls it (modern.py:2029-2034: one 131072-sample complex64 chunk from host memory per
call, then decode) -- the per-chunk latency against the chunk's 54.6 ms of air at 2.4 MSps.

Times, per chunk (median of --reps calls after warm-up):
  * etsi:   SignalProcessor(mode="etsi").process(x) + TetraDecoder(mode="etsi").decode(hard)
  * compat: SignalProcessor().process(x, f) + TetraDecoder().decode(hard)   (the reference's semantics,
            the default scipy-exact form); compat_blocked: the opt-in latency mode's process()
  * batch:  EtsiReceiver.demod_batch + EtsiLowerMac.decode_batch over C host channels at once
Host buffers in and out (H2D / D2H included): this is the drop-in's latency, not the HBM-resident
throughput bench.py reports.  usage: python tools/latency_c2.py [--reps 50]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tetraear-bladerf_amd"))


def med_ms(fn, reps):
    for _ in range(3):
        fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from tetraear.signal import SignalProcessor
    from tetraear.signal.etsi import synth, EtsiReceiver
    from tetraear.core import TetraDecoder
    from tetraear.core.etsi import EtsiLowerMac

    N, fs = 131072, 2.4e6
    air_ms = 1e3 * N / fs
    iq, cells, _, _, _ = synth(64, N, seed=7, snr_db=18.0, cfo_max=600.0)
    out = {"chunk_samples": N, "air_ms": round(air_ms, 2)}

    p = SignalProcessor(fs, mode="etsi")
    d = TetraDecoder(mode="etsi")
    d._etsi_rx().cell_state = np.array([cells[0]], np.uint32)   # as if acquired from an earlier chunk
    x = np.ascontiguousarray(iq[0])
    out["etsi_process_ms"] = med_ms(lambda: p.process(x), a.reps)
    hard = p.process(x)
    out["etsi_decode_ms"] = med_ms(lambda: d.decode(hard), a.reps)
    out["etsi_frames"] = len(d.decode(hard))

    pc = SignalProcessor(fs)
    dc = TetraDecoder(auto_decrypt=False)
    out["compat_process_ms"] = med_ms(lambda: pc.process(x, 1171.875), a.reps)
    hc = pc.process(x, 1171.875)
    out["compat_decode_ms"] = med_ms(lambda: dc.decode(hc), a.reps)
    pb = SignalProcessor(fs, decimator="blocked")   # the opt-in latency mode (not bit-exact)
    out["compat_blocked_process_ms"] = med_ms(lambda: pb.process(x, 1171.875), a.reps)

    rx, mac = EtsiReceiver(), EtsiLowerMac()
    for C in (1, 8, 64):
        xb = np.ascontiguousarray(iq[:C])

        def run():
            h, sb, sym, ns = rx.demod_batch(xb)
            mac.decode_batch(sb, h, ns, cells[:C])
        ms = med_ms(run, max(5, a.reps // 5))
        out[f"batch{C}_ms"] = round(ms, 3)
        out[f"batch{C}_realtime_x"] = round(C * air_ms / ms, 1)
    for k in list(out):
        if isinstance(out[k], float):
            out[k] = round(out[k], 3)
    out["etsi_realtime_x"] = round(air_ms / (out["etsi_process_ms"] + out["etsi_decode_ms"]), 1)
    out["compat_realtime_x"] = round(air_ms / (out["compat_process_ms"] + out["compat_decode_ms"]), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
