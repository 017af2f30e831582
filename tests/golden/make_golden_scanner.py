#!/usr/bin/env python3
"""Record the reference's scanner detector on seeded inputs (TEST INFRASTRUCTURE).

Run in the build container only (the reference does not exist on the GPU box):

    python tests/golden/make_golden_scanner.py     # writes tests/golden/g5_scanner.npz

Imports /root/reference/tetraear/signal/scanner.py's ``TetraSignalDetector`` (scanner.py:24-289),
with the oracle's ``bitstring`` shim on sys.path so its frame validation (scanner.py:149-202) can
import the reference's SignalProcessor / TetraDecoder, and records, per case:
calculate_power, detect_tetra_modulation, detect_sync_pattern, check_power_stability,
validate_frames and analyze_signal.  Only inputs and outputs are stored.

Cases: the shape of the reference's own ``sample_iq_samples`` fixture (tests/conftest.py:53-67,
seeded) and of its ``test_modulation_confidence_scaling`` inputs; TETRA chunks at 1.8 and 2.4 MSps
(the golden families' generator, on the SC16 grid); symbol walks whose frames the reference's own
process() + decode() validate (all CRC-good, some CRC-bad, a single frame); clipped captures pinned
to the diagonals (the +-pi wrap edge); lengths below 1000 and below 100 strided samples, an empty
chunk; a 72 kHz carrier row (D = 1); each as complex64 and complex128.
"""
import os
import sys
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("TETRA_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "oracle", "shim"))
sys.path.insert(0, REF)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from tetraear.signal import scanner as ref_scanner  # noqa: E402  (the reference)
from tetraear.signal.scanner import TetraSignalDetector  # noqa: E402

import _signals  # noqa: E402

warnings.simplefilter("ignore")

# analyze_signal's dict, in this order, as float64 (bools as 0/1)
AN_KEYS = ["power_db", "is_tetra", "confidence", "modulation_confidence", "sync_detected", "sync_correlation",
           "frames_validated", "crc_pass_rate", "power_stable", "signal_present"]
OUT_KEYS = ["power", "mod_flag", "mod_conf", "sync_flag", "sync_corr", "stable", "val_flag", "val_rate"] + \
           ["an_" + k for k in AN_KEYS]


def _steps_walk(sym, rep=130, off=65, tail=2000, phase0=0.3):
    """A constant-envelope walk whose symbol-to-symbol phase steps sit at the centres of the
    reference demod's decision regions (0 -> 0, 1 -> pi/2, 2 -> -pi/2, 3 -> pi; processor.py:152-161),
    held for rep = 130 samples per symbol: 2.4 MSps decimated by 10 gives the reference's integer 13
    samples per symbol (processor.py:183), so process() returns `sym` and decode() sees its frames.
    Returned as (constellation index per symbol, the 4 points, (rep, off))."""
    quarter = {0: 0, 1: 1, 2: 3, 3: 2}
    k = np.concatenate([[0], np.cumsum([quarter[int(v)] for v in sym])]) % 4
    k = np.concatenate([k, np.full(tail // rep + 1, k[-1])]).astype(np.uint8)
    pts = np.exp(1j * (phase0 + np.pi / 2 * np.arange(4))).astype(np.complex64)
    return k, pts, (rep, off)


def valid_frames_stream(rng, nfr, bad):
    """nfr 510-bit normal bursts with TS1 at bit 216 and a valid CRC-16 (make_golden's GF(2) fix),
    frames in `bad` with their CRC broken by 4 flipped data bits."""
    import make_golden as MG
    from tetraear.core.protocol import TetraProtocolParser
    parser = TetraProtocolParser()
    frames = []
    for k in range(nfr):
        f = rng.integers(0, 2, 510).astype(np.uint8)
        f[216:238] = _signals.TS_N
        f[255:277] = 0
        f = MG._crc_fix(parser, f, list(range(150, 200)))
        if k in bad:
            f[[20, 41, 63, 87]] ^= 1
        frames.append(f)
    bits = np.concatenate(frames)
    return (bits[0::2] << 1 | bits[1::2]).astype(np.uint8)


def cases():
    """(name, sample_rate, stored input) -- stored as ("c"|"q"|"k", arrays); each case also runs as
    complex128."""
    out = []
    for seed in range(2):   # tests/conftest.py:53-67: a baseband tone plus 0.1 complex noise, 10 ms at 2.4 MSps
        rng = np.random.default_rng(700 + seed)
        t = np.arange(0, 0.01, 1 / 2.4e6)
        iq = np.exp(1j * 2 * np.pi * 0 * t) + (rng.standard_normal(len(t)) + 1j * rng.standard_normal(len(t))) * 0.1
        out.append((f"conftest_{seed}", 2.4e6, ("c", iq.astype(np.complex64))))
    rng = np.random.default_rng(710)   # test_frequency_scanner.py: noise and a slow phase ramp, 2000 samples
    noise = (rng.standard_normal(2000) + 1j * rng.standard_normal(2000)).astype(np.complex64)
    out.append(("noise_2000", 2.4e6, ("c", noise)))
    out.append(("ramp_2000", 2.4e6, ("c", np.exp(1j * np.linspace(0, 4 * np.pi, 2000)).astype(np.complex64))))
    for fs, seed in ((2.4e6, 720), (1.8e6, 721)):
        _, q = _signals.family("tetra", np.random.default_rng(seed), 32768, fs)
        out.append((f"tetra_{int(fs / 1e3)}k_{seed}", fs, ("q", q)))
    # frames the reference decodes: all CRC-good, some CRC-bad (the pass rate must exceed 0.5), one
    # frame (validation needs two)
    for name, nfr, bad in (("valid_6of6", 6, ()), ("valid_3of6", 6, (1, 2, 4)), ("valid_2of3", 3, (1,)),
                           ("valid_2of4", 4, (0, 2)), ("valid_1of1", 1, ())):
        sym = valid_frames_stream(np.random.default_rng(760 + nfr), nfr, bad)
        out.append((name, 2.4e6, ("k",) + _steps_walk(sym)))
    rng = np.random.default_rng(730)   # clipped capture: every sample on a diagonal, steps of exactly 0, +-pi/2, pi
    diag = (rng.choice([-1.0, 1.0], 20000) + 1j * rng.choice([-1.0, 1.0], 20000)).astype(np.complex64)
    out.append(("clipped_diagonals", 2.4e6, ("c", diag)))
    rng = np.random.default_rng(731)   # half the samples clipped, half small noise
    mix = (0.05 * (rng.standard_normal(20000) + 1j * rng.standard_normal(20000))).astype(np.complex64)
    mix[::2] = diag[::2]
    out.append(("half_clipped", 2.4e6, ("c", mix)))
    _, q = _signals.family("tetra", np.random.default_rng(740), 20000, 2.4e6)
    out.append(("short_999", 2.4e6, ("q", q[:999])))             # < 1000: no modulation test
    out.append(("short_1000", 2.4e6, ("q", q[:1000])))
    out.append(("strided_99", 2.4e6, ("q", q[:13 * 99])))        # 99 strided samples: no sync test
    out.append(("strided_100", 2.4e6, ("q", q[:13 * 99 + 1])))
    out.append(("stability_4999", 2.4e6, ("q", q[:4999])))       # < 5 x 1000: never stable
    out.append(("empty", 2.4e6, ("c", np.zeros(0, np.complex64))))
    rng = np.random.default_rng(750)   # a 72 kHz carrier row (D = 1): pi/4-DQPSK at 4 samples per symbol + noise
    steps = rng.choice([1, 3, -1, -3], 3000) * np.pi / 4
    y = np.repeat(np.exp(1j * (0.4 + np.cumsum(steps))), 4)
    y = y + 0.05 * (rng.standard_normal(len(y)) + 1j * rng.standard_normal(len(y)))
    out.append(("carrier_72k", 72000.0, ("c", y.astype(np.complex64))))
    return out


def record(fs, x):
    det = TetraSignalDetector(sample_rate=fs)
    pw = det.calculate_power(x)
    mf, mc = det.detect_tetra_modulation(x)
    sf, sc = det.detect_sync_pattern(x)
    st = det.check_power_stability(x)
    vf, vr = det.validate_frames(x)
    an = det.analyze_signal(x)
    row = [pw, mf, mc, sf, sc, st, vf, vr] + [an[k] for k in AN_KEYS]
    return np.array([float(v) for v in row], np.float64)


def main():
    assert ref_scanner.DECODER_AVAILABLE, "the reference's frame validation needs its decoder (bitstring shim)"
    arrays, names, rates, dts, outs, idx = {}, [], [], [], [], []
    for i, (name, fs, (kind, *data)) in enumerate(cases()):
        if kind == "k":
            arrays[f"k_{i}"], arrays[f"p_{i}"], arrays[f"r_{i}"] = data[0], data[1], np.array(data[2], np.int64)
        else:
            arrays[f"{kind}_{i}"] = data[0]
        x = _signals.scanner_input(_Z(arrays), i)
        for dt in (np.complex64, np.complex128):
            names.append(name)
            rates.append(fs)
            idx.append(i)
            dts.append(64 if dt == np.complex64 else 128)
            outs.append(record(fs, x.astype(dt)))
            print(f"{name:20s} c{dts[-1]:<4d} " + " ".join(f"{k}={v:.6g}" for k, v in zip(OUT_KEYS[:8], outs[-1])))
    np.savez_compressed(os.path.join(HERE, "g5_scanner.npz"), **arrays, case=np.array(names), fs=np.array(rates),
                        dtype=np.array(dts), input=np.array(idx), out=np.stack(outs), out_keys=np.array(OUT_KEYS),
                        numpy_version=np.array(np.__version__))


class _Z(dict):
    """The arrays dict read like an NpzFile (files + item access) by _signals.scanner_input."""
    @property
    def files(self):
        return list(self)


if __name__ == "__main__":
    main()
