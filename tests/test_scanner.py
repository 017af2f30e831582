"""The scanner's TETRA signal detector (/root/reference/tetraear/signal/
scanner.py:42-147, 204-289): oracle known answers on the CPU, GPU counts against the oracle.

Parity: the modulation and sync counts are integers; they are equal to the oracle's except where a
phase difference sits within EDGE rad of a decision edge (the device atan2 and the host's libm
atan2f may round the last ulp differently), and the tests count those edges in the oracle and
allow at most that many disagreements.  Powers within 1e-9 relative (float64 sums on the device,
float32 pairwise means in numpy: 1e-6 dB)."""
import numpy as np
import pytest

import scanner as O

FS = 2.4e6
EDGE = 1e-5


def _dqpsk_walk(nsym, sps, rng, phase0=0.3):
    """Ideal pi/4-DQPSK: constant-amplitude symbols held for sps samples (phase steps of odd
    multiples of pi/4 between symbols, 0 within one)."""
    steps = rng.choice([1, 3, -1, -3], nsym) * np.pi / 4
    ph = phase0 + np.cumsum(steps)
    return np.repeat(np.exp(1j * ph), sps)


def _sync_walk(D, before=40, after=80, rng=None):
    """A phase walk whose samples strided by D differ by 0 for a 1 bit and pi/2 for a 0 bit, spelling
    the sync pattern after `before` random bits."""
    rng = rng or np.random.default_rng(0)
    bits = np.concatenate([rng.integers(0, 2, before), O.SYNC_PATTERN, rng.integers(0, 2, after)])
    ph = np.concatenate([[0.0], np.cumsum(np.where(bits == 1, 0.0, np.pi / 2))])
    return np.repeat(np.exp(1j * (0.2 + ph)), D), bits


def _edge_count_mod(x):
    """Differences within EDGE of the cluster test's edges: the multiples of pi/4 +- pi/8, and the
    wrap point +-pi, where (d + pi) % 2 pi - pi sends a difference one ulp below -pi to just under
    +pi (no match) and one ulp above to -pi (a match).  Clipped captures hit that edge often: samples
    pinned to the diagonals (+-1, +-1) differ by exactly -pi up to the last ulp of atan2."""
    x = np.asarray(x)
    x = x / (np.abs(x).max() + 1e-10)
    d = np.diff(np.angle(x)).astype(np.float64)
    w = O._wrap(np.diff(np.angle(x))).astype(np.float64)
    edges = np.pi / 8 + np.pi / 4 * np.arange(-8, 8)
    near = (np.abs(w[:, None] - edges[None, :]).min(axis=1) < EDGE) | (np.abs(np.abs(w) - np.pi) < EDGE)
    near |= np.abs(np.abs(d) - np.pi) < EDGE   # the raw difference at +-pi itself
    return int(near.sum())


# ----------------------------------------------------------------------------- CPU: oracle KATs
def test_oracle_known_answers():
    rng = np.random.default_rng(1)
    x = _dqpsk_walk(1000, 1, rng).astype(np.complex64)   # one sample per symbol: every step is pi/4-odd
    assert O.detect_tetra_modulation(x) == (True, 1.0)
    assert O.detect_tetra_modulation(x[:999]) == (False, 0.0)   # < 1000 samples
    D = max(1, int(FS / 18000 / 10))
    assert D == 13
    y, bits = _sync_walk(D)
    found, corr = O.detect_sync_pattern(y.astype(np.complex64), FS)
    assert found and corr == 1.0
    got, _ = O.sync_bits(y.astype(np.complex64), FS)
    assert np.array_equal(got[:len(bits)], bits)
    # every difference is within pi/8 of a multiple of pi/4 except in (7pi/8, pi): +pi is not among
    # the expected phases.  Tones stepping 7pi/8 -+ 1e-3 per sample: all / none match
    n = np.arange(2000)
    assert O.modulation_counts(np.exp(1j * (7 * np.pi / 8 - 1e-3) * n).astype(np.complex64))[0] == 1999
    assert O.modulation_counts(np.exp(1j * (7 * np.pi / 8 + 1e-3) * n).astype(np.complex64))[0] == 0
    # +pi is not among the expected phases: steps of (pi - 0.05) wrap to (7pi/8, pi) -> no match
    assert O.modulation_counts(np.exp(1j * (np.pi - 0.05) * n).astype(np.complex64))[0] == 0
    assert O.check_power_stability(np.ones(5000)) and not O.check_power_stability(np.ones(4999))
    burst = np.ones(10000, np.complex64)
    burst[:2000] *= 1e-4   # a 80 dB step: the window powers spread by > 10 dB
    assert not O.check_power_stability(burst)


# ----------------------------------------------------------------------------- GPU
def _compare_counts(st, x, fs):
    from tetraear.signal import scanner as S
    m, nd = O.modulation_counts(x)
    assert st[S.F_DIFFS] == nd
    assert abs(st[S.F_MOD] - m) <= _edge_count_mod(x), (st[S.F_MOD], m)
    bits, nsym = O.sync_bits(x, fs)
    best, npos = O.sync_best(bits)
    assert st[S.F_BITS] == len(bits) and st[S.F_WIN] == npos
    assert abs(st[S.F_SYNC] - best) <= 1, (st[S.F_SYNC], best)   # one edge bit at most moves the best window by 1
    p = np.mean(np.abs(x.astype(np.complex128)) ** 2)
    assert abs(st[S.F_POW] - p) <= 1e-9 * p
    ws = len(x) // 5
    # rows shorter than 5 samples have empty windows (np.mean -> nan); the detector's surface never
    # reads them there (check_power_stability needs 5000 samples, scanner.py:80-87)
    for i in range(5 if ws else 0):
        pw = np.mean(np.abs(x[i * ws:(i + 1) * ws].astype(np.complex128)) ** 2)
        assert abs(st[S.F_POW_W0 + i] - pw) <= 1e-9 * max(pw, 1e-30)


@pytest.mark.gpu
def test_gpu_detector_known_answers():
    """The GPU detector on the KATs: ideal pi/4-DQPSK walk -> modulation confidence 1.0; the planted
    sync pattern -> correlation 1.0; the cluster-edge tones; the reference surface's length rules."""
    from tetraear.signal import TetraSignalDetector
    det = TetraSignalDetector(FS)
    rng = np.random.default_rng(1)
    x = _dqpsk_walk(1000, 1, rng).astype(np.complex64)
    assert det.detect_tetra_modulation(x) == (True, 1.0)
    assert det.detect_tetra_modulation(x[:999]) == (False, 0.0)
    y, _ = _sync_walk(13)
    assert det.detect_sync_pattern(y.astype(np.complex64)) == (True, 1.0)
    assert det.detect_sync_pattern(y[:13 * 99].astype(np.complex64)) == (False, 0.0)   # < 100 strided samples
    n = np.arange(2000)
    assert det.detect_tetra_modulation(np.exp(1j * (7 * np.pi / 8 - 1e-3) * n).astype(np.complex64))[1] == 1.0
    assert det.detect_tetra_modulation(np.exp(1j * (7 * np.pi / 8 + 1e-3) * n).astype(np.complex64))[1] == 0.0
    assert det.detect_tetra_modulation(np.exp(1j * (np.pi - 0.05) * n).astype(np.complex64))[1] == 0.0
    assert det.check_power_stability(np.ones(5000, np.complex64)) and not det.check_power_stability(np.ones(4999))
    assert det.calculate_power(np.zeros(0)) == -85.0
    assert abs(det.calculate_power(np.full(1000, 0.1, np.complex64)) - O.calculate_power(np.full(1000, 0.1))) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", [np.complex64, np.complex128])
def test_gpu_counts_vs_oracle(fmt):
    """Batch of candidate channels -- TETRA bursts (the ETSI synthesiser at 2.4 MSps, 10-30 dB),
    noise, a tone, silence -- in one launch: every count equal to the oracle's up to the edge
    tolerance, every power to 1e-9."""
    from tetraear.signal.etsi import synth
    from tetraear.signal import scanner as S
    N = 131072
    rng = np.random.default_rng(5)
    rows = [synth(1, N, seed=s, snr_db=snr)[0][0] for s, snr in ((1, 30.0), (2, 10.0))]
    rows.append((0.01 * (rng.standard_normal(N) + 1j * rng.standard_normal(N))).astype(np.complex64))
    rows.append(np.exp(2j * np.pi * 0.01 * np.arange(N)).astype(np.complex64))
    rows.append(np.zeros(N, np.complex64))
    x = np.stack(rows).astype(fmt)
    st = S.scan_counts(x, FS)
    for c in range(len(x)):
        _compare_counts(st[c], x[c], FS)


@pytest.mark.gpu
def test_analyze_batch_matches_single_and_validates_frames():
    """analyze_batch over candidates equals analyze_signal one by one; a TETRA chunk in the
    reference-compatible chain validates frames as the GPU process()/decode() decides, and noise
    never does."""
    from tetraear.signal import TetraSignalDetector
    from tetraear.signal import SignalProcessor
    from tetraear.core import TetraDecoder
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import _signals
    rng = np.random.default_rng(2)
    tetra = [_signals.family("tetra", rng, 131072, FS)[0] for _ in range(2)]
    noise = (0.05 * (rng.standard_normal(131072) + 1j * rng.standard_normal(131072))).astype(np.complex64)
    x = np.stack(tetra + [noise]).astype(np.complex64)
    det = TetraSignalDetector(FS)
    batch = det.analyze_batch(x)
    for c in range(len(x)):
        one = det.analyze_signal(x[c])
        assert one == batch[c], c
        frames = TetraDecoder(auto_decrypt=False).decode(SignalProcessor(FS, mode="compat").process(x[c]))
        crc = sum(f['burst_crc'] is True for f in frames) / max(len(frames), 1) if frames else 0.0
        assert batch[c]['crc_pass_rate'] == crc
        assert batch[c]['frames_validated'] == (len(frames) >= 2 and crc > 0.5)
    assert not batch[2]['frames_validated']


@pytest.mark.gpu
def test_scan_wideband_carriers():
    """scan_wideband: the C3 channeliser's 800 carriers of a synthetic 20 MSps capture as candidate
    channels at 72 kHz (D = 1: every sample), one detector launch; the counts of a sample of carriers
    equal the oracle's on the same 72 kHz rows, and the TETRA carriers read as pi/4-DQPSK."""
    from tetraear.signal.scanner import scan_wideband, scan_counts
    from tetraear.signal.wideband import synth_wideband
    x = synth_wideband(400_000, seed=3, snr_db=30.0)[0]
    res, y = scan_wideband(x)
    assert len(res) == 800 and y.shape[0] == 800
    st = scan_counts(y, 72000.0)
    for k in (0, 1, 399, 400, 799):
        _compare_counts(st[k], y[k], 72000.0)
    conf = np.array([r['modulation_confidence'] for r in res])
    assert conf.min() > 0.4


# ----------------------------------------------------------------------------- the reference's outputs
def _g5():
    import os
    import sys
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    if here not in sys.path:
        sys.path.insert(0, here)
    import _signals
    z = np.load(os.path.join(here, "g5_scanner.npz"))
    keys = [str(k) for k in z["out_keys"]]
    for j in range(len(z["case"])):
        x = _signals.scanner_input(z, int(z["input"][j]))
        x = x.astype(np.complex64 if int(z["dtype"][j]) == 64 else np.complex128)
        yield str(z["case"][j]), float(z["fs"][j]), x, dict(zip(keys, z["out"][j]))


AN_KEYS = ["power_db", "is_tetra", "confidence", "modulation_confidence", "sync_detected", "sync_correlation",
           "frames_validated", "crc_pass_rate", "power_stable", "signal_present"]


def test_oracle_matches_reference_fixture():
    """oracle/scanner.py against the reference TetraSignalDetector's recorded outputs
    (tests/golden/g5_scanner.npz, 20 cases x complex64/complex128): every count-derived value and
    decision equal, the powers to 1e-12 dB (the same numpy expression)."""
    n = 0
    for name, fs, x, want in _g5():
        got = [O.calculate_power(x), *O.detect_tetra_modulation(x), *O.detect_sync_pattern(x, fs),
               O.check_power_stability(x), *O.validate_frames(x, fs)]
        for k, g in zip(["power", "mod_flag", "mod_conf", "sync_flag", "sync_corr", "stable", "val_flag",
                         "val_rate"], got):
            tol = 1e-12 if k == "power" else 0.0
            assert abs(float(g) - want[k]) <= tol, (name, x.dtype, k, g, want[k])
        an = O.analyze_signal(x, fs)
        for k in AN_KEYS:
            tol = 1e-12 if k == "power_db" else 0.0
            assert abs(float(an[k]) - want["an_" + k]) <= tol, (name, x.dtype, k, an[k], want["an_" + k])
        n += 1
    assert n == 40


@pytest.mark.gpu
def test_gpu_detector_matches_reference_fixture():
    """The GPU detector (tetra_scan_detect + the GPU process()/decode() validation) against the
    reference TetraSignalDetector's recorded outputs: decisions, validation and CRC rates equal;
    powers within 1e-6 dB (float64 device sums vs numpy's float32 pairwise mean); the modulation
    match count off by at most the phase differences within EDGE of a decision edge (device atan2
    ulps), the sync count by at most one; each disagreement counted and reported."""
    from tetraear.signal import TetraSignalDetector
    from tetraear.signal import scanner as S
    edges = []
    for name, fs, x, want in _g5():
        det = TetraSignalDetector(sample_rate=fs)
        assert abs(det.calculate_power(x) - want["power"]) <= 1e-6, (name, x.dtype)
        mf, mc = det.detect_tetra_modulation(x)
        sf, sc = det.detect_sync_pattern(x)
        if len(x) >= 1000 and mc != want["mod_conf"]:
            st = S.scan_counts(x, fs)[0]
            dm = abs(st[S.F_MOD] - want["mod_conf"] * st[S.F_DIFFS])
            assert dm <= _edge_count_mod(x) + 0.5, (name, x.dtype, mc, want["mod_conf"])
            edges.append((name, str(x.dtype), "mod", int(round(dm))))
        else:
            assert (mf, mc) == (bool(want["mod_flag"]), want["mod_conf"]), (name, x.dtype)
        if sc != want["sync_corr"]:
            assert abs(sc - want["sync_corr"]) * 31 <= 1 + 1e-9, (name, x.dtype, sc, want["sync_corr"])
            edges.append((name, str(x.dtype), "sync", 1))
        else:
            assert sf == bool(want["sync_flag"]), (name, x.dtype)
        assert det.check_power_stability(x) == bool(want["stable"]), (name, x.dtype)
        assert det.validate_frames(x) == (bool(want["val_flag"]), want["val_rate"]), (name, x.dtype)
        an = det.analyze_signal(x)
        assert abs(an["power_db"] - want["an_power_db"]) <= 1e-6
        if not any(e[0] == name and e[1] == str(x.dtype) for e in edges):
            for k in AN_KEYS[1:]:
                assert float(an[k]) == want["an_" + k], (name, x.dtype, k, an[k], want["an_" + k])
    print("edge disagreements (case, dtype, count, size):", edges)
    assert len(edges) <= 4, edges
