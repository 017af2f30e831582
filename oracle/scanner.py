"""CPU oracle for the scanner's TETRA signal detector (TEST INFRASTRUCTURE -- only tests/ use it).

SURVEY.md §8f rank 2: /root/reference/tetraear/signal/scanner.py:42-147 (calculate_power,
detect_tetra_modulation, detect_sync_pattern) and :204-231 (check_power_stability), restated in
numpy from that survey row's description of them, in the dtype numpy computes them in (complex64 ->
float32 angles, differences and wrap; the cluster distance in float64).  Vectorised: the reference's
per-sample loops become array expressions with the same comparisons.

validate_frames (:149-202) and analyze_signal (:233-289) run the compat oracle's process() and
decode() (oracle/compat.py) for the frame validation.

Pinned (round 5) to the reference's own outputs: tests/golden/g5_scanner.npz records the reference
TetraSignalDetector's six methods on 20 seeded cases x {complex64, complex128}
(tests/golden/make_golden_scanner.py); tests/test_scanner.py checks this module against every one,
and the analytic known answers (an ideal pi/4-DQPSK walk gives modulation confidence 1.0, a phase walk
whose strided differences spell the sync pattern gives correlation 1.0, tones at the decision edges).
"""
import numpy as np

SYNC_PATTERN = np.array([0, 1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0,
                         1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0])


def _wrap(d):
    """(d + pi) % (2 pi) - pi in d's dtype (numpy's weak Python-float scalars)."""
    return (d + np.pi) % (2 * np.pi) - np.pi


def calculate_power(x, bottom=-85.0):
    x = np.asarray(x)
    if x.size == 0:
        return float(bottom)
    return float(10 * np.log10(np.mean(np.abs(x) ** 2) + 1e-10))


def modulation_counts(x):
    """(matches, differences) of the pi/4 cluster test on the normalised samples."""
    x = np.asarray(x)
    x = x / (np.abs(x).max() + 1e-10)
    d = _wrap(np.diff(np.angle(x)))
    e = np.array([-np.pi, -3 * np.pi / 4, -np.pi / 2, -np.pi / 4, 0, np.pi / 4, np.pi / 2, 3 * np.pi / 4])
    dist = np.abs(e[None, :] - d.astype(np.float64)[:, None]).min(axis=1)
    return int(np.sum(dist < np.pi / 8)), len(d)


def detect_tetra_modulation(x):
    if len(x) < 1000:
        return False, 0.0
    m, n = modulation_counts(x)
    conf = m / n
    return conf > 0.4, conf


def sync_bits(x, fs):
    D = max(1, int(fs / 18000 / 10))
    s = np.asarray(x)[::D]
    d = _wrap(np.diff(np.angle(s)))
    q = d / (np.pi / 4)
    return (np.abs(q) <= 0.5).astype(np.int64), len(s)   # round(q) == 0, round half to even


def sync_best(bits):
    """Best match count of the 31-bit pattern over window starts 0 .. len(bits) - 32."""
    n = len(bits) - 31
    if n <= 0:
        return 0, 0
    w = np.lib.stride_tricks.sliding_window_view(bits, 31)[:n]
    return int((w == SYNC_PATTERN[None, :]).sum(axis=1).max()), n


def detect_sync_pattern(x, fs):
    bits, nsym = sync_bits(x, fs)
    if nsym < 100 or len(bits) < 31:
        return False, 0.0
    best, n = sync_best(bits)
    corr = best / 31 if n > 0 else 0.0
    return corr > 0.75, corr


def check_power_stability(x, num_windows=5):
    x = np.asarray(x)
    if len(x) < num_windows * 1000:
        return False
    ws = len(x) // num_windows
    p = [calculate_power(x[i * ws:(i + 1) * ws]) for i in range(num_windows)]
    return bool(np.std(p) < 10.0)


def validate_frames(x, fs):
    """(frames_valid, crc_pass_rate): process() + decode() of the chunk (scanner.py:149-202) -- at
    least 10000 samples and 255 symbols; valid with >= 2 frames and a CRC pass rate above 0.5."""
    import compat
    x = np.asarray(x)
    if len(x) < 10000:
        return False, 0.0
    try:
        hard = compat.SignalProcessor(fs).process(x)
        if len(hard) < 255:
            return False, 0.0
        frames = compat.decode_with_mac(hard)
    except Exception:
        return False, 0.0
    if not frames:
        return False, 0.0
    passed = 0.0
    for f in frames:
        bc = f.get('burst_crc')
        if bc is True:
            passed += 1
        elif bc is not False and 'type' in f and 'number' in f:
            passed += 0.5
    rate = passed / max(len(frames), 1)
    return len(frames) >= 2 and rate > 0.5, rate


def analyze_signal(x, fs, bottom=-85.0):
    """The detector's verdict dict (scanner.py:233-289)."""
    power = calculate_power(x, bottom)
    is_mod, mod_conf = detect_tetra_modulation(x)
    has_sync, sync_corr = detect_sync_pattern(x, fs)
    frames_valid, crc_rate = validate_frames(x, fs)
    stable = check_power_stability(x)
    if has_sync and is_mod:
        confidence = mod_conf * 0.4 + sync_corr * 0.4 + crc_rate * 0.2
    elif has_sync:
        confidence = sync_corr * 0.6
    elif is_mod:
        confidence = mod_conf * 0.5
    else:
        confidence = 0.0
    is_tetra = bool(is_mod and has_sync and stable)
    if frames_valid:
        is_tetra = True
        confidence = max(confidence, 0.7)
    return {'power_db': power, 'is_tetra': is_tetra, 'confidence': confidence, 'modulation_confidence': mod_conf,
            'sync_detected': has_sync, 'sync_correlation': sync_corr, 'frames_validated': frames_valid,
            'crc_pass_rate': crc_rate, 'power_stable': stable, 'signal_present': power > bottom}
