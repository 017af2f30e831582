"""The scanner's TETRA signal detector on the GPU.

Surface of /root/reference/tetraear/signal/scanner.py:24-289 (``TetraSignalDetector``: same
constructor, method names, argument meaning and return values).  The reference runs two per-sample
Python loops per candidate frequency -- the pi/4-DQPSK phase-cluster test (:57-96) and the 31-bit
sync search (:98-147) -- and decodes frames for validation (:149-202).  Here every candidate of a
batch is measured in one tetra_scan_detect launch (one workgroup per channel: the cluster counts, the
sync bits packed by ballots and the best 31-bit match by XOR/popcount, the chunk and window powers),
and validation is the GPU process() / decode() (``process_batch`` / ``decode_batch``).  The host only
turns the counts into the reference's decisions.

``scan_wideband`` feeds the detector from the C3 channeliser: each of the 800 carriers of a 20 MSps
capture, as 72 kHz samples, is a candidate channel of one batch.

The hardware sweep (``FrequencyScanner``: tuning the BladeRF, dwell, retries; scanner.py:292-554) is
the reference's: with its package root on sys.path after this build's, ``FrequencyScanner`` here is
the reference's class from its own file, its detector swapped for this module's GPU
``TetraSignalDetector`` (tetraear/_overlay.py).
"""
import logging

import numpy as np

from tetraear import _hip, _overlay

logger = logging.getLogger(__name__)

SYNC_PATTERN = [0, 1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0, 1, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 0, 1, 0, 0]
SYNC_WORD = sum(b << j for j, b in enumerate(SYNC_PATTERN))   # bit j = pattern bit j
F_MOD, F_DIFFS, F_SYNC, F_WIN, F_BITS, F_POW, F_POW_W0 = range(7)
SCAN_FIELDS = F_POW_W0 + 5


def scan_counts(iq, sample_rate):
    """tetra_scan_detect over a [C][N] (or [N]) batch of complex samples: [C][SCAN_FIELDS] float64."""
    a = iq if hasattr(iq, "data_ptr") else np.asarray(iq)
    one = a.ndim == 1
    if hasattr(a, "data_ptr"):
        import torch
        fmt = _hip.TETRA_CF64 if a.dtype == torch.complex128 else _hip.TETRA_CF32
        a = a.contiguous()
        stats = torch.zeros((1 if one else a.shape[0], SCAN_FIELDS), dtype=torch.float64, device=a.device)
    else:
        fmt = _hip.TETRA_CF64 if a.dtype == np.complex128 else _hip.TETRA_CF32
        a = np.ascontiguousarray(a, np.complex128 if fmt == _hip.TETRA_CF64 else np.complex64)
        stats = np.zeros((1 if one else a.shape[0], SCAN_FIELDS), np.float64)
    C, N = (1, a.shape[0]) if one else a.shape[:2]
    D = max(1, int(sample_rate / 18000 / 10))   # scanner.py:109
    c = _hip.ctx()
    c.check(c.lib.tetra_scan_detect(c.handle, _hip.ptr(a), fmt, C, N, D, SYNC_WORD, _hip.ptr(stats)),
            "tetra_scan_detect")
    return stats


class TetraSignalDetector:
    """Detects TETRA signals in captured samples (scanner.py:24)."""

    def __init__(self, sample_rate=2.4e6, noise_floor=-45, bottom_threshold=-85):
        self.sample_rate = sample_rate
        self.symbol_rate = 18000
        self.channel_bandwidth = 25000
        self.noise_floor = noise_floor
        self.bottom_threshold = bottom_threshold

    # ------------------------------------------------------------- decisions from the counts
    def _power_db(self, mean_p):
        return float(10 * np.log10(mean_p + 1e-10))

    def _modulation(self, st, n):
        if n < 1000:
            return False, 0.0
        conf = st[F_MOD] / st[F_DIFFS]
        return bool(conf > 0.4), float(conf)

    def _sync(self, st, n):
        nsym = int(st[F_BITS]) + 1 if n > 0 else 0
        if nsym < 100 or int(st[F_BITS]) < 31:
            return False, 0.0
        corr = st[F_SYNC] / 31 if st[F_WIN] > 0 else 0.0
        return bool(corr > 0.75), float(corr)

    def _stable(self, st, n, num_windows=5):
        if n < num_windows * 1000:
            return False
        p = [self._power_db(st[F_POW_W0 + i]) for i in range(num_windows)]
        return bool(np.std(p) < 10.0)

    # ------------------------------------------------------------- reference surface
    def calculate_power(self, samples):
        """Mean power in dB (scanner.py:42-55)."""
        x = np.asarray(samples)
        if x.size == 0:
            return float(self.bottom_threshold)
        return self._power_db(scan_counts(x.ravel(), self.sample_rate)[0, F_POW])

    def detect_tetra_modulation(self, samples):
        """(is_tetra, confidence): the share of consecutive phase differences within pi/8 of a
        multiple of pi/4 (scanner.py:57-96); > 0.4 counts as pi/4-DQPSK."""
        x = np.asarray(samples)
        if len(x) < 1000:
            return False, 0.0
        return self._modulation(scan_counts(x, self.sample_rate)[0], len(x))

    def detect_sync_pattern(self, samples):
        """(found_sync, correlation): best agreement of the 31-bit sync pattern with the phase-step
        bits of the samples strided to ~10x the symbol rate (scanner.py:98-147); > 0.75 is a sync."""
        x = np.asarray(samples)
        if len(x) == 0:
            return False, 0.0
        return self._sync(scan_counts(x, self.sample_rate)[0], len(x))

    def check_power_stability(self, samples, num_windows=5):
        """Std of the five window powers below 10 dB (scanner.py:204-231)."""
        x = np.asarray(samples)
        if num_windows != 5:
            if len(x) < num_windows * 1000:
                return False
            ws = len(x) // num_windows
            return bool(np.std([self.calculate_power(x[i * ws:(i + 1) * ws]) for i in range(num_windows)]) < 10.0)
        if len(x) < 5000:
            return False
        return self._stable(scan_counts(x, self.sample_rate)[0], len(x))

    def validate_frames(self, samples):
        """(frames_valid, crc_pass_rate) from decoding the chunk (scanner.py:149-202): GPU process()
        + decode(); >= 2 frames with a CRC pass rate above 0.5."""
        return self.validate_batch(np.asarray(samples)[None, :])[0]

    def validate_batch(self, iq):
        """validate_frames for every row of a [C][N] batch: one process_batch + decode_batch."""
        from tetraear.signal.processor import SignalProcessor
        from tetraear.core.decoder import TetraDecoder
        iq = np.asarray(iq)
        C, N = iq.shape
        if N < 10000:
            return [(False, 0.0)] * C
        try:
            p = SignalProcessor(sample_rate=self.sample_rate)
            if p.mode == "etsi":
                streams = [p.process(iq[c]) for c in range(C)]
            else:
                hard, _, ns = p.process_batch(iq)
                streams = [hard[c, :max(0, int(ns[c]) - 1)] for c in range(C)]
            dec = TetraDecoder(auto_decrypt=False)
            out = []
            # a fresh decoder per candidate, as scanner.py:171 builds one per call (the ETSI decoder
            # carries the cell it acquired; the compat batch's parser state cannot change the frames)
            frames_all = dec.decode_batch([s if len(s) >= 255 else s[:0] for s in streams]) if dec.mode != "etsi" \
                else [TetraDecoder(auto_decrypt=False).decode(s) if len(s) >= 255 else [] for s in streams]
            for s, frames in zip(streams, frames_all):
                if len(s) < 255 or not frames:
                    out.append((False, 0.0))
                    continue
                passed = 0.0
                for f in frames:
                    bc = f.get('burst_crc')
                    if bc is True:
                        passed += 1
                    elif bc is not False and 'type' in f and 'number' in f:   # unknown CRC: half credit
                        passed += 0.5
                rate = passed / max(len(frames), 1)
                out.append((len(frames) >= 2 and rate > 0.5, rate))
            return out
        except Exception as e:   # scanner.py:200-202
            logger.debug(f"Frame validation error: {e}")
            return [(False, 0.0)] * C

    def analyze_signal(self, samples):
        """The detector's verdict for one chunk (scanner.py:233-289)."""
        return self.analyze_batch(np.asarray(samples)[None, :])[0]

    def analyze_batch(self, iq, validate=True):
        """analyze_signal for every candidate channel of a [C][N] batch: one detector launch, one
        validation pass; a list of the reference's analysis dicts."""
        iq = np.asarray(iq)
        C, N = iq.shape
        st = scan_counts(iq, self.sample_rate) if N else np.zeros((C, SCAN_FIELDS))
        val = self.validate_batch(iq) if validate else [(False, 0.0)] * C
        out = []
        for c in range(C):
            s = st[c]
            power = self._power_db(s[F_POW]) if N else float(self.bottom_threshold)
            is_mod, mod_conf = self._modulation(s, N)
            has_sync, sync_corr = self._sync(s, N) if N else (False, 0.0)
            frames_valid, crc_rate = val[c]
            stable = self._stable(s, N)
            if has_sync and is_mod:
                confidence = mod_conf * 0.4 + sync_corr * 0.4 + crc_rate * 0.2
            elif has_sync:
                confidence = sync_corr * 0.6
            elif is_mod:
                confidence = mod_conf * 0.5
            else:
                confidence = 0.0
            is_tetra = is_mod and has_sync and stable
            if frames_valid:
                is_tetra = True
                confidence = max(confidence, 0.7)
            out.append({'power_db': power, 'is_tetra': is_tetra, 'confidence': confidence,
                        'modulation_confidence': mod_conf, 'sync_detected': has_sync,
                        'sync_correlation': sync_corr, 'frames_validated': frames_valid, 'crc_pass_rate': crc_rate,
                        'power_stable': stable, 'signal_present': power > self.bottom_threshold})
        return out


def scan_wideband(x, fs=20e6, validate=False):
    """Candidate-channel scan of a wideband capture: the C3 channeliser splits the capture into its
    800 carriers at 72 kHz (tetra_channelize), and the detector measures all of them in one launch.
    Returns (analyses [800 dicts], y [800][n72])."""
    from tetraear.signal.wideband import WidebandReceiver
    y = WidebandReceiver(fs).channelize(x)
    return TetraSignalDetector(sample_rate=72000.0).analyze_batch(y, validate=validate), y


def __getattr__(name):
    """``FrequencyScanner`` (scanner.py:292): the reference's sweep over this module's detector."""
    if name == "FrequencyScanner":
        mod = _overlay.reference_module("signal/scanner", patch={"TetraSignalDetector": TetraSignalDetector})
        return mod.FrequencyScanner
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
