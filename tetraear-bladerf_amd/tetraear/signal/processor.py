"""MI355X SignalProcessor -- the reference's demod surface, computed by libtetra_hip.so.

Surface mirrors /root/reference/tetraear/signal/processor.py:18-273 (same class, attributes,
method names, argument meaning, return dtypes and swallow-and-continue error behaviour).
This module only PLANS: it makes the reference's control decisions (decimate or not, filter or
not, samples per symbol, phase step) and its scipy filter designs, then hands every sample
computation to the HIP library.  There is no CPU fallback: without the library or a gfx950
device, the first numeric call raises ``TetraHipError``.

``mode="etsi"`` selects the ETSI EN 300 392-2 receiver (polyphase RRC channel filter, Gardner
timing recovery, correct pi/4-DQPSK decision with soft bits) instead of the reference-compatible
("compat") chain; see tetraear.signal.etsi.  Callers that construct ``SignalProcessor(sample_rate)``
unchanged (/root/reference/tetraear/ui/modern.py:1886, scanner.py:164) pick the chain with the
environment: ``TETRAEAR_DEMOD=compat|etsi`` (default compat).  ``TETRAEAR_BACKEND`` may only be
``hip`` (the default): this build has no CPU path.
"""
import functools
import logging
import math
import os

import numpy as np
from scipy import signal as _design   # filter DESIGN only (coefficients), as the reference does

from tetraear import _hip

logger = logging.getLogger(__name__)

SYMBOL_RATE = 18000
TARGET_RATE = 240000
# decision thresholds evaluated exactly as processor.py:152-158 writes them
THRESHOLDS = (-5 * np.pi / 8, -3 * np.pi / 8, 3 * np.pi / 8, 5 * np.pi / 8)


def demod_mode(mode=None):
    """The chain a SignalProcessor / TetraDecoder runs: `mode`, else $TETRAEAR_DEMOD, else compat."""
    m = mode if mode is not None else os.environ.get("TETRAEAR_DEMOD", "compat")
    if m not in ("compat", "etsi"):
        raise ValueError(f"mode / TETRAEAR_DEMOD must be 'compat' or 'etsi', not {m!r}")
    backend = os.environ.get("TETRAEAR_BACKEND", "hip")
    if backend != "hip":
        raise _hip.TetraHipError(f"TETRAEAR_BACKEND={backend!r}: this build computes on the GPU only (hip); "
                                 f"the CPU path is the reference itself")
    return m


def _fmt_of(x):
    """(library sample format, reference dtype class) for an input array."""
    if x.dtype in (np.complex64, np.float32):
        return _hip.TETRA_CF32
    return _hip.TETRA_CF64


def _tensor_fmt(x):
    """Library sample format of a torch tensor batch: complex64 [C, N] or float32 [C, N, 2] is cf32,
    complex128 [C, N] or float64 [C, N, 2] is cf64; anything else is refused (never reinterpreted)."""
    import torch
    if x.dim() == 2 and x.dtype in (torch.complex64, torch.complex128):
        return _hip.TETRA_CF32 if x.dtype == torch.complex64 else _hip.TETRA_CF64
    if x.dim() == 3 and x.shape[2] == 2 and x.dtype in (torch.float32, torch.float64):
        return _hip.TETRA_CF32 if x.dtype == torch.float32 else _hip.TETRA_CF64
    raise TypeError(f"process_batch: a tensor batch must be complex64/complex128 [C, N] or float32/float64 "
                    f"[C, N, 2], not {x.dtype} {tuple(x.shape)}")


def _as_complex(x, fmt):
    t = np.complex64 if fmt == _hip.TETRA_CF32 else np.complex128
    return np.ascontiguousarray(x, dtype=t)


@functools.lru_cache(maxsize=64)
def _decimator_design(q, real=False):
    """scipy.signal.decimate's filter (ftype='iir', n=8) in both working precisions.  decimate casts
    the sos to the input's dtype (scipy _signaltools.decimate) and sosfiltfilt derives its initial
    state from that array, so a real input's state comes from the real dtype: at q = 7 the float32
    and complex64 sosfilt_zi differ in one element's last bit."""
    sos = _design.cheby1(8, 0.05, 0.8 / q, output="sos")
    out = {}
    for name, t in (("f32", np.float32 if real else np.complex64), ("f64", np.float64 if real else np.complex128)):
        s = np.asarray(sos, dtype=t)
        out[name] = (s.real.copy(), _design.sosfilt_zi(s).real.copy())
    return out


@functools.lru_cache(maxsize=64)
def _lowpass_design(bandwidth, fs):
    """filter_signal's butter(4) design (processor.py:69-78)."""
    nyquist = fs / 2
    cutoff = min(0.99, max(0.01, (bandwidth / 2) / nyquist))
    b, a = _design.butter(4, cutoff, btype="low")
    return b, a, _design.lfilter_zi(b, a)


def _fill(arr, vals):
    for i, v in enumerate(np.asarray(vals).ravel()):
        arr[i] = v


DECIMATORS = {"auto": 0, "sequential": _hip.COMPAT_SEQUENTIAL, "blocked": _hip.COMPAT_BLOCKED}


def default_decimator():
    """The compat decimator form of a SignalProcessor built without one: $TETRAEAR_COMPAT_DECIMATOR
    (an operator's opt-in to the latency mode for unchanged callers, modern.py:1886), else "auto"
    (= scipy's sequential order, bit-identical to the reference)."""
    d = os.environ.get("TETRAEAR_COMPAT_DECIMATOR", "auto")
    if d not in DECIMATORS:
        raise ValueError(f"TETRAEAR_COMPAT_DECIMATOR must be one of {sorted(DECIMATORS)}, not {d!r}")
    return d


def compat_forms(plan, C, N):
    """The kernels tetra_demod_compat runs for `plan` on a [C, N] batch (host-only query):
    {"decimate": "blocked"|"sequential", "filtfilt": ..., "power_prepass": bool}."""
    import ctypes
    f = ctypes.c_int32(0)
    if _hip.lib().tetra_compat_forms(plan, int(C), int(N), ctypes.byref(f)) != 0:
        raise ValueError("tetra_compat_forms: invalid plan")
    v = f.value
    return {"decimate": "blocked" if v & _hip.FORM_DEC_BLOCKED else "sequential",
            "filtfilt": "blocked" if v & _hip.FORM_LF_BLOCKED else "sequential",
            "power_prepass": bool(v & _hip.FORM_POW_PREPASS)}


_PLANS = {}   # compat_plan results of the warning-free cases (the GUI's repeated chunk shape)


def compat_plan(sample_rate, n, fmt, bandwidth=25000, decimator="auto", real=False, cache=True):
    """Build the device plan for process() on n samples (processor.py:239-273 decisions).
    Plans of calls that log nothing are cached by their arguments (~40 us of filter design per
    chunk otherwise); the plan is read-only to the library.

    ``decimator`` picks the form of decimate's sosfiltfilt and of filtfilt (include/tetra_hip.h,
    TETRA_COMPAT_*): "sequential" (and "auto", the default) is scipy's operation order, bit-identical
    to the reference; "blocked" is the opt-in latency mode -- 256-/128-sample tiles recursed in
    parallel, ~40x lower latency for one chunk, but only within the cheby1 filter's fp32 noise of
    scipy (up to ~1.5e-5 on .symbols near the chunk start; a decision with a ~1e-6 rad margin can
    flip), so it is never chosen for the caller.
    ``real``: the samples are real (decimate's initial state in the real dtype).  ``cache=False``
    returns a private plan the caller may modify."""
    key = (float(sample_rate), int(n), int(fmt), bandwidth, decimator, bool(real))
    hit = _PLANS.get(key) if cache else None
    if hit is not None:
        return hit
    warned = False
    p = _hip.CompatPlan()
    p.flags = DECIMATORS[decimator]
    rate = sample_rate
    p.q = 0
    if rate > TARGET_RATE * 2:
        q = int(rate / TARGET_RATE)
        if q > 1:
            if n > 27:   # sosfiltfilt padlen = 3*(2*4+1); decimate raises for len <= 27
                p.q = q
                rate = rate / q
            else:
                warned = True
                logger.warning("Decimation failed: The length of the input vector x must be greater "
                               "than padlen, which is 27.")
    m = -(-n // p.q) if p.q > 1 else n
    p.dec_f64 = int(fmt == _hip.TETRA_CF64)
    if p.q > 1:
        d = _decimator_design(p.q, bool(real))
        _fill(p.sos_f32, d["f32"][0])
        _fill(p.zi_f32, d["f32"][1])
        _fill(p.sos_f64, d["f64"][0])
        _fill(p.zi_f64, d["f64"][1])
    b, a, zi = _lowpass_design(bandwidth, rate)
    p.ntaps = len(b)
    p.filt = int(m > 3 * max(len(a), len(b)))
    if not p.filt:
        warned = True
        logger.warning("Filter design failed, using unfiltered samples: The length of the input vector x "
                       "must be greater than padlen, which is %d.", 3 * max(len(a), len(b)))
    _fill(p.b, b)
    _fill(p.a, a)
    _fill(p.lzi, zi)
    sps = int(rate / SYMBOL_RATE)
    p.sps = sps if sps > 1 else 1
    p.phase_step = max(1, sps // 8) if sps > 1 else 1
    p.fs_dec = rate
    _fill(p.thr, THRESHOLDS)
    if not warned and cache:
        if len(_PLANS) >= 64:
            _PLANS.clear()
        _PLANS[key] = (p, m, rate)
    return p, m, rate


def mixer_coefficient(freq_offset):
    """Imaginary part of -1j*2*np.pi*freq_offset, evaluated as processor.py:99 evaluates it."""
    c = -1j * 2 * np.pi * freq_offset
    return float(np.imag(c))


class SignalProcessor:
    """Processes raw IQ samples for TETRA demodulation (processor.py:18)."""

    def __init__(self, sample_rate=2.4e6, mode=None, decimator=None):
        self.sample_rate = sample_rate
        self.symbol_rate = SYMBOL_RATE
        self.samples_per_symbol = int(sample_rate / self.symbol_rate)
        self.symbols = None
        self.mode = demod_mode(mode)
        decimator = default_decimator() if decimator is None else decimator
        if decimator not in DECIMATORS:
            raise ValueError(f"decimator must be one of {sorted(DECIMATORS)}, not {decimator!r}")
        # compat process(): the decimator form (compat_plan); "auto"/"sequential" is scipy's exact
        # order for every batch size, "blocked" the opt-in latency mode (not bit-exact)
        self.decimator = decimator
        self._etsi = None

    # --------------------------------------------------------------- component methods
    def resample(self, samples, target_rate):
        """FFT resampling (processor.py:35-49: scipy.signal.resample to int(len * target / fs)
        samples) on the GPU: tetra_resample (rocFFT forward, scipy's spectrum truncation/padding
        and Nyquist split/join, rocFFT inverse).  complex64 stays complex64, complex128 stays
        complex128; real input runs the complex transform and returns the real part, which is
        scipy's rfft path up to rounding."""
        x = np.asarray(samples)
        new_n = int(len(x) * target_rate / self.sample_rate)
        if new_n <= 0 or len(x) == 0:
            raise ValueError(f"resample: cannot resample {len(x)} samples to {new_n}")   # scipy errors too
        real = not np.iscomplexobj(x)
        if x.dtype in (np.complex64, np.float32, np.float16):
            fmt, dt = _hip.TETRA_CF32, np.complex64
        else:
            fmt, dt = _hip.TETRA_CF64, np.complex128
        xc = np.ascontiguousarray(x, dt)
        y = np.empty(new_n, dt)
        c = _hip.ctx()
        c.check(c.lib.tetra_resample(c.handle, _hip.ptr(xc), fmt, 1, len(xc), new_n, _hip.ptr(y)), "tetra_resample")
        return y.real.copy() if real else y

    def filter_signal(self, samples, bandwidth=25000, sample_rate=None):
        """Butterworth-4 filtfilt low-pass (processor.py:51-83), on the GPU.

        ETSI mode: the receiver's channel filter instead -- 2.4 MSps in, the RRC(0.35)-matched
        72 kHz samples (4 per symbol) out (`bandwidth` is fixed at the TETRA channel's)."""
        if self.mode == "etsi":
            fs = sample_rate if sample_rate is not None else self.sample_rate
            if fs != self.sample_rate:
                raise ValueError("ETSI mode filters the receiver's own input rate")
            return self._etsi_rx().chanfilt(samples)
        if len(samples) == 0:
            return samples
        fs = sample_rate if sample_rate is not None else self.sample_rate
        x = np.asarray(samples)
        try:
            b, a, zi = _lowpass_design(bandwidth, fs)
            if len(x) <= 3 * max(len(a), len(b)):
                raise ValueError("The length of the input vector x must be greater than padlen, "
                                 f"which is {3 * max(len(a), len(b))}.")
        except Exception as e:
            logger.warning(f"Filter design failed, using unfiltered samples: {e}")
            return samples
        p, _, _ = compat_plan(fs, len(x), _fmt_of(x), bandwidth, cache=False)   # its taps are replaced below
        _fill(p.b, b)
        _fill(p.a, a)
        _fill(p.lzi, zi)
        p.ntaps = len(b)
        fmt = _fmt_of(x)
        xc = _as_complex(x, fmt)
        out = np.empty(len(x), np.complex128)
        c = _hip.ctx()
        c.check(c.lib.tetra_filtfilt(c.handle, p, _hip.ptr(xc), fmt, 1, len(x), _hip.ptr(out)), "tetra_filtfilt")
        return out if np.iscomplexobj(x) else out.real.copy()

    def frequency_shift(self, samples, freq_offset, sample_rate=None):
        """Complex mixer x*exp(-j*2*pi*f*n/fs) (processor.py:85-100), on the GPU."""
        fs = sample_rate if sample_rate is not None else self.sample_rate
        x = np.asarray(samples)
        if len(x) == 0:
            return np.zeros(0, np.complex128)
        fmt = _fmt_of(x)
        xc = _as_complex(x, fmt)
        out = np.empty(len(x), np.complex128)
        cf = np.array([mixer_coefficient(freq_offset)], np.float64)
        c = _hip.ctx()
        c.check(c.lib.tetra_frequency_shift(c.handle, _hip.ptr(xc), fmt, 1, len(x), _hip.ptr(cf), float(fs),
                                            _hip.ptr(out)), "tetra_frequency_shift")
        return out

    def demodulate_dqpsk(self, samples):
        """Differential decision with the reference's thresholds (processor.py:102-166).

        ETSI mode: the Table 5.1 decision regions of the docstring at processor.py:106-110
        (00 +pi/4, 01 +3pi/4, 11 -3pi/4, 10 -pi/4) on the given symbols (tetra_etsi_decide)."""
        if self.mode == "etsi":
            return self._etsi_rx().decide(samples)
        if len(samples) < 2:
            return np.array([], dtype=np.uint8)
        x = np.asarray(samples)
        fmt = _fmt_of(x)
        if np.iscomplexobj(x):
            xc = _as_complex(x, fmt)
        else:   # real samples: real division and product, as numpy runs them on a real array
            fmt = _hip.TETRA_F32 if fmt == _hip.TETRA_CF32 else _hip.TETRA_F64
            xc = np.ascontiguousarray(x, np.float32 if fmt == _hip.TETRA_F32 else np.float64)
        out = np.empty(len(x) - 1, np.uint8)
        thr = np.array(THRESHOLDS, np.float64)
        c = _hip.ctx()
        c.check(c.lib.tetra_demod_dqpsk(c.handle, _hip.ptr(xc), fmt, 1, len(x), _hip.ptr(thr), _hip.ptr(out)),
                "tetra_demod_dqpsk")
        return out

    def extract_symbols(self, samples, sample_rate=None):
        """Best integer sampling phase by mean power, then decimate (processor.py:168-219).

        ETSI mode: timing recovery (Oerder-Meyr + block Gardner) on the channel filter's 72 kHz
        samples (sample_rate 72000), or on raw input at the receiver's rate (filtered first)."""
        if self.mode == "etsi":
            fs = sample_rate if sample_rate is not None else 72000.0
            x = np.asarray(samples)
            y = x if fs == 72000.0 else self.filter_signal(x, sample_rate=fs)
            return self._etsi_rx().timing(y)[1]
        if len(samples) == 0:
            return np.array([], dtype=complex)
        fs = sample_rate if sample_rate is not None else self.sample_rate
        sps = int(fs / self.symbol_rate)
        if sps <= 1:
            return samples
        x = np.asarray(samples)
        fmt = _fmt_of(x)
        xc = _as_complex(x, fmt)
        smax = len(x) // sps + 1
        sym = np.empty(smax, xc.dtype)
        ns = np.zeros(1, np.int32)
        c = _hip.ctx()
        c.check(c.lib.tetra_extract_symbols(c.handle, _hip.ptr(xc), fmt, 1, len(x), sps, max(1, sps // 8),
                                            _hip.ptr(sym), _hip.ptr(ns), None, smax), "tetra_extract_symbols")
        out = sym[:int(ns[0])]
        return out if np.iscomplexobj(x) else out.real.astype(x.dtype)

    # --------------------------------------------------------------- pipeline
    def process(self, samples, freq_offset=0):
        """Complete demodulation of one chunk (processor.py:221-273); sets ``self.symbols``."""
        if self.mode == "etsi":
            try:
                rx = self._etsi_rx()
            except ValueError as e:   # a rate with no channel-filter plan: log and go on (processor.py:253-257)
                logger.warning(f"ETSI demodulation unavailable: {e}")
                self.symbols = np.zeros(0, np.complex64)
                return np.zeros(0, np.uint8)
            hard, self.symbols = rx.process(np.asarray(samples), freq_offset)
            return hard
        if len(samples) == 0:
            self.symbols = np.array([], dtype=complex)
            return np.array([], dtype=np.uint8)
        x = np.asarray(samples)
        real_in = not np.iscomplexobj(x)
        fmt = _fmt_of(x)
        xc = _as_complex(x, fmt)
        plan, m, _ = compat_plan(self.sample_rate, len(x), fmt, decimator=self.decimator, real=real_in)
        smax = m // plan.sps + 1
        soft = np.empty(smax, np.complex128)
        hard = np.empty(smax, np.uint8)
        ns = np.zeros(1, np.int32)
        f32 = ctypes_int()
        mc = np.array([mixer_coefficient(freq_offset) if freq_offset != 0 else 0.0], np.float64)
        mo = np.array([1 if freq_offset != 0 else 0], np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_demod_compat(c.handle, plan, _hip.ptr(xc), fmt, 1, len(x), _hip.ptr(mc), _hip.ptr(mo),
                                         _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), smax, f32),
                "tetra_demod_compat")
        n = int(ns[0])
        if f32.value:
            sym = soft.view(np.complex64)[:n].copy()
        else:
            sym = soft[:n].copy()
        if real_in and freq_offset == 0:
            sym = sym.real.copy() if plan.filt else sym.real.astype(np.float32 if fmt == _hip.TETRA_CF32 else np.float64)
            self.symbols = sym
            return self.demodulate_dqpsk(sym)   # the reference decides real symbols with real arithmetic
        self.symbols = sym
        return hard[:max(0, n - 1)].copy()

    def process_batch(self, samples, freq_offsets=None):
        """process() over a [C, N] batch of independent chunks in one launch sequence.

        Returns (hard [C, S-1] uint8, symbols [C, S] complex128, nsym [C]); row c holds what
        process(samples[c], freq_offsets[c]) returns / stores in .symbols, in its first
        nsym[c]-1 / nsym[c] entries.  ``freq_offsets``: None (no mixer), [C] Hz on the host, a [C]
        torch tensor of Hz on the GPU (the mixer inputs are derived on the device), or ``"afc"``: the
        capture loop's signal-present / AFC gate (modern.py:1952-2028, spectrum.afc_gate) runs on
        the device on each channel's first 2048 samples and feeds its offset straight into the demod
        (no host round trip); the gate's per-channel results are kept in ``self.gate`` (the loop
        only demodulates channels with ``self.gate["present"]``)."""
        x = np.asarray(samples) if not hasattr(samples, "data_ptr") else samples
        C, N = x.shape[:2]
        dev_offsets = hasattr(freq_offsets, "data_ptr")
        afc = isinstance(freq_offsets, str)
        if afc and freq_offsets != "afc":
            raise ValueError("freq_offsets must be None, an array of Hz, a device tensor or 'afc'")
        real_in = False
        if hasattr(x, "data_ptr"):
            fmt = _tensor_fmt(x)
            xc = x.contiguous()
        else:
            fmt = _fmt_of(x)
            real_in = not np.iscomplexobj(x)
            xc = _as_complex(x, fmt)
        plan, m, _ = compat_plan(self.sample_rate, N, fmt, decimator=self.decimator, real=real_in)
        smax = m // plan.sps + 1
        soft = np.empty((C, smax), np.complex128)
        hard = np.empty((C, smax), np.uint8)
        ns = np.zeros(C, np.int32)
        f32 = ctypes_int()
        c = _hip.ctx()
        gate = None
        if afc or dev_offsets:
            import torch
            dev = torch.device("cuda", torch.cuda.current_device()) if not dev_offsets else freq_offsets.device
            if not hasattr(xc, "data_ptr"):
                xc = torch.from_numpy(np.ascontiguousarray(xc)).to(dev)   # staged once for gate + demod
            if afc:
                from tetraear.signal.spectrum import afc_gate
                torch.cuda.current_stream(dev).synchronize()   # the library runs on its own stream
                gate = afc_gate(xc, self.sample_rate, mixer=True)
                mc, mo = gate["mixer_coef"], gate["mixer_on"]
            else:
                f = freq_offsets.to(torch.float64)
                mc = torch.where(f != 0, f * (-2 * np.pi), torch.zeros_like(f))   # mixer_coefficient, on device
                mo = (f != 0).to(torch.uint8)
                torch.cuda.current_stream(dev).synchronize()
        else:
            fo = np.zeros(C) if freq_offsets is None else np.asarray(freq_offsets, np.float64)
            mc = np.array([mixer_coefficient(f) if f != 0 else 0.0 for f in fo], np.float64)
            mo = (fo != 0).astype(np.uint8)
        split = False
        if not plan.filt:
            # a chunk too short for filtfilt (processor.py:81-83 returns it unfiltered): the library
            # takes such a batch only with the mixer on for all channels or for none, so a mixed
            # batch runs as those two batches
            on = (mo.cpu().numpy() if hasattr(mo, "data_ptr") else mo).astype(bool)
            if on.any() and not on.all():
                split = True
                mc_h = mc.cpu().numpy() if hasattr(mc, "data_ptr") else mc
                for rows in (np.flatnonzero(on), np.flatnonzero(~on)):
                    h, s, n = self._compat_rows(plan, xc, fmt, rows, mc_h[rows], on[rows], smax)
                    hard[rows], soft[rows], ns[rows] = h, s, n
        if not split:
            c.check(c.lib.tetra_demod_compat(c.handle, plan, _hip.ptr(xc), fmt, C, N, _hip.ptr(mc), _hip.ptr(mo),
                                             _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), smax, f32),
                    "tetra_demod_compat")
            if f32.value:   # unfiltered cf32 without the mixer: complex64 symbols, rows smax apart
                soft = soft.reshape(-1).view(np.complex64)[:C * smax].reshape(C, smax).astype(np.complex128)
        if real_in:
            # real rows whose mixer stays off keep real symbols in the reference: decide them as
            # process() does (real arithmetic), whichever way the offsets came -- host Hz, a device
            # tensor or the AFC gate -- and whether or not the batch was split above
            off = (mo.cpu().numpy() if hasattr(mo, "data_ptr") else np.asarray(mo)).astype(bool) == 0
            rt = np.float32 if (not plan.filt and fmt == _hip.TETRA_CF32) else np.float64
            for r in np.flatnonzero(off):
                if ns[r] >= 2:
                    hard[r, :ns[r] - 1] = self.demodulate_dqpsk(soft[r, :ns[r]].real.astype(rt))
        if gate is not None:
            self.gate = {k: v.cpu().numpy() for k, v in gate.items()}
        return hard, soft, ns

    def _compat_rows(self, plan, xc, fmt, rows, mc, on, smax):
        """tetra_demod_compat over the channels ``rows`` of ``xc`` (host or device), mixer
        coefficients ``mc`` and flags ``on`` (all set or all clear); symbols returned as complex128."""
        xs = xc[rows.tolist()] if hasattr(xc, "data_ptr") else np.ascontiguousarray(xc[rows])
        if hasattr(xs, "data_ptr"):
            xs = xs.contiguous()
        R, N = len(rows), xs.shape[1]
        mc = np.ascontiguousarray(mc, np.float64)
        mo = np.ascontiguousarray(on, np.uint8)
        soft = np.empty((R, smax), np.complex128)
        hard = np.empty((R, smax), np.uint8)
        ns = np.zeros(R, np.int32)
        f32 = ctypes_int()
        c = _hip.ctx()
        c.check(c.lib.tetra_demod_compat(c.handle, plan, _hip.ptr(xs), fmt, R, N, _hip.ptr(mc), _hip.ptr(mo),
                                         _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), smax, f32),
                "tetra_demod_compat")
        if f32.value:
            soft = soft.reshape(-1).view(np.complex64)[:R * smax].reshape(R, smax).astype(np.complex128)
        return hard, soft, ns

    def _etsi_rx(self):
        if self._etsi is None:
            from tetraear.signal.etsi import EtsiReceiver
            self._etsi = EtsiReceiver(self.sample_rate)
        return self._etsi


def ctypes_int():
    import ctypes
    return ctypes.c_int32(0)
