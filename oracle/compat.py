"""CPU oracle for the reference's compat hot path (TEST INFRASTRUCTURE -- never shipped).

Restates, function by function, what the reference computes on the path that
BASELINE.json's north_star names, with the same numerics:

  SignalProcessor  /root/reference/tetraear/signal/processor.py:18-273
  TetraDecoder     /root/reference/tetraear/core/decoder.py:140-295, 835-888 (lower-MAC part)
  TetraProtocolParser.parse_burst/_check_crc/_calculate_crc16
                   /root/reference/tetraear/core/protocol.py:192-347

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It is pinned bit-exact against golden vectors produced by running the reference itself
(tests/golden/make_golden.py; tests/test_oracle_golden.py checks the pin).

Heavy loops live in compat_oracle.c (liboracle.so, built by oracle/Makefile); vector math
uses the same numpy/scipy calls the reference makes, so third-party numerics (scipy 1.15.3
filter design, numpy's SIMD complex kernels) are inherited, not re-derived.
"""
import ctypes
import os

import numpy as np
from scipy import signal as _ss

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        import subprocess
        try:   # keep the checker in step with its sources (no-op when up to date)
            subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
        except (OSError, subprocess.CalledProcessError):
            if not os.path.exists(path):
                raise
        L = ctypes.CDLL(path)
        f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
        L.orc_sosfilt_f32.argtypes = [f32p, ctypes.c_int, f32p, f32p, ctypes.c_long]
        L.orc_sosfilt_f64.argtypes = [f64p, ctypes.c_int, f64p, f64p, ctypes.c_long]
        L.orc_lfilter_f64.argtypes = [f64p, f64p, ctypes.c_int, f64p, f64p, ctypes.c_long]
        vp = ctypes.c_void_p
        for nm in ("orc_sos_tiles_f32", "orc_sos_tiles_f64"):
            getattr(L, nm).argtypes = [vp, ctypes.c_int, vp, ctypes.c_long, ctypes.c_int, vp, vp, vp]
        L.orc_lf_tiles_f64.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_long, ctypes.c_int, vp, vp, vp]
        L.orc_sync_counts.argtypes = [u8p, ctypes.c_long, u8p, u8p]
        L.orc_find_sync_greedy.argtypes = [u8p, u8p, ctypes.c_long, ctypes.c_int, i64p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_int)]
        L.orc_find_sync_greedy.restype = ctypes.c_int
        L.orc_crc16.argtypes = [u8p, ctypes.c_long, ctypes.c_int]
        L.orc_crc16.restype = ctypes.c_uint32
        L.orc_check_crc.argtypes = [u8p, ctypes.c_long]
        L.orc_check_crc.restype = ctypes.c_int
        _LIB = L
    return _LIB


# ----------------------------------------------------------------------------- filters

def _odd_ext(x, n):
    """scipy.signal._arraytools.odd_ext along the last axis, in x's own dtype."""
    left = 2 * x[0:1] - x[n:0:-1]
    right = 2 * x[-1:] - x[-2:-(n + 2):-1]
    return np.concatenate((left, x, right))


def _components(v):
    return (v.real, v.imag) if np.iscomplexobj(v) else (v,)


def _run_per_component(ext, dtype, init_state, step):
    """Run a real recursion `step(comp, state)` over each component of ext (forward+reverse)."""
    real_t = np.float32 if dtype in (np.float32, np.complex64) else np.float64
    outs = []
    for comp in _components(ext.astype(dtype)):
        c = np.ascontiguousarray(comp, dtype=real_t)
        step(c, init_state(c[0]))
        c = np.ascontiguousarray(c[::-1])
        step(c, init_state(c[0]))
        outs.append(c[::-1])
    if np.iscomplexobj(np.zeros(0, dtype)):
        return (outs[0] + 1j * outs[1]).astype(dtype)
    return outs[0].astype(dtype)


def sosfiltfilt(sos, x):
    """scipy.signal.sosfiltfilt(sos, x) with default odd padding (scipy 1.15.3)."""
    ns = sos.shape[0]
    ntaps = 2 * ns + 1 - min(int((sos[:, 2] == 0).sum()), int((sos[:, 5] == 0).sum()))
    edge = 3 * ntaps
    if x.shape[0] <= edge:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {edge}.")
    dtype = np.result_type(sos, x)
    zi = _ss.sosfilt_zi(sos)
    real_t = np.float32 if dtype in (np.float32, np.complex64) else np.float64
    zr = np.ascontiguousarray(zi.real, dtype=real_t)
    coef = np.ascontiguousarray(np.asarray(sos).real, dtype=real_t)
    fn = lib().orc_sosfilt_f32 if real_t is np.float32 else lib().orc_sosfilt_f64
    ext = _odd_ext(x, edge)
    y = _run_per_component(ext, dtype, lambda x0: np.ascontiguousarray(zr * x0, dtype=real_t),
                           lambda c, st: fn(coef, ns, st, c, len(c)))
    return y[edge:-edge]


def decimate(x, q):
    """scipy.signal.decimate(x, q) (IIR, zero phase), scipy 1.15.3 _signaltools.decimate."""
    x = np.asarray(x)
    rt = x.dtype
    if not np.issubdtype(rt, np.inexact) or rt.type == np.float16:
        rt = np.float64
    sos = np.asarray(_ss.cheby1(8, 0.05, 0.8 / q, output="sos"), dtype=rt)
    return sosfiltfilt(sos, x)[::q]


def filtfilt(b, a, x):
    """scipy.signal.filtfilt(b, a, x) with default odd padding, a[0] == 1."""
    assert a[0] == 1.0
    edge = 3 * max(len(a), len(b))
    if x.shape[0] <= edge:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {edge}.")
    zi = np.ascontiguousarray(_ss.lfilter_zi(b, a), dtype=np.float64)
    ext = _odd_ext(x, edge)
    dtype = np.result_type(b, a, ext, zi[:1] * ext[:1])
    bb = np.ascontiguousarray(b, np.float64)
    aa = np.ascontiguousarray(a, np.float64)
    y = _run_per_component(ext, dtype, lambda x0: np.ascontiguousarray(zi * x0),
                           lambda c, st: lib().orc_lfilter_f64(bb, aa, len(bb), st, c, len(c)))
    return y[edge:-edge]


# ----------------------------------------------------------------------------- time-blocked decimate
# The product's latency-mode decimator (tetraear-bladerf_amd/csrc/compat_demod.hip, k_sosb_*), restated
# operation for operation, so the GPU can be checked bit for bit; its distance from the reference's
# sequential decimate is checked against the reference's own fixtures (tests/test_compat_blocked.py).
# Not a reference function: the reference only has the sequential scipy.signal.decimate
# (/root/reference/tetraear/signal/processor.py:254).
SB_B, SB_MAXT, SB_NPOW, SB_MAXC, SB_MAXQ = 256, 1024, 10, 64, 16


def blocked_fits(C, N, q):
    """The shapes tetra_demod_compat decimates time-blocked by default (compat_demod.hip: blocked_fits)."""
    return 1 <= C <= SB_MAXC and 2 <= q <= SB_MAXQ and N > 27 and -(-(N + 54) // SB_B) <= SB_MAXT


def blocked_table(coef):
    """Phi^(2^r), r < SB_NPOW (Phi = A^SB_B, A the cascade's one-sample zero-input transition in scipy's
    _sosfilt order), as float64 [SB_NPOW, 8, 8]; every product summed in k order, no FMA -- the
    host loops of compat_demod.hip: blocked_table."""
    c = [float(v) for v in np.asarray(coef, np.float64).ravel()]
    A = [[0.0] * 8 for _ in range(8)]
    for k in range(8):
        z = [0.0] * 8
        z[k] = 1.0
        zn = [0.0] * 8
        u = 0.0
        for s in range(4):
            b0, b1, b2, a1, a2 = c[6 * s], c[6 * s + 1], c[6 * s + 2], c[6 * s + 4], c[6 * s + 5]
            xn = b0 * u + z[2 * s]
            zn[2 * s] = (b1 * u - a1 * xn) + z[2 * s + 1]
            zn[2 * s + 1] = b2 * u - a2 * xn
            u = xn
        for i in range(8):
            A[i][k] = zn[i]

    def square(P):
        out = [[0.0] * 8 for _ in range(8)]
        for i in range(8):
            for j in range(8):
                acc = 0.0
                for k in range(8):
                    acc = acc + P[i][k] * P[k][j]
                out[i][j] = acc
        return out

    b = 1
    while b < SB_B:
        A = square(A)
        b <<= 1
    tab = [A]
    for _ in range(1, SB_NPOW):
        tab.append(square(tab[-1]))
    return np.array(tab, np.float64)


def _blocked_pass(coef, zi, c, real_t, tab):
    """sosfilt of one real sequence c from state zi * c[0], time-blocked: every tile of SB_B samples
    from zero state (end states e_k), the start states by the float64 Hillis-Steele scan
    w_k += Phi^d w_{k-d}, every tile again from its start state."""
    L = len(c)
    Tn = -(-L // SB_B)
    tiles = lib().orc_sos_tiles_f32 if real_t is np.float32 else lib().orc_sos_tiles_f64
    c = np.ascontiguousarray(c, real_t)
    coef = np.ascontiguousarray(coef, real_t)
    s0 = np.ascontiguousarray(zi * c[0], dtype=real_t)
    w = np.zeros((Tn, 8), np.float64)
    w[0] = s0.astype(np.float64)
    # every tile from zero state -> its end state (compat_oracle.c: orc_sos_tiles_*, the loop
    # "for k < Tn - 1: sosfilt(tile k, z = 0); w[k + 1] = z")
    tiles(coef.ctypes.data, 4, c.ctypes.data, L, SB_B, w.ctypes.data, None, None)
    r = 0
    while (1 << r) < Tn:
        d = 1 << r
        u = w[:-d].copy()
        acc = w[d:].copy()
        for j in range(8):
            acc = acc + tab[r][None, :, j] * u[:, j:j + 1]
        w[d:] = acc
        r += 1
    out = np.empty(L, real_t)
    w = np.ascontiguousarray(w)
    tiles(coef.ctypes.data, 4, c.ctypes.data, L, SB_B, None, w.ctypes.data, out.ctypes.data)   # tile k from w[k]
    return out


def decimate_blocked(x, q):
    """decimate(x, q) as the product's time-blocked decimator computes it (see above)."""
    x = np.asarray(x)
    dtype = x.dtype
    real_t = np.float32 if dtype in (np.float32, np.complex64) else np.float64
    sos = np.asarray(_ss.cheby1(8, 0.05, 0.8 / q, output="sos"), dtype=dtype)
    zr = np.ascontiguousarray(_ss.sosfilt_zi(sos).real, dtype=real_t).ravel()
    coef = np.ascontiguousarray(sos.real, dtype=real_t).ravel()
    tab = blocked_table(coef)
    edge = 27
    if x.shape[0] <= edge:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {edge}.")
    ext = _odd_ext(x, edge)
    outs = []
    for comp in _components(ext):
        f = _blocked_pass(coef, zr, np.ascontiguousarray(comp, real_t), real_t, tab)
        b = _blocked_pass(coef, zr, np.ascontiguousarray(f[::-1]), real_t, tab)
        outs.append(b[::-1])
    y = (outs[0] + 1j * outs[1]).astype(dtype) if np.iscomplexobj(ext) else outs[0].astype(dtype)
    return y[edge:-edge][::q]


LB_B, LB_NS = 128, 4


def lf_blocked_fits(C, M, ntaps=5):
    """The shapes whose filtfilt tetra_demod_compat runs time-blocked in latency mode."""
    return 1 <= C <= SB_MAXC and ntaps == LB_NS + 1 and -(-(M + 6 * ntaps) // LB_B) <= SB_MAXT


def lfilter_table(b, a):
    """Psi^(2^r) (Psi = B^LB_B, B scipy lfilter's one-sample zero-input transition of its 4 DF-II-T
    states), float64 [SB_NPOW, 4, 4], in compat_demod.hip: lfilter_table's operation order."""
    b = [float(v) for v in b]
    a = [float(v) for v in a]
    K = LB_NS
    Bm = [[0.0] * K for _ in range(K)]
    for c in range(K):
        z = [0.0] * K
        z[c] = 1.0
        xn = 0.0
        yn = z[0] + b[0] * xn
        zn = [0.0] * K
        for k in range(K - 1):
            zn[k] = (z[k + 1] + xn * b[k + 1]) - yn * a[k + 1]
        zn[K - 1] = xn * b[K] - yn * a[K]
        for i in range(K):
            Bm[i][c] = zn[i]

    def square(P):
        out = [[0.0] * K for _ in range(K)]
        for i in range(K):
            for j in range(K):
                acc = 0.0
                for k in range(K):
                    acc = acc + P[i][k] * P[k][j]
                out[i][j] = acc
        return out

    n = 1
    while n < LB_B:
        Bm = square(Bm)
        n <<= 1
    tab = [Bm]
    for _ in range(1, SB_NPOW):
        tab.append(square(tab[-1]))
    return np.array(tab, np.float64)


def _lf_blocked_pass(bb, aa, zi, c, tab):
    """lfilter of one real float64 sequence c from state zi * c[0], time-blocked (tiles of LB_B)."""
    L = len(c)
    Tn = -(-L // LB_B)
    c = np.ascontiguousarray(c, np.float64)
    w = np.zeros((Tn, LB_NS), np.float64)
    w[0] = zi * c[0]
    lib().orc_lf_tiles_f64(bb.ctypes.data, aa.ctypes.data, len(bb), c.ctypes.data, L, LB_B, w.ctypes.data, None, None)
    r = 0
    while (1 << r) < Tn:
        d = 1 << r
        u = w[:-d].copy()
        acc = w[d:].copy()
        for j in range(LB_NS):
            acc = acc + tab[r][None, :, j] * u[:, j:j + 1]
        w[d:] = acc
        r += 1
    out = np.empty(L, np.float64)
    w = np.ascontiguousarray(w)
    lib().orc_lf_tiles_f64(bb.ctypes.data, aa.ctypes.data, len(bb), c.ctypes.data, L, LB_B, None, w.ctypes.data,
                           out.ctypes.data)
    return out


def filtfilt_blocked(b, a, x):
    """filtfilt(b, a, x) as the product's latency mode computes it (compat_demod.hip: k_lfb_*)."""
    assert a[0] == 1.0
    edge = 3 * max(len(a), len(b))
    if x.shape[0] <= edge:
        raise ValueError(f"The length of the input vector x must be greater than padlen, which is {edge}.")
    zi = np.ascontiguousarray(_ss.lfilter_zi(b, a), dtype=np.float64)
    ext = _odd_ext(x, edge)
    dtype = np.result_type(b, a, ext, zi[:1] * ext[:1])
    bb = np.ascontiguousarray(b, np.float64)
    aa = np.ascontiguousarray(a, np.float64)
    tab = lfilter_table(bb, aa)
    outs = []
    for comp in _components(ext.astype(dtype)):
        f = _lf_blocked_pass(bb, aa, zi, np.ascontiguousarray(comp, np.float64), tab)
        r = _lf_blocked_pass(bb, aa, zi, np.ascontiguousarray(f[::-1]), tab)
        outs.append(r[::-1])
    y = (outs[0] + 1j * outs[1]).astype(dtype) if np.iscomplexobj(ext.astype(dtype)) else outs[0].astype(dtype)
    return y[edge:-edge]


# ----------------------------------------------------------------------------- demod

def _pairwise_sum(v):
    """numpy's pairwise summation for float64 (np.add.reduce on a contiguous 1-D array)."""
    return np.add.reduce(v)


class SignalProcessor:
    """Restatement of processor.py:18-273."""

    def __init__(self, sample_rate=2.4e6, decimator="sequential"):
        self.sample_rate = sample_rate
        self.symbol_rate = 18000
        self.samples_per_symbol = int(sample_rate / self.symbol_rate)
        self.symbols = None
        # "sequential" / "auto": the reference's decimate and filtfilt (the product's default form);
        # "blocked": the product's opt-in latency mode (time-blocked decimate and filtfilt where
        # they fit one channel: blocked_fits / lf_blocked_fits)
        self.decimator = decimator

    def filter_signal(self, samples, bandwidth=25000, sample_rate=None):
        if len(samples) == 0:
            return samples
        fs = sample_rate if sample_rate is not None else self.sample_rate
        cutoff = min(0.99, max(0.01, (bandwidth / 2) / (fs / 2)))
        try:
            b, a = _ss.butter(4, cutoff, btype="low")
            return filtfilt(b, a, np.asarray(samples))
        except Exception:
            return samples

    def _filter_blocked(self, samples, fs):
        """filter_signal(samples, 25000, fs) with the latency mode's time-blocked filtfilt."""
        if len(samples) == 0:
            return samples
        cutoff = min(0.99, max(0.01, (25000 / 2) / (fs / 2)))
        try:
            b, a = _ss.butter(4, cutoff, btype="low")
            return filtfilt_blocked(b, a, np.asarray(samples))
        except Exception:
            return samples

    def frequency_shift(self, samples, freq_offset, sample_rate=None):
        fs = sample_rate if sample_rate is not None else self.sample_rate
        t = np.arange(len(samples)) / fs
        return samples * np.exp(-1j * 2 * np.pi * freq_offset * t)

    def demodulate_dqpsk(self, samples):
        if len(samples) < 2:
            return np.array([], dtype=np.uint8)
        samples = np.asarray(samples)
        m = np.max(np.abs(samples))
        if m > 0:
            samples = samples / m
        s = samples[1:]
        p = samples[:-1]
        if np.iscomplexobj(samples):
            sr, si, pr, pi = s.real, s.imag, p.real, -p.imag
            # numpy scalar complex multiply (no FMA): (sr*pr - si*pi, sr*pi + si*pr)
            dr = sr * pr - si * pi
            di = sr * pi + si * pr
        else:
            dr = s * p
            di = np.zeros_like(dr)
        ph = np.arctan2(di, dr)
        out = np.full(len(ph), 3, np.uint8)
        out[ph < 5 * np.pi / 8] = 1
        out[ph < 3 * np.pi / 8] = 0
        out[ph < -3 * np.pi / 8] = 2
        out[ph < -5 * np.pi / 8] = 3
        return out

    def extract_symbols(self, samples, sample_rate=None):
        if len(samples) == 0:
            return np.array([], dtype=complex)
        fs = sample_rate if sample_rate is not None else self.sample_rate
        sps = int(fs / self.symbol_rate)
        if sps <= 1:
            return samples
        best, maxp = 0, -1
        for ph in range(0, sps, max(1, sps // 8)):
            ns = (len(samples) - ph) // sps
            if ns <= 0:
                continue
            p = np.mean(np.abs(samples[ph + np.arange(ns) * sps]) ** 2)
            if p > maxp:
                maxp, best = p, ph
        ns = (len(samples) - best) // sps
        return samples[best + np.arange(ns) * sps]

    def process(self, samples, freq_offset=0):
        if len(samples) == 0:
            self.symbols = np.array([], dtype=complex)
            return np.array([], dtype=np.uint8)
        rate = self.sample_rate
        if rate > 240000 * 2:
            q = int(rate / 240000)
            if q > 1:
                try:
                    blk = self.decimator == "blocked"   # (the product refuses it past blocked_fits)
                    samples = decimate_blocked(samples, q) if blk else decimate(samples, q)
                    rate = rate / q
                except Exception:
                    pass
        if freq_offset != 0:
            samples = self.frequency_shift(samples, freq_offset, sample_rate=rate)
        if self.decimator == "blocked" and lf_blocked_fits(1, len(samples)):   # opt-in latency mode
            filtered = self._filter_blocked(samples, rate)
        else:
            filtered = self.filter_signal(samples, bandwidth=25000, sample_rate=rate)
        sym = self.extract_symbols(filtered, sample_rate=rate)
        self.symbols = sym
        return self.demodulate_dqpsk(sym)


# ----------------------------------------------------------------------------- lower MAC

SYNC_CONT = np.array([1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0], np.uint8)
SYNC_DISC = np.array([0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 0, 0, 1, 1], np.uint8)


def count_threshold(thr):
    """Least integer count c with c/22 >= thr (the float comparison of decoder.py:240-245)."""
    for c in range(23):
        if c / 22 >= thr:
            return c
    return 23


def symbols_to_bits(symbols):
    """decoder.py:140-169 (returns int64 arrays like np.array(list_of_ints))."""
    symbols = np.asarray(symbols)
    if len(symbols) == 0:
        return np.array([]), np.array([])
    if np.max(symbols) <= 3:
        val = symbols.astype(np.int64) & 0x3
    else:
        lut = np.array([0, 0, 0, 1, 1, 3, 2, 2], np.int64)
        s = symbols.astype(np.int64)
        val = np.where((s >= 0) & (s <= 7), lut[np.clip(s, 0, 7)], 0)
    bits = np.stack([val >> 1, val & 1], axis=1).reshape(-1)
    return bits, val


def find_sync(bits, threshold=0.85, return_max_corr=False):
    """decoder.py:171-295."""
    bits = np.ascontiguousarray(np.asarray(bits), dtype=np.uint8) if len(bits) else np.zeros(0, np.uint8)
    if len(bits) < 22:
        return ([], 0.0) if return_max_corr else []
    nw = len(bits) - 21
    c1 = np.empty(nw, np.uint8)
    c2 = np.empty(nw, np.uint8)
    lib().orc_sync_counts(bits, len(bits), c1, c2)
    pos = np.zeros(nw // 250 + 2, np.int64)
    mc = ctypes.c_int(0)
    n = lib().orc_find_sync_greedy(c1, c2, nw, count_threshold(threshold), pos, len(pos), ctypes.byref(mc))
    sync = [int(p) for p in pos[:n]]
    max_corr = mc.value / 22
    if not sync and max_corr > 0.75 and max_corr >= (threshold - 0.15):
        adaptive = max(0.75, max_corr - 0.02)
        if adaptive < threshold:
            m = np.maximum(c1, c2)
            k = count_threshold(adaptive)
            last = -10 ** 9
            for i in np.nonzero(m >= k)[0]:
                if i >= last + 250:
                    sync.append(int(i))
                    last = int(i)
    return (sync, max_corr) if return_max_corr else sync


def decode_syncs(bits):
    """The threshold cascade of decoder.py:845-857."""
    sp, mc = find_sync(bits, threshold=0.90, return_max_corr=True)
    if not sp:
        sp, mc = find_sync(bits, threshold=0.85, return_max_corr=True)
        if not sp:
            sp, mc = find_sync(bits, threshold=0.80, return_max_corr=True)
            if not sp and mc >= 0.75:
                sp, _ = find_sync(bits, threshold=max(0.75, mc - 0.02), return_max_corr=True)
    return sp


def calculate_crc16(bits):
    b = np.ascontiguousarray(np.asarray(bits) & 1, dtype=np.uint8)
    c = lib().orc_crc16(b, len(b), 0)
    return np.array([(c >> i) & 1 for i in range(15, -1, -1)])


def check_crc(bits):
    b = np.ascontiguousarray(np.asarray(bits) & 1, dtype=np.uint8)
    return bool(lib().orc_check_crc(b, len(b)))


def parse_burst_fields(symbols):
    """parse_burst (protocol.py:192-244) -> (burst_type value, training_sequence, data_bits, crc_ok)."""
    if len(symbols) < 255:
        return None
    s = np.asarray(symbols)[:255].astype(np.int64)
    bits = np.stack([(s >> 1) & 1, s & 1], axis=1).reshape(-1)
    w = bits[255:277]
    corr = max(np.sum(w == SYNC_CONT) / 22, np.sum(w == SYNC_DISC) / 22)
    if corr > 0.8:
        btype, ts, data = 5, bits[108:130], bits
    else:
        btype, ts, data = 2, bits[108:122], np.concatenate([bits[0:108], bits[122:230]])
    return btype, ts, data, check_crc(data)


def decode_frames(symbols):
    """Lower-MAC part of decode()/decode_frame() (decoder.py:835-888, 890-992)."""
    bits, mapped = symbols_to_bits(symbols)
    frames = []
    for pos in decode_syncs(bits):
        start = pos - 216
        if start < 0 or start // 2 + 255 > len(mapped):
            continue
        fb = bits[start:start + 510]
        f = dict(pos=pos, start=start, number=start // 510, nbits=len(fb))
        if len(fb) >= 510:
            btype, ts, data, ok = parse_burst_fields(mapped[start // 2:start // 2 + 255])
            f.update(burst_type=btype, ts=ts, data=data, crc_ok=ok,
                     header="".join(str(int(v)) for v in fb[:32]), pdu_type=int(fb[0] * 2 + fb[1]),
                     enc_mode=int(fb[2] * 2 + fb[3]))
        frames.append(f)
    return frames


_ENC_MODES = {1: ("TEA1", "Class 2 (SCK)"), 2: ("TEA2", "Class 3 (DCK)"), 3: ("TEA3", "Reserved")}
_PDU_NAMES = {0: "MAC_RESOURCE", 1: "MAC_FRAG", 2: "MAC_END", 3: "MAC_BROADCAST"}


def decode_with_mac(symbols, mac_parser=None):
    """decode() through decode_frame's MAC PDU stage (decoder.py:835-888, 890-1100) with the
    oracle's parse_mac_pdu (oracle/mac.py): [dict(number, header, burst_crc, encrypted,
    encryption_algorithm, encryption_mode, mac_pdu)] of the frames the reference keeps.

    decoder.py:1093-1095: no MAC PDU and a failed CRC drops the frame.  decoder.py:1008-1053: a PDU
    settles 'encrypted' / 'encryption_algorithm' from its mode, or by the data-entropy rule."""
    from mac import MacParser
    mp = mac_parser if mac_parser is not None else MacParser()
    out = []
    for f in decode_frames(symbols):
        if f["nbits"] < 510:
            continue
        enc = f["enc_mode"]
        alg, mode_txt = _ENC_MODES.get(enc, (None, None))
        d = dict(number=f["number"], header=f["header"], burst_crc=bool(f["crc_ok"]), encrypted=enc > 0,
                 encryption_algorithm=alg, encryption_mode=mode_txt, mac_pdu=None)
        pdu = mp.parse(f["data"])
        if pdu is None:
            if not f["crc_ok"]:
                continue
            out.append(d)
            continue
        d["mac_pdu"] = dict(type=_PDU_NAMES[pdu["pdu_type"]], encrypted=bool(pdu["encrypted"]),
                            address=pdu["address"], length=pdu["length"], data=bytes(pdu["data"]).hex())
        if pdu["encrypted"]:
            d["encrypted"] = True
            if pdu["encryption_mode"] in _ENC_MODES:
                d["encryption_algorithm"], d["encryption_mode"] = _ENC_MODES[pdu["encryption_mode"]]
            elif not d["encryption_algorithm"]:
                d["encryption_algorithm"] = "TEA1"
        else:
            data = bytes(pdu["data"])
            if len(data) > 0 and len(set(data)) / max(len(data), 1) > 0.7 and len(data) > 8:
                d["encrypted"] = True
            else:
                d["encrypted"], d["encryption_algorithm"] = False, None
        out.append(d)
    return out
