"""ETSI EN 300 392-2 demodulator (north-star chain) on the GPU.

The reference demodulates with integer samples/symbol and shifted decision regions
(/root/reference/tetraear/signal/processor.py:152-183).  This receiver is the
standard one BASELINE.json's north_star names: polyphase channel filter + RRC(0.35) matched
filter resampled to 4 samples/symbol, Oerder-Meyr timing acquisition with block-Gardner
tracking, pi/4-DQPSK differential decision per Table 5.1 with a 4th-power CFO correction, and
int8 soft bits for the channel decoder.  All sample work runs in libtetra_hip.so
(k_chanfilt, k_timing); this module designs the filters and moves arrays.
"""
import ctypes
import os
import functools

import numpy as np
from scipy import signal as _design

from tetraear import _hip

SYMBOL_RATE = 18000.0


def rrc(t, alpha=0.35):
    """Root-raised-cosine impulse response at t symbol periods (unit-energy pulse)."""
    t = np.asarray(t, np.float64)
    out = np.empty_like(t)
    z = np.abs(t) < 1e-9
    out[z] = 1.0 - alpha + 4 * alpha / np.pi
    s = np.abs(np.abs(4 * alpha * t) - 1.0) < 1e-9
    out[s] = (alpha / np.sqrt(2)) * ((1 + 2 / np.pi) * np.sin(np.pi / (4 * alpha))
                                     + (1 - 2 / np.pi) * np.cos(np.pi / (4 * alpha)))
    o = ~(z | s)
    tt = t[o]
    out[o] = (np.sin(np.pi * tt * (1 - alpha)) + 4 * alpha * tt * np.cos(np.pi * tt * (1 + alpha))) / \
        (np.pi * tt * (1 - (4 * alpha * tt) ** 2))
    return out


def rate_design(fs):
    """(q1, L1, up, down, Lp) of the receiver for input rate fs: stage 1 decimates by q1 (L1-tap FIR,
    fs1 = fs / q1 >= 180 kHz), stage 2 resamples fs1 x up/down to 72 kHz (4 samples/symbol) with an
    8-symbol RRC prototype of Lp = 32 down + 1 taps at up * fs1 = 4 down x 18 kHz.  Among the q1 <= 13
    whose plan fits the kernels (Lp <= 4096, a stage-2 window of < 254 taps) the smallest `down` (the
    shortest prototype) wins, then the larger q1.  2.4 MSps gives the canonical 10, 48, 3/10, 321;
    the reference CLI's 1.8-2.4 MSps (modern.py:5518-5519, 5630-5638) give q1 = 10 / 10 / 10 / 7 / 11
    / 10 / 10.  Raises ValueError for a rate no such plan serves (e.g. 20 MSps: that is the wideband
    channeliser's input)."""
    from fractions import Fraction
    fs_i = int(round(fs))
    if abs(fs - fs_i) > 1e-6 or fs_i < 72000:
        raise ValueError(f"ETSI receiver: unsupported sample rate {fs!r} (integer Hz >= 72 kHz required)")
    best = None
    for q1 in range(1, 14):
        if q1 > 1 and fs_i / q1 < 180000.0:
            break
        r = Fraction(72000 * q1, fs_i)
        up, down = r.numerator, r.denominator
        Lp = 32 * down + 1
        if Lp > 4096 or (Lp - 1) // up + 2 >= 254:
            continue
        L1 = 1 if q1 == 1 else min(64, 2 * int(round(2.4 * q1)))
        if best is None or (down, -q1) < best[0]:
            best = ((down, -q1), (q1, L1, up, down, Lp))
    if best is None:
        raise ValueError(f"ETSI receiver: no channel-filter plan for {fs_i} Sps")
    return best[1]


@functools.lru_cache(maxsize=16)
def etsi_plan(fs=2.4e6, force_generic=False):
    """Receiver design for input rate fs (rate_design): stage-1 Kaiser FIR (60 kHz cutoff), RRC(0.35)
    prototype scaled by 240 kHz / fs1 (1 at the canonical 2.4 MSps), loop constants."""
    q1, L1, up, down, Lp = rate_design(fs)
    p = _hip.EtsiPlan()
    p.q1, p.L1, p.Lp, p.up, p.down = q1, L1, Lp, up, down
    p.gain, p.soft_scale = 1.5, 64.0
    p.flags = _hip.ETSI_FORCE_GENERIC if force_generic else 0
    h1 = (_design.firwin(L1, 60e3, fs=fs, window=("kaiser", 6.0)) if q1 > 1 else np.ones(1)).astype(np.float32)
    hp = (rrc((np.arange(Lp) - (Lp - 1) / 2) / (4.0 * down)) * (240000.0 * q1 / fs)).astype(np.float32)
    for i, v in enumerate(h1):
        p.h1[i] = v
    for i, v in enumerate(hp):
        p.hp[i] = v
    return p


def lengths(plan, n):
    m1, m2, sm = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    _hip.lib().tetra_etsi_lengths(plan, n, ctypes.byref(m1), ctypes.byref(m2), ctypes.byref(sm))
    return m1.value, m2.value, sm.value


class SoftSymbols(np.ndarray):
    """uint8 hard dibit symbols (what process() returns) that also carry ``soft_bits`` (int8, >0 = 0)
    so TetraDecoder(mode='etsi').decode() can run the soft-decision Viterbi on them."""

    def __new__(cls, hard, soft_bits):
        obj = np.asarray(hard, np.uint8).view(cls)
        obj.soft_bits = soft_bits
        return obj

    def __array_finalize__(self, obj):
        self.soft_bits = getattr(obj, "soft_bits", None)


RESERVE, MARGIN = _hip.ETSI_RESERVE, _hip.ETSI_MARGIN
TRACK = _hip.ETSI_TRACK


def stream_window(plan, x_total, y_done, n):
    """tetra_etsi_stream_window: (s, W, yoff, y_done_next) of the next chunk of n samples."""
    v = [ctypes.c_int64() for _ in range(4)]
    rc = _hip.lib().tetra_etsi_stream_window(plan, int(x_total), int(y_done), int(n), *[ctypes.byref(x) for x in v])
    if rc:
        raise ValueError("tetra_etsi_stream_window: invalid arguments")
    return tuple(x.value for x in v)


def _sc16_to_cf32(x):
    """[C, N, 2] int16 -> [C, N] complex64 scaled 1/32768 (capture.py:241-269; exact)."""
    return ((x[..., 0].astype(np.float32) + 1j * x[..., 1].astype(np.float32)) / np.float32(32768)).astype(
        np.complex64)


class EtsiStream:
    """The demod half of the streaming receiver: consecutive chunks of C channels' continuous
    captures (the reference's capture loops, /root/reference/tetraear/ui/modern.py:1901-1919,
    continuous_capture.py:20) demodulated as ONE symbol stream per channel.

    Each chunk's channel filter runs over a window that starts before the chunk -- the previous
    chunks' last samples are kept here (``HIST``) -- at a multiple of q1 * down input samples, so its
    polyphase phases are those of a run over the whole capture (tetra_etsi_stream_window); the timing
    loop of every channel is carried in ``track`` (tetra_etsi_track: base, delta, last symbol); the
    AFC mixer (``freq_offsets``) runs on the window with the capture's global sample index, so its
    phase is continuous too.  Row c of the outputs holds the carried last symbol of the previous
    chunk first (once the channel's loop is acquired), so its nsym-1 dibits start with the one across
    the seam -- exactly the row layout demod_batch returns, ready for EtsiLowerMac.decode_stream.
    oracle/etsi.py Stream restates it."""

    HIST = 4096   # input samples kept per channel (a window re-reads < 1600 at every supported rate)

    def __init__(self, sample_rate=2.4e6, channels=1):
        self.sample_rate = sample_rate
        self.plan = etsi_plan(sample_rate)
        self.C = int(channels)
        self.reset()

    def reset(self):
        """A new capture: the next chunk acquires timing (Oerder-Meyr) and starts the chains."""
        self.track = np.zeros(self.C, TRACK)
        self.x_total = self.y_done = 0
        self.hist = None
        self.diag = None

    def demod(self, iq, freq_offsets=None):
        """[C, n] complex or [C, n, 2] int16 SC16 (n even) -> (hard [C, smax] u8, soft_bits
        [C, 2*smax] i8, symbols [C, smax] c64, nsym [C]) of this chunk, rows as described above."""
        iq = np.asarray(iq)
        if iq.dtype == np.int16:
            if iq.ndim != 3 or iq.shape[-1] != 2:
                raise ValueError("SC16 input must be [C, N, 2] int16")
            fmt, x = _hip.TETRA_SC16, np.ascontiguousarray(iq)
        else:
            fmt, x = _hip.TETRA_CF32, np.ascontiguousarray(iq, dtype=np.complex64)
        if x.shape[0] != self.C:
            raise ValueError(f"EtsiStream of {self.C} channels given {x.shape[0]}")
        n = x.shape[1]
        if n % 2:
            raise ValueError("streaming chunks must hold an even number of samples")
        # SC16 -> cf32 is exact (the SC16 kernels compute on the same scaled samples, bit for bit), so a
        # stream whose chunks mix the formats -- or SC16 with the mixer on for some chunks, which takes
        # cf32 -- continues in cf32
        if fmt == _hip.TETRA_SC16 and (freq_offsets is not None or
                                       (self.hist is not None and self.hist.dtype != np.int16)):
            x, fmt = _sc16_to_cf32(x), _hip.TETRA_CF32
        if self.hist is not None and self.hist.dtype == np.int16 and fmt == _hip.TETRA_CF32:
            self.hist = _sc16_to_cf32(self.hist)
        s, W, yoff, y_next = stream_window(self.plan, self.x_total, self.y_done, n)
        h = self.x_total - s
        if h > (0 if self.hist is None else self.hist.shape[1]):
            raise RuntimeError(f"stream window needs {h} samples of history")
        win = x if h == 0 else np.concatenate([self.hist[:, self.hist.shape[1] - h:], x], axis=1)
        win = np.ascontiguousarray(win)
        c = _hip.ctx()
        if freq_offsets is not None:
            from tetraear.signal.processor import mixer_coefficient
            fo = np.broadcast_to(np.asarray(freq_offsets, np.float64), (self.C,))
            mc = np.array([mixer_coefficient(f) for f in fo], np.float64)
            mixed = np.empty((self.C, W), np.complex64)
            c.check(c.lib.tetra_etsi_mix(c.handle, _hip.ptr(win), self.C, W, W, _hip.ptr(mc), float(self.sample_rate),
                                         int(s), _hip.ptr(mixed)), "tetra_etsi_mix")
            dwin = mixed
        else:
            dwin = win
        _, M2, sm = lengths(self.plan, W)
        smax = max(sm + 1, 2)
        sym = np.zeros((self.C, smax), np.complex64)
        soft = np.zeros((self.C, 2 * smax), np.int8)
        hard = np.zeros((self.C, smax), np.uint8)
        ns = np.zeros(self.C, np.int32)
        diag = np.zeros((self.C, 4), np.float32)
        c.check(c.lib.tetra_demod_etsi_stream(c.handle, self.plan, _hip.ptr(dwin), fmt, self.C, W, W, int(yoff),
                                              _hip.ptr(self.track), _hip.ptr(sym), _hip.ptr(soft), _hip.ptr(hard),
                                              _hip.ptr(ns), smax, smax, _hip.ptr(diag)), "tetra_demod_etsi_stream")
        keep = min(self.HIST, win.shape[1])
        self.hist = np.ascontiguousarray(win[:, win.shape[1] - keep:])
        self.x_total += n
        self.y_done = y_next
        self.diag = diag
        return hard, soft, sym, ns


class EtsiReceiver:
    def __init__(self, sample_rate=2.4e6):
        self.sample_rate = sample_rate
        self.plan = etsi_plan(sample_rate)
        self.diag = None
        self._stream = None
        self._odd = None   # a streamed chunk's odd last sample, carried to the front of the next one

    def reset(self):
        """process() starts a new capture (a retune): timing is acquired afresh on the next chunk."""
        self._stream = None
        self._odd = None

    def demod_batch(self, iq):
        """[C, N] complex, or [C, N, 2] int16 SC16 capture samples (scaled 1/32768 in the channel
        filter, as capture.py:241-269 scales them) -> (hard [C, smax] u8, soft_bits [C, 2*smax] i8,
        symbols [C, smax] c64, nsym [C])."""
        iq = np.asarray(iq)
        if iq.dtype == np.int16:
            if iq.ndim != 3 or iq.shape[-1] != 2:
                raise ValueError("SC16 input must be [C, N, 2] int16")
            fmt, x = _hip.TETRA_SC16, np.ascontiguousarray(iq)
        else:
            fmt, x = _hip.TETRA_CF32, np.ascontiguousarray(iq, dtype=np.complex64)
        C, N = x.shape[:2]
        if N % 2:
            x = np.ascontiguousarray(x[:, :N - 1])
            N -= 1
        _, M2, smax = lengths(self.plan, N)
        smax = max(smax, 1)
        sym = np.zeros((C, smax), np.complex64)
        soft = np.zeros((C, 2 * smax), np.int8)
        hard = np.zeros((C, smax), np.uint8)
        ns = np.zeros(C, np.int32)
        diag = np.zeros((C, 4), np.float32)
        if C == 0 or M2 <= 0:   # shorter than the channel filter: no symbols in any channel (as process())
            self.diag = diag
            return hard, soft, sym, ns
        c = _hip.ctx()
        c.check(c.lib.tetra_demod_etsi_fmt(c.handle, self.plan, _hip.ptr(x), fmt, C, N, _hip.ptr(sym),
                                           _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(ns), smax, _hip.ptr(diag)),
                "tetra_demod_etsi")
        self.diag = diag
        return hard, soft, sym, ns

    def process(self, samples, freq_offset=0, stream=True):
        """One chunk -> (SoftSymbols hard dibits, complex64 symbol-rate samples).

        ``stream`` (default): the chunk continues the capture the previous process() calls fed
        (the reference's callers stream one capture chunk by chunk, modern.py:1901-1919): an
        EtsiStream of one channel carries the filter history, the timing loop and the mixer phase,
        so the symbols continue across the seam -- the returned symbols then start with the
        previous chunk's last one and the dibits with the one across the seam (len(hard) ==
        len(symbols) - 1 either way).  An odd chunk's last sample is carried into the next call.
        reset() starts a new capture.  ``stream=False``: the chunk on its own (demod_batch)."""
        x = np.ascontiguousarray(samples, np.complex64)
        if stream:
            # the stream takes whole sample pairs (the kernels load two at a time): an odd chunk's last
            # sample goes in front of the next chunk instead of being dropped, so no sample slips
            if self._odd is not None:
                x = np.concatenate([self._odd, x])
                self._odd = None
            if len(x) % 2:
                self._odd = x[-1:].copy()
                x = x[:-1]
            if len(x) == 0:
                return SoftSymbols(np.zeros(0, np.uint8), np.zeros(0, np.int8)), np.zeros(0, np.complex64)
            if self._stream is None:
                self._stream = EtsiStream(self.sample_rate, 1)
            hard, soft, sym, ns = self._stream.demod(x[None, :], [freq_offset] if freq_offset else None)
            self.diag = self._stream.diag
            n = int(ns[0])
            nd = max(0, n - 1)
            return SoftSymbols(hard[0, :nd].copy(), soft[0, :2 * nd].copy()), sym[0, :n].copy()
        if freq_offset and len(x):   # AFC mixer on the GPU (same kernel as frequency_shift)
            from tetraear.signal.processor import mixer_coefficient
            out = np.empty(len(x), np.complex128)
            cf = np.array([mixer_coefficient(freq_offset)], np.float64)
            c = _hip.ctx()
            c.check(c.lib.tetra_frequency_shift(c.handle, _hip.ptr(x), _hip.TETRA_CF32, 1, len(x), _hip.ptr(cf),
                                                float(self.sample_rate), _hip.ptr(out)), "tetra_frequency_shift")
            x = out.astype(np.complex64)
        _, _, smax = lengths(self.plan, len(x) - len(x) % 2)
        if len(x) < 2 or smax <= 2 or lengths(self.plan, len(x) - len(x) % 2)[1] < 16:
            return SoftSymbols(np.zeros(0, np.uint8), np.zeros(0, np.int8)), np.zeros(0, np.complex64)
        hard, soft, sym, ns = self.demod_batch(x[None, :])
        n = int(ns[0])
        nd = max(0, n - 1)
        return SoftSymbols(hard[0, :nd].copy(), soft[0, :2 * nd].copy()), sym[0, :n].copy()

    def decide(self, symbols):
        """Table 5.1 differential decision on given symbol-spaced samples (tetra_etsi_decide):
        uint8 dibits, one fewer than the symbols (the fused demod's decision without its CFO
        rotation; ETSI-mode demodulate_dqpsk)."""
        x = np.asarray(symbols)
        if x.dtype in (np.float32, np.float64) and x.ndim == 2:   # interleaved I/Q: [n, 2] -> [n] complex
            if x.shape[1] != 2:
                raise ValueError("real-valued 2-D symbols must be interleaved I/Q of shape [n, 2]")
            x = np.ascontiguousarray(x).view(np.complex64 if x.dtype == np.float32 else np.complex128)[:, 0]
        elif not np.iscomplexobj(x):   # 1-D real samples: zero imaginary part, as numpy's angle() reads them
            x = x.astype(np.complex64 if x.dtype == np.float32 else np.complex128)
        if len(x) < 2:
            return np.array([], dtype=np.uint8)
        fmt = _hip.TETRA_CF32 if x.dtype == np.complex64 else _hip.TETRA_CF64
        xc = np.ascontiguousarray(x, np.complex64 if fmt == _hip.TETRA_CF32 else np.complex128)
        out = np.empty(len(x) - 1, np.uint8)
        c = _hip.ctx()
        c.check(c.lib.tetra_etsi_decide(c.handle, _hip.ptr(xc), fmt, len(xc), _hip.ptr(out)), "tetra_etsi_decide")
        return out

    def chanfilt(self, samples):
        """Channel filter: 2.4 MSps samples -> the RRC-matched 72 kHz samples (4 per symbol) the
        timing stage reads (tetra_etsi_chanfilt); ETSI-mode filter_signal."""
        x = np.ascontiguousarray(samples, np.complex64)
        x = x[:len(x) - len(x) % 2]
        _, M2, _ = lengths(self.plan, len(x))
        y = np.zeros(max(M2, 0), np.complex64)
        if M2 <= 0:
            return y
        c = _hip.ctx()
        c.check(c.lib.tetra_etsi_chanfilt(c.handle, self.plan, _hip.ptr(x), 1, len(x), _hip.ptr(y)),
                "tetra_etsi_chanfilt")
        return y

    def timing(self, y):
        """Timing recovery on 72 kHz samples: (SoftSymbols hard dibits, complex64 symbol-spaced
        samples) (tetra_etsi_timing); ETSI-mode extract_symbols returns the samples."""
        y = np.ascontiguousarray(y, np.complex64)
        M2 = len(y)
        smax = M2 // 4 + 2
        if M2 < 16:
            return SoftSymbols(np.zeros(0, np.uint8), np.zeros(0, np.int8)), np.zeros(0, np.complex64)
        sym = np.zeros(smax, np.complex64)
        soft = np.zeros(2 * smax, np.int8)
        hard = np.zeros(smax, np.uint8)
        ns = np.zeros(1, np.int32)
        c = _hip.ctx()
        c.check(c.lib.tetra_etsi_timing(c.handle, self.plan, _hip.ptr(y), 1, M2, _hip.ptr(sym), _hip.ptr(soft),
                                        _hip.ptr(hard), _hip.ptr(ns), smax, None), "tetra_etsi_timing")
        n = int(ns[0])
        nd = max(0, n - 1)
        return SoftSymbols(hard[:nd].copy(), soft[:2 * nd].copy()), sym[:n].copy()


def synth(C, N, fs=2.4e6, seed=1, snr_db=None, cfo_max=600.0, device_arrays=None):
    """Device-generated synthetic capture (host copies returned).  See tetra_synth_etsi."""
    nb = _hip.lib().tetra_synth_bursts_per_channel(N, fs)
    iq = np.zeros((C, N), np.complex64)
    cells = np.zeros(C, np.uint32)
    kinds = np.zeros((C, nb), np.int32)
    payload = np.zeros((C, nb, 2, 268), np.uint8)
    t0 = np.zeros(C, np.float64)
    c = _hip.ctx()
    c.check(c.lib.tetra_synth_etsi(c.handle, C, N, fs, seed, 1000.0 if snr_db is None else float(snr_db),
                                   float(cfo_max), _hip.ptr(iq), _hip.ptr(cells), _hip.ptr(kinds),
                                   _hip.ptr(payload), _hip.ptr(t0)), "tetra_synth_etsi")
    return iq, cells, kinds, payload, t0


def _on_stream(c):
    """torch ops enqueued on library context c's stream (ordered with its kernels)."""
    import torch
    ptr = c.lib.tetra_get_stream(c.handle)
    return torch.cuda.stream(torch.cuda.ExternalStream(ptr) if ptr else torch.cuda.default_stream())


class BenchStep:
    """bench.py workload: device-resident synthetic capture -> fused demod -> lower MAC."""

    dtype = "f32 (DSP), int8/int32 (Viterbi)"

    def __init__(self, c, C, N, fs, seed, device, snr_db=18.0, iq_format="cf32", demod="fused", cells="given",
                 chunks=1):
        import torch
        self.c, self.C, self.N, self.fs = c, C, N, fs
        # "acquire": the lower MAC finds each channel's cell in its BSCH (tetra_lmac_etsi_acquire,
        # per-channel state carried from step to step, as a receiver streaming chunks would);
        # "given": the synthesised cells are configured up front (tetra_etsi_set_cells)
        self.cells_mode = cells
        # "fused": k_chanfilt<.., true> (timing on the LDS-resident 72 kHz samples, wave 0 of the
        # workgroup); "split": k_chanfilt<.., false> writes y (0.24 B per input sample) and k_timing
        # runs as its own launch -- with the pipeline, beside the next batch's channel filter
        self.demod_mode = demod
        self.fmt = {"cf32": _hip.TETRA_CF32, "sc16": _hip.TETRA_SC16}[iq_format]
        self.plan = etsi_plan(fs)
        _, self.M2, self.smax = lengths(self.plan, N)
        # chunks > 1: every channel is one continuous capture of chunks x N samples, resident in HBM
        # as [C, chunks N] rows, and decoded as ONE stream (streaming receiver: step k demodulates
        # chunk k's window -- the previous chunk's last samples re-read in place, tetra_etsi_stream_window
        # -- with every channel's timing loop carried, and the lower MAC resumes each channel's burst
        # scan on the dibits the previous step left unconsumed, tetra_lmac_etsi_stream), the cell
        # state of protocol.py:479-485 kept as a receiver streaming 128 Ki chunks (modern.py:1919)
        # does.  A run longer than the capture starts it again as a new capture (stream_resets).
        self.chunks = max(1, int(chunks))
        self.stream = self.chunks > 1
        if self.stream and demod != "fused":
            raise ValueError("the streaming bench runs the fused demod")
        NT = N * self.chunks
        nb = c.lib.tetra_synth_bursts_per_channel(NT, fs)
        self.cells = torch.empty(C, dtype=torch.int32, device=device)
        self.kinds = torch.empty((C, nb), dtype=torch.int32, device=device)
        self.payload = torch.empty((C, nb, 2, 268), dtype=torch.uint8, device=device)
        if self.stream:
            # synthesised straight into the capture rows, in channel slices (SC16: through a float slice)
            sc16 = self.fmt == _hip.TETRA_SC16
            self.cap = torch.empty((C, NT, 2), dtype=torch.int16 if sc16 else torch.float32, device=device)
            S = max(1, min(C, (1 << 30) // NT))
            for s0 in range(0, C, S):
                n = min(S, C - s0)
                dst = torch.empty((n, NT, 2), dtype=torch.float32, device=device) if sc16 else self.cap[s0:s0 + n]
                c.check(c.lib.tetra_synth_etsi(c.handle, n, NT, fs, seed + 7919 * (s0 // S), snr_db, 600.0,
                                               _hip.ptr(dst), _hip.ptr(self.cells[s0:]), _hip.ptr(self.kinds[s0:]),
                                               _hip.ptr(self.payload[s0:]), None), "synth")
                if sc16:
                    c.synchronize()
                    self.cap[s0:s0 + n].copy_(torch.round(dst * 32768).clamp_(-32768, 32767).to(torch.int16))
                    del dst
            self.iqs = [self.cap]
        elif self.chunks == 1:
            self.iqs = [torch.empty((C, N, 2), dtype=torch.float32, device=device)]
            c.check(c.lib.tetra_synth_etsi(c.handle, C, N, fs, seed, snr_db, 600.0, _hip.ptr(self.iqs[0]),
                                           _hip.ptr(self.cells), _hip.ptr(self.kinds), _hip.ptr(self.payload), None),
                    "synth")
        else:
            # synthesised in channel slices (a slice's whole capture, then cut into the chunk batches)
            self.iqs = [torch.empty((C, N, 2), dtype=torch.float32, device=device) for _ in range(self.chunks)]
            S = max(1, min(C, (1 << 30) // NT))
            for s0 in range(0, C, S):
                n = min(S, C - s0)
                x = torch.empty((n, NT, 2), dtype=torch.float32, device=device)
                c.check(c.lib.tetra_synth_etsi(c.handle, n, NT, fs, seed + 7919 * (s0 // S), snr_db, 600.0, _hip.ptr(x),
                                               _hip.ptr(self.cells[s0:]), _hip.ptr(self.kinds[s0:]),
                                               _hip.ptr(self.payload[s0:]), None), "synth")
                c.synchronize()   # the copies below run on torch's stream, which need not be the context's
                for k in range(self.chunks):
                    self.iqs[k][s0:s0 + n].copy_(x[:, k * N:(k + 1) * N])
                del x
        c.check(c.lib.tetra_etsi_set_cells(c.handle, _hip.ptr(self.cells), C), "set_cells")
        c.synchronize()   # the synthesised batches are read by torch's ops below (SC16 conversion)
        from tetraear.core.etsi import UNKNOWN_CELL
        self.cell_state = torch.full((C,), UNKNOWN_CELL, dtype=torch.int32, device=device)
        if self.fmt == _hip.TETRA_SC16 and not self.stream:   # the synth output is on the SC16 grid: exact
            self.iqs = [torch.round(x * 32768).clamp_(-32768, 32767).to(torch.int16) for x in self.iqs]
        self.iq = self.iqs[0]
        self.kchunk = 0
        if self.stream:
            # output rows: TETRA_ETSI_RESERVE dibits for the carried tail, then a window's symbols
            # (a window is the chunk + < 1600 samples of the previous one)
            _, self.M2, sm1 = lengths(self.plan, N + 4096)
            self.smax = sm1 + 1
            self.stride = RESERVE + self.smax
            self.track = torch.zeros((C, TRACK.itemsize // 4), dtype=torch.int32, device=device)
            self.lead = torch.full((C,), 2 * RESERVE, dtype=torch.int32, device=device)
            self.x_total = self.y_done = 0
            self.resets = 0
            self._next_k, self._origin = 0, 0   # the chunk the stream continues into; its capture's start
            self.bufs = [self._stream_bufs(device) for _ in range(2)]
            self.sym, self.soft, self.hard, self.nsym = self.bufs[0]
        sm = self.smax
        if not self.stream:
            self.sym = torch.empty((C, sm, 2), dtype=torch.float32, device=device)
            self.soft = torch.empty((C, 2 * sm), dtype=torch.int8, device=device)
            self.hard = torch.empty((C, sm), dtype=torch.uint8, device=device)
            self.nsym = torch.empty(C, dtype=torch.int32, device=device)
        self.nburst = torch.empty(C, dtype=torch.int32, device=device)
        self.bursts = torch.empty((C, _hip.ETSI_MAXB, 2), dtype=torch.int32, device=device)
        self.nblock = torch.empty(C, dtype=torch.int32, device=device)
        self.blocks = torch.empty((C, _hip.ETSI_MAXJ, 4), dtype=torch.int32, device=device)
        self.type1 = torch.empty((C, _hip.ETSI_MAXJ, 268), dtype=torch.uint8, device=device)
        if demod == "split":
            self.y = [torch.empty((C, self.M2, 2), dtype=torch.float32, device=device)]
        self.pipelined = False
        # buffers made by torch (on torch's stream) are complete before any kernel of the context's
        # stream -- a Context() of its own runs on a non-blocking stream that does not wait for torch's
        c.synchronize()
        torch.cuda.current_stream(device).synchronize()

    def _stream_bufs(self, device):
        import torch
        C, st = self.C, self.stride
        return (torch.zeros((C, st, 2), dtype=torch.float32, device=device),
                torch.zeros((C, 2 * st), dtype=torch.int8, device=device),
                torch.zeros((C, st), dtype=torch.uint8, device=device),
                torch.zeros(C, dtype=torch.int32, device=device))

    def pipeline(self):
        """Stream the batches through a two-stage software pipeline: the fused demod (HBM-bound
        channel filter + timing) of batch k+1 runs on a front stream while the lower MAC (sync,
        Viterbi) of batch k runs on a back stream.  The symbol-rate outputs are double-buffered;
        each stage waits only on the event that protects its buffer.  Every step still does the
        whole chain."""
        import torch
        dev = self.iq.device
        self.back = _hip.Context()
        self.s_front = torch.cuda.current_stream(dev)
        self.s_back = torch.cuda.Stream(device=dev)
        self.back.check(self.back.lib.tetra_set_stream(self.back.handle, ctypes.c_void_p(self.s_back.cuda_stream)),
                        "set_stream")
        self.back.check(self.back.lib.tetra_etsi_set_cells(self.back.handle, _hip.ptr(self.cells), self.C), "set_cells")
        if not self.stream:
            self.bufs = [(self.sym, self.soft, self.hard, self.nsym),
                         tuple(torch.empty_like(t) for t in (self.sym, self.soft, self.hard, self.nsym))]
        if self.demod_mode == "split":   # y is what crosses the streams; the symbol buffers stay on the back one
            self.y.append(torch.empty_like(self.y[0]))
        self.ev_front = [torch.cuda.Event() for _ in range(2)]
        self.ev_back = [torch.cuda.Event() for _ in range(2)]
        for e in self.ev_back:
            e.record(self.s_back)
        # TETRA_ETSI_FRONT2=1 (fused demod, device-resident input): consecutive batches' demods on two
        # front streams (contexts), so one batch's last workgroups and the next batch's first ones overlap
        # instead of draining the chip at every launch boundary
        self.front2 = None
        if (os.environ.get("TETRA_ETSI_FRONT2") == "1" and self.demod_mode == "fused"
                and not getattr(self, "hostfed", False)):
            self.front2 = _hip.Context()
            self.s_front2 = torch.cuda.Stream(device=dev)
            self.front2.check(self.front2.lib.tetra_set_stream(self.front2.handle,
                                                               ctypes.c_void_p(self.s_front2.cuda_stream)), "set_stream")
        self.k = 0
        self.pipelined = True
        return self

    def contexts(self):
        return ([self.c] + ([self.back] if self.pipelined else [])
                + ([self.front2] if getattr(self, "front2", None) is not None else []))

    def host_feed(self):
        """PCIe-inclusive mode (bench.py --host-input): every step's batch starts in pinned host
        memory and is copied host -> device on a copy stream, double-buffered, so batch k+1's copy
        overlaps batch k's demod -- the rate a host-fed receiver (SDR capture buffers) would see.
        Never the headline `value` (that is measured with the input resident in HBM)."""
        import torch
        if self.chunks > 1:
            raise ValueError("host-fed mode streams one resident batch (chunks=1)")
        dev = self.iq.device
        self.host = self.iq.cpu().pin_memory()
        self.dbuf = [self.iq, torch.empty_like(self.iq)]
        self.s_copy = torch.cuda.Stream(device=dev)
        self.ev_copied = [torch.cuda.Event() for _ in range(2)]
        self.ev_used = [torch.cuda.Event() for _ in range(2)]
        for e in self.ev_used:
            e.record(torch.cuda.current_stream(dev))
        self.kin = 0
        self.hostfed = True
        return self

    def _input(self):
        """Device input of this step: the resident batch, or (host-fed) the freshly copied buffer."""
        if not getattr(self, "hostfed", False):
            x = self.iqs[self.kchunk % self.chunks]
            self.kchunk += 1
            return x
        import torch
        i = self.kin & 1
        self.kin += 1
        with torch.cuda.stream(self.s_copy):
            self.s_copy.wait_event(self.ev_used[i])            # the demod two steps back is done with it
            self.dbuf[i].copy_(self.host, non_blocking=True)
            self.ev_copied[i].record(self.s_copy)
        front = self.s_front if self.pipelined else torch.cuda.current_stream(self.iq.device)
        front.wait_event(self.ev_copied[i])
        self._used = (self.ev_used[i], front)
        return self.dbuf[i]

    def _demod(self, c, sym, soft, hard, nsym):
        if self.stream:
            self._demod_stream(c, sym, soft, hard, nsym)
            return
        x = self._input()
        c.check(c.lib.tetra_demod_etsi_fmt(c.handle, self.plan, _hip.ptr(x), self.fmt, self.C, self.N,
                                           _hip.ptr(sym), _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), self.smax,
                                           None), "demod_etsi")
        if getattr(self, "hostfed", False):
            ev, st = self._used
            ev.record(st)

    def _demod_stream(self, c, sym, soft, hard, nsym):
        """Chunk kchunk of every channel's capture: its window in place in the capture rows."""
        k = self.kchunk % self.chunks
        # the stream continues only into the chunk after the last one; anything else -- past the
        # capture's end, or a caller that moved kchunk -- starts a new capture at chunk k (the
        # windows never leave the resident capture)
        if k != self._next_k:
            self.x_total = self.y_done = 0
            with _on_stream(c):
                self.track.zero_()
            self._reset_lead = True
            self.resets += 1
            self._origin = k * self.N
        self._next_k = k + 1
        self.kchunk += 1
        s, W, yoff, y_next = stream_window(self.plan, self.x_total, self.y_done, self.N)
        bps = 4 if self.fmt == _hip.TETRA_SC16 else 8
        _, _, sm = lengths(self.plan, W)
        off = self._origin + s
        assert off + W <= self.N * self.chunks, (off, W)
        c.check(c.lib.tetra_demod_etsi_stream(
            c.handle, self.plan, ctypes.c_void_p(self.cap.data_ptr() + bps * off), self.fmt, self.C,
            self.N * self.chunks, W, int(yoff), _hip.ptr(self.track), ctypes.c_void_p(sym.data_ptr() + 8 * RESERVE),
            ctypes.c_void_p(soft.data_ptr() + 2 * RESERVE), ctypes.c_void_p(hard.data_ptr() + RESERVE),
            _hip.ptr(nsym), min(sm + 1, self.smax), self.stride, None), "demod_etsi_stream")
        self.x_total += self.N
        self.y_done = y_next

    def _lmac(self, c, soft, hard, nsym):
        if self.stream:
            i = [b[2].data_ptr() for b in self.bufs].index(hard.data_ptr())
            nsoft, nhard = self.bufs[i ^ 1][1], self.bufs[i ^ 1][2]
            if getattr(self, "_reset_lead", False):   # a new capture: no carried dibits
                with _on_stream(c):
                    self.lead.fill_(2 * RESERVE)
                self._reset_lead = False
            acq = self.cells_mode == "acquire"
            c.check(c.lib.tetra_lmac_etsi_stream(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), self.C,
                                                 self.stride, _hip.ptr(self.lead), _hip.ptr(nsoft), _hip.ptr(nhard),
                                                 _hip.ptr(self.cell_state) if acq else None, _hip.ptr(self.nburst),
                                                 _hip.ptr(self.bursts), _hip.ptr(self.nblock), _hip.ptr(self.blocks),
                                                 _hip.ptr(self.type1)), "lmac_etsi_stream")
            return
        if self.cells_mode == "acquire":
            c.check(c.lib.tetra_lmac_etsi_acquire(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), self.C,
                                                  self.smax, _hip.ptr(self.cell_state), _hip.ptr(self.nburst),
                                                  _hip.ptr(self.bursts), _hip.ptr(self.nblock), _hip.ptr(self.blocks),
                                                  _hip.ptr(self.type1)), "lmac_etsi_acquire")
            return
        c.check(c.lib.tetra_lmac_etsi(c.handle, _hip.ptr(soft), _hip.ptr(hard), _hip.ptr(nsym), self.C, self.smax,
                                      _hip.ptr(self.nburst), _hip.ptr(self.bursts), _hip.ptr(self.nblock),
                                      _hip.ptr(self.blocks), _hip.ptr(self.type1)), "lmac_etsi")

    def _chanfilt(self, c, y):
        x = self._input()
        c.check(c.lib.tetra_etsi_chanfilt_fmt(c.handle, self.plan, _hip.ptr(x), self.fmt, self.C, self.N,
                                              _hip.ptr(y)), "chanfilt")
        if getattr(self, "hostfed", False):
            ev, st = self._used
            ev.record(st)

    def _timing(self, c, y):
        c.check(c.lib.tetra_etsi_timing(c.handle, self.plan, _hip.ptr(y), self.C, self.M2, _hip.ptr(self.sym),
                                        _hip.ptr(self.soft), _hip.ptr(self.hard), _hip.ptr(self.nsym), self.smax,
                                        None), "timing")

    def __call__(self):
        split = self.demod_mode == "split"
        if not self.pipelined:
            if split:
                self._chanfilt(self.c, self.y[0])
                self._timing(self.c, self.y[0])
            elif self.stream:   # the rows alternate: a chunk's lower MAC puts its tail in front of the next's
                sym, soft, hard, nsym = self.bufs[self.kchunk & 1]
                self._demod(self.c, sym, soft, hard, nsym)
                self._lmac(self.c, soft, hard, nsym)
                return
            else:
                self._demod(self.c, self.sym, self.soft, self.hard, self.nsym)
            self._lmac(self.c, self.soft, self.hard, self.nsym)
            return
        i = self.k & 1
        if split:
            self.k += 1
            self.s_front.wait_event(self.ev_back[i])    # timing of batch k-2 has consumed y[i]
            self._chanfilt(self.c, self.y[i])
            self.ev_front[i].record(self.s_front)
            self.s_back.wait_event(self.ev_front[i])
            self._timing(self.back, self.y[i])
            self._lmac(self.back, self.soft, self.hard, self.nsym)
            self.ev_back[i].record(self.s_back)
            return
        self.k += 1
        sym, soft, hard, nsym = self.bufs[i]
        fc, fs = (self.front2, self.s_front2) if self.front2 is not None and i else (self.c, self.s_front)
        fs.wait_event(self.ev_back[i])                  # lower MAC of batch k-2 has consumed buffer i
        self._demod(fc, sym, soft, hard, nsym)
        self.ev_front[i].record(fs)
        self.s_back.wait_event(self.ev_front[i])
        self._lmac(self.back, soft, hard, nsym)
        self.ev_back[i].record(self.s_back)

    def kernel_info(self):
        """(symbol, static LDS bytes) of the channel-filter kernel this step's demod launches, asked
        from the library (tetra_etsi_kernel_info), so the bench follows the kernels as they change."""
        name = ctypes.create_string_buffer(64)
        lds = ctypes.c_int64(0)
        self.c.check(self.c.lib.tetra_etsi_kernel_info(self.c.handle, self.plan, self.fmt, self.N,
                                                       int(self.demod_mode == "fused"), name, 64, ctypes.byref(lds)),
                     "tetra_etsi_kernel_info")
        return name.value.decode(), lds.value

    def dominant(self):
        # fused demod: reads 8 B (cf32) or 4 B (SC16) per input sample; writes per symbol (0.0075 per
        # input sample) 8 B cf32 symbol + 2 B soft bits + 1 B hard dibit.  split: the same reads,
        # writes y (8 B per 72 kHz sample = 0.24 B per input sample).
        rd = 4.0 if self.fmt == _hip.TETRA_SC16 else 8.0
        sym = self.kernel_info()[0]
        if self.demod_mode == "split":
            return ("etsi_chanfilt", rd + 8.0 * self.M2 / self.N, sym)
        return ("etsi_demod", rd + 11.0 * 18000.0 / self.fs, sym)

    def floor_args(self):
        """bench.py's read floor over this batch: one row per channel at the demod kernel's own LDS
        footprint (so as many workgroups per CU as the kernel gets)."""
        row = self.N * (4 if self.fmt == _hip.TETRA_SC16 else 8)
        if self.stream:   # rows of the resident capture are chunks N apart: the floor reads one chunk
            x = self.cap[:, :self.N].contiguous() if not hasattr(self, "_floor_x") else self._floor_x
            self._floor_x = x
            return _hip.ptr(x), self.C, row, self.kernel_info()[1]
        return _hip.ptr(self.iq), self.C, row, self.kernel_info()[1]

    def quality(self):
        """Decoded-block statistics of the last step (device results, checked on the host); with
        cell acquisition also how many channels hold the synthesised cell.  Streaming: the bursts the
        step decoded per channel against the slots on air in one chunk (N / 34000 at 2.4 MSps: a
        255-symbol slot is 34000 samples) -- the fraction of the transmitted bursts decoded."""
        nb = self.nblock.cpu().numpy()
        blocks = self.blocks.cpu().numpy()
        ok = sum(int(blocks[i, :nb[i], 1].sum()) for i in range(self.C))
        q = dict(blocks=int(nb.sum()), crc_ok=ok, bursts=int(self.nburst.sum().item()),
                 crc_ok_frac=round(ok / max(1, int(nb.sum())), 5))
        if self.chunks > 1:
            q["chunk"] = (self.kchunk - 1) % self.chunks   # the batch the last step decoded
        if self.stream:
            on_air = self.N * 18000.0 / 255.0 / self.fs
            q["stream"] = True
            q["bursts_per_channel_chunk"] = round(q["bursts"] / self.C, 4)
            q["on_air_per_channel_chunk"] = round(on_air, 4)
            q["decoded_frac"] = round(q["bursts"] / self.C / on_air, 4)
            q["stream_resets"] = self.resets
        if self.cells_mode == "acquire":
            q["cells_acquired"] = int((self.cell_state == self.cells).sum().item())
        return q


def smoke_check():
    """Tiny ETSI round trip on the GPU (used by __graft_entry__.smoke)."""
    from tetraear.core.etsi import EtsiLowerMac
    iq, cells, kinds, payload, t0 = synth(2, 131072, seed=7, snr_db=20.0)
    rx = EtsiReceiver()
    lm = EtsiLowerMac()
    hard, soft, sym, ns = rx.demod_batch(iq)
    res = lm.decode_batch(soft, hard, ns, cells)
    nok = 0
    for ch, frames in enumerate(res):
        sent = {tuple(p) for bb in payload[ch] for p in bb}
        for f in frames:
            for b in f["blocks"]:
                if b["crc_ok"]:
                    nok += 1
                    padded = tuple(np.pad(b["bits"], (0, 268 - len(b["bits"]))))
                    assert padded in sent, "decoded payload is not a transmitted block"
    assert nok >= 4, f"ETSI smoke: only {nok} blocks passed CRC"
