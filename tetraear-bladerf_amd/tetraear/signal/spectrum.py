"""Waterfall / live spectrum on the GPU (BASELINE.json north_star
"waterfall FFT").

The reference computes its live spectrum inline in the capture loop
(/root/reference/tetraear/ui/modern.py:1928-1941): x[:2048] * numpy.hanning(2048), FFT, fftshift,
20 log10(|X| / 2048 + 1e-20) dBFS, and emits (freqs + centre frequency, power) to the GUI.
``spectrum()`` returns that same pair from libtetra_hip.so's fused kernel (k_waterfall: window +
LDS FFT + shift + dB in one pass over HBM); ``waterfall()`` batches frames over channels and
time (a [C][N] batch, or a wideband capture at hop 2048).  Host arrays (numpy) or device arrays
(torch tensors on the GPU) in; the output lives where the input did.  No CPU fallback.
"""
import numpy as np

from tetraear import _hip

N_FFT = 2048


def _fmt(a):
    """(TETRA format, [C][N] view, is_device) of a sample array."""
    if hasattr(a, "data_ptr"):   # torch tensor: complex64, complex128, or [..., 2] int16 / float32 pairs
        import torch
        if a.dtype == torch.complex64:
            return _hip.TETRA_CF32, a, True
        if a.dtype == torch.complex128:
            return _hip.TETRA_CF64, a, True
        if a.dtype == torch.int16 and a.shape[-1] == 2:
            return _hip.TETRA_SC16, a[..., 0], True
        if a.dtype == torch.float32 and a.shape[-1] == 2:
            return _hip.TETRA_CF32, a[..., 0], True
        raise TypeError(f"unsupported tensor dtype {a.dtype} (complex64/complex128 or [..., 2] int16/float32)")
    a = np.asarray(a)
    if a.dtype == np.int16 and a.shape[-1] == 2:
        return _hip.TETRA_SC16, a[..., 0], False
    if a.dtype == np.complex128:
        return _hip.TETRA_CF64, a, False
    return _hip.TETRA_CF32, a, False


def waterfall(iq, hop=N_FFT, nframes=None, nfft=N_FFT):
    """iq [C][N] or [N] samples (complex64/complex128, or int16 [..., 2] SC16 as captured) ->
    float32 dBFS rows [C][nframes][nfft] (or [nframes][nfft]); frame f covers samples
    [f hop, f hop + nfft).  nframes defaults to every whole frame."""
    fmt, shape_of, dev = _fmt(iq)
    if not dev:
        want = {_hip.TETRA_CF32: np.complex64, _hip.TETRA_CF64: np.complex128, _hip.TETRA_SC16: np.int16}[fmt]
        iq = np.ascontiguousarray(iq, want)
    else:
        iq = iq.contiguous()
    one = len(shape_of.shape) == 1
    C = 1 if one else shape_of.shape[0]
    N = shape_of.shape[-1]
    if N < nfft:
        raise ValueError(f"{N} samples are fewer than one {nfft}-point frame")
    if nframes is None:
        nframes = (N - nfft) // hop + 1
    if dev:
        import torch
        out = torch.empty((C, nframes, nfft), dtype=torch.float32, device=iq.device)
    else:
        out = np.empty((C, nframes, nfft), np.float32)
    c = _hip.ctx()
    c.check(c.lib.tetra_waterfall(c.handle, _hip.ptr(iq), fmt, C, N, nfft, hop, nframes, _hip.ptr(out)), "waterfall")
    return out[0] if one else out


def spectrum(samples, sample_rate, center_freq=0.0, nfft=N_FFT):
    """(freqs_actual, power) of samples[:nfft] as the reference's capture loop emits them
    (modern.py:1928-1941): the frequency axis is fftshift(fftfreq(nfft, 1/fs)) + centre."""
    if not hasattr(samples, "data_ptr"):
        samples = np.asarray(samples)[:nfft]   # 1-D complex chunk, or [N, 2] int16 SC16
    power = waterfall(samples, hop=nfft, nframes=1, nfft=nfft)[0]
    freqs = np.fft.fftshift(np.fft.fftfreq(nfft, 1 / sample_rate)) + center_freq
    return freqs, power


GATE_FIELDS = ("valid", "signal", "peak", "peak_bin", "peak_freq", "noise", "snr", "above", "present", "afc")


def afc_gate(iq, sample_rate, power=False, mixer=False):
    """The capture loop's signal-present / AFC gate (modern.py:1952-2028) for every channel of a
    [C][N] batch (or one [N] chunk), on the GPU (tetra_afc_gate: fused into the waterfall kernel's
    frame-0 row).  Returns a dict of [C] arrays over GATE_FIELDS -- band mean ``signal``, ``peak`` and
    ``peak_bin`` / ``peak_freq``, ``noise`` floor, ``snr``, ``above`` (peak - mean), ``present`` and
    ``afc`` (the freq_offset the loop hands process()) -- plus ``power`` [C][2048] (power=True) and the
    compat demod's mixer inputs ``mixer_coef`` / ``mixer_on`` (mixer=True).  Device (torch) input
    keeps every output on the device."""
    fmt, shape_of, dev = _fmt(iq)
    if not dev:
        want = {_hip.TETRA_CF32: np.complex64, _hip.TETRA_CF64: np.complex128, _hip.TETRA_SC16: np.int16}[fmt]
        iq = np.ascontiguousarray(iq, want)
    else:
        iq = iq.contiguous()
    one = len(shape_of.shape) == 1
    C = 1 if one else shape_of.shape[0]
    N = shape_of.shape[-1]
    if dev:
        import torch
        mk = lambda shape, dt: torch.zeros(shape, dtype=getattr(torch, dt), device=iq.device)   # noqa: E731
    else:
        mk = lambda shape, dt: np.zeros(shape, getattr(np, dt))   # noqa: E731
    stats = mk((C, len(GATE_FIELDS)), "float64")
    pw = mk((C, N_FFT), "float32") if power and N >= N_FFT else None
    mc = mk((C,), "float64") if mixer else None
    mo = mk((C,), "uint8") if mixer else None
    c = _hip.ctx()
    c.check(c.lib.tetra_afc_gate(c.handle, _hip.ptr(iq), fmt, C, N, float(sample_rate),
                                 _hip.ptr(pw) if pw is not None else None, _hip.ptr(stats),
                                 _hip.ptr(mc) if mc is not None else None, _hip.ptr(mo) if mo is not None else None),
            "tetra_afc_gate")
    out = {k: (stats[0, i] if one else stats[:, i]) for i, k in enumerate(GATE_FIELDS)}
    if pw is not None:
        out["power"] = pw[0] if one else pw
    if mixer:
        out["mixer_coef"], out["mixer_on"] = mc, mo
    return out
