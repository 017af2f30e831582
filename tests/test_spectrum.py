"""Waterfall spectrum (SURVEY.md §8d C3 "2048-pt Hann waterfall"): oracle known answers on the CPU,
GPU parity against oracle/spectrum.py.

Tolerance (the GPU computes window + FFT in fp32, the oracle in float64 as numpy does):
  * linear: | |X|/N (GPU) - |X|/N (oracle) | <= MAG_TOL x the frame's largest |X|/N;
  * dB: within DB_TOL for every bin within 40 dB of the frame's peak.
An fp32 FFT of this size lands near 4e-8 of the peak (numpy complex64 FFT, measured here).
"""
import numpy as np
import pytest

import spectrum as S

MAG_TOL = 1e-6
DB_TOL = 5e-3


def _signal(rng, C, N, fmt_scale=0.4):
    n = np.arange(N)
    x = np.zeros((C, N), np.complex128)
    for c in range(C):
        for _ in range(3):
            f = rng.uniform(-0.5, 0.5)
            x[c] += rng.uniform(0.05, fmt_scale) * np.exp(2j * np.pi * (f * n + rng.uniform()))
        x[c] += 1e-3 * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
    return x.astype(np.complex64)


def _compare(got, x, hop, nframes):
    mag = S.waterfall(x, hop, nframes, magnitude=True)
    db = S.waterfall(x, hop, nframes)
    got_mag = 10.0 ** (got.astype(np.float64) / 20.0) - 1e-20
    peak = mag.max(axis=-1, keepdims=True)
    err = np.abs(got_mag - mag) / peak
    assert err.max() <= MAG_TOL, f"linear error {err.max():.3g} of the frame peak"
    strong = db >= 20 * np.log10(peak) - 40
    assert np.abs(got - db)[strong].max() <= DB_TOL


# ------------------------------------------------------------------------- CPU: oracle pinned
def test_oracle_matches_direct_dft():
    rng = np.random.default_rng(3)
    x = _signal(rng, 1, 2048)[0]
    assert np.abs(S.frame_power(x) - S.dft_power(x)).max() < 1e-6


def test_oracle_hann_known_answers():
    """A tone of amplitude A exactly on bin k: Hann coherent gain (N-1)/(2N) at shifted index
    k + N/2 (exact: sum(hanning(N)) = (N-1)/2), about half of that on both neighbours (the
    symmetric window is not the periodic one: +0.07 %), leakage 75 dB down elsewhere."""
    N, k, A = 2048, 300, 0.25
    x = A * np.exp(2j * np.pi * k * np.arange(N) / N)
    m = S.frame_magnitude(x)
    assert np.isclose(m[k + N // 2], A * (N - 1) / (2 * N), rtol=1e-12)
    assert np.isclose(m[k + N // 2 - 1], A * (N - 1) / (4 * N), rtol=1e-3)
    assert np.isclose(m[k + N // 2 + 1], A * (N - 1) / (4 * N), rtol=1e-3)
    far = np.delete(m, [k + N // 2 - 1, k + N // 2, k + N // 2 + 1])
    assert far.max() < 2e-4 * m.max()
    assert np.isclose(S.frame_power(np.zeros(N))[0], -400.0)


def test_waterfall_frames_layout():
    rng = np.random.default_rng(4)
    x = _signal(rng, 2, 6000)
    w = S.waterfall(x, hop=1000)
    assert w.shape == (2, 4, 2048)
    assert np.array_equal(w[1, 2], S.frame_power(x[1, 2000:4048]))


# ------------------------------------------------------------------------- GPU parity
@pytest.mark.gpu
def test_waterfall_cf32_vs_oracle():
    from tetraear.signal.spectrum import waterfall
    rng = np.random.default_rng(5)
    x = _signal(rng, 3, 20000)
    hop = 1500   # overlapping frames
    got = waterfall(x, hop=hop)
    assert got.shape == (3, (20000 - 2048) // hop + 1, 2048) and got.dtype == np.float32
    _compare(got, x, hop, got.shape[1])


@pytest.mark.gpu
def test_waterfall_formats_bit_identical():
    """SC16 (int16 pairs scaled 1/32768 on the device) and complex128 (rounded to fp32 on the
    device) give exactly the cf32 result of the same fp32 samples."""
    from tetraear.signal.spectrum import waterfall
    rng = np.random.default_rng(6)
    q = rng.integers(-20000, 20000, size=(2, 8192, 2), dtype=np.int16)
    x32 = (q[..., 0].astype(np.float32) / 32768 + 1j * (q[..., 1].astype(np.float32) / 32768)).astype(np.complex64)
    a = waterfall(q, hop=2048)
    b = waterfall(x32, hop=2048)
    c = waterfall(x32.astype(np.complex128), hop=2048)
    assert np.array_equal(a, b) and np.array_equal(b, c)
    _compare(b, x32, 2048, 4)


@pytest.mark.gpu
def test_spectrum_matches_reference_display():
    """spectrum() = the (freqs + centre, power) pair of the reference's capture loop for a 128 Ki
    chunk (only x[:2048] is used), including an all-zero chunk (-400 dB everywhere)."""
    from tetraear.signal.spectrum import spectrum
    rng = np.random.default_rng(7)
    x = _signal(rng, 1, 131072)[0]
    f, p = spectrum(x, 2.4e6, 390.5e6)
    assert np.array_equal(f, np.fft.fftshift(np.fft.fftfreq(2048, 1 / 2.4e6)) + 390.5e6)
    _compare(p[None, None], x[None, :2048], 2048, 1)
    _, z = spectrum(np.zeros(4096, np.complex64), 2.4e6)
    assert np.allclose(z, -400.0, atol=1e-3)


@pytest.mark.gpu
def test_waterfall_device_tensor_and_many_frames():
    """Device (torch) input at a C3-sized frame count: same bits as the host path, and Parseval
    per frame (sum |X|^2 = N sum |x w|^2) as a size-independent check on every frame."""
    import torch
    from tetraear.signal.spectrum import waterfall
    rng = np.random.default_rng(8)
    nfr = 4882                       # 10 M samples of a 20 MSps capture at hop 2048
    x = (0.3 * (rng.standard_normal(nfr * 2048) + 1j * rng.standard_normal(nfr * 2048))).astype(np.complex64)
    d = waterfall(torch.from_numpy(x).cuda())
    h = waterfall(x)
    assert d.shape == (nfr, 2048) and np.array_equal(d.cpu().numpy(), h)
    w = np.hanning(2048)
    xw = x.reshape(nfr, 2048).astype(np.complex128) * w
    e_time = 2048 * np.sum(np.abs(xw) ** 2, axis=1)
    e_freq = np.sum((10.0 ** (h.astype(np.float64) / 20.0) * 2048) ** 2, axis=1)
    assert np.abs(e_freq / e_time - 1).max() < 1e-5
    # spot-check frames against the oracle
    for f in (0, 1, 2047, nfr - 1):
        _compare(h[f][None, None], x[None, f * 2048:(f + 1) * 2048], 2048, 1)


@pytest.mark.gpu
def test_waterfall_rejects_bad_requests():
    from tetraear import _hip
    from tetraear.signal.spectrum import waterfall
    x = np.zeros(4096, np.complex64)
    with pytest.raises(_hip.TetraHipError):
        waterfall(x, hop=2048, nframes=3)     # the third frame runs past the end
    with pytest.raises(_hip.TetraHipError):
        waterfall(x, nfft=1024)
    with pytest.raises(ValueError):
        waterfall(np.zeros(100, np.complex64))
