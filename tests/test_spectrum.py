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


# ------------------------------------------------------------------ signal-present / AFC gate
# SURVEY.md §8f rank 1 (/root/reference/tetraear/ui/modern.py:1952-2028).  Known answers: a comb
# filling the 25 kHz centre band (alternating-sign tones on every band bin, so the Hann leakage
# adds up flat) with one bin raised by g, plus white noise sigma.  Each case flips one threshold.
GATE_FS = 2.4e6
BIN_HZ = GATE_FS / 2048   # 1171.875


def _comb(A, g, kp, sigma, N=131072, seed=0, fs=GATE_FS):
    rng = np.random.default_rng(seed)
    n = np.arange(N)
    start, end, _, _ = S.gate_bins(fs)
    x = np.zeros(N, np.complex128)
    for b in range(start, end):
        x += A * (g if b == kp else 1.0) * (-1.0) ** b * np.exp(2j * np.pi * (b - 1024) * n / 2048)
    x += sigma * (rng.standard_normal(N) + 1j * rng.standard_normal(N))
    return x.astype(np.complex64)


# (A, g, peak bin, sigma) -> (present, the threshold it sits on)
GATE_KATS = [
    ((0.01, 4, 1030, 1e-4), True, "present, peak 6 bins up"),
    ((0.01, 4, 1014, 1e-4), True, "present, peak on the band's first bin"),
    ((0.001, 4, 1030, 0.01), True, "snr 17 > 15"),
    ((0.001, 4, 1030, 0.02), False, "snr 11 < 15"),
    ((3e-4, 4, 1020, 1e-6), True, "peak -62.5 > -70"),
    ((1e-4, 4, 1020, 1e-6), False, "peak -72 < -70"),
    ((0.01, 2, 1020, 1e-4), True, "peak - mean 3.4 > 3"),
    ((0.01, 1.6, 1020, 1e-4), False, "peak - mean 2.3 < 3"),
]


def test_gate_oracle_known_answers():
    """The oracle gate on the comb KATs: band = bins 1014..1033 at 2.4 MSps (int(25000 / 1171.875) = 21
    bins, 10 each side of bin 1024, the upper one exclusive), noise from bins < 1004 and >= 1044;
    the peak bin's offset is (bin - 1024) x 1171.875 Hz and is the AFC offset exactly when the three
    thresholds pass; each threshold flips the decision on its own."""
    assert S.gate_bins(GATE_FS) == (1014, 1034, 1004, 1044)
    assert S.gate_bins(1.8e6) == (1010, 1038, 1000, 1048)   # 878.9 Hz bins: 28
    for args, present, why in GATE_KATS:
        g = S.gate_iq(_comb(*args), GATE_FS)
        assert g["valid"] == 1.0 and bool(g["present"]) == present, (why, g)
        assert g["peak_bin"] == args[2] and g["peak_freq"] == (args[2] - 1024) * BIN_HZ, why
        assert g["afc"] == (g["peak_freq"] if present else 0.0), why
    assert S.gate_iq(np.zeros(2047, np.complex64), GATE_FS)["valid"] == 0.0   # < 2048 samples: no detection


def _gate_vs_oracle(got, x, fs, i=None):
    """GPU gate row vs the float64 oracle: dB statistics within GATE_DB_TOL; the decision and peak
    bin equal whenever the oracle's margins exceed that tolerance (no case here sits in the band)."""
    want = S.gate_iq(x, fs)
    pick = (lambda k: float(got[k])) if i is None else (lambda k: float(got[k][i]))
    for k in ("signal", "peak", "noise", "snr", "above"):
        assert abs(pick(k) - want[k]) <= GATE_DB_TOL, (k, pick(k), want[k])
    assert pick("valid") == want["valid"] and pick("present") == want["present"]
    assert pick("peak_bin") == want["peak_bin"] and pick("peak_freq") == want["peak_freq"]
    assert pick("afc") == want["afc"]
    return want


GATE_DB_TOL = 2e-3   # fp32 FFT vs float64, averaged dB over the band / the noise bins (measured ~1e-4)


@pytest.mark.gpu
def test_gate_gpu_known_answers_and_formats():
    """tetra_afc_gate (fused into the waterfall kernel) on the KATs, one batch: statistics within
    GATE_DB_TOL of the oracle, decisions / peak bins / AFC offsets identical; SC16 input (the
    capture's wire format) and complex128 give the same decisions; fewer than 2048 samples: no
    detection."""
    from tetraear.signal.spectrum import afc_gate
    x = np.stack([_comb(*args, seed=i) for i, (args, _, _) in enumerate(GATE_KATS)])
    got = afc_gate(x, GATE_FS, power=True, mixer=True)
    for i, (args, present, why) in enumerate(GATE_KATS):
        want = _gate_vs_oracle(got, x[i], GATE_FS, i)
        assert bool(got["present"][i]) == present, why
        f = want["afc"]
        assert got["mixer_on"][i] == (f != 0) and got["mixer_coef"][i] == (-2 * np.pi * f if f else 0.0)
    ref = np.stack([S.frame_power(v) for v in x])
    near = ref >= ref.max(axis=1, keepdims=True) - 80.0   # the fused row is the waterfall's (tolerances above)
    assert np.abs(got["power"] - ref)[near].max() < 0.05
    sc = np.stack([np.rint(x.real * 32768), np.rint(x.imag * 32768)], -1).clip(-32768, 32767).astype(np.int16)
    g16 = afc_gate(sc, GATE_FS)
    big = [i for i, (a, _, _) in enumerate(GATE_KATS) if a[0] >= 1e-3]   # the SC16 grid (3e-5) hides the weak ones
    assert np.array_equal(g16["present"][big], got["present"][big])
    g64 = afc_gate(x.astype(np.complex128), GATE_FS)
    assert np.array_equal(g64["present"], got["present"]) and np.array_equal(g64["peak_bin"], got["peak_bin"])
    short = afc_gate(x[:, :2047], GATE_FS, mixer=True)
    assert not short["valid"].any() and not short["present"].any() and not short["mixer_on"].any()


@pytest.mark.gpu
@pytest.mark.parametrize("fs", [1.8e6, 2.4e6])
def test_gate_gpu_tetra_chunks_vs_oracle(fs):
    """The gate on TETRA-like chunks (the ETSI synthesiser's pi/4-DQPSK bursts, CFO up to 600 Hz,
    Es/N0 10-25 dB, and pure-noise channels): GPU equals the oracle (tolerance above) channel by
    channel at both ends of the reference's rate range."""
    from tetraear.signal.etsi import synth
    from tetraear.signal.spectrum import afc_gate
    N = 2 * int(131072 * fs / 2.4e6 / 2)
    xs = [synth(4, N, fs=fs, seed=s, snr_db=snr)[0] for s, snr in ((1, 25.0), (2, 10.0))]
    rng = np.random.default_rng(9)
    noise = (1e-3 * (rng.standard_normal((2, N)) + 1j * rng.standard_normal((2, N)))).astype(np.complex64)
    x = np.concatenate(xs + [noise])
    got = afc_gate(x, fs)
    npres = 0
    for i in range(len(x)):
        npres += _gate_vs_oracle(got, x[i], fs, i)["present"]
    assert not got["present"][-2:].any()   # noise alone: never present


@pytest.mark.gpu
def test_process_batch_afc_feeds_the_demod_on_device():
    """SignalProcessor.process_batch(x, 'afc'): the gate's offsets go to the compat demod as device
    arrays.  Every channel equals process(x[c], freq_offset = the gate's AFC offset) -- what the
    capture loop does per chunk (modern.py:2028-2029) -- and a device tensor of offsets gives the
    same rows as the host array."""
    import torch
    from tetraear.signal import SignalProcessor
    offs = [0, 3, -5, 7]
    x = np.stack([_comb(0.01, 4, 1024 + k, 1e-4, seed=k + 20) for k in offs])
    p = SignalProcessor(GATE_FS, mode="compat")
    hard, soft, ns = p.process_batch(x, "afc")
    assert np.array_equal(p.gate["afc"], np.array(offs) * BIN_HZ) and p.gate["present"].all()
    for c in range(len(x)):
        h = p.process(x[c], freq_offset=float(p.gate["afc"][c]))
        n = int(ns[c])
        assert np.array_equal(hard[c, :n - 1], h), c
    fo = torch.tensor(np.array(offs) * BIN_HZ, dtype=torch.float64, device="cuda")
    h2, s2, n2 = p.process_batch(x, fo)
    h3, s3, n3 = p.process_batch(x, np.array(offs) * BIN_HZ)
    assert np.array_equal(h2, hard) and np.array_equal(s2, soft) and np.array_equal(h3, hard) and np.array_equal(n3, ns)
    # device-tensor samples: the format follows the dtype, a strided view is made contiguous first
    xt = torch.from_numpy(x).to("cuda")
    h4, s4, n4 = p.process_batch(xt, fo)
    assert np.array_equal(h4, hard) and np.array_equal(s4, soft) and np.array_equal(n4, ns)
    h5, _, n5 = p.process_batch(torch.view_as_real(xt), fo)                      # float32 [C, N, 2]
    assert np.array_equal(h5, hard) and np.array_equal(n5, ns)
    wide = torch.zeros((len(x), 2 * x.shape[1]), dtype=torch.complex64, device="cuda")
    wide[:, ::2] = xt
    h6, _, n6 = p.process_batch(wide[:, ::2], fo)                                # non-contiguous view
    assert np.array_equal(h6, hard) and np.array_equal(n6, ns)
    x128 = x.astype(np.complex128)
    h7, s7, n7 = p.process_batch(torch.from_numpy(x128).to("cuda"), fo)          # complex128: the cf64 chain
    h8, s8, n8 = p.process_batch(x128, np.array(offs) * BIN_HZ)
    assert np.array_equal(h7, h8) and np.array_equal(s7, s8) and np.array_equal(n7, n8)
    with pytest.raises(TypeError):
        p.process_batch(torch.zeros((2, 4096), dtype=torch.int32, device="cuda"), fo[:2])
